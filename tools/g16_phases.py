"""Phase spans of the last Groth16 prove in a rocprofv3 kernel trace
(tools/prof_g16.py run): witness map, then each MSM (k_decompose_var starts)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if "k_assign" in r["Kernel_Name"]]
last = sorted(rows[idx[-1]:], key=lambda r: int(r["Start_Timestamp"]))
t0 = int(last[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in last)
marks = [r for r in last if any(k in r["Kernel_Name"] for k in ("k_decompose_var", "k_assign", "k_qap", "k_xyzz_to_affine"))]
for r in marks:
    print("%8.3f %s" % ((int(r["Start_Timestamp"]) - t0) / 1e6, r["Kernel_Name"][:70]))
print("end %8.3f ms, %d kernels" % ((end - t0) / 1e6, len(last)))
agg = defaultdict(lambda: [0, 0])
for r in last:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    agg[n][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[n][1] += 1
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:16]:
    print("%8.3f ms %4d  %s" % (v[0] / 1e6, v[1], k))
