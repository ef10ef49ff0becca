"""Timeline of the last span of a rocprofv3 kernel trace starting at the last
launch whose name contains START (e.g. k_assign for a Groth16 prove): queue,
start (ms from the span's start), duration, kernel, grid.

    python tools/span_timeline.py TRACE.csv START [LIMIT]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
             r.get("Queue_Id", "?")) for r in rows)
i0 = max(i for i, e in enumerate(ev) if sys.argv[2] in e[2])
seg = ev[i0:]
lim = int(sys.argv[3]) if len(sys.argv) > 3 else len(seg)
short = lambda n: re.sub(r"tpst::|\(anonymous namespace\)::|unsigned int|unsigned long|const|\*|void|\(.*", "", n)[:58]
t0 = seg[0][0]
print("span %.3f ms, %d kernels" % ((max(e[1] for e in seg) - t0) / 1e6, len(seg)))
for s, e, n, g, q in seg[:lim]:
    print("q%-3s %8.3f %7.3f  %-58s grid %d" % (q, (s - t0) / 1e6, (e - s) / 1e6, short(n), g))
