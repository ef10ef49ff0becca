"""Timeline of the last variable-base MSM in a rocprofv3 kernel trace (from its
k_decompose_hist to the end of its k_window_chain): queue, start (ms from the
MSM's start), duration, kernel, grid -- to read the accumulation / reduction /
chain overlap of the window-grouped pipeline (csrc/msm.hip msm_var)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
             r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows)
starts = [i for i, e in enumerate(ev) if "k_decompose" in e[2]]
i0 = starts[-2] if len(starts) > 1 else starts[-1]  # the last complete MSM
i1 = starts[starts.index(i0) + 1] if starts.index(i0) + 1 < len(starts) else len(ev)
seg = ev[i0:i1]
short = lambda n: re.sub(r"tpst::|unsigned int|unsigned long|const|\*|void|\(.*", "", n)[:60]
t0 = seg[0][0]
end = max(e[1] for e in seg)
print("MSM span %.3f ms, %d kernels" % ((end - t0) / 1e6, len(seg)))
for s, e, n, g, q in seg:
    print("q%-3s %8.3f %7.3f  %-60s grid %d" % (q, (s - t0) / 1e6, (e - s) / 1e6, short(n), g))
