"""Timeline of the last sqrt-PST open in a rocprofv3 kernel trace
(tools/prof_open.py): every kernel after the last commit's IPP final
exponentiation, with its queue, start offset and duration (ms), then the
per-queue busy time -- the opening runs on four streams, so the critical
path is read off the start/end offsets, not from summed durations.
    python tools/open_timeline.py run_kernel_trace.csv [max_lines]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 400
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?"),
             int(r.get("Grid_Size_X", r.get("Grid_Size", 0)))) for r in rows)
short = lambda n: re.sub(r"tpst::|unsigned int|unsigned long|const|\*|void |Fp<FqCfg>", "", n).split("(")[0][:48]
commits = [i for i, e in enumerate(ev) if "k_batch_sort" in e[2]]
i0 = commits[-1]
# the open starts at the first kernel after the commit's final exponentiation
j = i0
while j < len(ev) and "k_final_wave" not in ev[j][2] and "k_chain_final" not in ev[j][2]:
    j += 1
seg = ev[j + 1:]
t0 = seg[0][0]
end = max(e[1] for e in seg)
print("open span %.2f ms, %d kernels" % ((end - t0) / 1e6, len(seg)))
busy = {}
for n, e in enumerate(seg):
    busy[e[3]] = busy.get(e[3], 0) + e[1] - e[0]
    if n < lim:
        print("q%-3s %8.3f %7.3f  %-48s grid %d" % (e[3], (e[0] - t0) / 1e6, (e[1] - e[0]) / 1e6, short(e[2]), e[4]))
for q, b in sorted(busy.items()):
    print("queue %s busy %.2f ms" % (q, b / 1e6))
