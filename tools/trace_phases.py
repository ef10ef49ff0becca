"""Summarise the last commit+open of a rocprofv3 kernel trace (tools/prof_open.py):
per-kernel busy time and the idle gaps, split at the last k_batch_sort (commit start)
and the first MIPP kernel after it (open start)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
       int(r["Workgroup_Size_X"]), r["VGPR_Count"], r["LDS_Block_Size"]) for r in rows]
ev.sort()
starts = [i for i, e in enumerate(ev) if "k_batch_sort" in e[2]]
i0 = starts[-1]
seg = ev[i0:]
short = lambda n: re.sub(r"tpst::|unsigned int|unsigned long|const|\*", "", n)[:70]


def summ(name, s):
    if not s:
        return
    span = s[-1][1] - s[0][0]
    busy = sum(e[1] - e[0] for e in s)
    print("== %s: span %.2f ms busy %.2f ms idle %.2f ms, %d launches" % (name, span / 1e6, busy / 1e6,
          (span - busy) / 1e6, len(s)))
    agg = {}
    for e in s:
        a = agg.setdefault(short(e[2]), [0, 0, e[3], e[4], e[5], e[6]])
        a[0] += 1
        a[1] += e[1] - e[0]
    for n, a in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
        print("  %-70s %4d %9.3f ms  grid %8d wg %4d vgpr %s lds %s" % (n, a[0], a[1] / 1e6, a[2], a[3], a[4], a[5]))


# commit = from batch_sort until the first k_final_wave completes (IPP final exp)
j = next(k for k in range(len(seg)) if "k_final_wave" in seg[k][2] or "k_chain_final" in seg[k][2])
summ("commit", seg[:j + 1])
summ("open", seg[j + 1:])
if len(sys.argv) > 2:
    t0 = seg[j + 1][0]
    for e in seg[j + 1:]:
        print("%9.3f %8.3f  %s" % ((e[0] - t0) / 1e6, (e[1] - e[0]) / 1e6, short(e[2])))
