"""Median commit / open per (size, label) of tools/ab_env.sh-style outputs
(t{20,24}_{label}_{pass}.txt, lines "commit S open S"; the first call of
each file dropped).   python tools/ab_summary.py gpurun_out/TAG"""
import glob
import os
import re
import statistics as st
import sys

res = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "t2*_*.txt"))):
    m = re.match(r"t(\d+)_(\w+)_(\d+)\.txt", os.path.basename(f))
    n, lab, _ = m.groups()
    vals = [tuple(map(float, re.findall(r"[\d.]+", ln))) for ln in open(f) if ln.startswith("commit")][1:]
    res.setdefault((n, lab), []).extend(vals)
for (n, lab), v in sorted(res.items()):
    print("2^%s %-10s open median %.2f ms  commit median %.2f ms  opens: %s" % (
        n, lab, 1e3 * st.median(x[1] for x in v), 1e3 * st.median(x[0] for x in v),
        " ".join("%.1f" % (1e3 * x[1]) for x in v)))
