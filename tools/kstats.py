"""Summarise a rocprofv3 rocpd database: per-kernel count / total / avg, optionally
only dispatches after the N-th launch of a marker kernel (skip warm-up)."""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
after = sys.argv[3] if len(sys.argv) > 3 else None
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
if after:
    idx = [i for i, r in enumerate(rows) if after in r[0]]
    rows = rows[idx[skip]:] if len(idx) > skip else rows
agg = {}
for n, s, e in rows:
    a = agg.setdefault(n, [0, 0])
    a[0] += 1
    a[1] += e - s
tot = sum(v[1] for v in agg.values())
span = (rows[-1][2] - rows[0][1]) if rows else 0
print("kernels %d  busy %.2f ms  span %.2f ms" % (len(rows), tot / 1e6, span / 1e6))
for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print("%-72s %6d %9.2f ms %9.1f us" % (n[:72], k, t / 1e6, t / k / 1e3))
