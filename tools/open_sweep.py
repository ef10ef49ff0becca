"""Median sqrt-PST open time at 2^n under environment variants, one child
process per variant (the tunables are read once per process):
    python tools/open_sweep.py 20 'TPST_COMMIT_TABLE=0' 'TPST_LIB_PATH=/path/to/other/libtpst.so' ..."""
import os
import subprocess
import sys

CHILD = r'''
import sys, time, statistics, os
sys.path.insert(0, os.environ["TPST_REPO"])
from testudo_amd.engine import Context
from testudo_amd import sqrt_pst as S
n = int(sys.argv[1])
ctx = Context(0)
S.srs_setup(ctx, (n + 1) // 2, 0x7E57D1)
Z, k = S.fr_stream(0x7E57D0, 1 << n)
pt, _ = S.fr_stream(0x7E57D0, n, k)
pl = S.Polynomial.from_evaluations(ctx, Z)
pl.eval(pt)
comms, T = pl.commit()
ts = []
for _ in range(6):
    t = time.perf_counter(); pl.open(S.PoseidonTranscript(), comms, pt, T); ts.append(time.perf_counter() - t)
print("%.2f" % (1e3 * statistics.median(ts[1:])))
'''

n = sys.argv[1]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for var in ["base"] + sys.argv[2:]:
    env = dict(os.environ, TPST_REPO=repo)
    if var != "base":
        for kv in var.split(","):
            k, v = kv.split("=")
            env[k] = v
    r = subprocess.run([sys.executable, "-c", CHILD, n], env=env, capture_output=True, text=True, timeout=300)
    print("%-40s open %s ms %s" % (var, r.stdout.strip(), r.stderr.strip()[-200:] if r.returncode else ""), flush=True)
