"""Profile target: sqrt-PST commit + open at 2^n (default 20) for rocprofv3."""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from testudo_amd.engine import Context  # noqa: E402
from testudo_amd import sqrt_pst as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ctx = Context(0)
S.srs_setup(ctx, (n + 1) // 2, 0x7E57D1)
Z, k = S.fr_stream(0x7E57D0, 1 << n)
pt, _ = S.fr_stream(0x7E57D0, n, k)
pl = S.Polynomial.from_evaluations(ctx, Z)
pl.eval(pt)
for _ in range(reps):
    t = time.perf_counter()
    comms, T = pl.commit()
    t1 = time.perf_counter()
    pl.open(S.PoseidonTranscript(), comms, pt, T)
    t2 = time.perf_counter()
    print("commit %.4f open %.4f" % (t1 - t, t2 - t1), flush=True)
