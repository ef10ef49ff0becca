"""Throughput / latency of the field and curve primitives (microbench kinds):
0 Fq mul, 1 G1 XYZZ mixed add, 2 Fq inverse, 5 G1 XYZZ doubling."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from testudo_amd import Context
ctx = Context(0)
ctx.microbench(0, 64, 1)
for kind, name, it in ((0, "fq_mul", 200), (1, "g1_madd", 50), (2, "fq_inv", 10), (5, "g1_dbl", 50)):
    lat = min(ctx.microbench(kind, 64, it) for _ in range(2)) * 1e3 / it
    thr = 256 * 16 * 64
    ms = min(ctx.microbench(kind, thr, it) for _ in range(2))
    print("%-8s lone-wave latency %.3f us | 16 w/CU %.3f G/s" % (name, lat, thr * it / ms / 1e6), flush=True)
