"""First-contact GPU probe: field microbenchmarks, MSM / pairing parity
against the Python oracle, and a first 2^20 MSM timing.  Diagnostic only."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))

from testudo_amd import Context  # noqa: E402
from testudo_amd.encoding import fr_array, g1_array, g1_from_array, g2_array, g2_from_array, gt_from_array  # noqa
import bls377 as O  # noqa: E402
from pst import fr_stream  # noqa: E402

ctx = Context(0)
print("devices ok", flush=True)

# microbench: latency (1 wave) and throughput (full chip)
for kind, name in ((0, "fq_mul"), (1, "g1_madd")):
    it = 2000
    ms1 = ctx.microbench(kind, 64, it)
    print("%s latency: %.3f us/op (1 wave)" % (name, ms1 * 1e3 / it), flush=True)
    for waves_per_cu in (4, 8, 16):
        thr = 256 * waves_per_cu * 64
        it2 = 200
        ms = ctx.microbench(kind, thr, it2)
        print("%s throughput @%d waves/CU: %.2f Gop/s" % (name, waves_per_cu, thr * it2 / ms / 1e6), flush=True)

# MSM parity small
for n in (1, 7, 100, 1000):
    s, k = fr_stream(1234 + n, n)
    b, _ = fr_stream(999 + n, n)
    bases = [O.g1_mul(O.G1_GEN, x) for x in b]
    t = time.time()
    got = g1_from_array(ctx.g1_msm(g1_array(bases), fr_array(s)))[0]
    dt = time.time() - t
    exp = O.g1_mul(O.G1_GEN, sum(x * y for x, y in zip(s, b)) % O.R)
    print("g1 msm n=%d ok=%s (%.1f ms)" % (n, got == exp, dt * 1e3), flush=True)

# G2 MSM small
n = 50
s, _ = fr_stream(77, n)
b, _ = fr_stream(78, n)
bases = [O.g2_mul(O.G2_GEN, x) for x in b]
got = g2_from_array(ctx.g2_msm(g2_array(bases), fr_array(s)))[0]
exp = O.g2_mul(O.G2_GEN, sum(x * y for x, y in zip(s, b)) % O.R)
print("g2 msm n=%d ok=%s" % (n, got == exp), flush=True)

# pairing
ps = [O.g1_mul(O.G1_GEN, 11 + i) for i in range(3)]
qs = [O.g2_mul(O.G2_GEN, 101 + i) for i in range(3)]
got = gt_from_array(ctx.multi_pairing(g1_array(ps), g2_array(qs)))
exp = O.fq12_to_tower(O.multi_pairing(ps, qs))
print("multi_pairing ok=%s" % (got == exp), flush=True)

# large MSM, property check
for lg in (16, 20):
    n = 1 << lg
    s, _ = fr_stream(5, n)
    b, _ = fr_stream(6, n)
    t = time.time()
    bases = ctx.g1_mul_generator(fr_array(b))
    print("gen bases 2^%d: %.2f s" % (lg, time.time() - t), flush=True)
    sc = fr_array(s)
    for rep in range(3):
        t = time.time()
        got = g1_from_array(ctx.g1_msm(bases, sc))[0]
        dt = time.time() - t
        print("g1 msm 2^%d host-call %.2f ms" % (lg, dt * 1e3), flush=True)
    exp = O.g1_mul(O.G1_GEN, sum(x * y for x, y in zip(s, b)) % O.R)
    print("g1 msm 2^%d ok=%s" % (lg, got == exp), flush=True)
