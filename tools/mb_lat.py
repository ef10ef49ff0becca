"""Fq multiply / XYZZ doubling latency (one wave) and throughput (full chip)
for the microbench kinds: 0 = product scanning (field.h), 3 = two interleaved
chains, 4 = independent columns + word-serial REDC, 5 = G1 XYZZ doubling,
2 = Fq inverse."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import Context  # noqa: E402

ctx = Context(0)
for kind, iters in ((0, 400), (3, 400), (4, 400), (5, 100), (2, 20)):
    ctx.microbench(kind, 64, 4)
    lat = min(ctx.microbench(kind, 64, iters) for _ in range(3)) / iters * 1e3
    thr_threads = 256 * 16 * 64
    ms = min(ctx.microbench(kind, thr_threads, iters // 4) for _ in range(3))
    print("kind %d: lone-wave latency %.3f us/op, chip throughput %.2f G op/s" %
          (kind, lat, thr_threads * (iters // 4) / ms / 1e6), flush=True)
