"""Chip throughput of the Fq product / square / XYZZ mixed add in field.h's
12 x 32-bit form (kinds 0, -, 1) and field29.h's 13 x 29-bit form (kinds 12,
14, 13), plus the lone-wave latency of each product.  JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import Context  # noqa: E402

ctx = Context(0)
thr = 256 * 16 * 64
for kind, name, iters in ((0, "fq_mul", 200), (12, "fq29_mul", 200), (14, "fq29_sqr", 200), (1, "madd", 40),
                          (13, "madd29", 40)):
    ctx.microbench(kind, thr, 4)
    ms = min(ctx.microbench(kind, thr, iters) for _ in range(3))
    lone = min(ctx.microbench(kind, 64, iters) for _ in range(3))
    print(json.dumps({"kind": kind, "op": name, "chip_G_per_s": round(thr * iters / (ms * 1e-3) / 1e9, 3),
                      "lone_wave_us": round(lone * 1e3 / iters, 3)}), flush=True)
