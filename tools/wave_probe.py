"""Per-stage latency of the wave-cooperative tower ops (tpst_microbench 16+op)
and the lone-wave Fq multiply for reference."""
import re
import sys

import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.chdir(ROOT)
from testudo_amd.engine import Context  # noqa: E402

ops = re.findall(r"OP_(\w+)", open("testudo_amd/csrc/wave_ops.inc").read().split("enum OpId {")[1].split("}")[0])
ops = [o for o in ops if o != "N_OPS" and not o.startswith("N_")]
ctx = Context(0)
it = 2000
ctx.microbench(0, 64, 10)
ms = ctx.microbench(0, 64, it)
print("lone-wave Fq mul: %.3f us" % (ms * 1e3 / it))
ms = ctx.microbench(0, 64 * 1024, it)
print("64K-thread Fq mul: %.3f us per chain step" % (ms * 1e3 / it))
for th in (1, 64, 4096):
    ctx.microbench(2, th, 2)
    ms = ctx.microbench(2, th, 20)
    print("Fq inverse, %d threads: %.1f us" % (th, ms * 1e3 / 20))
for i, name in enumerate(ops):
    ctx.microbench(16 + i, 1, 10)
    ms = ctx.microbench(16 + i, 1, it)
    print("%-10s %.3f us/stage" % (name, ms * 1e3 / it))

import numpy as np  # noqa: E402
from testudo_amd.encoding import ptr  # noqa: E402
print("phase cycles per stage: forms, mul, store+sync, out-forms, reduce+store+sync")
for i, name in enumerate(ops):
    cy = np.zeros(5, dtype=np.uint64)
    ctx.check(ctx.lib.tpst_microbench_wave_phases(ctx.h, i, 500, ptr(cy)), "phases")
    print("%-10s %s" % (name, " ".join("%7.0f" % (c / 500) for c in cy)))
