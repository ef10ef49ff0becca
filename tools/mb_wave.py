"""Wave-engine stage latency (one lone wave) per op, plus the phase split
(X/Y forms, product, store+sync, output forms, reduce+store+sync) in cycles;
and the scalar microbenchmarks of tools/mb_lat.py.  Output: JSON lines."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import Context  # noqa: E402

OPS = ["F12_MUL", "F12_SQR", "CYC_SQR", "LINE_PREP", "SQR_LP1", "SQR_LP2", "MUL034", "FROB1", "FROB2", "FROB3",
       "CONJ", "COPY", "INV1", "INV2", "INV3", "INV4", "INV5", "INV6", "INV7", "G2_DBL1", "G2_DBL2", "G2_DBL3",
       "G2_DBL4", "G2_ADD1", "G2_ADD2", "G2_ADD3", "G2_ADD4"]

ctx = Context(0)
for kind, iters in ((0, 400),):
    ctx.microbench(kind, 64, 4)
    lat = min(ctx.microbench(kind, 64, iters) for _ in range(3)) / iters * 1e3
    print(json.dumps({"kind": kind, "lone_wave_us": round(lat, 3)}), flush=True)
for op in ("F12_MUL", "CYC_SQR", "SQR_LP1", "MUL034", "G2_DBL1", "G2_DBL3", "CONJ"):
    k = OPS.index(op)
    ctx.microbench(16 + k, 64, 4)
    iters = 200
    us = min(ctx.microbench(16 + k, 64, iters) for _ in range(3)) / iters * 1e3
    cyc = np.zeros(5, dtype=np.uint64)
    ctx.lib.tpst_microbench_wave_phases(ctx.h, k, 100, cyc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    print(json.dumps({"op": op, "stage_us": round(us, 3),
                      "phase_cycles": [int(c) // 100 for c in cyc]}), flush=True)
# instruction issue: 8 independent chains per lane; lone wave and full chip
for kind, name in ((6, "v_mad_u64_u32"), (7, "v_mad_u32_u24"), (8, "v_mul_lo_u32"), (9, "v_add_u32"),
                   (10, "v_fma_f64"), (11, "v_mul_hi_u32")):
    iters = 2000
    ctx.microbench(kind, 64, 4)
    lone = min(ctx.microbench(kind, 64, iters) for _ in range(3))
    thr = 256 * 4 * 8 * 64
    chip = min(ctx.microbench(kind, thr, iters) for _ in range(3))
    print(json.dumps({"insn": name, "lone_wave_ns_per_insn": round(lone * 1e6 / (iters * 32), 3),
                      "chip_wave_insn_per_ns": round(thr / 64 * iters * 32 / (chip * 1e6), 2)}), flush=True)
