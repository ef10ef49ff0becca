"""RNS engine stage timing (csrc/rns_engine.h, microbench kinds 64 + op):
per-stage latency of one 12-wave workgroup (two chains) and the stage time
when 64 .. 2048 workgroups run at once, with the extension rows in VGPRs
(one workgroup per CU) and in LDS (two per CU).  Output: JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import Context  # noqa: E402

RNS_OPS = ["F12_MUL", "F12_SQR", "CYC_SQR"]  # rns_ops.inc OpId order
ctx = Context(0)
for op, base, tag in [(o, 64, "vgpr_rows") for o in RNS_OPS] + [("F12_MUL", 80, "lds_rows"), ("CYC_SQR", 80, "lds_rows")]:
    kind = base + RNS_OPS.index(op)
    for wgs in (1, 64, 256, 512, 1024, 2048):
        iters = 100
        ctx.microbench(kind, 768 * wgs, 4)
        ms = min(ctx.microbench(kind, 768 * wgs, iters) for _ in range(3))
        us = ms * 1e3 / iters
        print(json.dumps({"op": op, "lane_rows": tag, "wgs": wgs, "stage_us": round(us, 3),
                          "chain_stages_per_us": round(2 * wgs / us, 2)}), flush=True)
