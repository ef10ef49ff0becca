"""Issue rates of the 64-bit integer VALU instructions in the radix-2^29
Montgomery product (v_lshl_add_u64 column carry adds, v_lshrrev_b64 column
shifts) against v_add_u32 / v_mad_u64_u32 / v_alignbit_b32 / v_add3_u32:
chip-wide wave-instructions per ns (8 independent chains per lane, 8 waves per
SIMD) and a lone wave's ns per instruction.  JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import Context  # noqa: E402

ctx = Context(0)
for kind, name in ((9, "v_add_u32"), (6, "v_mad_u64_u32"), (112, "v_lshl_add_u64"), (113, "v_lshrrev_b64"),
                   (114, "v_alignbit_b32"), (115, "v_add3_u32")):
    iters = 2000
    ctx.microbench(kind, 64, 4)
    lone = min(ctx.microbench(kind, 64, iters) for _ in range(3))
    thr = 256 * 4 * 8 * 64
    chip = min(ctx.microbench(kind, thr, iters) for _ in range(3))
    print(json.dumps({"insn": name, "lone_wave_ns_per_insn": round(lone * 1e6 / (iters * 32), 3),
                      "chip_wave_insn_per_ns": round(thr / 64 * iters * 32 / (chip * 1e6), 2)}), flush=True)
