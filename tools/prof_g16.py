"""Groth16 prove at 2^log_cons (tools/gpu_g16.sh profiles it): setup, then
`reps` proves, printing per-prove wall time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import Context, _lib  # noqa: E402
from testudo_amd import groth16 as D  # noqa: E402
from testudo_amd import r1cs as S  # noqa: E402
from testudo_amd.encoding import fr_array  # noqa: E402

log_cons = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
_lib.load()
ctx = Context(0)
inst, v, x = S.R1CSInstance.produce_synthetic_r1cs(ctx, 1 << log_cons, 1 << log_cons, 10, 7)
pk = D.ProvingKey.setup(inst, fr_array([11, 12, 13, 14, 15]))
for _ in range(reps):
    ctx.synchronize()
    t = time.perf_counter()
    p = D.prove(pk, inst, v, x, fr_array([3]), fr_array([4]))
    print("prove_s %.4f" % (time.perf_counter() - t), flush=True)
