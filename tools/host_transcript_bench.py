"""Host Poseidon transcript cost on this machine: append_bytes of one MIPP
round's t_l || t_r (1152 B) plus the challenge squeeze, as tpst_poly_open runs
it between device phases (the per-round host gap of the opening)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import sqrt_pst as S  # noqa: E402

t = S.PoseidonTranscript()
b = (bytes(range(256)) * 5)[:1152]
for _ in range(20):
    t.append_bytes(b)
    t.challenge_scalar()
N = 500
t0 = time.perf_counter()
for _ in range(N):
    t.append_bytes(b)
    t.challenge_scalar()
dt = (time.perf_counter() - t0) / N
print("append(1152 B) + challenge: %.1f us (%d reps)" % (dt * 1e6, N))
