"""The exact model of the wave-cooperative Fq inverse (csrc/inv_wave.h):
both the Bernstein-Yang variable-time form the device runs and the Pornin
form it replaced, against Python's modular inverse (CPU only)."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import inv_wave_model as M  # noqa: E402


def test_inv_wave_model_by_and_pornin():
    random.seed(7)
    ys = [1, 2, M.P - 1, (1 << 376) + 5] + [random.randrange(1, M.P) for _ in range(40)]
    for y in ys:
        r, batches, _ = M.inv_model_by(y)
        assert r * y % M.P == 1
        assert batches <= 73  # the 1091-divstep bound; inv_wave.h BY_MAX_BATCHES = 80
        assert M.inv_model(y) * y % M.P == 1
