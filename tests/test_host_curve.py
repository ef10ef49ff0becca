"""Host-side point validation (host_curve.h, 64-bit limbs) through
tpst_g1_check / tpst_g2_check -- the Valid::check the verifier, the Groth16
verifier and the MultilinearPC checks run on every proof element -- against
the oracle's on-curve / subgroup predicates.  No GPU: host code only."""
import numpy as np

import bls377 as O
import serialize as SZ
from testudo_amd import _lib
from testudo_amd.encoding import g1_array, g2_array, limbs_to_int


def _chk(p, g2=False):
    lib = _lib.load()
    a = np.ascontiguousarray(p, dtype=np.uint64)
    return (lib.tpst_g2_check if g2 else lib.tpst_g1_check)(a.ctypes.data_as(_lib._u64p)) == 0


def _g1_non_subgroup():
    x = 5
    while True:
        y = SZ._fq_sqrt((x ** 3 + 1) % O.P)
        if y is not None and not O.g1_in_subgroup((x, y)):
            return (x, y)
        x += 1


def _g2_non_subgroup():
    k = 1
    while True:
        x = (k, 1)
        y = SZ._fq2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(x), x), O.G2_B))
        if y is not None and not O.g2_in_subgroup((x, y)):
            return (x, y)
        k += 1


def test_g1_check_matches_oracle():
    pts = [O.g1_mul(O.G1_GEN, k) for k in (1, 2, 12345, O.R - 1)]
    for p in pts:
        assert _chk(g1_array([p])[0])
    assert _chk(np.zeros(12, dtype=np.uint64))  # infinity
    ns = _g1_non_subgroup()
    assert O.g1_on_curve(ns) and not _chk(g1_array([ns])[0])
    off = g1_array([pts[1]])[0]
    off[6] ^= 1
    assert not _chk(off)
    big = g1_array([pts[2]])[0]  # x + p: same point mod p, non-canonical limbs
    xi = limbs_to_int(big[:6]) + O.P
    big[:6] = [(xi >> (64 * i)) & (2 ** 64 - 1) for i in range(6)]
    assert not _chk(big)


def test_g2_check_matches_oracle():
    pts = [O.g2_mul(O.G2_GEN, k) for k in (1, 3, 98765)]
    for p in pts:
        assert _chk(g2_array([p])[0], g2=True)
    assert _chk(np.zeros(24, dtype=np.uint64), g2=True)
    ns = _g2_non_subgroup()
    assert not _chk(g2_array([ns])[0], g2=True)
    off = g2_array([pts[0]])[0]
    off[12] ^= 1
    assert not _chk(off, g2=True)
