"""Known answers the reference itself holds for the path's field / transcript
layer (fixtures: tests/golden/transcript_ref.json, kat_unipoly_chi.json, made
by oracle/py/gen_kat_ref.py).

* The Poseidon squeeze literal of prova.rs:132 / prova2.rs:143 / prova3.rs:143
  and the three absorb_test flows around it: the oracle and the library's host
  transcript (C-ABI) agree on every flow; the literal itself matches none of
  them under either limb reading, which the fixture records.
* UniPoly::from_evals KATs (unipoly.rs:119-173) through the oracle and
  ``tpst_unipoly_from_evals``.
* The chi-table identities of dense_mlpoly.rs:626-736 (MSB-first
  compute_chis_at_r == EqPolynomial::evals == L (x) R) on the oracle, and on
  the device kernel (``tpst_eq_evals``) under ``-m gpu``.
"""
import hashlib

import numpy as np
import pytest

import bls377 as O
import gen_kat_ref as K
import golden_io as G
import r1cs as Q
from testudo_amd.encoding import fr_array, limbs_to_int

R = O.R


def _digest(tab):
    return hashlib.sha256(np.ascontiguousarray(tab, dtype=np.uint64).tobytes()).hexdigest()


def test_reference_literal_recorded_and_unmatched():
    d = G.load("transcript_ref.json")
    ref = sum(int(x) << (64 * k) for k, x in enumerate(d["reference_literal"]["limbs_u64"]))
    assert G.i(d["reference_literal"]["as_canonical"]) == ref
    assert G.i(d["reference_literal"]["as_montgomery_to_canonical"]) == ref * pow(2 ** 256, -1, R) % R
    readings = {ref, ref * pow(2 ** 256, -1, R) % R}
    for name, f in d["flows"].items():
        c = G.i(f["challenge"])
        assert f["matches_reference_literal"] == (c in readings), name
    assert d["verdict"] == "unmatched"


def test_oracle_reproduces_transcript_flows():
    d = G.load("transcript_ref.json")
    g1 = K.GN.g1_rand(K.GN.ChaCha12Rng(K.TEST_RNG_SEED))
    assert [G.i(x) for x in d["flows"]["prova2_g1_test_rng"]["g1"]] == list(g1)
    assert O.g1_to_bytes(g1, compress=False).hex() == d["flows"]["prova2_g1_test_rng"]["input_hex"]
    gt = O.pairing(O.G1_GEN, O.G2_GEN)
    assert O.fq12_to_bytes(gt).hex() == d["flows"]["prova3_gt_generators"]["input_hex"]
    for name, f in d["flows"].items():
        assert K.squeeze_after(bytes.fromhex(f["input_hex"])) == G.i(f["challenge"]), name


def test_host_transcript_reproduces_flows():
    """The library's PoseidonTranscript (C-ABI, host) on the same three flows:
    append_bytes of the serialisations, and the typed append_g1 / append_gt."""
    from testudo_amd.encoding import g1_array
    from testudo_amd.sqrt_pst import PoseidonTranscript
    d = G.load("transcript_ref.json")
    for name, f in d["flows"].items():
        t = PoseidonTranscript()
        t.append_bytes(bytes.fromhex(f["input_hex"]))
        assert limbs_to_int(t.challenge_scalar()) == G.i(f["challenge"]), name
    t = PoseidonTranscript()
    t.append_g1(g1_array([tuple(G.i(x) for x in d["flows"]["prova2_g1_test_rng"]["g1"])])[0])
    assert limbs_to_int(t.challenge_scalar()) == G.i(d["flows"]["prova2_g1_test_rng"]["challenge"])
    t = PoseidonTranscript()
    t.append_gt(G.gt_array(d["flows"]["prova3_gt_generators"]["gt"]))
    assert limbs_to_int(t.challenge_scalar()) == G.i(d["flows"]["prova3_gt_generators"]["challenge"])
    t = PoseidonTranscript()  # empty vector: the length prefix alone
    t.append_bytes(b"")
    assert limbs_to_int(t.challenge_scalar()) == K.squeeze_after(b"")


@pytest.mark.parametrize("kind", ["quad", "cubic"])
def test_unipoly_from_evals_kat(kind):
    from testudo_amd.r1cs import UniPoly
    k = G.load("kat_unipoly_chi.json")["unipoly"][kind]
    assert Q.unipoly_from_evals(k["evals"]) == k["coeffs"]
    assert Q.unipoly_eval(k["coeffs"], k["at"]) == k["value"]
    cs = UniPoly.from_evals(fr_array(k["evals"]))
    assert [limbs_to_int(c) for c in cs] == k["coeffs"]
    with pytest.raises(ValueError):
        UniPoly.from_evals(fr_array([1, 2]))


def test_unipoly_from_evals_random_vs_oracle():
    from testudo_amd.r1cs import UniPoly
    import pst as P
    vals, _ = P.fr_stream(77, 70)
    for n in (3, 4):
        for k in range(0, 70 - n, n):
            e = vals[k:k + n]
            assert [limbs_to_int(c) for c in UniPoly.from_evals(fr_array(e))] == Q.unipoly_from_evals(e)


def test_chi_identities_oracle():
    c = G.load("kat_unipoly_chi.json")["chi"]
    r = [G.i(x) for x in c["r"]]
    chis = K.chis_at_r(r)
    assert K.digest(chis) == c["chis_sha256"]
    assert Q.eq_evals(r) == chis
    L, Rv = K.factored_chis_at_r(r)
    assert (K.digest(L), K.digest(Rv)) == (c["L_sha256"], c["R_sha256"])
    assert Q.eq_evals(r[:5]) == L and Q.eq_evals(r[5:]) == Rv  # compute_factored_evals
    assert [a * b % R for a in L for b in Rv] == chis


@pytest.mark.gpu
def test_chi_table_device(ctx):
    """EqPolynomial::evals on the device (the phase-one tau table kernel) ==
    compute_chis_at_r of the fixture, and its factored halves == L, R."""
    from testudo_amd.r1cs import EqPolynomial
    c = G.load("kat_unipoly_chi.json")["chi"]
    r = [G.i(x) for x in c["r"]]
    tab = EqPolynomial(fr_array(r)).evals(ctx)
    assert _digest(tab) == c["chis_sha256"]
    assert [limbs_to_int(x) for x in tab[:4]] == [G.i(x) for x in c["chis_head"]]
    assert _digest(EqPolynomial(fr_array(r[:5])).evals(ctx)) == c["L_sha256"]
    assert _digest(EqPolynomial(fr_array(r[5:])).evals(ctx)) == c["R_sha256"]
    # a larger table against the oracle's memoised evals
    import pst as P
    r16, _ = P.fr_stream(4242, 16)
    tab = EqPolynomial(fr_array(r16)).evals(ctx)
    assert [limbs_to_int(x) for x in tab] == Q.eq_evals(r16)
    assert EqPolynomial(fr_array([])).evals(ctx).tolist() == [[1, 0, 0, 0]]


def test_gt_membership_and_frobenius_split_facts():
    """The facts the verifier's GT exponentiation rests on (pairing.hip
    k_gt_pow_wave): p = x (mod r), so f^p = f^x on GT; e < r < x^4 has exact
    base-x digits; gcd(p - x, Phi12(p)) = r, so a cyclotomic f with f^p = f^x
    is in GT; and the 4-way split agrees with plain exponentiation."""
    from math import gcd
    P_, X_ = O.P, O.X
    assert P_ % R == X_ % R and X_ ** 4 > R
    assert gcd(P_ - X_, P_ ** 4 - P_ ** 2 + 1) == R
    f = O.pairing(O.G1_GEN, O.G2_GEN)
    assert O.f12_frob(f, 1) == O.f12_pow(f, X_)
    e = R - 12345
    d, q = [], e
    for _ in range(4):
        d.append(q % X_)
        q //= X_
    assert q == 0
    acc = O.f12_one()
    for j in range(4):
        acc = O.f12_mul(acc, O.f12_pow(O.f12_frob(f, j) if j else f, d[j]))
    assert acc == O.f12_pow(f, e)
