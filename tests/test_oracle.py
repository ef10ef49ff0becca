"""CPU tests: the oracles against the golden vectors and the reference KAT.

These pin the oracle before it is trusted as the GPU parity checker
(oracle/py = first-principles Python, oracle/cpu = arkworks-shaped C++).
"""
import numpy as np
import pytest

import bls377 as O
import golden_io as G
import orc
import pst as P
from testudo_amd.encoding import fr_array, g1_array, g1_from_array, g2_array, g2_from_array, gt_from_array, limbs_to_int


def test_reference_kat_dense_eval():
    d = G.load("kat_dense_eval.json")  # dense_mlpoly.rs:609-623
    assert P.dense_evaluate(d["Z"], d["r"]) == d["eval"] == 28
    pl = P.Polynomial([z % O.R for z in d["Z"]])
    assert pl.eval(d["r"]) == 28


def test_curve_constants():
    assert O.R == O.X ** 4 - O.X ** 2 + 1
    assert O.P == (O.X - 1) ** 2 * O.R // 3 + O.X
    assert O.g1_on_curve(O.G1_GEN) and O.g2_on_curve(O.G2_GEN)
    assert O.g1_in_subgroup(O.G1_GEN) and O.g2_in_subgroup(O.G2_GEN)
    # final-exponentiation chain exponent == 3 (p^12 - 1) / r
    x, p = O.X, O.P
    assert (3 + (x - 1) ** 2 * (x + p) * (x * x + p * p - 1)) * O.R == 3 * (p ** 4 - p ** 2 + 1)


def test_pairing_restatements_agree():
    d = G.load("pairing.json")
    ps = [G.g1(p) for p in d["g1"]]
    qs = [G.g2(q) for q in d["g2"]]
    e = O.multi_pairing(ps, qs)
    assert O.fq12_to_tower(e) == G.gt(d["gt"])
    assert O.pairing_textbook(ps[0], qs[0]) == O.pairing(ps[0], qs[0])
    eg = O.pairing(O.G1_GEN, O.G2_GEN)
    assert O.f12_pow(eg, O.R) == O.f12_one() and eg != O.f12_one()
    assert O.pairing(O.g1_mul(O.G1_GEN, 6), O.G2_GEN) == O.f12_pow(eg, 6)


def test_python_oracle_msm_golden():
    d = G.load("msm.json")
    g1 = d["g1"]
    assert O.g1_msm([G.g1(p) for p in g1["bases"]], [G.i(s) for s in g1["scalars"]]) == G.g1(g1["out"])


def test_cpp_oracle_msm_golden():
    d = G.load("msm.json")
    g1 = d["g1"]
    out = orc.g1_msm(G.g1_arr(g1["bases"]), G.fr_arr(g1["scalars"]))
    assert g1_from_array(out)[0] == G.g1(g1["out"])
    g2 = d["g2"]
    out2 = orc.g2_msm(G.g2_arr(g2["bases"]), G.fr_arr(g2["scalars"]))
    assert g2_from_array(out2)[0] == G.g2(g2["out"])


def test_cpp_oracle_pairing_golden():
    d = G.load("pairing.json")
    out = orc.multi_pairing(G.g1_arr(d["g1"]), G.g2_arr(d["g2"]))
    assert gt_from_array(out) == G.gt(d["gt"])


def test_stream_generators_agree():
    a, k1 = orc.fr_stream(P.SEED, 20)
    b, k2 = P.fr_stream(P.SEED, 20)
    assert [limbs_to_int(r) for r in a] == b and k1 == k2


def test_transcript_golden():
    d = G.load("transcript.json")
    tr = P.PoseidonTranscript()
    tr.append_g1(G.g1(d["append_g1"]))
    assert tr.challenge_scalar() == G.i(d["c1"])
    tr.append_gt(O.fq12_from_tower(G.gt(d["append_gt"])))
    assert tr.challenge_scalar() == G.i(d["c2"])
    assert tr.challenge_scalar() == G.i(d["c3"])


@pytest.mark.parametrize("n", [4, 5, 6, 7])
def test_cpp_oracle_sqrt_pst_golden(n):
    d = G.load("sqrt_pst_n%d.json" % n)
    srs = orc.SRS(d["srs_nv"], d["srs_seed"])
    assert np.array_equal(srs.export(), G.srs_flat(d))
    Z = G.fr_arr(d["Z"])
    pt = G.fr_arr(d["point"])
    assert limbs_to_int(orc.pst_eval(Z, n, pt)) == G.i(d["eval"])
    comms, T = orc.pst_commit(srs, Z, n)
    assert np.array_equal(comms, G.g1_arr(d["comms"]))
    assert np.array_equal(T, G.gt_array(d["T"]))
    pr = orc.pst_open(srs, Z, n, pt, comms)
    assert np.array_equal(pr["U"], G.g1_arr([d["U"]])[0])
    assert np.array_equal(pr["pst_proof"], G.g2_arr(d["pst_proof"]))
    assert np.array_equal(pr["comms_u"].reshape(-1, 12), G.g1_arr([p for pair in d["comms_u"] for p in pair]))
    assert np.array_equal(pr["comms_t"].reshape(-1, 72),
                          np.stack([G.gt_array(t) for pair in d["comms_t"] for t in pair]))
    assert np.array_equal(pr["final_a"], G.g1_arr([d["final_a"]])[0])
    assert np.array_equal(pr["final_h"], G.g2_arr([d["final_h"]])[0])
    assert np.array_equal(pr["pst_proof_h"], G.g1_arr(d["pst_proof_h"]))
    v = fr_array([G.i(d["eval"])])[0]
    assert orc.pst_verify(srs, n, pt, v, pr, T)
    bad = dict(pr)
    bad["final_a"] = orc.g1_mul_gen(fr_array([3]))[0]
    assert not orc.pst_verify(srs, n, pt, v, bad, T)


def test_cpp_oracle_batch_msm_matches_single():
    s, _ = orc.fr_stream(7, 64)
    b, _ = orc.fr_stream(8, 8)
    bases = orc.g1_mul_gen(b)
    rows = orc.g1_msm_batch(bases, s, 8, 1, 8)  # strided column view
    for r in range(8):
        assert np.array_equal(rows[r], orc.g1_msm(bases, s[r::8][:8]))


def test_msm_linearity_large():
    """size-independent property at 2^12: MSM(k_i G) == (sum s_i k_i) G."""
    n = 1 << 12
    s, _ = orc.fr_stream(21, n)
    k, _ = orc.fr_stream(22, n)
    bases = orc.g1_mul_gen(k)
    got = g1_from_array(orc.g1_msm(bases, s))[0]
    tot = sum(limbs_to_int(a) * limbs_to_int(b) for a, b in zip(s, k)) % O.R
    assert got == g1_from_array(orc.g1_mul_gen(fr_array([tot])))[0]


# ---- MultiCommitGens::new oracle (oracle/py/gens.py) ----
def test_chacha_block_known_answers():
    """The ChaCha block of oracle/py/gens.py (shared by the 12-round StdRng)
    against the published ChaCha20 vectors: the all-zero key stream (RFC 7539
    A.1 #1, = rand_chacha's zero-seed ChaCha20 output) and RFC 7539 §2.3.2."""
    import gens as GN
    assert GN.chacha_block([0] * 8, 0, rounds=20)[:4] == [0xADE0B876, 0x903DF1A0, 0xE56A5D40, 0x28BD8653]
    key = [int.from_bytes(bytes(range(4 * i, 4 * i + 4)), "little") for i in range(8)]
    out = GN.chacha_block(key, 1 | (0x09000000 << 32), rounds=20, nonce=(0x4A000000, 0))
    assert out[:4] == [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3]


def test_gens_oracle_points_valid():
    import gens as GN
    G, h = GN.multi_commit_gens(3, b"gens_test")
    for p in G + [h]:
        assert O.g1_on_curve(p) and O.g1_in_subgroup(p)
    assert len(set(G + [h])) == 4


def test_gens_seeds_match_oracle():
    """Host Poseidon<Fr> sponge of tpst_gens_new (no GPU) vs oracle/py/gens.py."""
    import ctypes as C
    import gens as GN
    from serialize import ser_g1
    from testudo_amd import _lib
    for n, label in ((3, b"gens_test"), (0, b""), (40, b"gens_pc")):
        buf = C.create_string_buffer(32 * (n + 1))
        assert _lib.load().tpst_gens_seeds(n, label, len(label), buf) == 0
        sp = GN.FrSponge()
        sp.absorb_bytes(label)
        sp.absorb_bytes(ser_g1(O.G1_GEN))
        assert buf.raw == b"".join(sp.squeeze_bytes(32) for _ in range(n + 1))


def test_cpp_r1cs_sumchecks_match_python_oracle():
    """oracle/cpu orc_r1cs_sumchecks (the bench's R1CS CPU leg) == oracle/py/r1cs.py."""
    import r1cs as Q
    num_cons, num_vars, ni, seed = 64, 16, 5, 1064
    mats, v, x = Q.synthetic_r1cs(num_cons, num_vars, ni, seed)
    out = Q.r1cs_prove(mats, num_cons, num_vars, v, x, P.SRS(2, 0x7E57D1), P.PoseidonTranscript())
    T = np.zeros((12, 6), dtype=np.uint64)
    for k, c in enumerate(O.fq12_to_tower(out["T"])):
        T[k] = [(c >> (64 * q)) & (2 ** 64 - 1) for q in range(6)]
    r = orc.r1cs_sumchecks(num_cons, num_vars, ni, seed, T.reshape(-1))
    ints = lambda a: [limbs_to_int(z) for z in np.asarray(a).reshape(-1, 4)]  # noqa: E731
    assert [ints(p) for p in r["sc1"]] == out["sc1"] and [ints(p) for p in r["sc2"]] == out["sc2"]
    assert ints(r["rx"]) == out["rx"] and ints(r["ry"]) == out["ry"]
    assert ints(r["claims_phase2"]) == list(out["claims_phase2"])
    assert limbs_to_int(r["sat_state"]) == out["transcript_sat_state"]
