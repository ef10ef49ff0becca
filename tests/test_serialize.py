"""arkworks wire format (f2): the C++ writer/reader of csrc/serialize.hip
(host-only C-ABI, no GPU) against the independent Python restatement in
oracle/py/serialize.py, on the golden proofs (tests/golden/sqrt_pst_n*.json),
plus sizes (benches/pst.rs:43-46,64-74), round trips and rejection of invalid
encodings (Validate::Yes).  Parity against arkworks itself is unpinned (no
Rust toolchain; the reference holds no serialized fixture)."""
import numpy as np
import pytest

import bls377 as O
import golden_io as G
import serialize as OS
from testudo_amd import serialize as S
from testudo_amd.encoding import g1_array, g2_array
from testudo_amd.sqrt_pst import MippProof


def _golden_proof(d):
    pst = G.g2_arr(d["pst_proof"])
    mipp = MippProof(comms_t=np.stack([np.stack([G.gt_array(a), G.gt_array(b)]) for a, b in d["comms_t"]]),
                     comms_u=np.stack([G.g1_arr(p) for p in d["comms_u"]]),
                     final_a=G.g1_arr([d["final_a"]])[0], final_h=G.g2_arr([d["final_h"]])[0],
                     pst_proof_h=G.g1_arr(d["pst_proof_h"]))
    return pst, mipp


@pytest.mark.parametrize("n", [4, 5, 6, 7])
def test_proof_bytes_match_oracle_and_round_trip(n):
    d = G.load("sqrt_pst_n%d.json" % n)
    pst, mipp = _golden_proof(d)
    b_pst, b_mipp = S.ser_pst_proof(pst, mipp), S.ser_mipp_proof(pst, mipp)
    assert b_pst == OS.ser_pst_proof([G.g2(q) for q in d["pst_proof"]])
    assert b_mipp == OS.ser_mipp_proof([(G.gt(a), G.gt(b)) for a, b in d["comms_t"]],
                                       [(G.g1(a), G.g1(b)) for a, b in d["comms_u"]],
                                       G.g1(d["final_a"]), G.g2(d["final_h"]),
                                       [G.g1(q) for q in d["pst_proof_h"]])
    m_col, m_row = n // 2, n - n // 2
    assert len(b_pst) == 8 + 96 * m_row
    assert len(b_mipp) == 8 + 1152 * m_col + 8 + 96 * m_col + 48 + 96 + 8 + 48 * m_col
    pst2, mipp2 = S.de_open_proof(b_pst, b_mipp)
    assert np.array_equal(pst2, pst)
    for f in ("comms_t", "comms_u", "final_a", "final_h", "pst_proof_h"):
        assert np.array_equal(getattr(mipp2, f), getattr(mipp, f)), f
    # U as a Commitment { nv, g_product } (sqrt_pst.rs:201: nv = m_col)
    U = G.g1_arr([d["U"]])[0]
    assert S.ser_commitment(m_col, U) == OS.ser_commitment(m_col, G.g1(d["U"]))


def test_proof_size_at_baseline_n20():
    """13 128 B MippProof + 968 B Proof = 14 096 B at n = 20
    (structure only: every point at infinity, every GT zero -- all valid)."""
    m = 10
    pst = np.zeros((m, 24), dtype=np.uint64)
    mipp = MippProof(comms_t=np.zeros((m, 2, 72), dtype=np.uint64), comms_u=np.zeros((m, 2, 12), dtype=np.uint64),
                     final_a=np.zeros(12, dtype=np.uint64), final_h=np.zeros(24, dtype=np.uint64),
                     pst_proof_h=np.zeros((m, 12), dtype=np.uint64))
    assert len(S.ser_mipp_proof(pst, mipp)) == 13128
    assert S.proof_size(pst, mipp) == 14096


def test_committer_key_matches_oracle():
    d = G.load("sqrt_pst_n5.json")
    s, nv = d["srs"], d["srs_nv"]
    b = S.ser_committer_key(nv, G.srs_flat(d))
    ref = OS.ser_committer_key(nv, [[G.g1(p) for p in lv] for lv in s["powers_of_g"]],
                               [[G.g2(p) for p in lv] for lv in s["powers_of_h"]], G.g1(s["g"]), G.g2(s["h"]))
    assert b == ref
    pts = (1 << (nv + 1)) - 2
    assert len(b) == 8 + (8 + 8 * nv + 48 * pts) + (8 + 8 * nv + 96 * pts) + 48 + 96


def test_point_codec_edge_cases():
    g, h = O.G1_GEN, O.G2_GEN
    for k in (1, 2, 3, O.R - 1, 12345):
        p, q = O.g1_mul(g, k), O.g2_mul(h, k)
        bp, bq = S.ser_g1(g1_array([p])[0]), S.ser_g2(g2_array([q])[0])
        assert bp == OS.ser_g1(p) and bq == OS.ser_g2(q)
        assert np.array_equal(S.de_g1(bp), g1_array([p])[0]) and OS.de_g1(bp) == p
        assert np.array_equal(S.de_g2(bq), g2_array([q])[0]) and OS.de_g2(bq) == q
    # -P flips exactly the sign flag
    p = O.g1_mul(g, 77)
    a, b = OS.ser_g1(p), OS.ser_g1(O.g1_neg(p))
    assert a[:47] == b[:47] and (a[47] ^ b[47]) == 0x80
    # infinity
    assert S.ser_g1(np.zeros(12, dtype=np.uint64)) == bytes(47) + b"\x40"
    assert not S.de_g1(bytes(47) + b"\x40").any()
    assert not S.de_g2(bytes(95) + b"\x40").any()


def test_invalid_encodings_rejected():
    p = O.g1_mul(O.G1_GEN, 5)
    good = bytearray(OS.ser_g1(p))
    bad_flags = bytes(good[:47]) + bytes([good[47] | 0xC0])
    with pytest.raises(S.SerializationError):
        S.de_g1(bad_flags)
    over = (O.P + 3).to_bytes(48, "little")  # x >= p
    with pytest.raises(S.SerializationError):
        S.de_g1(over)
    # x with x^3 + 1 a non-residue: no point
    x = next(x for x in range(2, 200) if pow((x ** 3 + 1) % O.P, (O.P - 1) // 2, O.P) == O.P - 1)
    with pytest.raises(S.SerializationError):
        S.de_g1(x.to_bytes(48, "little"))
    # on the curve but outside the order-r subgroup
    x = next(x for x in range(2, 200) if pow((x ** 3 + 1) % O.P, (O.P - 1) // 2, O.P) == 1)
    with pytest.raises(S.SerializationError):
        S.de_g1(x.to_bytes(48, "little"))
    with pytest.raises(ValueError):
        OS.de_g1(x.to_bytes(48, "little"))
    # non-canonical limbs are refused by the writer
    with pytest.raises(S.SerializationError):
        S.ser_g1(np.array([0xFFFFFFFFFFFFFFFF] * 12, dtype=np.uint64))
    # truncated / trailing bytes
    d = G.load("sqrt_pst_n4.json")
    pst, mipp = _golden_proof(d)
    b_pst, b_mipp = S.ser_pst_proof(pst, mipp), S.ser_mipp_proof(pst, mipp)
    with pytest.raises(S.SerializationError):
        S.de_open_proof(b_pst[:-1], b_mipp)
    with pytest.raises(S.SerializationError):
        S.de_open_proof(b_pst, b_mipp + b"\x00")


def test_committer_key_length_checked():
    """tpst_ser_committer_key takes the flat length and rejects a mismatch
    (short array or wrong nv) instead of reading past the buffer."""
    d = G.load("sqrt_pst_n5.json")
    flat = G.srs_flat(d)
    nv = d["srs_nv"]
    assert len(S.ser_committer_key(nv, flat)) > 0
    with pytest.raises(S.SerializationError):
        S.ser_committer_key(nv, flat[:-1])
    with pytest.raises(S.SerializationError):
        S.ser_committer_key(nv + 1, flat)


def test_multilinear_pc_rejects_non_power_of_two():
    """MultilinearPC calls raise on a non-power-of-two evaluation vector (the
    reference's MultilinearExtension has 2^nv evaluations) before any device
    work: no context is needed to see the error."""
    from testudo_amd.engine import TpstError
    from testudo_amd.sqrt_pst import MultilinearPC
    bad = np.zeros((3, 4), dtype=np.uint64)
    for fn in (MultilinearPC.commit, MultilinearPC.commit_g2):
        with pytest.raises(TpstError):
            fn(None, bad)
    for fn in (MultilinearPC.open, MultilinearPC.open_g1):
        with pytest.raises(TpstError):
            fn(None, bad, np.zeros((1, 4), dtype=np.uint64))
    with pytest.raises(TpstError):
        MultilinearPC.commit(None, np.zeros((0, 4), dtype=np.uint64))
