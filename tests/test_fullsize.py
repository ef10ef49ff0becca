"""Parity at the BASELINE sizes (configs[2]: n = 20, configs[3]: n = 24 on one
GPU) against fixtures the C++ CPU oracle produced over the bench's exact
inputs (oracle/gen_fullsize.py, shaped like benches/pst.rs:48-62), plus the
reference's own known-answer test through the device eval.

Every output of Polynomial::{commit, eval, open} (sqrt_pst.rs:105-230) is
compared bit-exact: T, v, U, the PST proof and every MippProof element in
full, the 2^m_col-point comm_list by SHA-256 digest and sampled rows.
"""
import hashlib

import numpy as np
import pytest

import golden_io as G
from testudo_amd.encoding import fr_array, limbs_to_int

R = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001


def _arr(hexs, shape):
    return np.frombuffer(bytes.fromhex(hexs), dtype=np.uint64).reshape(shape)


def test_fullsize_fixture_inputs_cpu():
    """The committed fixtures name the bench's inputs: the point is the stream
    continuation after Z and the recorded eval matches the CPU oracle."""
    import orc
    d = G.load("fullsize_n20.json")
    n = d["n"]
    Z, k = orc.fr_stream(d["seed_z"], 1 << n)
    pt, _ = orc.fr_stream(d["seed_z"], n, k)
    assert np.array_equal(pt, _arr(d["point"], (n, 4)))
    assert np.array_equal(orc.pst_eval(Z, n, pt), _arr(d["eval"], (4,)))
    assert {"n": 24, "srs_nv": 12}.items() <= G.load("fullsize_n24.json").items()


@pytest.mark.gpu
def test_reference_kat_dense_eval_gpu(ctx):
    """dense_mlpoly.rs:609-623 (Z = [1, 2, 1, 4], r = [4, 3] -> 28) through
    Polynomial::from_evaluations + eval on the device."""
    from testudo_amd import sqrt_pst as S
    d = G.load("kat_dense_eval.json")
    pl = S.Polynomial.from_evaluations(ctx, fr_array(d["Z"]))
    assert limbs_to_int(pl.eval(fr_array(d["r"]))) == d["eval"] == 28


def _check_fullsize(ctx, n):
    from testudo_amd import sqrt_pst as S
    d = G.load("fullsize_n%d.json" % n)
    m_col, m_row = n // 2, n - n // 2
    S.srs_setup(ctx, d["srs_nv"], d["seed_srs"])
    Z, k = S.fr_stream(d["seed_z"], 1 << n)
    pt, _ = S.fr_stream(d["seed_z"], n, k)
    assert np.array_equal(pt, _arr(d["point"], (n, 4)))
    pl = S.Polynomial.from_evaluations(ctx, Z)
    del Z
    comms, T = pl.commit()
    assert hashlib.sha256(comms.tobytes()).hexdigest() == d["comms_sha256"]
    for r, h in zip(d["comms_rows"], d["comms_sampled"]):
        assert np.array_equal(comms[r], _arr(h, (12,))), r
    assert np.array_equal(T, _arr(d["T"], (72,)))
    v = pl.eval(pt)
    assert np.array_equal(v, _arr(d["eval"], (4,)))
    U, pst_proof, mipp = pl.open(S.PoseidonTranscript(), comms, pt, T)
    assert np.array_equal(U, _arr(d["U"], (12,)))
    assert np.array_equal(pst_proof, _arr(d["pst_proof"], (m_row, 24)))
    assert np.array_equal(mipp.comms_t, _arr(d["comms_t"], (m_col, 2, 72)))
    assert np.array_equal(mipp.comms_u, _arr(d["comms_u"], (m_col, 2, 12)))
    assert np.array_equal(mipp.final_a, _arr(d["final_a"], (12,)))
    assert np.array_equal(mipp.final_h, _arr(d["final_h"], (24,)))
    assert np.array_equal(mipp.pst_proof_h, _arr(d["pst_proof_h"], (m_col, 12)))
    assert S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, mipp, T)
    # wire format (benches/pst.rs:64-74): sizes, and verify on the decoded proof
    from testudo_amd import serialize as W
    b_pst, b_mipp = W.ser_pst_proof(pst_proof, mipp), W.ser_mipp_proof(pst_proof, mipp)
    assert len(b_pst) + len(b_mipp) == 8 + 96 * m_row + 24 + 1296 * m_col + 144
    if n == 20:
        assert len(b_pst) + len(b_mipp) == 14096
    pst2, mipp2 = W.de_open_proof(b_pst, b_mipp)
    assert S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst2, mipp2, T)
    bad = fr_array([(limbs_to_int(v) + 1) % R])[0]
    assert not S.verify(ctx, S.PoseidonTranscript(), U, pt, bad, pst_proof, mipp, T)


@pytest.mark.gpu
def test_fullsize_commit_open_n20(ctx):
    """BASELINE configs[2]: 2^20-variable commit + open, bit-exact."""
    _check_fullsize(ctx, 20)


@pytest.mark.gpu
def test_fullsize_commit_open_n24(ctx):
    """BASELINE configs[3] on one GPU: 2^24-variable commit + open, bit-exact."""
    _check_fullsize(ctx, 24)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_fullsize_sharded_n24(ctx, world):
    """BASELINE configs[3] in its sharded form (sqrt_pst.rs:121-143 row MSMs +
    IPP, :198 c_u, then the opening), the world-`world` split run rank by rank
    in one process on one GPU: each rank uploads only its column block
    (from_evaluations_cols, 512 rows at world 8), writes [row commitments |
    Miller partial] into its row of one (world, R*12+72) device tensor -- the
    all-gather buffer of distributed.sharded_commit -- and its z_q / c_u
    shares; rank 0's combines (final exponentiation read from the gathered
    device buffer, mod-r sum, G1 sum) and the opening from q alone must give
    the fixture's comm_list, T, v, U, PST proof and every MippProof element."""
    import torch
    from testudo_amd import sqrt_pst as S
    n = 24
    d = G.load("fullsize_n%d.json" % n)
    m_col, m_row = n // 2, n - n // 2
    S.srs_setup(ctx, d["srs_nv"], d["seed_srs"])
    Z, k = S.fr_stream(d["seed_z"], 1 << n)
    pt, _ = S.fr_stream(d["seed_z"], n, k)
    C, N = 1 << m_col, 1 << m_row
    R = C // world
    dev = torch.device("cuda", 0)
    gathered = torch.empty((world, R * 12 + 72), dtype=torch.int64, device=dev)
    zq_parts = torch.empty((world, N * 4), dtype=torch.int64, device=dev)
    cu = []
    for g in range(world):
        sl = S.Polynomial.from_evaluations_cols(ctx, Z, g * R, (g + 1) * R)
        sl.commit_rows_partial_into(g * R, (g + 1) * R, gathered[g])
        sl.get_q_partial_into(pt, g * R, (g + 1) * R, zq_parts[g])
        own = gathered[g, :12 * R].cpu().numpy().view(np.uint64).reshape(R, 12)
        cu.append(S.cu_partial(ctx, n, pt, g * R, (g + 1) * R, own))
        del sl
    del Z
    comms = gathered[:, :12 * R].cpu().numpy().view(np.uint64).reshape(C, 12).copy()
    assert hashlib.sha256(comms.tobytes()).hexdigest() == d["comms_sha256"]
    T = S.gt_final_exp_product_gathered(ctx, gathered, R)
    assert np.array_equal(T, _arr(d["T"], (72,)))
    zq = S.fr_sum(ctx, zq_parts)
    U = S.g1_sum(ctx, np.stack(cu))
    assert np.array_equal(U, _arr(d["U"], (12,)))
    pq = S.Polynomial.from_q(ctx, n, pt, zq, U)
    v = pq.eval(pt)
    assert np.array_equal(v, _arr(d["eval"], (4,)))
    U2, pst_proof, mipp = pq.open(S.PoseidonTranscript(), comms, pt, T)
    assert np.array_equal(U2, U)
    assert np.array_equal(pst_proof, _arr(d["pst_proof"], (m_row, 24)))
    assert np.array_equal(mipp.comms_t, _arr(d["comms_t"], (m_col, 2, 72)))
    assert np.array_equal(mipp.comms_u, _arr(d["comms_u"], (m_col, 2, 12)))
    assert np.array_equal(mipp.final_a, _arr(d["final_a"], (12,)))
    assert np.array_equal(mipp.final_h, _arr(d["final_h"], (24,)))
    assert np.array_equal(mipp.pst_proof_h, _arr(d["pst_proof_h"], (m_col, 12)))
    assert S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, mipp, T)


@pytest.mark.gpu
def test_fullsize_groth16_2p20(ctx):
    """Groth16 at the R1CS leg's size (2^20 constraints and variables, 10
    inputs, domain 2^21): the device proof satisfies the pairing equation, a
    wrong public input or a broken witness does not."""
    from testudo_amd import groth16 as D
    from testudo_amd import r1cs as S
    inst, vars_, inputs = S.R1CSInstance.produce_synthetic_r1cs(ctx, 1 << 20, 1 << 20, 10, 2024)
    pk = D.ProvingKey.setup(inst, fr_array([3, 5, 7, 11, 13]))
    assert pk.domain_size == 1 << 21
    vk = pk.vk()
    proof = D.prove(pk, inst, vars_, inputs, fr_array([17]), fr_array([19]))
    assert D.verify(ctx, vk, inputs, proof)
    bad = inputs.copy()
    bad[9, 0] ^= 2
    assert not D.verify(ctx, vk, bad, proof)
    v2 = vars_.copy()
    v2[(1 << 20) - 1, 1] ^= 1
    assert not D.verify(ctx, vk, inputs, D.prove(pk, inst, v2, inputs, fr_array([17]), fr_array([19])))
