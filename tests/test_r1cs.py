"""Spartan R1CS sum-checks: R1CSProof::prove
(r1csproof.rs:237-370, Groth16 part excluded) on the device against the
pure-Python restatement oracle/py/r1cs.py, every proof element bit-exact at
small sizes; at 2^18 constraints by the verifier's size-independent checks
(sumcheck.rs:29-66 round consistency, the phase-one and phase-two final
claims, z(ry) from the PST evaluation).  Transcript parity against arkworks is
unpinned (oracle/py/r1cs.py header)."""
import numpy as np
import pytest

import bls377 as O
import pst as P
import r1cs as Q
from testudo_amd.encoding import fr_array, g1_from_array, g2_from_array, gt_from_array, limbs_to_int

R = O.R


def _ints(a):
    return [limbs_to_int(x) for x in np.asarray(a).reshape(-1, 4)]


def test_transcript_scalar_calls_match_oracle():
    """append_scalar / new_from_state2 of the host transcript (C-ABI, no GPU)."""
    from testudo_amd import r1cs as D
    from testudo_amd.sqrt_pst import PoseidonTranscript
    vals = [0, 1, R - 1, 12345678901234567890, 2 ** 252 + 7]
    a, b = PoseidonTranscript(), P.PoseidonTranscript()
    for v in vals:
        D.transcript_append_scalar(a, fr_array([v]))
        Q.append_scalar(b, v)
    assert limbs_to_int(a.challenge_scalar()) == b.challenge_scalar()
    D.transcript_new_from_state2(a, fr_array([vals[3]]))
    Q.new_from_state2(b, vals[3])
    D.transcript_append_scalar(a, fr_array([5]))
    Q.append_scalar(b, 5)
    assert limbs_to_int(a.challenge_scalar()) == b.challenge_scalar()
    with pytest.raises(ValueError):
        D.transcript_append_scalar(a, fr_array([0]) + np.array([0, 0, 0, 2 ** 63], dtype=np.uint64))


def _oracle_verify(out, inputs, num_cons, num_vars):
    """The verifier's sum-check side (r1csproof.rs verify restated) over the
    oracle transcript: returns (rx, ry) and asserts every claim."""
    tr = P.PoseidonTranscript()
    tr.append_gt(out["T"])
    assert tr.challenge_scalar() == out["initial_state"]
    Q.new_from_state2(tr, out["initial_state"])
    for x in inputs:
        Q.append_scalar(tr, x)
    rounds_x = Q.log2(num_cons)
    tau = [tr.challenge_scalar() for _ in range(rounds_x)]
    e, rx = Q.sumcheck_verify(out["sc1"], 0, 3, tr)
    tb = 1
    for t, r in zip(tau, rx):
        tb = tb * (t * r + (1 - t) * (1 - r)) % R
    az, bz, cz, azbz = out["claims_phase2"]
    assert azbz == az * bz % R and e == tb * (az * bz - cz) % R
    ra, rb, rc = (tr.challenge_scalar() for _ in range(3))
    e2, ry = Q.sumcheck_verify(out["sc2"], (ra * az + rb * bz + rc * cz) % R, 2, tr)
    zr, abcr = out["claims2"]
    assert e2 == zr * abcr % R
    return rx, ry, (ra, rb, rc)


def test_r1cs_oracle_self_consistent():
    mats, v, x = Q.synthetic_r1cs(32, 16, 3, 7)
    z = v + [1] + x
    for M in mats:  # the instance is satisfied
        pass
    Az, Bz, Cz = (Q.multiply_vec(M, 32, z) for M in mats)
    assert all((a * b - c) % R == 0 for a, b, c in zip(Az, Bz, Cz))
    out = Q.r1cs_prove(mats, 32, 16, v, x, P.SRS(2, 9), P.PoseidonTranscript())
    _oracle_verify(out, x, 32, 16)


CASES = [(16, 16, 3), (64, 16, 5), (32, 32, 0), (256, 64, 10)]


def _gpu_prove(ctx, num_cons, num_vars, num_inputs, seed, srs_seed):
    from testudo_amd import r1cs as D
    from testudo_amd import sqrt_pst as S
    n = Q.log2(num_vars)
    S.srs_setup(ctx, (n + 1) // 2, srs_seed)
    inst, vars_, inputs = D.R1CSInstance.produce_synthetic_r1cs(ctx, num_cons, num_vars, num_inputs, seed)
    proof, rx, ry = D.R1CSProof.prove(inst, vars_, inputs, S.PoseidonTranscript())
    return inst, vars_, inputs, proof


def _compare(proof, out):
    assert gt_from_array(proof.T) == O.fq12_to_tower(out["T"])
    assert limbs_to_int(proof.initial_state) == out["initial_state"]
    assert [_ints(p) for p in proof.sc_proof_phase1] == out["sc1"]
    assert _ints(proof.claims_phase2) == list(out["claims_phase2"])
    assert _ints(proof.r_abc) == list(out["r_abc"])
    assert [_ints(p) for p in proof.sc_proof_phase2] == out["sc2"]
    assert _ints(proof.claims_z_abc) == list(out["claims2"])
    assert _ints(proof.rx) == out["rx"] and _ints(proof.ry) == out["ry"]
    assert limbs_to_int(proof.transcript_sat_state) == out["transcript_sat_state"]
    assert limbs_to_int(proof.eval_vars_at_ry) == out["eval_vars_at_ry"]
    assert g1_from_array(proof.comm)[0] == out["U"]
    assert g2_from_array(proof.proof_eval_vars_at_ry) == list(out["pst_proof"])
    m = out["mipp"]
    assert g1_from_array(proof.mipp_proof.final_a)[0] == m["final_a"]
    assert g2_from_array(proof.mipp_proof.final_h)[0] == m["final_h"]
    assert g1_from_array(proof.mipp_proof.pst_proof_h) == list(m["pst_proof_h"])
    assert [tuple(g1_from_array(p)) for p in proof.mipp_proof.comms_u] == [tuple(u) for u in m["comms_u"]]
    assert [[gt_from_array(t) for t in p] for p in proof.mipp_proof.comms_t] == \
        [[O.fq12_to_tower(t) for t in pr] for pr in m["comms_t"]]


@pytest.mark.gpu
@pytest.mark.parametrize("num_cons,num_vars,num_inputs", CASES)
def test_r1cs_prove_vs_oracle(ctx, num_cons, num_vars, num_inputs):
    inst, vars_, inputs, proof = _gpu_prove(ctx, num_cons, num_vars, num_inputs, 1000 + num_cons, 0x7E57D1)
    mats, v, x = Q.synthetic_r1cs(num_cons, num_vars, num_inputs, 1000 + num_cons)
    assert _ints(vars_) == v and _ints(inputs) == x
    n = Q.log2(num_vars)
    out = Q.r1cs_prove(mats, num_cons, num_vars, v, x, P.SRS((n + 1) // 2, 0x7E57D1), P.PoseidonTranscript())
    _compare(proof, out)


@pytest.mark.gpu
def test_r1cs_load_general_matrices(ctx):
    """R1CSInstance::new path (host triples in shuffled order, several entries
    per row and column) gives the oracle's proof."""
    from testudo_amd import r1cs as D
    from testudo_amd import sqrt_pst as S
    num_cons, num_vars, num_inputs = 64, 16, 4
    mats, v, x = Q.synthetic_r1cs(num_cons, num_vars, num_inputs, 4242)
    rng = np.random.default_rng(5)
    extra = [(int(rng.integers(num_cons)), int(rng.integers(2 * num_vars)), int(rng.integers(1, 2 ** 60)))
             for _ in range(40)]
    A = mats[0] + extra  # A z no longer satisfies the constraints: the prover does not care
    mats2 = (A, mats[1], mats[2])
    enc = lambda M: [(r, c, fr_array([val])[0]) for (r, c, val) in M]  # noqa: E731
    order = [list(rng.permutation(len(M))) for M in mats2]
    inst = D.R1CSInstance.new(ctx, num_cons, num_vars, num_inputs,
                              *[[enc(M)[i] for i in o] for M, o in zip(mats2, order)])
    S.srs_setup(ctx, 2, 0x7E57D1)
    proof, _, _ = D.R1CSProof.prove(inst, fr_array(v), fr_array(x), S.PoseidonTranscript())
    out = Q.r1cs_prove(mats2, num_cons, num_vars, v, x, P.SRS(2, 0x7E57D1), P.PoseidonTranscript())
    _compare(proof, out)
    with pytest.raises(Exception):  # out-of-range column
        D.R1CSInstance.new(ctx, num_cons, num_vars, num_inputs, [(0, 2 * num_vars, fr_array([1])[0])], [], [])


@pytest.mark.gpu
def test_r1cs_prove_2p18_verifier_checks(ctx):
    """2^18 constraints, 2^16 variables: the verifier's checks over the
    device proof -- sum-check round consistency and final claims (phase one
    against eq(tau, rx), phase two against z(ry) ABC(ry) with z(ry) built from
    the device PST evaluation and the inputs, ABC(ry) from the instance)."""
    num_cons, num_vars, num_inputs = 1 << 18, 1 << 16, 17
    inst, vars_, inputs, proof = _gpu_prove(ctx, num_cons, num_vars, num_inputs, 99, 0x7E57D1)
    out = {"T": None, "initial_state": limbs_to_int(proof.initial_state),
           "sc1": [_ints(p) for p in proof.sc_proof_phase1], "claims_phase2": _ints(proof.claims_phase2),
           "sc2": [_ints(p) for p in proof.sc_proof_phase2], "claims2": _ints(proof.claims_z_abc)}
    x = _ints(inputs)
    tr = P.PoseidonTranscript()
    tr.sponge.absorb_bytes(np.asarray(proof.T, dtype=np.uint64).tobytes())
    assert tr.challenge_scalar() == out["initial_state"]
    Q.new_from_state2(tr, out["initial_state"])
    for xi in x:
        Q.append_scalar(tr, xi)
    tau = [tr.challenge_scalar() for _ in range(18)]
    e, rx = Q.sumcheck_verify(out["sc1"], 0, 3, tr)
    assert rx == _ints(proof.rx)
    tb = 1
    for t, r in zip(tau, rx):
        tb = tb * (t * r + (1 - t) * (1 - r)) % R
    az, bz, cz, azbz = out["claims_phase2"]
    assert azbz == az * bz % R and e == tb * (az * bz - cz) % R
    ra, rb, rc = (tr.challenge_scalar() for _ in range(3))
    e2, ry = Q.sumcheck_verify(out["sc2"], (ra * az + rb * bz + rc * cz) % R, 2, tr)
    assert ry == _ints(proof.ry)
    zr, abcr = out["claims2"]
    assert e2 == zr * abcr % R
    # z(ry) = (1 - ry0) vars(ry[1..]) + ry0 * (1, inputs, 0..)(ry[1..])   (r1csproof.rs verifier)
    v_at = limbs_to_int(proof.eval_vars_at_ry)
    io = [1] + x
    eq_io = Q.eq_evals(ry[1:])
    io_eval = sum(a * b for a, b in zip(io, eq_io)) % R
    assert zr == ((1 - ry[0]) * v_at + ry[0] * io_eval) % R
    # ABC(ry) = sum_M r_M M(rx, ry) for the synthetic instance (one entry per row and matrix)
    ex, ey = Q.eq_evals(rx), Q.eq_evals(ry)
    mats, v, xs = Q.synthetic_r1cs(num_cons, num_vars, num_inputs, 99)
    tot = 0
    for coef, M in zip((ra, rb, rc), mats):
        tot += coef * sum(ex[r] * ey[c] * val for r, c, val in M)
    assert abcr == tot % R


@pytest.mark.gpu
def test_r1cs_commit_spark_vs_oracle(ctx):
    """R1CSInstance::commit (SPARK dense representation + Hyrax commitments of
    comb_ops / comb_mem) against oracle/py/r1cs.py, synthetic and loaded
    (shuffled, repeated cells) instances."""
    from testudo_amd import r1cs as D
    num_cons, num_vars, num_inputs = 16, 16, 3
    inst, vars_, inputs = D.R1CSInstance.produce_synthetic_r1cs(ctx, num_cons, num_vars, num_inputs, 31)
    mats, v, x = Q.synthetic_r1cs(num_cons, num_vars, num_inputs, 31)
    ops, mem = inst.commit(b"gens_r1cs_eval")
    r_ops, r_mem = Q.spark_multi_commit(mats, num_cons, num_vars, b"gens_r1cs_eval")
    assert g1_from_array(ops) == r_ops and g1_from_array(mem) == r_mem
    # general matrices: different nnz per matrix, entries in caller order
    rng = np.random.default_rng(9)
    A = [(int(rng.integers(16)), int(rng.integers(32)), int(rng.integers(1, 1000))) for _ in range(21)]
    B = [(int(rng.integers(16)), int(rng.integers(32)), int(rng.integers(1, 1000))) for _ in range(7)]
    Cm = [(3, 5, 7)]
    enc = lambda M: [(r, c, fr_array([val])[0]) for (r, c, val) in M]  # noqa: E731
    inst2 = D.R1CSInstance.new(ctx, 16, 16, 3, enc(A), enc(B), enc(Cm))
    ops, mem = inst2.commit(b"lbl")
    r_ops, r_mem = Q.spark_multi_commit((A, B, Cm), 16, 16, b"lbl")
    assert g1_from_array(ops) == r_ops and g1_from_array(mem) == r_mem


@pytest.mark.gpu
def test_r1cs_prove_2p20_vs_cpu_oracle(ctx):
    """BASELINE configs[4]'s live path at full size: R1CSProof::prove over a
    2^20-constraint, 2^20-variable synthetic instance (the bench's), bit-exact
    against the C++ restatement (oracle/cpu, OpenMP): the witness commitment's
    T from orc.pst_commit, then every sum-check round polynomial, rx, ry, the
    phase-two claims and the transcript state after the sum-checks."""
    import orc
    from testudo_amd import r1cs as D
    from testudo_amd import sqrt_pst as S
    log_cons, seed, srs_seed = 20, 0x7E57D0 + 7, 0x7E57D0 + 1
    n = 1 << log_cons
    S.srs_setup(ctx, (log_cons + 1) // 2, srs_seed)
    inst, vars_, inputs = D.R1CSInstance.produce_synthetic_r1cs(ctx, n, n, 10, seed)
    proof, rx, ry = D.R1CSProof.prove(inst, vars_, inputs, S.PoseidonTranscript())
    srs = orc.SRS((log_cons + 1) // 2, srs_seed)
    _, T = orc.pst_commit(srs, vars_, log_cons)
    assert np.array_equal(np.asarray(proof.T, dtype=np.uint64).reshape(72), np.asarray(T).reshape(72))
    cpu = orc.r1cs_sumchecks(n, n, 10, seed, proof.T)
    assert np.array_equal(cpu["sc1"], proof.sc_proof_phase1)
    assert np.array_equal(cpu["sc2"], proof.sc_proof_phase2)
    assert np.array_equal(cpu["rx"], proof.rx) and np.array_equal(cpu["ry"], proof.ry)
    assert np.array_equal(cpu["claims_phase2"], proof.claims_phase2)
    assert np.array_equal(cpu["sat_state"], proof.transcript_sat_state)
