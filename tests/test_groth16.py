"""Groth16 over BLS12-377 (r1csproof.rs:374-434,
Groth16::<E>::prove at :421): the device key generation, QAP witness map
(NTTs) and prover against the pure-Python restatement oracle/py/groth16.py --
h, the verifying key and the proof bit-exact for the same toxic waste and
(r, s) -- and the pairing verification equation at every size (the property
that pins the restatement, whose arkworks parity is unpinned)."""
import numpy as np
import pytest

import bls377 as O
import groth16 as G
import r1cs as Q
from testudo_amd.encoding import fr_array, g1_from_array, g2_array, g2_from_array, limbs_to_int

R = O.R
TOXIC = (0x1234567, 0xA1FA, 0xBE7A, 0x6A33A, 0xDE17A)


def _ints(a):
    return [limbs_to_int(x) for x in np.asarray(a).reshape(-1, 4)]


# ------------------------------------------------------------ CPU (oracle) --
def test_oracle_groth16_verifies():
    mats, v, x = Q.synthetic_r1cs(8, 8, 2, 5)
    z = G.assignment(v, x)
    pk = G.setup(mats, 8, 8, 2, TOXIC)
    A, B, C, h = G.prove(pk, mats, 8, z, 77, 88)
    assert G.qap_divides(mats, 8, 8, 2, z, pk["n"], h, 0xC0FFEE)
    assert G.verify(pk, x, (A, B, C))
    assert not G.verify(pk, [x[0] + 1, x[1]], (A, B, C))
    assert not G.verify(pk, x, (A, B, O.g1_add(C, O.G1_GEN)))


def test_oracle_qap_rejects_unsatisfied():
    """an assignment that breaks a constraint leaves a remainder: h is then
    not a quotient, the divisibility check fails."""
    mats, v, x = Q.synthetic_r1cs(8, 8, 1, 9)
    z = G.assignment(v, x)
    z[0] = (z[0] + 1) % R
    n = G.domain_size(8, 1)
    h = G.witness_map(mats, 8, 8, 1, z, n)
    assert not G.qap_divides(mats, 8, 8, 1, z, n, h, 0xC0FFEE)


def test_oracle_domain_matches_arkworks_root():
    """the two-adic root of unity the kernels hard-code (csrc/groth16.hip
    FR_ROOT47) is GENERATOR^((r - 1) / 2^47) and has order exactly 2^47."""
    w = G.root_of_unity(2 ** 47)
    assert w == 0x11d4b7f60cb92cc160c69477d1a8a12f9b506ee363e3f04a476ef4a4ec2a895e
    assert pow(w, 2 ** 46, R) == R - 1
    assert G.domain_size(8, 2) == 16 and G.domain_size(13, 2) == 16 and G.domain_size(14, 2) == 32


# ------------------------------------------------------------------ GPU -----
def _gpu(ctx, num_cons, num_vars, num_inputs, seed):
    from testudo_amd import groth16 as D
    from testudo_amd import r1cs as S
    inst, vars_, inputs = S.R1CSInstance.produce_synthetic_r1cs(ctx, num_cons, num_vars, num_inputs, seed)
    pk = D.ProvingKey.setup(inst, fr_array(TOXIC))
    return D, inst, vars_, inputs, pk


@pytest.mark.gpu
@pytest.mark.parametrize("num_cons,num_vars,num_inputs", [(8, 8, 2), (16, 4, 1), (4, 8, 0)])
def test_groth16_vs_oracle(ctx, num_cons, num_vars, num_inputs):
    D, inst, vars_, inputs, pk = _gpu(ctx, num_cons, num_vars, num_inputs, 31 + num_cons)
    mats, v, x = Q.synthetic_r1cs(num_cons, num_vars, num_inputs, 31 + num_cons)
    assert _ints(vars_) == v and _ints(inputs) == x
    z = G.assignment(v, x)
    opk = G.setup(mats, num_cons, num_vars, num_inputs, TOXIC)
    assert pk.domain_size == opk["n"]
    # witness map
    h = pk.witness_map(vars_, inputs)
    assert _ints(h) == G.witness_map(mats, num_cons, num_vars, num_inputs, z, opk["n"])
    # verifying key
    vk = pk.vk()
    assert g1_from_array(vk.alpha_g1)[0] == opk["alpha_g1"]
    assert g2_from_array(vk.beta_g2)[0] == opk["beta_g2"]
    assert g2_from_array(vk.gamma_g2)[0] == opk["gamma_g2"]
    assert g2_from_array(vk.delta_g2)[0] == opk["delta_g2"]
    assert g1_from_array(vk.gamma_abc_g1) == opk["gamma_abc_g1"]
    # proof
    r, s = 0xABCDEF12345, 0x5EED5EED
    proof = D.prove(pk, inst, vars_, inputs, fr_array([r]), fr_array([s]))
    A, B, C, _ = G.prove(opk, mats, num_cons, z, r, s)
    assert g1_from_array(proof.a)[0] == A
    assert g2_from_array(proof.b)[0] == B
    assert g1_from_array(proof.c)[0] == C
    assert D.verify(ctx, vk, inputs, proof)


@pytest.mark.gpu
def test_groth16_verify_rejects(ctx):
    D, inst, vars_, inputs, pk = _gpu(ctx, 32, 16, 3, 77)
    vk = pk.vk()
    proof = D.prove(pk, inst, vars_, inputs, fr_array([5]), fr_array([6]))
    assert D.verify(ctx, vk, inputs, proof)
    bad = inputs.copy()
    bad[0, 0] ^= 1
    assert not D.verify(ctx, vk, bad, proof)
    swapped = D.Proof(proof.a, proof.b, vk.alpha_g1)
    assert not D.verify(ctx, vk, inputs, swapped)
    # a witness that breaks a constraint gives a proof that does not verify
    v2 = vars_.copy()
    v2[1, 0] ^= 1
    assert not D.verify(ctx, vk, inputs, D.prove(pk, inst, v2, inputs, fr_array([5]), fr_array([6])))
    with pytest.raises(ValueError):
        D.verify(ctx, vk, inputs[:-1], proof)


@pytest.mark.gpu
def test_groth16_general_matrices_and_randomness(ctx):
    """R1CSInstance::new path with extra entries in padding columns (value-0
    variables): the oracle's proof for two different (r, s)."""
    from testudo_amd import groth16 as D
    from testudo_amd import r1cs as S
    num_cons, num_vars, num_inputs = 32, 8, 2
    mats, v, x = Q.synthetic_r1cs(num_cons, num_vars, num_inputs, 606)
    rng = np.random.default_rng(3)
    pad = [(int(rng.integers(num_cons)), int(rng.integers(num_vars + num_inputs + 1, 2 * num_vars)),
            int(rng.integers(1, 2 ** 60))) for _ in range(6)]
    mats2 = (mats[0] + pad, mats[1], mats[2])
    enc = lambda M: [(r, c, fr_array([val])[0]) for (r, c, val) in M]  # noqa: E731
    inst = S.R1CSInstance.new(ctx, num_cons, num_vars, num_inputs, *[enc(M) for M in mats2])
    pk = D.ProvingKey.setup(inst, fr_array(TOXIC))
    opk = G.setup(mats2, num_cons, num_vars, num_inputs, TOXIC)
    z = G.assignment(v, x)
    for r, s in ((1, 2), (R - 1, 0)):
        proof = D.prove(pk, inst, fr_array(v), fr_array(x), fr_array([r]), fr_array([s]))
        A, B, C, _ = G.prove(opk, mats2, num_cons, z, r, s)
        assert (g1_from_array(proof.a)[0], g2_from_array(proof.b)[0], g1_from_array(proof.c)[0]) == (A, B, C)
        assert D.verify(ctx, pk.vk(), fr_array(x), proof)


@pytest.mark.gpu
def test_groth16_setup_rejects(ctx):
    from testudo_amd import groth16 as D
    from testudo_amd import r1cs as S
    inst, _, _ = S.R1CSInstance.produce_synthetic_r1cs(ctx, 8, 8, 2, 1)
    with pytest.raises(Exception):
        D.ProvingKey.setup(inst, fr_array([1, 2, 3, 0, 5]))  # gamma = 0
    w = G.root_of_unity(16)
    with pytest.raises(Exception):
        D.ProvingKey.setup(inst, fr_array([pow(w, 3, R), 2, 3, 4, 5]))  # tau in the domain


@pytest.mark.gpu
def test_groth16_2p14_verifies(ctx):
    """2^14 constraints (domain 2^15): device prove + pairing verification."""
    D, inst, vars_, inputs, pk = _gpu(ctx, 1 << 14, 1 << 13, 7, 4)
    assert pk.domain_size == 1 << 15
    proof = D.prove(pk, inst, vars_, inputs, fr_array([0x1111]), fr_array([0x2222]))
    assert D.verify(ctx, pk.vk(), inputs, proof)


@pytest.mark.gpu
def test_groth16_verify_rejects_malformed_elements(ctx):
    """tpst_groth16_verify validates before pairing: an off-curve
    A, a B on the twist but outside the r-torsion subgroup, a coordinate >= p,
    an input >= r and a malformed verifying-key point are invalid proofs."""
    import serialize as SZ
    D, inst, vars_, inputs, pk = _gpu(ctx, 32, 16, 3, 78)
    vk = pk.vk()
    proof = D.prove(pk, inst, vars_, inputs, fr_array([5]), fr_array([6]))
    assert D.verify(ctx, vk, inputs, proof)
    off = proof.a.copy()
    off[6] ^= 1  # y + - 1: off the curve
    assert not O.g1_on_curve(g1_from_array(off)[0])
    assert not D.verify(ctx, vk, inputs, D.Proof(off, proof.b, proof.c))
    # a twist point of the full group order (no cofactor clearing)
    k = 1
    while True:
        x = (k, 1)
        y2 = O.f2_add(O.f2_mul(O.f2_sqr(x), x), O.G2_B)
        y = SZ._fq2_sqrt(y2)
        if y is not None and not O.g2_in_subgroup((x, y)):
            break
        k += 1
    bad_b = g2_array([(x, y)])[0]
    assert not D.verify(ctx, vk, inputs, D.Proof(proof.a, bad_b, proof.c))
    big = proof.c.copy()
    big[:6] = np.array([(O.P >> (64 * i)) & (2 ** 64 - 1) for i in range(6)], dtype=np.uint64)
    assert not D.verify(ctx, vk, inputs, D.Proof(proof.a, proof.b, big))
    ge_r = inputs.copy()
    ge_r[0] = fr_array([0])[0] + np.array([(O.R >> (64 * i)) & (2 ** 64 - 1) for i in range(4)], dtype=np.uint64)
    assert not D.verify(ctx, vk, ge_r, proof)
    vk2 = D.VerifyingKey(vk.alpha_g1, vk.beta_g2, vk.gamma_g2, bad_b, vk.gamma_abc_g1)
    assert not D.verify(ctx, vk2, inputs, proof)


@pytest.mark.gpu
def test_groth16_key_bound_to_context(ctx):
    """A proving key or instance presented through a context other than the
    one that built it is an argument error (TPST_E_ARG), never a launch on
    another context's stream and arena."""
    from testudo_amd import Context
    from testudo_amd.encoding import ptr
    D, inst, vars_, inputs, pk = _gpu(ctx, 16, 16, 2, 79)
    other = Context(0)
    try:
        bufs = [np.zeros(w, dtype=np.uint64) for w in (12, 24, 24, 24, 36)]
        assert other.lib.tpst_groth16_vk(other.h, pk.h, *[ptr(b) for b in bufs]) == -1
        a, b, c = (np.zeros(w, dtype=np.uint64) for w in (12, 24, 12))
        rs = fr_array([5, 6])
        assert other.lib.tpst_groth16_prove(other.h, pk.h, inst.h, ptr(np.ascontiguousarray(vars_)),
                                            ptr(np.ascontiguousarray(inputs)), ptr(rs), ptr(a), ptr(b), ptr(c)) == -1
    finally:
        other.close()
