"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Pure-Python restatement of R1CSProof::prove (r1csproof.rs:237-370) -- the
Spartan sum-checks around the sqrt-PST commitment --
for small instances: the checker of testudo_amd/csrc/r1cs.hip.

  synthetic_r1cs        R1CSInstance::produce_synthetic_r1cs (r1csinstance.rs:166-242),
                        with a seeded SplitMix64 Fr stream instead of thread_rng
  multiply_vec          SparseMatPolynomial::multiply_vec (sparse_mlpoly.rs:462-476)
  eval_table_sparse     SparseMatPolynomial::compute_eval_table_sparse (:478-488)
  eq_evals              EqPolynomial::evals (dense_mlpoly.rs:231-250), MSB-first
  bound_top             DensePolynomial::bound_poly_var_top (dense_mlpoly.rs:389-396)
  unipoly_from_evals    UniPoly::from_evals (unipoly.rs:15-45)
  prove_cubic_additive  SumcheckInstanceProof::prove_cubic_with_additive_term (sumcheck.rs:67-148)
  prove_quad            SumcheckInstanceProof::prove_quad (sumcheck.rs:387-444)
  sumcheck_verify       SumcheckInstanceProof::verify (sumcheck.rs:29-66)
  r1cs_prove            R1CSProof::prove (r1csproof.rs:237-370), the Groth16 part excluded

Transcript (PoseidonTranscript<Fq>, poseidon_transcript.rs): append_scalar
absorbs an Fr as ONE Fq element with the same integer value (ark-crypto-
primitives Absorb of a prime-field element cast by value, exact since r < p);
new_from_state2 restarts the sponge and absorbs the 32-byte uncompressed Fr.
Parity unpinned against arkworks (no Rust toolchain; the reference holds no
R1CS fixture and its snapshot may not compile).
"""
from __future__ import annotations

import bls377 as O
import pst as P

R = O.R


def synthetic_r1cs(num_cons, num_vars, num_inputs, seed):
    """-> (A, B, C as lists of (row, col, val)), vars, inputs."""
    size_z = num_vars + num_inputs + 1
    Z, _ = P.fr_stream(seed, size_z)
    Z = list(Z)
    Z[num_vars] = 1
    A, B, C = [], [], []
    for i in range(num_cons):
        a_idx, b_idx, c_idx = i % size_z, (i + 2) % size_z, (i + 3) % size_z
        A.append((i, a_idx, 1))
        B.append((i, b_idx, 1))
        ab = Z[a_idx] * Z[b_idx] % R
        if Z[c_idx] == 0:
            C.append((i, num_vars, ab))
        else:
            C.append((i, c_idx, ab * pow(Z[c_idx], -1, R) % R))
    return (A, B, C), Z[:num_vars], Z[num_vars + 1:]


def multiply_vec(M, num_rows, z):
    out = [0] * num_rows
    for row, col, val in M:
        out[row] = (out[row] + z[col] * val) % R
    return out


def eval_table_sparse(M, rx, num_cols):
    out = [0] * num_cols
    for row, col, val in M:
        out[col] = (out[col] + rx[row] * val) % R
    return out


def eq_evals(r):
    ell = len(r)
    evals = [1] * (1 << ell)
    size = 1
    for j in range(ell):
        size *= 2
        for i in range(size - 1, 0, -2):
            s = evals[i // 2]
            evals[i] = s * r[j] % R
            evals[i - 1] = (s - evals[i]) % R
    return evals


def bound_top(Z, r):
    n = len(Z) // 2
    return [(Z[i] + (Z[i + n] - Z[i]) * r) % R for i in range(n)]


def unipoly_from_evals(e):
    i2, i6 = pow(2, -1, R), pow(6, -1, R)
    if len(e) == 3:
        c = e[0]
        a = i2 * (e[2] - 2 * e[1] + c) % R
        b = (e[1] - c - a) % R
        return [c, b, a]
    d = e[0]
    a = i6 * (e[3] - 3 * e[2] + 3 * e[1] - e[0]) % R
    b = i2 * (2 * e[0] - 5 * e[1] + 4 * e[2] - e[3]) % R
    c = (e[1] - d - a - b) % R
    return [d, c, b, a]


def unipoly_eval(cs, r):
    out, pw = cs[0], r
    for c in cs[1:]:
        out = (out + pw * c) % R
        pw = pw * r % R
    return out


def append_scalar(tr, s):
    tr.sponge.absorb_elems([s % R])


def new_from_state2(tr, s):
    tr.sponge = P.PoseidonSponge()
    tr.sponge.absorb_bytes((s % R).to_bytes(32, "little"))


def prove_cubic_additive(claim, rounds, tau, A, B, C, tr):
    comb = lambda t, a, b, c: t * (a * b - c)  # noqa: E731  r1csproof.rs:193-197
    e, rs, polys = claim, [], []
    for _ in range(rounds):
        n = len(tau) // 2
        e0 = e2 = e3 = 0
        for i in range(n):
            e0 += comb(tau[i], A[i], B[i], C[i])
            t2, a2, b2, c2 = (2 * X[n + i] - X[i] for X in (tau, A, B, C))
            e2 += comb(t2, a2, b2, c2)
            t3, a3, b3, c3 = (x2 + X[n + i] - X[i] for x2, X in zip((t2, a2, b2, c2), (tau, A, B, C)))
            e3 += comb(t3, a3, b3, c3)
        e0, e2, e3 = e0 % R, e2 % R, e3 % R
        cs = unipoly_from_evals([e0, (e - e0) % R, e2, e3])
        for c in cs:
            append_scalar(tr, c)
        r = tr.challenge_scalar()
        rs.append(r)
        tau, A, B, C = (bound_top(X, r) for X in (tau, A, B, C))
        e = unipoly_eval(cs, r)
        polys.append(cs)
    return polys, rs, [tau[0], A[0], B[0], C[0]]


def prove_quad(claim, rounds, A, B, tr):
    e, rs, polys = claim, [], []
    for _ in range(rounds):
        n = len(A) // 2
        e0 = e2 = 0
        for i in range(n):
            e0 += A[i] * B[i]
            e2 += (2 * A[n + i] - A[i]) * (2 * B[n + i] - B[i])
        e0, e2 = e0 % R, e2 % R
        cs = unipoly_from_evals([e0, (e - e0) % R, e2])
        for c in cs:
            append_scalar(tr, c)
        r = tr.challenge_scalar()
        rs.append(r)
        A, B = bound_top(A, r), bound_top(B, r)
        e = unipoly_eval(cs, r)
        polys.append(cs)
    return polys, rs, [A[0], B[0]]


def sumcheck_verify(polys, claim, degree, tr):
    """sumcheck.rs:29-66 over the same transcript calls as the prover
    (append_scalar of every coefficient, as prove_* write them)."""
    e, rs = claim, []
    for cs in polys:
        assert len(cs) - 1 == degree
        assert (cs[0] + sum(cs)) % R == e
        for c in cs:
            append_scalar(tr, c)
        r = tr.challenge_scalar()
        rs.append(r)
        e = unipoly_eval(cs, r)
    return e, rs


def log2(n):
    return n.bit_length() - 1


def r1cs_prove(mats, num_cons, num_vars, vars_, inputs, srs, tr):
    """R1CSProof::prove (r1csproof.rs:237-370) without prove_verifier (Groth16)."""
    A, B, C = mats
    n_vars = log2(num_vars)
    pl = P.Polynomial(list(vars_))
    comms, T = pl.commit(srs)
    tr.append_gt(T)
    initial_state = tr.challenge_scalar()
    new_from_state2(tr, initial_state)
    for x in inputs:
        append_scalar(tr, x)
    z = list(vars_) + [1] + list(inputs) + [0] * (num_vars - len(inputs) - 1)
    rounds_x, rounds_y = log2(num_cons), log2(len(z))
    tau = [tr.challenge_scalar() for _ in range(rounds_x)]
    poly_tau = eq_evals(tau)
    Az, Bz, Cz = (multiply_vec(M, num_cons, z) for M in (A, B, C))
    p1, rx, cl1 = prove_cubic_additive(0, rounds_x, poly_tau, Az, Bz, Cz, tr)
    _, az, bz, cz = cl1
    r_A, r_B, r_C = tr.challenge_scalar(), tr.challenge_scalar(), tr.challenge_scalar()
    claim2 = (r_A * az + r_B * bz + r_C * cz) % R
    erx = eq_evals(rx)
    eA, eB, eC = (eval_table_sparse(M, erx, len(z)) for M in (A, B, C))
    abc = [(r_A * a + r_B * b + r_C * c) % R for a, b, c in zip(eA, eB, eC)]
    p2, ry, cl2 = prove_quad(claim2, rounds_y, z, abc, tr)
    sat_state = tr.challenge_scalar()
    new_from_state2(tr, sat_state)
    point = ry[1:]
    U, pst_proof, mipp = pl.open(tr, comms, srs, point, T)
    v = pl.eval(point)
    return {"comms": comms, "T": T, "initial_state": initial_state, "sc1": p1, "rx": rx,
            "claims_phase2": (az, bz, cz, az * bz % R), "sc2": p2, "ry": ry, "claims2": cl2,
            "r_abc": (r_A, r_B, r_C), "transcript_sat_state": sat_state, "eval_vars_at_ry": v,
            "U": U, "pst_proof": pst_proof, "mipp": mipp, "n_vars": n_vars}


def spark_multi_commit(mats, num_cons, num_vars, label):
    """R1CSInstance::commit (r1csinstance.rs:313-344) = SparseMatPolynomial::
    multi_commit (sparse_mlpoly.rs:373-437, 490-517): dense representation
    (sparse_to_dense_vecs, AddrTimestamps::new, DensePolynomial::merge) and two
    DensePolynomial::commit (dense_mlpoly.rs:349-377, zero blinds) over
    PolyCommitmentGens::setup's Hyrax generators (nizk/mod.rs:25-28: the first R
    of MultiCommitGens::new(R + 1, label))."""
    import gens as GN
    nnz = max(len(M) for M in mats)
    N = 1
    while N < nnz:
        N *= 2
    vx, vy = log2(num_cons), log2(2 * num_vars)
    cells = 1 << max(vx, vy)

    def dense(M):
        rows = [e[0] for e in M] + [0] * (N - len(M))
        cols = [e[1] for e in M] + [0] * (N - len(M))
        vals = [e[2] % R for e in M] + [0] * (N - len(M))
        return rows, cols, vals

    reps = [dense(M) for M in mats]

    def timestamps(ops):
        audit = [0] * cells
        read = []
        for inst in ops:
            r = []
            for a in inst:
                r.append(audit[a])
                audit[a] += 1
            read.append(r)
        return read, audit

    row_ops = [r[0] for r in reps]
    col_ops = [r[1] for r in reps]
    row_read, row_audit = timestamps(row_ops)
    col_read, col_audit = timestamps(col_ops)
    comb_ops = sum(row_ops, []) + sum(row_read, []) + sum(col_ops, []) + sum(col_read, []) + sum([r[2] for r in reps], [])
    size = 1
    while size < len(comb_ops):
        size *= 2
    comb_ops += [0] * (size - len(comb_ops))
    comb_mem = row_audit + col_audit

    def hyrax(Z):
        ell = log2(len(Z))
        Lr, Rn = 1 << (ell // 2), 1 << (ell - ell // 2)
        G, _ = GN.multi_commit_gens(Rn + 1, label)
        return [O.g1_msm(G[:Rn], Z[Rn * i:Rn * (i + 1)]) for i in range(Lr)]

    return hyrax(comb_ops), hyrax(comb_mem)

