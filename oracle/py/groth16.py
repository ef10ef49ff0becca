"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Pure-Python restatement of Groth16 over BLS12-377 as R1CSProof::prove_verifier
calls it (r1csproof.rs:374-434, ``Groth16::<E>::prove`` at :421) for small
instances: the checker of testudo_amd/csrc/groth16.hip.

The algorithm lives in the dependency ark-groth16 (Cargo.toml:32, version
0.4.0, patched to the arkworks-rs/groth16 git head at Cargo.toml:81), absent
from /root/reference; restated from its published code:

  r1cs_to_qap.rs  LibsnarkReduction
    instance_map_with_evaluation  Lagrange coefficients u_i at tau over the
                                  radix-2 domain of size next_pow2(num_cons +
                                  num_instance); a/b/c_j(tau) = sum_i M[i][j] u_i,
                                  plus u[num_cons + k] in a for instance var k
    witness_map_from_matrices     a/b/c = M z (a[num_cons + k] = instance k),
                                  iFFT, coset FFT (offset Fr::GENERATOR = 22),
                                  (a b - c) / (g^n - 1), coset iFFT
    h_query_scalars               zt / delta * tau^i, i < n - 1
  generator.rs    generate_parameters_with_qap (gamma_abc over the instance
                  variables / gamma, l over the witness / delta, k * G queries)
  prover.rs       create_proof_with_assignment:
                  A = alpha + sum z_i a_i + r delta, B = beta + sum z_i b_i + s delta,
                  C = s A + r B_g1 - r s delta + sum w_i l_i + sum h_i H_i
  verifier.rs     e(A, B) = e(alpha, beta) e(IC, gamma) e(C, delta)

Variables in the Spartan z order (vars, 1, inputs): instance = z[nv .. nv+ni],
witness = z[0 .. nv).  Parity against arkworks unpinned (no Rust toolchain, no
Groth16 fixture in the reference); the restatement is pinned by the
verification equation and the QAP divisibility check in tests/test_groth16.py.
"""
from __future__ import annotations

import bls377 as O

R = O.R
GENERATOR = 22


def domain_size(num_cons, num_inputs):
    n = 1
    while n < num_cons + num_inputs + 1:
        n *= 2
    return n


def root_of_unity(n):
    """Radix2EvaluationDomain::group_gen: GENERATOR^((r - 1) / n)."""
    return pow(GENERATOR, (R - 1) // n, R)


def dft(coeffs, w):
    """evaluations at w^j (O(n^2): small domains only)."""
    n = len(coeffs)
    return [sum(c * pow(w, i * j, R) for i, c in enumerate(coeffs)) % R for j in range(n)]


def ifft(evals, w):
    n = len(evals)
    ninv = pow(n, -1, R)
    return [x * ninv % R for x in dft(evals, pow(w, -1, R))]


def coset_fft(coeffs, w, g=GENERATOR):
    return dft([c * pow(g, i, R) % R for i, c in enumerate(coeffs)], w)


def coset_ifft(evals, w, g=GENERATOR):
    gi = pow(g, -1, R)
    return [c * pow(gi, i, R) % R for i, c in enumerate(ifft(evals, w))]


def lagrange_at(tau, n):
    w = root_of_unity(n)
    zt = (pow(tau, n, R) - 1) % R
    c = zt * pow(n, -1, R) % R
    return [c * pow(w, i, R) * pow((tau - pow(w, i, R)) % R, -1, R) % R for i in range(n)]


def qap_at(mats, num_cons, nv, ni, tau, n):
    """a/b/c_j(tau) for j < nq = nv + ni + 1."""
    u = lagrange_at(tau, n)
    nq = nv + ni + 1
    out = []
    for M in mats:
        t = [0] * nq
        for row, col, val in M:
            if col < nq:
                t[col] = (t[col] + u[row] * val) % R
        out.append(t)
    for k in range(ni + 1):
        out[0][nv + k] = (out[0][nv + k] + u[num_cons + k]) % R
    return out


def setup(mats, num_cons, nv, ni, toxic):
    tau, alpha, beta, gamma, delta = (t % R for t in toxic)
    n = domain_size(num_cons, ni)
    a, b, c = qap_at(mats, num_cons, nv, ni, tau, n)
    zt = (pow(tau, n, R) - 1) % R
    di, gi = pow(delta, -1, R), pow(gamma, -1, R)
    G1, G2 = O.G1_GEN, O.G2_GEN
    lin = lambda j, s: (beta * a[j] + alpha * b[j] + c[j]) * s % R  # noqa: E731
    return {
        "n": n, "nv": nv, "ni": ni,
        "a_query": [O.g1_mul(G1, x) for x in a],
        "b_g1_query": [O.g1_mul(G1, x) for x in b],
        "b_g2_query": [O.g2_mul(G2, x) for x in b],
        "h_query": [O.g1_mul(G1, zt * di * pow(tau, i, R)) for i in range(n - 1)],
        "l_query": [O.g1_mul(G1, lin(j, di)) for j in range(nv)],
        "gamma_abc_g1": [O.g1_mul(G1, lin(nv + k, gi)) for k in range(ni + 1)],
        "alpha_g1": O.g1_mul(G1, alpha), "beta_g1": O.g1_mul(G1, beta), "delta_g1": O.g1_mul(G1, delta),
        "beta_g2": O.g2_mul(G2, beta), "gamma_g2": O.g2_mul(G2, gamma), "delta_g2": O.g2_mul(G2, delta),
    }


def assignment(vars_, inputs):
    return [v % R for v in vars_] + [1] + [x % R for x in inputs]


def witness_map(mats, num_cons, nv, ni, z, n):
    w = root_of_unity(n)
    tabs = []
    for M in mats:
        t = [0] * n
        for row, col, val in M:
            t[row] = (t[row] + val * (z[col] if col < len(z) else 0)) % R
        tabs.append(t)
    for k in range(ni + 1):
        tabs[0][num_cons + k] = z[nv + k]
    a, b, c = (coset_fft(ifft(t, w), w) for t in tabs)
    vinv = pow((pow(GENERATOR, n, R) - 1) % R, -1, R)
    ab = [(x * y - v) * vinv % R for x, y, v in zip(a, b, c)]
    return coset_ifft(ab, w)[: n - 1]


def prove(pk, mats, num_cons, z, r, s):
    nv, ni, n = pk["nv"], pk["ni"], pk["n"]
    h = witness_map(mats, num_cons, nv, ni, z, n)
    A = O.g1_add(O.g1_add(pk["alpha_g1"], O.g1_msm(pk["a_query"], z)), O.g1_mul(pk["delta_g1"], r))
    B = O.g2_add(O.g2_add(pk["beta_g2"], O.g2_msm(pk["b_g2_query"], z)), O.g2_mul(pk["delta_g2"], s))
    B1 = O.g1_add(O.g1_add(pk["beta_g1"], O.g1_msm(pk["b_g1_query"], z)), O.g1_mul(pk["delta_g1"], s))
    C = O.g1_msm(pk["l_query"], z[:nv])
    C = O.g1_add(C, O.g1_msm(pk["h_query"], h))
    C = O.g1_add(C, O.g1_mul(A, s))
    C = O.g1_add(C, O.g1_mul(B1, r))
    C = O.g1_add(C, O.g1_neg(O.g1_mul(pk["delta_g1"], r * s)))
    return A, B, C, h


def verify(pk, inputs, proof):
    A, B, C = proof
    ic = pk["gamma_abc_g1"][0]
    for k, x in enumerate(inputs):
        ic = O.g1_add(ic, O.g1_mul(pk["gamma_abc_g1"][k + 1], x))
    g1s = [A, O.g1_neg(pk["alpha_g1"]), O.g1_neg(ic), O.g1_neg(C)]
    g2s = [B, pk["beta_g2"], pk["gamma_g2"], pk["delta_g2"]]
    keep = [(p, q) for p, q in zip(g1s, g2s) if p is not None and q is not None]
    return O.multi_pairing([p for p, _ in keep], [q for _, q in keep]) == O.f12_one()


def qap_divides(mats, num_cons, nv, ni, z, n, h, x):
    """a(x) b(x) - c(x) == h(x) (x^n - 1) at a point x off the domain, with
    a, b, c the interpolants of the witness-map tables (independent of the FFTs)."""
    u = lagrange_at(x, n)
    vals = []
    for mi, M in enumerate(mats):
        t = [0] * n
        for row, col, val in M:
            t[row] = (t[row] + val * (z[col] if col < len(z) else 0)) % R
        if mi == 0:
            for k in range(ni + 1):
                t[num_cons + k] = z[nv + k]
        vals.append(sum(ti * ui for ti, ui in zip(t, u)) % R)
    hx = sum(hi * pow(x, i, R) for i, hi in enumerate(h)) % R
    return (vals[0] * vals[1] - vals[2]) % R == hx * (pow(x, n, R) - 1) % R
