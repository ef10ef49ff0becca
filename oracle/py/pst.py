"""sqrt-PST commit / open / verify + MIPP + Poseidon transcript, restated in
pure Python.  TEST INFRASTRUCTURE ONLY (golden-vector generator and checker);
never imported by the product.

Every function cites the reference line it follows.  Upstream semantics that
are not in the tree (ark-poly-commit fork ``MultilinearPC``, ark-crypto-
primitives ``PoseidonSponge``) are restated from their published algorithm
and pinned by the reference's call sites.
"""

from __future__ import annotations

import json
import os

from bls377 import (P, R, G1_GEN, G2_GEN, g1_add, g1_neg, g1_mul, g1_msm, g2_add,
                    g2_neg, g2_mul, g2_msm, multi_pairing, pairing, f12_mul, f12_pow,
                    f12_one, g1_to_bytes, fq12_to_bytes)

# ----------------------------------------------------------- input stream --
GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
SEED = 0x7E57D0


def splitmix_word(seed, i):
    """Word i of the SplitMix64 stream started at ``seed``."""
    z = (seed + (i + 1) * GOLDEN) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def fr_stream(seed, n, start=0):
    """n uniform Fr by rejection: candidate k = words 4k..4k+3 (LE limbs),
    top limb masked to 253 bits, rejected if >= r.  Returns (values, next_k)."""
    out = []
    k = start
    while len(out) < n:
        v = 0
        for j in range(4):
            v |= splitmix_word(seed, 4 * k + j) << (64 * j)
        v &= (1 << 253) - 1
        k += 1
        if v < R:
            out.append(v)
    return out, k


# --------------------------------------------------------------- Poseidon --
_PARAMS = None


def poseidon_params():
    """get_bls12377_fq_params (parameters.rs:309-338): FR table read into Fq."""
    global _PARAMS
    if _PARAMS is None:
        here = os.path.dirname(os.path.abspath(__file__))
        path = os.path.join(here, "..", "..", "testudo_amd", "data", "poseidon_bls12_377.json")
        d = json.load(open(path))
        _PARAMS = {
            "ark": [[int(v) % P for v in row] for row in d["ark"]],
            "mds": [[int(v) % P for v in row] for row in d["mds"]],
            "rate": d["rate"], "capacity": d["capacity"], "alpha": d["alpha"],
            "full": d["full_rounds"], "partial": d["partial_rounds"],
        }
    return _PARAMS


class PoseidonSponge:
    """ark-crypto-primitives 0.4 ``PoseidonSponge<Fq>`` (duplex, state =
    capacity ‖ rate, absorb/squeeze modes) restated."""

    def __init__(self):
        self.p = poseidon_params()
        self.state = [0] * (self.p["rate"] + self.p["capacity"])
        self.mode = ("absorb", 0)

    def permute(self):
        p = self.p
        st = self.state[:]
        half = p["full"] // 2
        total = p["full"] + p["partial"]
        for rnd in range(total):
            st = [(s + a) % P for s, a in zip(st, p["ark"][rnd])]
            if rnd < half or rnd >= half + p["partial"]:
                st = [pow(s, p["alpha"], P) for s in st]
            else:
                st[0] = pow(st[0], p["alpha"], P)
            st = [sum(m * s for m, s in zip(row, st)) % P for row in p["mds"]]
        self.state = st

    def _absorb_internal(self, idx, elems):
        rate, cap = self.p["rate"], self.p["capacity"]
        rem = list(elems)
        while True:
            if idx + len(rem) <= rate:
                for i, e in enumerate(rem):
                    self.state[cap + i + idx] = (self.state[cap + i + idx] + e) % P
                self.mode = ("absorb", idx + len(rem))
                return
            n = rate - idx
            for i, e in enumerate(rem[:n]):
                self.state[cap + i + idx] = (self.state[cap + i + idx] + e) % P
            self.permute()
            rem = rem[n:]
            idx = 0

    def _squeeze_internal(self, idx, n):
        rate, cap = self.p["rate"], self.p["capacity"]
        out = []
        while True:
            if idx + (n - len(out)) <= rate:
                k = n - len(out)
                out += self.state[cap + idx:cap + idx + k]
                self.mode = ("squeeze", idx + k)
                return out
            k = rate - idx
            out += self.state[cap + idx:cap + idx + k]
            if len(out) < n:
                self.permute()
            idx = 0

    def absorb_elems(self, elems):
        if not elems:
            return
        mode, idx = self.mode
        if mode == "absorb":
            if idx == self.p["rate"]:
                self.permute()
                idx = 0
            self._absorb_internal(idx, elems)
        else:
            self.permute()
            self._absorb_internal(0, elems)

    def absorb_bytes(self, data: bytes):
        """``Absorb for Vec<u8>``: u64 LE length prefix, then
        ``[u8]::to_field_elements`` in 47-byte chunks ((377-1)/8)."""
        buf = len(data).to_bytes(8, "little") + data
        elems = [int.from_bytes(buf[i:i + 47], "little") for i in range(0, len(buf), 47)]
        self.absorb_elems(elems)

    def squeeze_native(self, n):
        mode, idx = self.mode
        if mode == "absorb":
            self.permute()
            return self._squeeze_internal(0, n)
        if idx == self.p["rate"]:
            self.permute()
            idx = 0
        return self._squeeze_internal(idx, n)

    def squeeze_fr(self):
        """Non-native ``squeeze_field_elements::<Fr>(1)``: one Fq element,
        its low 376 usable bits, truncated to Fr::MODULUS_BIT_SIZE-1 = 252."""
        e = self.squeeze_native(1)[0]
        return e & ((1 << 252) - 1)


class PoseidonTranscript:
    """poseidon_transcript.rs:17-34 — append = serialize(Compress::No) then
    absorb bytes; challenge_scalar = squeeze one Fr."""

    def __init__(self):
        self.sponge = PoseidonSponge()

    def append_g1(self, pt):
        self.sponge.absorb_bytes(g1_to_bytes(pt, compress=False))

    def append_gt(self, f):
        self.sponge.absorb_bytes(fq12_to_bytes(f))

    def challenge_scalar(self):
        return self.sponge.squeeze_fr()


# ------------------------------------------------------------ MultilinearPC --
def eq_table_lsb(t):
    """eq(t, x) for x in {0,1}^len(t), bit j of x <-> t[j] (ark-poly order)."""
    tab = [1]
    for tj in t:
        tab = [v * (1 - tj) % R for v in tab] + [v * tj % R for v in tab]
    return tab


class SRS:
    """MultilinearPC::setup + trim semantics from a
    seeded trapdoor: powers_of_g[i][x] = g^{eq(t[i..], x)}, g_mask[i]=g^{t_i},
    h likewise.  g = k_g * G1gen, h = k_h * G2gen."""

    def __init__(self, nv, seed=SEED + 1):
        vals, _ = fr_stream(seed, nv + 2)
        self.nv = nv
        kg, kh, t = vals[0], vals[1], vals[2:]
        self.t = t
        self.g = g1_mul(G1_GEN, kg)
        self.h = g2_mul(G2_GEN, kh)
        self.powers_of_g = []
        self.powers_of_h = []
        for i in range(nv):
            tab = eq_table_lsb(t[i:])
            self.powers_of_g.append([g1_mul(self.g, s) for s in tab])
            self.powers_of_h.append([g2_mul(self.h, s) for s in tab])
        self.g_mask = [g1_mul(self.g, ti) for ti in t]
        self.h_mask = [g2_mul(self.h, ti) for ti in t]


def pst_commit(srs, evals):
    """MultilinearPC::commit: msm(powers_of_g[ck.nv - nv], evals)."""
    nv = len(evals).bit_length() - 1
    return g1_msm(srs.powers_of_g[srs.nv - nv], evals)


def pst_commit_g2(srs, evals):
    nv = len(evals).bit_length() - 1
    return g2_msm(srs.powers_of_h[srs.nv - nv], evals)


def pst_quotients(evals, point):
    """The open recurrence: for i in 0..nv, k = nv-i,
    q_k[b] = r_k[2b+1]-r_k[2b]; r_{k-1}[b] = r_k[2b](1-pt_i)+r_k[2b+1]pt_i."""
    rk = list(evals)
    qs = []
    for a in point:
        half = len(rk) // 2
        q = [(rk[2 * b + 1] - rk[2 * b]) % R for b in range(half)]
        rk = [(rk[2 * b] * (1 - a) + rk[2 * b + 1] * a) % R for b in range(half)]
        qs.append(q)
    return qs, rk[0]


def pst_open(srs, evals, point):
    """MultilinearPC::open: pi_i = msm_G2(powers_of_h[i], [q_k[x>>1]])."""
    qs, _ = pst_quotients(evals, point)
    off = srs.nv - len(point)
    return [g2_msm(srs.powers_of_h[off + i], [q[x >> 1] for x in range(2 * len(q))])
            for i, q in enumerate(qs)]


def pst_open_g1(srs, evals, point):
    qs, _ = pst_quotients(evals, point)
    off = srs.nv - len(point)
    return [g1_msm(srs.powers_of_g[off + i], [q[x >> 1] for x in range(2 * len(q))])
            for i, q in enumerate(qs)]


def pst_check(srs, comm, point, value, proofs):
    """MultilinearPC::check (circuit_verifier.rs:245-314):
    e(C - g^v, h) == prod e(g_mask[nv-len+i] - g^{pt_i}, pi_i)."""
    left = pairing(g1_add(comm, g1_neg(g1_mul(srs.g, value))), srs.h)
    # level offset as in check_2 (0 for the full-level polynomials sqrt_pst.rs:261 checks)
    off = srs.nv - len(point)
    lefts = [g1_add(srs.g_mask[off + i], g1_neg(g1_mul(srs.g, point[i]))) for i in range(len(point))]
    return left == multi_pairing(lefts, proofs)


def pst_check_2(srs, comm_h, point, value, proofs):
    """check_2 (circuit_verifier.rs:175-243):
    e(g, C_h - h^v) == prod e(pi_i, h_mask[nv-len+i] - h^{pt_i})."""
    left = pairing(srs.g, g2_add(comm_h, g2_neg(g2_mul(srs.h, value))))
    off = srs.nv - len(point)
    rights = [g2_add(srs.h_mask[off + i], g2_neg(g2_mul(srs.h, point[i]))) for i in range(len(point))]
    return left == multi_pairing(proofs, rights)


# ----------------------------------------------------------------- MIPP ----
def polynomial_evaluations_from_transcript(cs_inv):
    """mipp.rs:159-180: evals[i] = prod_{bit j of i} cs_inv[m-1-j]."""
    m = len(cs_inv)
    out = []
    for i in range(1 << m):
        v = 1
        for j in range(m):
            if (i >> j) & 1:
                v = v * cs_inv[m - j - 1] % R
        out.append(v)
    return out


def mipp_prove(tr, srs, a, y, h, U):
    """MippProof::prove (mipp.rs:31-153)."""
    m_a, m_y, m_h = list(a), list(y), list(h)
    comms_t, comms_u, xs_inv = [], [], []
    tr.append_g1(U)
    while len(m_a) > 1:
        s = len(m_a) // 2
        a_l, a_r = m_a[:s], m_a[s:]
        y_l, y_r = m_y[:s], m_y[s:]
        h_l, h_r = m_h[:s], m_h[s:]
        u_l = g1_msm(a_l, y_r)          # mipp.rs:82
        u_r = g1_msm(a_r, y_l)          # mipp.rs:84
        t_l = multi_pairing(a_l, h_r)   # mipp.rs:90
        t_r = multi_pairing(a_r, h_l)   # mipp.rs:92
        tr.append_g1(u_l)
        tr.append_g1(u_r)
        tr.append_gt(t_l)
        tr.append_gt(t_r)
        c_inv = tr.challenge_scalar()   # mipp.rs:101
        c = pow(c_inv, -1, R)           # mipp.rs:106
        m_a = [g1_add(a_l[i], g1_mul(a_r[i], c)) for i in range(s)]       # compress
        m_y = [(y_l[i] + y_r[i] * c_inv) % R for i in range(s)]            # compress_field
        m_h = [g2_add(h_l[i], g2_mul(h_r[i], c_inv)) for i in range(s)]    # compress
        comms_t.append((t_l, t_r))
        comms_u.append((u_l, u_r))
        xs_inv.append(c_inv)
    final_a, final_h = m_a[0], m_h[0]
    poly = polynomial_evaluations_from_transcript(xs_inv)
    assert pst_commit_g2(srs, poly) == final_h  # mipp.rs:134 invariant
    rs = [tr.challenge_scalar() for _ in range(len(xs_inv))]
    pst_proof_h = pst_open_g1(srs, poly, rs)
    return {"comms_t": comms_t, "comms_u": comms_u, "final_a": final_a,
            "final_h": final_h, "pst_proof_h": pst_proof_h}


def mipp_verify(srs, tr, proof, point, U, T):
    """MippProof::verify (mipp.rs:182-320)."""
    tr.append_g1(U)
    xs, xs_inv = [], []
    final_y = 1
    for i, ((u_l, u_r), (t_l, t_r)) in enumerate(zip(proof["comms_u"], proof["comms_t"])):
        tr.append_g1(u_l)
        tr.append_g1(u_r)
        tr.append_gt(t_l)
        tr.append_gt(t_r)
        c_inv = tr.challenge_scalar()
        c = pow(c_inv, -1, R)
        xs.append(c)
        xs_inv.append(c_inv)
        final_y = final_y * (1 + c_inv * point[i] - point[i]) % R
    tc, uc = T, U
    for (t_l, t_r), (u_l, u_r), c, ci in zip(proof["comms_t"], proof["comms_u"], xs, xs_inv):
        tc = f12_mul(tc, f12_mul(f12_pow(t_l, ci), f12_pow(t_r, c)))
        uc = g1_add(uc, g1_add(g1_mul(u_l, ci), g1_mul(u_r, c)))
    m = len(xs_inv)
    rs = [tr.challenge_scalar() for _ in range(m)]
    v = 1
    for i in range(m):
        v = v * (1 + rs[i] * xs_inv[m - i - 1] - rs[i]) % R
    check_h = pst_check_2(srs, proof["final_h"], rs, v, proof["pst_proof_h"])
    final_u = g1_mul(proof["final_a"], final_y)
    final_t = pairing(proof["final_a"], proof["final_h"])
    return check_h and tc == final_t and uc == final_u


# ------------------------------------------------------------- sqrt-PST ----
def get_chi_i(b, i):
    """sqrt_pst.rs:152-166, MSB-first."""
    m = len(b)
    prod = 1
    for j in range(m):
        prod = prod * (b[j] if (i >> (m - j - 1)) & 1 else (1 - b[j])) % R
    return prod


def dense_evaluate(Z, r):
    """DensePolynomial::evaluate (dense_mlpoly.rs:408-414), MSB-first chi."""
    return sum(z * get_chi_i(r, j) for j, z in enumerate(Z)) % R


class Polynomial:
    """sqrt_pst.rs:14-265."""

    def __init__(self, Z):
        """from_evaluations, sqrt_pst.rs:32-75: polys[i].Z[j] = Z[(j<<m_col)|i]."""
        n = len(Z).bit_length() - 1
        assert 1 << n == len(Z)
        self.m_col = n // 2
        self.m_row = n - self.m_col
        self.odd = n % 2
        self.polys = [[Z[(j << self.m_col) | i] for j in range(1 << self.m_row)]
                      for i in range(1 << self.m_col)]
        self.q = None
        self.chis_b = None

    def get_q(self, point):
        """sqrt_pst.rs:81-101."""
        b = point[self.m_col + self.odd:]
        chis = [get_chi_i(b, i) for i in range(1 << self.m_col)]
        self.q = [sum(self.polys[i][j] * chis[i] for i in range(1 << self.m_col)) % R
                  for j in range(1 << self.m_row)]
        self.chis_b = chis

    def eval(self, point):
        """sqrt_pst.rs:105-115."""
        a = point[:len(point) // 2 + self.odd]
        if self.q is None:
            self.get_q(point)
        return sum(qj * get_chi_i(a, j) for j, qj in enumerate(self.q)) % R

    def commit(self, srs):
        """sqrt_pst.rs:117-149."""
        comms = [pst_commit(srs, p) for p in self.polys]
        h_vec = srs.powers_of_h[self.odd]
        T = multi_pairing(comms, h_vec)
        return comms, T

    def open(self, tr, comms, srs, point, T):
        """sqrt_pst.rs:168-230."""
        a = point[:self.m_col + self.odd]
        if self.q is None:
            self.get_q(point)
        c_u = g1_msm(comms, self.chis_b)
        assert c_u == pst_commit(srs, self.q)  # sqrt_pst.rs:206 invariant
        h_vec = srs.powers_of_h[self.odd]
        mipp = mipp_prove(tr, srs, comms, self.chis_b, h_vec, c_u)
        pst_proof = pst_open(srs, self.q, a[::-1])
        return c_u, pst_proof, mipp

    @staticmethod
    def verify(tr, srs, U, point, v, pst_proof, mipp, T):
        """sqrt_pst.rs:232-264."""
        n = len(point)
        odd = n % 2
        a = point[:n // 2 + odd]
        b = point[n // 2 + odd:]
        ok_mipp = mipp_verify(srs, tr, mipp, b, U, T)
        return ok_mipp and pst_check(srs, U, a[::-1], v, pst_proof)
