"""GPU tests of the drop-in boundary beyond the sqrt-PST flow (include/tpst.h):

* shared-base strided batch MSM and Pedersen / Hyrax commitments
  (commitments.rs:79-86, dense_mlpoly.rs:314-329) against the C++ oracle;
* the length-checked multiexponentiation (mipp.rs:385-394);
* the single-call MultilinearPC surface against the
  Python oracle and through its own checks;
* proof-element validation in verify: p-shifted encodings, off-curve and
  non-subgroup points are rejected before the transcript absorbs them.
"""
import numpy as np
import pytest

import bls377 as O
import golden_io as G
import orc
import pst as P
from testudo_amd.encoding import fr_array, g1_array, g1_from_array, g2_from_array, limbs_to_int

pytestmark = pytest.mark.gpu


def _pts(seed, n):
    k, _ = orc.fr_stream(seed, n)
    return orc.g1_mul_gen(k)


# ------------------------------------------------------ batch / Pedersen --
@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 5), (17, 33), (64, 1024)])
def test_g1_msm_batch_strided_vs_oracle(ctx, rows, cols):
    from testudo_amd import Gens
    bases = _pts(900 + cols, cols)
    bases[min(2, cols - 1)] = 0  # an infinity generator
    gens = Gens(ctx, bases)
    Z, _ = orc.fr_stream(901 + rows, rows * cols)
    # contiguous rows (commit_inner) and the column view of sqrt-PST (Z[(j << m) | i])
    for rs, cs in ((cols, 1), (1, rows)):
        got = gens.msm_batch(Z, rows, rs, cs)
        assert np.array_equal(got, orc.g1_msm_batch(bases, Z, rows, rs, cs)), (rs, cs)
    gens.close()


def test_pedersen_commit_slice_and_rows_vs_oracle(ctx):
    from testudo_amd import Gens, TpstError
    n, L = 64, 16
    G_ = _pts(910, n + 1)
    gens = Gens(ctx, G_[:n], G_[n])
    Z, _ = orc.fr_stream(911, L * n)
    blinds, _ = orc.fr_stream(912, L)
    blinds[3] = 0  # zero blind (random_blinds = false, dense_mlpoly.rs:361)
    rows = gens.commit_rows(Z, blinds)
    for i in range(L):
        ref = orc.g1_msm(G_, np.concatenate([Z[i * n:(i + 1) * n], blinds[i:i + 1]]))
        assert np.array_equal(rows[i], ref), i
        assert np.array_equal(gens.commit_slice(Z[i * n:(i + 1) * n], blinds[i]), ref)
    with pytest.raises(TpstError):  # scalars.len() != gens.n (commitments.rs:84)
        gens.commit_slice(Z[:n - 1], blinds[0])
    nh = Gens(ctx, G_[:n])
    with pytest.raises(TpstError):  # no blinding base
        nh.commit_slice(Z[:n], blinds[0])


def test_multiexponentiation_length_check(ctx):
    from testudo_amd import TpstError
    bases = _pts(920, 40)
    s, _ = orc.fr_stream(921, 41)
    assert np.array_equal(ctx.multiexp(bases, s[:40]), orc.g1_msm(bases, s[:40]))
    with pytest.raises(TpstError):
        ctx.multiexp(bases, s)
    h = orc.g2_mul_gen(s[:3])
    assert np.array_equal(ctx.multiexp(h, s[:3], g2=True), orc.g2_msm(h, s[:3]))
    with pytest.raises(TpstError):
        ctx.multiexp(h, s[:2], g2=True)


# ------------------------------------------------------------ MultilinearPC --
def _lsb_eval(evals, point):
    tab = P.eq_table_lsb([limbs_to_int(x) for x in point])
    return sum(limbs_to_int(e) * t for e, t in zip(evals, tab)) % O.R


def test_multilinear_pc_single_calls(ctx):
    """commit / commit_g2 / open / open_g1 against the Python oracle at
    nv = 3 (the full level) and nv = 2 (a lower level of the variable CRS);
    check / check_2 accept the honest proofs and reject a wrong value."""
    from testudo_amd import sqrt_pst as S
    ck = 3
    seed = 0x7E57D1
    S.srs_setup(ctx, ck, seed)
    srs = P.SRS(ck, seed)
    for nv in (3, 2):
        ev, k = orc.fr_stream(930 + nv, 1 << nv)
        pt, _ = orc.fr_stream(930 + nv, nv, k)
        evi = [limbs_to_int(x) for x in ev]
        pti = [limbs_to_int(x) for x in pt]
        v = fr_array([_lsb_eval(ev, pt)])[0]
        c = S.MultilinearPC.commit(ctx, ev)
        assert g1_from_array(c)[0] == P.pst_commit(srs, evi)
        ch = S.MultilinearPC.commit_g2(ctx, ev)
        assert g2_from_array(ch)[0] == P.pst_commit_g2(srs, evi)
        pr = S.MultilinearPC.open(ctx, ev, pt)
        assert g2_from_array(pr) == P.pst_open(srs, evi, pti)
        pr1 = S.MultilinearPC.open_g1(ctx, ev, pt)
        assert g1_from_array(pr1) == P.pst_open_g1(srs, evi, pti)
        assert S.MultilinearPC.check(ctx, c, pt, v, pr), ctx.lib.tpst_last_error(ctx.h)
        assert S.MultilinearPC.check_2(ctx, ch, pt, v, pr1), ctx.lib.tpst_last_error(ctx.h)
        bad = fr_array([(limbs_to_int(v) + 1) % O.R])[0]
        assert not S.MultilinearPC.check(ctx, c, pt, bad, pr)
        assert not S.MultilinearPC.check_2(ctx, ch, pt, bad, pr1)


# ------------------------------------------------------- input validation --
def _sqrt_fq(a):
    """Tonelli-Shanks mod p (p - 1 = 2^46 * q)."""
    p = O.P
    if pow(a, (p - 1) // 2, p) != 1:
        return None
    q, s = p - 1, 0
    while q % 2 == 0:
        q //= 2
        s += 1
    z = 2
    while pow(z, (p - 1) // 2, p) == 1:
        z += 1
    m, c, t, r = s, pow(z, q, p), pow(a, q, p), pow(a, (q + 1) // 2, p)
    while t != 1:
        i, t2 = 0, t
        while t2 != 1:
            t2 = t2 * t2 % p
            i += 1
        b = pow(c, 1 << (m - i - 1), p)
        m, c, t, r = i, b * b % p, t * b * b % p, r * b % p
    return r


def _non_subgroup_point():
    x = 5
    while True:
        y = _sqrt_fq((x ** 3 + 1) % O.P)
        if y is not None and not O.g1_in_subgroup((x, y)):
            return (x, y)
        x += 1


def test_verify_rejects_malformed_proof_elements(ctx):
    from testudo_amd import sqrt_pst as S
    d = G.load("sqrt_pst_n5.json")
    S.srs_load(ctx, d["srs_nv"], G.srs_flat(d))
    pl = S.Polynomial.from_evaluations(ctx, G.fr_arr(d["Z"]))
    pt = G.fr_arr(d["point"])
    v = pl.eval(pt)
    comms, T = pl.commit()
    U, pst_proof, mipp = pl.open(S.PoseidonTranscript(), comms, pt, T)
    assert S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, mipp, T)
    pmod = np.array([(O.P >> (64 * i)) & (2**64 - 1) for i in range(6)], dtype=np.uint64)

    def shifted(a):  # same value mod p, different limbs (x + p < 2^384)
        out = a.copy()
        xi = limbs_to_int(out[:6]) + O.P
        out[:6] = [(xi >> (64 * i)) & (2**64 - 1) for i in range(6)]
        return out

    assert limbs_to_int(pmod) == O.P
    U2 = shifted(U)
    assert not S.verify(ctx, S.PoseidonTranscript(), U2, pt, v, pst_proof, mipp, T)
    off = U.copy()
    off[6] ^= 1  # y changed: off the curve
    assert not S.verify(ctx, S.PoseidonTranscript(), off, pt, v, pst_proof, mipp, T)
    ns = g1_array([_non_subgroup_point()])[0]
    assert not S.verify(ctx, S.PoseidonTranscript(), ns, pt, v, pst_proof, mipp, T)
    m2 = S.MippProof(mipp.comms_t.copy(), mipp.comms_u.copy(), mipp.final_a, mipp.final_h, mipp.pst_proof_h)
    m2.comms_u[0, 0] = shifted(mipp.comms_u[0, 0])
    assert not S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, m2, T)
    m3 = S.MippProof(mipp.comms_t.copy(), mipp.comms_u, mipp.final_a, mipp.final_h, mipp.pst_proof_h)
    m3.comms_t[0, 1] = shifted(mipp.comms_t[0, 1])
    assert not S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, m3, T)
    # comms_t outside GT: a canonical Fq12 that is not a pairing output (ark's
    # PairingOutput deserialisation rejects it), and a cyclotomic element of
    # the wrong order (t_l times a non-GT element of the cyclotomic subgroup)
    m4 = S.MippProof(mipp.comms_t.copy(), mipp.comms_u, mipp.final_a, mipp.final_h, mipp.pst_proof_h)
    m4.comms_t[0, 0] = G.gt_array([("%x" % (k + 2)) for k in range(12)])
    assert not S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, m4, T)
    t0 = O.fq12_from_tower([limbs_to_int(mipp.comms_t[0, 0][6 * i:6 * i + 6]) for i in range(12)])
    z = O.fq12_from_tower([k + 3 for k in range(12)])
    cyc = O.f12_mul(O.f12_frob(O.f12_mul(O.f12_conj(z), O.f12_inv(z)), 2), O.f12_mul(O.f12_conj(z), O.f12_inv(z)))
    assert O.f12_pow(cyc, O.R) != O.f12_one()  # cyclotomic, not in GT
    m5 = S.MippProof(mipp.comms_t.copy(), mipp.comms_u, mipp.final_a, mipp.final_h, mipp.pst_proof_h)
    m5.comms_t[0, 0] = G.gt_array(["%x" % c for c in O.fq12_to_tower(O.f12_mul(t0, cyc))])
    assert not S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, m5, T)
    # a valid GT element in the wrong place: t_l <-> t_r swapped
    m6 = S.MippProof(mipp.comms_t[:, ::-1].copy(), mipp.comms_u, mipp.final_a, mipp.final_h, mipp.pst_proof_h)
    assert not S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, m6, T)
    # a wrong-sized proof vector or an out-of-range scalar
    badpt = pt.copy()
    badpt[0] = fr_array([O.R - 1])[0]
    badpt[0, 3] = 0xFFFFFFFFFFFFFFFF
    assert not S.verify(ctx, S.PoseidonTranscript(), U, badpt, v, pst_proof, mipp, T)


# ---- MultiCommitGens::new (commitments.rs:17-39) ----------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("n,label", [(1, b""), (7, b"gens_r1cs_sat"), (40, b"gens_pc")])
def test_gens_new_matches_oracle(ctx, n, label):
    import gens as GN
    from testudo_amd.engine import Gens
    g = Gens.new(ctx, n, label)
    G, h = GN.multi_commit_gens(n, label)
    assert g1_from_array(g.G) == G and g1_from_array(g.h)[0] == h
    # the loaded set commits like commit_slice over the same points
    s, _ = orc.fr_stream(5, n)
    assert np.array_equal(g.msm_batch(s, 1, 0, 1)[0], orc.g1_msm(g.G, s))


@pytest.mark.gpu
@pytest.mark.parametrize("ell", [5, 8])
def test_dense_commit_hyrax(ctx, ell):
    """DensePolynomial::commit (dense_mlpoly.rs:349-377) over generators from
    MultiCommitGens::new: rows of 2^(ell - ell/2), zero and random blinds."""
    from testudo_amd.engine import Gens, dense_commit
    L, Rn = 1 << (ell // 2), 1 << (ell - ell // 2)
    g = Gens.new(ctx, Rn, b"gens_dense")
    Z, _ = orc.fr_stream(900 + ell, 1 << ell)
    got = dense_commit(g, Z)
    for i in range(L):
        assert np.array_equal(got[i], orc.g1_msm(g.G, Z[Rn * i:Rn * (i + 1)]))
    bl, _ = orc.fr_stream(950 + ell, L)
    got = dense_commit(g, Z, bl)
    for i in range(L):
        row = np.concatenate([g.G, g.h[None, :]])
        sc = np.concatenate([Z[Rn * i:Rn * (i + 1)], bl[i:i + 1]])
        assert np.array_equal(got[i], orc.g1_msm(row, sc))
