"""GPU parity tests: libtpst (HIP, gfx950) against the golden vectors and the
C++ CPU oracle, through the C-ABI.  Bit-exact on every output.

Sizes: golden vectors (n <= 7), oracle cross-checks at mid sizes that the
CPU oracle finishes in seconds, and size-independent properties (MSM
linearity, commit homomorphism, prove -> verify round trips) at the
BASELINE sizes.  Edge cases from the reference's domain: empty / length-
mismatched MSM inputs (msm_unchecked truncates, mipp.rs:389-393), infinity
bases, zero / one / r-1 scalars, repeated bases (bucket collisions), odd and
even variable counts (sqrt_pst.rs:297-304).
"""
import numpy as np
import pytest

import bls377 as O
import golden_io as G
import orc
from testudo_amd.encoding import fr_array, g1_array, g1_from_array, g2_array, g2_from_array, gt_from_array, limbs_to_int

pytestmark = pytest.mark.gpu


def _fr(v):
    return fr_array([v])[0]


# ------------------------------------------------------------ Fq inverse --
def test_fq_inverse_lane_and_wave(ctx):
    """csrc/inv_wave.h (one inverse per wave, 15-bit limbs across lanes) and
    field29.h's lone-lane inverse against Python's modular inverse, on
    Montgomery-form words (w = a R -> a^-1 R = R^2 / w); 0 -> 0"""
    p = O.P
    R = 1 << 384
    rng = np.random.default_rng(11)
    vals = [0, 1, 2, p - 1, p - 2, R % p, (1 << 376) + 12345, p // 2]
    vals += [int.from_bytes(rng.bytes(48), "little") % p for _ in range(120)]
    words = np.array([[(v >> (64 * i)) & ((1 << 64) - 1) for i in range(6)] for v in vals], dtype=np.uint64)
    ol, ow = ctx.selftest_inv(words)
    for v, a, b in zip(vals, ol, ow):
        want = 0 if v == 0 else R * R * pow(v, -1, p) % p
        assert limbs_to_int(a) == want, v
        assert limbs_to_int(b) == want, v


# ------------------------------------------------------------------- MSM --
def test_g1_msm_golden(ctx):
    d = G.load("msm.json")["g1"]
    out = ctx.g1_msm(G.g1_arr(d["bases"]), G.fr_arr(d["scalars"]))
    assert g1_from_array(out)[0] == G.g1(d["out"])


def test_g2_msm_golden(ctx):
    d = G.load("msm.json")["g2"]
    out = ctx.g2_msm(G.g2_arr(d["bases"]), G.fr_arr(d["scalars"]))
    assert g2_from_array(out)[0] == G.g2(d["out"])


@pytest.mark.parametrize("n", [0, 1, 2, 3, 31, 64, 255, 1000, 4097])
def test_g1_msm_vs_oracle(ctx, n):
    s, _ = orc.fr_stream(1000 + n, max(n, 1))
    k, _ = orc.fr_stream(2000 + n, max(n, 1))
    bases = orc.g1_mul_gen(k)[:n]
    s = s[:n]
    assert np.array_equal(ctx.g1_msm(bases, s), orc.g1_msm(bases, s))


def test_g1_msm_edge_scalars_and_collisions(ctx):
    n = 300
    k, _ = orc.fr_stream(31, n)
    bases = orc.g1_mul_gen(k)
    bases[10] = 0                      # infinity base
    bases[20:40] = bases[50]           # repeated bases -> same-bucket collisions
    vals = [0, 1, 2, O.R - 1, O.R - 2, (1 << 252), (1 << 16), (1 << 15) - 1, (1 << 15), (1 << 15) + 1]
    s = fr_array(vals * (n // len(vals)))
    assert np.array_equal(ctx.g1_msm(bases, s), orc.g1_msm(bases, s))
    # all-equal scalars: every point in one bucket per window
    s2 = fr_array([12345678901234567890123] * n)
    assert np.array_equal(ctx.g1_msm(bases, s2), orc.g1_msm(bases, s2))
    # P + (-P) cancellation inside one bucket
    neg = g1_array([None if p is None else (p[0], (O.P - p[1]) % O.P) for p in g1_from_array(bases[:2])])
    b3 = np.concatenate([bases[:2], neg])
    s3 = fr_array([5, 9, 5, 9])
    assert not ctx.g1_msm(b3, s3).any()


def test_msm_truncates_like_msm_unchecked(ctx):
    k, _ = orc.fr_stream(41, 50)
    s, _ = orc.fr_stream(42, 70)
    bases = orc.g1_mul_gen(k)
    assert np.array_equal(ctx.g1_msm(bases, s), orc.g1_msm(bases, s[:50]))


def test_g2_msm_vs_oracle(ctx):
    for n in (1, 17, 300):
        s, _ = orc.fr_stream(3000 + n, n)
        k, _ = orc.fr_stream(4000 + n, n)
        bases = orc.g2_mul_gen(k)
        assert np.array_equal(ctx.g2_msm(bases, s), orc.g2_msm(bases, s))


@pytest.mark.parametrize("lg", [16, 20, 21])
def test_g1_msm_linearity_full_size(ctx, lg):
    """BASELINE config 2 size: MSM(k_i G) == (sum s_i k_i) G (exact).  At 2^21
    the bucket sort has 8 193 bins and stages its scatter 2 entries per thread
    (k_sort_scatter_win<2>, the path of Groth16's 3.1 M-base MSMs)."""
    n = 1 << lg
    s, _ = orc.fr_stream(51, n)
    k, _ = orc.fr_stream(52, n)
    bases = ctx.g1_mul_generator(k)
    got = ctx.g1_msm(bases, s)
    si = [limbs_to_int(r) for r in s]
    ki = [limbs_to_int(r) for r in k]
    tot = sum(a * b for a, b in zip(si, ki)) % O.R
    assert np.array_equal(got, orc.g1_mul_gen(fr_array([tot]))[0])


@pytest.mark.parametrize("case", ["uniform", "clustered", "short", "boolean"])
def test_g1_msm_window_groups_vs_oracle(ctx, case):
    """n >= 2^17 takes the window-grouped pipeline (msm.hip msm_groups: per-group
    accumulation launches, group reductions + doubling chains on aux streams).
    'clustered' puts whole windows into a handful of buckets, so buckets span
    many chunks and the chunks straddling two window groups; its sort bins
    overflow the bin sort's LDS stage (k_sort_bin's direct-scatter path).
    'short' scalars (< 2^70) leave the top windows all zero digits: one large
    sentinel bin, and the lower windows' GLV digits skewed.  'boolean' puts
    half the points into one bucket (the long-bucket fixup)."""
    n = (1 << 17) + 37
    k, _ = orc.fr_stream(71, n)
    bases = ctx.g1_mul_generator(k)
    if case == "uniform":
        s, _ = orc.fr_stream(72, n)
    elif case == "boolean":
        # 0/1 scalars (witness bits): one bucket of ~65 K entries in window 0,
        # finished by k_bucket_fixup_long; every other window is sentinel
        rng = np.random.default_rng(74)
        s = np.zeros((n, 4), dtype=np.uint64)
        s[:, 0] = rng.integers(0, 2, n, dtype=np.uint64)
        assert 60000 < int(s[:, 0].sum()) < 71000
    elif case == "short":
        # scalars < 2^70: the top windows are all zero digits (sentinel bin)
        s, _ = orc.fr_stream(73, n)
        s[:, 1] &= np.uint64(0x3f)
        s[:, 2:] = 0
    else:
        assert case == "clustered"
        vals = [0, 1, 3, O.R - 1, (1 << 128) + 5, 12345678901234567890123]
        s = fr_array([vals[(i // 1000) % len(vals)] for i in range(n)])
        bases[100:3000] = bases[7]     # repeated bases inside the big buckets
    assert np.array_equal(ctx.g1_msm(bases, s), orc.g1_msm(bases, s, parallel=True))


def test_g2_msm_window_groups_long_buckets(ctx):
    """G2 at >= 2^17 points (window-grouped pipeline, pair-distributed Fq2
    accumulation): 0/1 and 0/1/2 scalars -> two long buckets in window 0,
    summed by the grouped pipeline's long-bucket fixup."""
    n = (1 << 17) + 37
    k, _ = orc.fr_stream(79, 4096)
    bases = np.concatenate([orc.g2_mul_gen(k)] * (n // 4096 + 1))[:n]
    rng = np.random.default_rng(80)
    s = np.zeros((n, 4), dtype=np.uint64)
    s[:, 0] = rng.integers(0, 3, n, dtype=np.uint64)
    assert np.array_equal(ctx.g2_msm(bases, s), orc.g2_msm(bases, s, parallel=True))


@pytest.mark.parametrize("g2", [False, True])
def test_msm_long_buckets_small_n(ctx, g2):
    """Below 2^17 points (one window group, the quad / pair fixups): all-ones
    scalars put every point into one bucket of window 0 -- n / 32 chunk pieces,
    summed by k_bucket_fixup_long -- and every other entry is a zero digit."""
    n = 20000
    k, _ = orc.fr_stream(75, n)
    bases = orc.g2_mul_gen(k[:2000]) if g2 else ctx.g1_mul_generator(k)
    if g2:
        bases = np.concatenate([bases] * (n // 2000))
    s = np.zeros((n, 4), dtype=np.uint64)
    s[:, 0] = 1
    s[::7, 0] = 2  # a second long bucket
    got = ctx.g2_msm(bases, s) if g2 else ctx.g1_msm(bases, s)
    ref = (orc.g2_msm if g2 else orc.g1_msm)(bases, s)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("world,lg", [(1, 16), (2, 16), (4, 16), (8, 16), (2, 18), (8, 20)])
def test_split_msm_shares_combine(ctx, world, lg):
    """Strong-scaled MSM pieces: the XYZZ shares of `world`
    equal point ranges (tpst_g1_msm_xyzz_dev), summed on the device
    (tpst_g1_xyzz_sum_dev), equal the MSM of all points.  (2, 18) and (8, 20)
    put exactly 2^17 points in each share -- the boundary of the
    window-grouped pipeline that configs[1] split over 8 GPUs hits; there the
    reference is (sum s_i k_i) G (bases k_i G)."""
    import torch
    from testudo_amd import sqrt_pst as S
    n = 1 << lg
    k, _ = orc.fr_stream(76, n)
    s, _ = orc.fr_stream(77, n)
    dev = torch.device("cuda", 0)
    d_k = torch.from_numpy(k.view(np.int64)).to(dev)
    d_s = torch.from_numpy(s.view(np.int64)).to(dev)
    d_b = torch.empty(n * 12, dtype=torch.int64, device=dev)
    ctx.torch_to_lib()
    ctx.g1_mul_generator_dev(d_k.data_ptr(), n, d_b.data_ptr())
    ctx.lib_to_torch()
    parts = torch.empty((world, 24), dtype=torch.int64, device=dev)
    R = n // world
    for g in range(world):
        S.g1_msm_partial_into(ctx, d_b.data_ptr(), d_s.data_ptr(), g * R, (g + 1) * R, parts[g])
    # a strided view of the shares (every other row of a wider buffer)
    wide = torch.zeros((2 * world, 24), dtype=torch.int64, device=dev)
    wide[::2] = parts
    out = S.g1_xyzz_combine(ctx, parts).cpu().numpy().view(np.uint64)
    out2 = S.g1_xyzz_combine(ctx, wide[::2]).cpu().numpy().view(np.uint64)
    if lg <= 16:
        ref = orc.g1_msm(orc.g1_mul_gen(k), s, parallel=True)
    else:
        si = [limbs_to_int(r) for r in s]
        ki = [limbs_to_int(r) for r in k]
        ref = orc.g1_mul_gen(fr_array([sum(a * b for a, b in zip(si, ki)) % O.R]))[0]
    assert np.array_equal(out, ref) and np.array_equal(out2, ref)


def test_msm_dev_pipelined_calls(ctx):
    """Back-to-back tpst_g1_msm_dev_async calls overlap (api.hip: call i+1's sort
    under call i's accumulation, its accumulation under call i's tail, three
    arenas in turn): five calls of mixed sizes -- window-grouped (tail
    off the bulk stream), single-group, empty -- into five outputs with no
    synchronisation in between, an entry point of another kind in the middle
    (it must see the pending results), then one tpst_synchronize.  Each output is
    (sum s_i k_i) G (bases k_i G)."""
    import torch
    n = (1 << 17) + 3
    k, _ = orc.fr_stream(81, n)
    dev = torch.device("cuda", 0)
    d_k = torch.from_numpy(k.view(np.int64)).to(dev)
    d_b = torch.empty(n * 12, dtype=torch.int64, device=dev)
    sets = [orc.fr_stream(82 + j, n)[0] for j in range(3)]
    d_s = [torch.from_numpy(s.view(np.int64)).to(dev) for s in sets]
    outs = torch.zeros((6, 12), dtype=torch.int64, device=dev)
    ctx.torch_to_lib()
    ctx.g1_mul_generator_dev(d_k.data_ptr(), n, d_b.data_ptr())
    calls = [(0, n), (1, 1000), (2, n), (0, 0), (1, n)]
    for o, (j, m) in enumerate(calls):
        ctx.g1_msm_dev_async(d_b.data_ptr(), d_s[j].data_ptr(), m, outs[o].data_ptr())
        if o == 2:  # another entry point between pipelined calls
            mid = ctx.g1_msm(orc.g1_mul_gen(k[:64]), sets[2][:64])
    ctx.g1_msm_dev_async(d_b.data_ptr(), d_s[2].data_ptr(), n, outs[5].data_ptr())
    ctx.synchronize()  # waits for the pending pipelined calls, not only the context stream
    got = outs.cpu().numpy().view(np.uint64)
    ki = [limbs_to_int(r) for r in k]

    def ref(j, m):
        si = [limbs_to_int(r) for r in sets[j][:m]]
        return orc.g1_mul_gen(fr_array([sum(a * b for a, b in zip(si, ki)) % O.R]))[0]

    for o, (j, m) in enumerate(calls + [(2, n)]):
        assert np.array_equal(got[o], ref(j, m)), (o, j, m)
    assert np.array_equal(mid, orc.g1_msm(orc.g1_mul_gen(k[:64]), sets[2][:64]))


def test_msm_dev_stream_ordered(ctx):
    """tpst_g1_msm_dev (the stream-safe form): work the caller
    queues straight on tpst_stream() after the calls -- a copy of the outputs,
    then overwriting the scalars -- is ordered after the MSMs without any
    further tpst_* call, so the copy holds the right results."""
    import torch
    n = (1 << 17) + 5
    k, _ = orc.fr_stream(91, n)
    dev = torch.device("cuda", 0)
    d_k = torch.from_numpy(k.view(np.int64)).to(dev)
    d_b = torch.empty(n * 12, dtype=torch.int64, device=dev)
    sets = [orc.fr_stream(92 + j, n)[0] for j in range(2)]
    d_s = [torch.from_numpy(s.view(np.int64)).to(dev) for s in sets]
    outs = torch.zeros((3, 12), dtype=torch.int64, device=dev)
    ctx.torch_to_lib()
    ctx.g1_mul_generator_dev(d_k.data_ptr(), n, d_b.data_ptr())
    calls = [(0, n), (1, n), (0, 777)]
    for o, (j, m) in enumerate(calls):
        ctx.g1_msm_dev(d_b.data_ptr(), d_s[j].data_ptr(), m, outs[o].data_ptr())
    lib = torch.cuda.ExternalStream(ctx.lib.tpst_stream(ctx.h), device=dev)
    with torch.cuda.stream(lib):
        snap = outs.clone()
        for t in d_s:
            t.zero_()
        outs.zero_()
    lib.synchronize()
    got = snap.cpu().numpy().view(np.uint64)
    ki = [limbs_to_int(r) for r in k]
    for o, (j, m) in enumerate(calls):
        si = [limbs_to_int(r) for r in sets[j][:m]]
        ref = orc.g1_mul_gen(fr_array([sum(a * b for a, b in zip(si, ki)) % O.R]))[0]
        assert np.array_equal(got[o], ref), (o, j, m)
    ctx.synchronize()


def test_xyzz_sum_rejects_misaligned_shares(ctx):
    """k_xyzz_sum reads shares with 16-byte loads: a share pointer or stride
    that is not 16-byte aligned is an argument error, not a misread."""
    import torch
    from testudo_amd import TpstError
    dev = torch.device("cuda", 0)
    buf = torch.zeros(3 * 26, dtype=torch.int64, device=dev)
    out = torch.empty(12, dtype=torch.int64, device=dev)
    with pytest.raises(TpstError):
        ctx.g1_xyzz_sum_dev(buf.data_ptr(), 2, 200, out.data_ptr())  # stride % 16 != 0
    with pytest.raises(TpstError):
        ctx.g1_xyzz_sum_dev(buf.data_ptr() + 8, 2, 208, out.data_ptr())  # base % 16 != 0
    ctx.torch_to_lib()
    ctx.g1_xyzz_sum_dev(buf.data_ptr(), 2, 208, out.data_ptr())  # zero shares: ZZ = 0, infinity
    ctx.lib_to_torch()
    assert not out.cpu().numpy().any()


def test_fr_sum_non_contiguous_gathered_view(ctx):
    """The C3 combine reads a torch-produced buffer on the library stream:
    a non-contiguous slice of a gathered tensor (the RCCL path's got[:, :N*4])
    is made contiguous on torch's stream and must be complete before
    tpst_fr_sum_dev reads it (tpst_wait_stream)."""
    import torch
    from testudo_amd import sqrt_pst as S
    k, w = 4, 1 << 14
    a, _ = orc.fr_stream(78, k * w)
    dev = torch.device("cuda", 0)
    for _ in range(3):
        big = torch.from_numpy(np.concatenate([a.reshape(k, -1), np.zeros((k, 12), np.uint64)], axis=1)
                               .view(np.int64)).to(dev)
        got = S.fr_sum(ctx, big[:, :w * 4]).cpu().numpy().view(np.uint64).reshape(-1, 4)
        ai = a.reshape(k, w, 4).astype(object)
        tot = sum(ai[:, :, t] << (64 * t) for t in range(4)).sum(axis=0) % O.R
        assert [limbs_to_int(x) for x in got] == list(tot)


def test_generator_muls_vs_oracle(ctx):
    k, _ = orc.fr_stream(61, 100)
    assert np.array_equal(ctx.g1_mul_generator(k), orc.g1_mul_gen(k))
    assert np.array_equal(ctx.g2_mul_generator(k[:20]), orc.g2_mul_gen(k[:20]))


# --------------------------------------------------------------- pairing --
def test_multi_pairing_golden(ctx):
    d = G.load("pairing.json")
    out = ctx.multi_pairing(G.g1_arr(d["g1"]), G.g2_arr(d["g2"]))
    assert gt_from_array(out) == G.gt(d["gt"])


def test_multi_pairing_vs_oracle_with_infinity(ctx):
    k, _ = orc.fr_stream(71, 40)
    g1 = orc.g1_mul_gen(k)
    g2 = orc.g2_mul_gen(k[::-1].copy())
    g1[3] = 0
    g2[7] = 0
    assert np.array_equal(ctx.multi_pairing(g1, g2), orc.multi_pairing(g1, g2))
    e = ctx.multi_pairing(g1[:0], g2[:0])  # empty product = 1
    assert e[0] == 1 and not e[1:].any()


def test_pairing_bilinearity(ctx):
    a, b = 123456789, 987654321
    P = orc.g1_mul_gen(fr_array([a]))
    Q = orc.g2_mul_gen(fr_array([b]))
    gen1 = orc.g1_mul_gen(fr_array([1]))
    gen2 = orc.g2_mul_gen(fr_array([a * b % O.R]))
    assert np.array_equal(ctx.multi_pairing(P, Q), ctx.multi_pairing(gen1, gen2))


# -------------------------------------------------------------- sqrt-PST --
def _golden_poly(ctx, n):
    from testudo_amd import sqrt_pst as S
    d = G.load("sqrt_pst_n%d.json" % n)
    S.srs_load(ctx, d["srs_nv"], G.srs_flat(d))
    pl = S.Polynomial.from_evaluations(ctx, G.fr_arr(d["Z"]))
    return d, pl


@pytest.mark.parametrize("n", [4, 5, 6, 7])
def test_sqrt_pst_golden(ctx, n):
    """benches/pst.rs flow at n = 4..7 against the Python oracle's values,
    every proof element bit-exact (incl. transcript-dependent MIPP values)."""
    from testudo_amd import sqrt_pst as S
    d, pl = _golden_poly(ctx, n)
    pt = G.fr_arr(d["point"])
    v = pl.eval(pt)
    assert limbs_to_int(v) == G.i(d["eval"])
    comms, T = pl.commit()
    assert np.array_equal(comms, G.g1_arr(d["comms"]))
    assert np.array_equal(T, G.gt_array(d["T"]))
    U, pst_proof, mipp = pl.open(S.PoseidonTranscript(), comms, pt, T)
    assert np.array_equal(U, G.g1_arr([d["U"]])[0])
    assert np.array_equal(pst_proof, G.g2_arr(d["pst_proof"]))
    assert np.array_equal(mipp.comms_u.reshape(-1, 12), G.g1_arr([p for pr in d["comms_u"] for p in pr]))
    assert np.array_equal(mipp.comms_t.reshape(-1, 72), np.stack([G.gt_array(t) for pr in d["comms_t"] for t in pr]))
    assert np.array_equal(mipp.final_a, G.g1_arr([d["final_a"]])[0])
    assert np.array_equal(mipp.final_h, G.g2_arr([d["final_h"]])[0])
    assert np.array_equal(mipp.pst_proof_h, G.g1_arr(d["pst_proof_h"]))
    assert S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, mipp, T)
    # tampering is caught
    bad_v = fr_array([(limbs_to_int(v) + 1) % O.R])[0]
    assert not S.verify(ctx, S.PoseidonTranscript(), U, pt, bad_v, pst_proof, mipp, T)


def test_srs_setup_matches_oracle(ctx):
    from testudo_amd import sqrt_pst as S
    for nv in (2, 3):
        S.srs_setup(ctx, nv, 0x7E57D1)
        assert np.array_equal(S.srs_export(ctx, nv), orc.SRS(nv, 0x7E57D1).export())


@pytest.mark.parametrize("n", [10, 11])
def test_sqrt_pst_vs_cpu_oracle(ctx, n):
    """benches/pst.rs-shaped config 1 (n = 10) and an odd size, full proof
    against the C++ oracle."""
    from testudo_amd import sqrt_pst as S
    nv = (n + 1) // 2
    S.srs_setup(ctx, nv, 0x7E57D1)
    srs = orc.SRS(nv, 0x7E57D1)
    Z, k = orc.fr_stream(0x7E57D0, 1 << n)
    pt, _ = orc.fr_stream(0x7E57D0, n, k)
    pl = S.Polynomial.from_evaluations(ctx, Z)
    v = pl.eval(pt)
    assert np.array_equal(v, orc.pst_eval(Z, n, pt))
    comms, T = pl.commit()
    c2, T2 = orc.pst_commit(srs, Z, n)
    assert np.array_equal(comms, c2) and np.array_equal(T, T2)
    U, pst_proof, mipp = pl.open(S.PoseidonTranscript(), comms, pt, T)
    pr = orc.pst_open(srs, Z, n, pt, comms)
    assert np.array_equal(U, pr["U"])
    assert np.array_equal(pst_proof, pr["pst_proof"])
    assert np.array_equal(mipp.comms_t, pr["comms_t"]) and np.array_equal(mipp.comms_u, pr["comms_u"])
    assert np.array_equal(mipp.final_a, pr["final_a"]) and np.array_equal(mipp.final_h, pr["final_h"])
    assert np.array_equal(mipp.pst_proof_h, pr["pst_proof_h"])
    assert orc.pst_verify(srs, n, pt, v, pr, T)


def test_commit_homomorphism_n20(ctx):
    """BASELINE config 3 size (2^20, 1024 x 1024), size-independent checks:
    sampled row commitments C_i == K2 MSM(powers_of_g[0], row_i); T == the IPP
    of the returned comm_list; and the sqrt_pst.rs:206 invariant
    c_u = MSM(comm_list, chi(b)) == commit(q) with q = Z^T chi(b) computed
    here on the host with Python integers."""
    from testudo_amd import sqrt_pst as S
    n = 20
    C = N = 1 << 10
    S.srs_setup(ctx, 10, 0x7E57D1)
    flat = S.srs_export(ctx, 10)
    pg0 = flat[36:36 + N * 12].reshape(N, 12)
    Z, k = S.fr_stream(0x7E57D0, 1 << n)
    pt, _ = S.fr_stream(0x7E57D0, n, k)
    pl = S.Polynomial.from_evaluations(ctx, Z)
    comms, T = pl.commit()
    for i in (0, 1, 517, 1023):
        row = Z[i::1024]
        assert np.array_equal(comms[i], ctx.g1_msm(pg0, row))
    assert np.array_equal(S.ipp(ctx, n, comms), T)
    # chi(b), b = point[m_row..], MSB-first (sqrt_pst.rs:152-166)
    b = [limbs_to_int(x) for x in pt[10:]]
    chis = [1] * C
    for i in range(C):
        for j in range(10):
            bit = (i >> (9 - j)) & 1
            chis[i] = chis[i] * (b[j] if bit else (1 - b[j])) % O.R
    zi = Z.astype(object)
    zv = (zi[:, 0] + (zi[:, 1] << 64) + (zi[:, 2] << 128) + (zi[:, 3] << 192)).reshape(N, C)
    q = [int(x) % O.R for x in zv.dot(np.array(chis, dtype=object))]
    pl.eval(pt)
    U, _, _ = pl.open(S.PoseidonTranscript(), comms, pt, T)
    assert np.array_equal(U, ctx.g1_msm(pg0, fr_array(q)))
    assert np.array_equal(U, ctx.g1_msm(comms, fr_array(chis)))


def test_commit_homomorphism_n23_long_chunks(ctx):
    """Batch commit at 2^23 (2048 rows x 4096): the accumulation runs 256-entry
    chunks (buckets of ~44 entries straddle chunk and workgroup boundaries,
    finished in-workgroup or by the workgroup fixup) and the bucket reduction
    runs L = 16 segments; sampled rows == the K2 MSM of the same row."""
    from testudo_amd import sqrt_pst as S
    n = 23
    S.srs_setup(ctx, 12, 0x7E57D1)
    flat = S.srs_export(ctx, 12)
    pg0 = flat[36:36 + 4096 * 12].reshape(4096, 12)
    Z, _ = S.fr_stream(0x7E57D0 + 23, 1 << n)
    pl = S.Polynomial.from_evaluations(ctx, Z)
    comms, T = pl.commit()
    C = 1 << (n // 2)
    for i in (0, 1, 1000, C - 1):
        assert np.array_equal(comms[i], ctx.g1_msm(pg0, Z[i::C])), i
    for i in (1, C - 1):  # and against the CPU oracle (not only HIP vs HIP)
        assert np.array_equal(comms[i], orc.g1_msm(pg0, np.ascontiguousarray(Z[i::C]), parallel=True)), i
    del pl


def test_commit_rows_and_ipp_match_full_commit(ctx):
    """The per-rank pieces of the sharded commit:
    row blocks concatenate to the full comm_list and ipp(comm_list) == T."""
    from testudo_amd import sqrt_pst as S
    for n in (9, 12):
        nv = (n + 1) // 2
        S.srs_setup(ctx, nv, 0x7E57D1)
        Z, _ = S.fr_stream(0x7E57D0 + n, 1 << n)
        pl = S.Polynomial.from_evaluations(ctx, Z)
        comms, T = pl.commit()
        C = 1 << (n // 2)
        parts = [pl.commit_rows(r, r + C // 4) for r in range(0, C, C // 4)]
        assert np.array_equal(np.concatenate(parts), comms)
        assert np.array_equal(S.ipp(ctx, n, comms), T)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_commit_rows_partial_world_split(ctx, world):
    """Row-sharded commit with the IPP split by rows: each
    share's Miller-loop partial equals the C++ oracle's unreduced product of
    the same pairs, and FE(prod of the shares) == T of the full commit."""
    from testudo_amd import sqrt_pst as S
    n = 11
    nv = (n + 1) // 2
    S.srs_setup(ctx, nv, 0x7E57D1)
    flat = S.srs_export(ctx, nv)
    C, Rn = 1 << (n // 2), 1 << nv
    off = 36 + Rn * 12  # powers_of_h[0]; n odd -> powers_of_h[1]
    off += Rn * 24 + (Rn // 2) * 12
    hvec = flat[off:off + C * 24].reshape(C, 24)
    Z, _ = S.fr_stream(0x7E57D0 + world, 1 << n)
    pl = S.Polynomial.from_evaluations(ctx, Z)
    comms, T = pl.commit()
    R = C // world
    shares = [pl.commit_rows_partial(r, r + R) for r in range(0, C, R)]
    assert np.array_equal(np.concatenate([c for c, _ in shares]), comms)
    ml = np.stack([m for _, m in shares])
    assert np.array_equal(ml[0], orc.miller_product(comms[:R], hvec[:R]))
    assert np.array_equal(S.gt_final_exp_product(ctx, ml), T)
    assert np.array_equal(orc.gt_final_exp_product(ml), T)


@pytest.mark.parametrize("g2", [False, True])
def test_fixed_base_grouped_msm_vs_oracle(ctx, g2):
    """csrc/fbt.h lookup-table MSM: plain (one group), MIPP-fold groups
    (D = 1) and cross-product groups (D = L/2), against the oracle MSM of
    each group's members; includes an infinity base and edge scalars."""
    n = 64
    k, _ = orc.fr_stream(81, n)
    s, _ = orc.fr_stream(82, n)
    bases = orc.g2_mul_gen(k) if g2 else orc.g1_mul_gen(k)
    bases[5] = 0
    s[0] = fr_array([O.R - 1])[0]
    s[1] = 0
    s[2] = fr_array([1])[0]
    ref_msm = orc.g2_msm if g2 else orc.g1_msm
    for L, D in ((n, n), (16, 1), (16, 8), (8, 2)):
        got = ctx.msm_fixed(bases, s, L, D, g2=g2)
        for g in range(L // D):
            idx = [(m // D) * L + g * D + m % D for m in range(n // L * D)]
            assert np.array_equal(got[g], ref_msm(bases[idx], s[idx])), (L, D, g)


@pytest.mark.parametrize("n,world", [(12, 4), (13, 2)])
def test_column_slice_upload_matches_full_commit(ctx, n, world):
    """Multi-GPU shard upload: a rank that uploads only its
    column block [c0, c1) of the strided view (one 2D copy) commits exactly
    the same rows and Miller partial as the whole-polynomial handle; the
    operations that need all of Z refuse a slice."""
    from testudo_amd import TpstError
    from testudo_amd import sqrt_pst as S
    nv = (n + 1) // 2
    S.srs_setup(ctx, nv, 0x7E57D1)
    Z, _ = S.fr_stream(0x7E57D0 + 3 * n, 1 << n)
    full = S.Polynomial.from_evaluations(ctx, Z)
    comms, T = full.commit()
    C = 1 << (n // 2)
    R = C // world
    parts = []
    for g in range(world):
        sl = S.Polynomial.from_evaluations_cols(ctx, Z, g * R, (g + 1) * R)
        c, ml = sl.commit_rows_partial(g * R, (g + 1) * R)
        c2, ml2 = full.commit_rows_partial(g * R, (g + 1) * R)
        assert np.array_equal(c, comms[g * R:(g + 1) * R]) and np.array_equal(ml, ml2)
        parts.append(ml)
        with pytest.raises(TpstError):
            sl.commit_rows(0 if g else R, (g + 2) * R if g + 2 <= world else C)  # outside the slice
        with pytest.raises(TpstError):
            sl.eval(np.zeros((n, 4), dtype=np.uint64))
    assert np.array_equal(S.gt_final_exp_product(ctx, np.stack(parts)), T)


@pytest.mark.parametrize("n,world", [(11, 4), (12, 2)])
def test_sharded_opening_matches_single_process(ctx, n, world):
    """Row-sharded opening: every rank's column-slice
    handle computes its rows' share of get_q's z_q and of c_u; the mod-r sum
    (tpst_fr_sum_dev) and the G1 sum give q and U; the opening-only handle
    (tpst_poly_from_q_dev) evaluates and opens to the same bytes as the
    whole-polynomial handle, and the proof verifies.  The device-buffer
    variants of the commit share and of the final exponentiation agree with
    the host ones."""
    import torch
    from testudo_amd import sqrt_pst as S
    nv = (n + 1) // 2
    S.srs_setup(ctx, nv, 0x7E57D1)
    Z, k = S.fr_stream(0x7E57D0 + 5 * n, 1 << n)
    pt, _ = S.fr_stream(0x7E57D0 + 5 * n, n, k)
    full = S.Polynomial.from_evaluations(ctx, Z)
    comms, T = full.commit()
    v = full.eval(pt)
    U, pst_proof, mipp = full.open(S.PoseidonTranscript(), comms, pt, T)
    C = 1 << (n // 2)
    N = 1 << (n - n // 2)
    R = C // world
    dev = torch.device("cuda", 0)
    zq_parts = torch.empty((world, N * 4), dtype=torch.int64, device=dev)
    cm_parts = torch.empty((world, R * 12 + 72), dtype=torch.int64, device=dev)
    cu = []
    for g in range(world):
        sl = S.Polynomial.from_evaluations_cols(ctx, Z, g * R, (g + 1) * R)
        sl.get_q_partial_into(pt, g * R, (g + 1) * R, zq_parts[g])
        host = sl.get_q_partial(pt, g * R, (g + 1) * R)
        assert np.array_equal(zq_parts[g].cpu().numpy().view(np.uint64).reshape(-1, 4), host)
        sl.commit_rows_partial_into(g * R, (g + 1) * R, cm_parts[g])
        c, ml = sl.commit_rows_partial(g * R, (g + 1) * R)
        got = cm_parts[g].cpu().numpy().view(np.uint64)
        assert np.array_equal(got[:12 * R].reshape(R, 12), c) and np.array_equal(got[12 * R:], ml)
        cu.append(S.cu_partial(ctx, n, pt, g * R, (g + 1) * R, c))
    assert np.array_equal(S.gt_final_exp_product_gathered(ctx, cm_parts, R), T)
    zq = S.fr_sum(ctx, zq_parts)
    Uc = S.g1_sum(ctx, np.stack(cu))
    assert np.array_equal(Uc, U)
    for Ugiven in (Uc, None):
        pq = S.Polynomial.from_q(ctx, n, pt, zq, Ugiven)
        assert np.array_equal(pq.eval(pt), v)
        U2, pst2, mipp2 = pq.open(S.PoseidonTranscript(), comms, pt, T)
        assert np.array_equal(U2, U) and np.array_equal(pst2, pst_proof)
        for f in ("comms_t", "comms_u", "final_a", "final_h", "pst_proof_h"):
            assert np.array_equal(getattr(mipp2, f), getattr(mipp, f)), f
    assert S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, mipp, T)
