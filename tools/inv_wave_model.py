"""Exact model of the wave-cooperative Fq inversion (field29.h inv_wave):
Pornin's binary GCD with 15-divstep batches on 32-bit approximations, the
big values a, b, u, v as 28 limbs of 15 bits, one limb per lane.  Every
lane-parallel step (limb products, the two local carry passes, the ballot
carry resolution, the shift that divides by 2^15) is modelled as the device
code computes it, so the model fixes the algorithm before the kernel.
    python tools/inv_wave_model.py      (random + edge inputs, asserts)"""
import random

P = 0x01AE3A4617C510EAC63B05C06CA1493B1A22D9F300F5138F1EF3622FBA094800170B5D44300000008508C00000000001
NL = 28          # limbs (420 bits: the update before / 2^15 reaches 2^401)
LB = 15          # bits per limb
LM = (1 << LB) - 1
K = 15           # divsteps per outer iteration
ITERS = -(-(2 * 377 - 1) // K)   # 51
P_L = [(P >> (LB * i)) & LM for i in range(NL)]


def to_limbs(x):
    assert 0 <= x < 1 << (LB * NL)
    return [(x >> (LB * i)) & LM for i in range(NL)]


def from_limbs(l):
    return sum(v << (LB * i) for i, v in enumerate(l))


def i32(x):
    assert -(1 << 31) <= x < (1 << 31), x
    return x


def normalize(t):
    """limb sums t_i (int32, |t_i| < 2^31) -> two's complement limbs of their
    value mod 2^(15 NL), as inv_wave computes them: a bias makes every limb
    nonnegative (2^31 into limb i, 2^16 out of limb i+1: the biases sum to
    2^(16 + 15 NL) = 0 mod 2^(15 NL)), two local carry passes leave limbs
    <= 2^15 + 3, and one ballot-mask pass resolves the remaining +1 ripples"""
    t = [i32(x) for x in t]
    u = [(t[i] + (1 << 31) - (0 if i == 0 else 1 << 16)) for i in range(NL)]
    assert all(0 <= x < 1 << 32 for x in u)
    for _ in range(2):
        c = [x >> LB for x in u]
        u = [(u[i] & LM) + (c[i - 1] if i else 0) for i in range(NL)]
    assert all(0 <= x <= LM + 4 for x in u)
    g = sum(1 << i for i in range(NL) if u[i] > LM)
    base = [x & LM for x in u]
    pr = sum(1 << i for i in range(NL) if base[i] == LM)
    cin = ((g << 1) + pr) ^ pr
    return [(base[i] + ((cin >> i) & 1)) & LM for i in range(NL)]


def div_signed(t):
    """(value of limb sums t) / 2^15 as (negative?, magnitude limbs)"""
    lim = normalize(t)
    neg = (lim[NL - 1] >> (LB - 1)) & 1 == 1
    if neg:  # magnitude: invert the limbs, add 1 (ballot ripple from lane 0)
        inv = [LM - x for x in lim]
        pr = sum(1 << i for i in range(NL) if inv[i] == LM)
        cin = (1 + pr) ^ pr
        lim = [(inv[i] + ((cin >> i) & 1)) & LM for i in range(NL)]
    assert lim[0] == 0, "not divisible"
    return neg, lim[1:] + [0]


def lincomb(xm, xs, f, ym, ys, g, kp=0):
    """(sign xs * xm * f + sign ys * ym * g + kp * p) / 2^15 -> (neg, magnitude limbs)"""
    ff = -f if xs else f
    gg = -g if ys else g
    t = [xm[i] * ff + ym[i] * gg + kp * P_L[i] for i in range(NL)]
    return div_signed(t)


def inv_model(y):
    a = to_limbs(y)
    b = P_L[:]
    u, us = to_limbs(1), False
    v, vs = to_limbs(0), False
    for it in range(ITERS):
        av, bv = from_limbs(a), from_limbs(b)
        nb = max(av.bit_length(), bv.bit_length())
        n = max(nb, 2 * K + 2)
        ab = (av & ((1 << K) - 1)) | (((av >> (n - K - 2)) & ((1 << (K + 2)) - 1)) << K)
        bb = (bv & ((1 << K) - 1)) | (((bv >> (n - K - 2)) & ((1 << (K + 2)) - 1)) << K)
        f0, g0, f1, g1 = 1, 0, 0, 1
        for _ in range(K):
            if ab & 1:
                if ab < bb:
                    ab, bb = bb, ab
                    f0, f1 = f1, f0
                    g0, g1 = g1, g0
                ab -= bb
                f0 -= f1
                g0 -= g1
            ab >>= 1
            f1 += f1
            g1 += g1
        assert abs(f0) + abs(g0) <= 1 << K and abs(f1) + abs(g1) <= 1 << K
        sa, na = lincomb(a, False, f0, b, False, g0)
        sb, nbl = lincomb(a, False, f1, b, False, g1)
        if sa:
            f0, g0 = -f0, -g0
        if sb:
            f1, g1 = -f1, -g1
        # u, v: signed values, Montgomery step k p clears the low 15 bits
        t0 = (-u[0] * f0 if us else u[0] * f0) + (-v[0] * g0 if vs else v[0] * g0)
        k0 = (-t0) & LM
        t1 = (-u[0] * f1 if us else u[0] * f1) + (-v[0] * g1 if vs else v[0] * g1)
        k1 = (-t1) & LM
        nus, nu = lincomb(u, us, f0, v, vs, g0, k0)
        nvs, nv = lincomb(u, us, f1, v, vs, g1, k1)
        a, b, u, us, v, vs = na, nbl, nu, nus, nv, nvs
    # b = 1 and b = v y (mod p): v = y^-1 (exactly tracked, |v| < 52 p)
    assert from_limbs(b) == 1, from_limbs(b)
    vv = from_limbs(v)
    assert vv < 52 * P
    vv = -vv if vs else vv
    return vv % P


def divsteps_var(eta, f0, g0):
    """Bernstein-Yang divsteps, variable time (libsecp256k1 modinv32's
    divsteps_30_var shape) on the low 30 bits of the signed f, g (uint32
    wraparound, as the scalar unit computes them): K divsteps -> eta and the
    transition matrix (u, v, q, r), |u| + |v| <= 2^K, f' = (u f + v g) / 2^K,
    g' = (q f + r g) / 2^K.  Each inner iteration skips g's trailing zeros and
    cancels up to min(eta + 1, i) low bits of g with one multiple of f (f^-1
    mod 2^16 by three Newton steps)."""
    M32 = (1 << 32) - 1
    u, v, q, r = 1, 0, 0, 1
    f, g = f0 & M32, g0 & M32
    i = K
    iters = 0
    while True:
        iters += 1
        gg = (g | (M32 << i)) & M32
        zeros = (gg & -gg).bit_length() - 1
        g >>= zeros
        u <<= zeros
        v <<= zeros
        eta -= zeros
        i -= zeros
        if i == 0:
            break
        if eta < 0:
            eta = -eta
            f, g = g, (-f) & M32
            u, q = q, -u
            v, r = r, -v
        limit = min(eta + 1, i)
        m = (1 << limit) - 1
        x = f
        for _ in range(3):
            x = (x * (2 - f * x)) & 0xFFFF
        w = ((-g) * x) & m
        g = (g + f * w) & M32
        q += u * w
        r += v * w
    assert abs(u) + abs(v) <= 1 << K and abs(q) + abs(r) <= 1 << K
    return eta, u, v, q, r, iters


def low30(mag, neg):
    x = mag[0] | (mag[1] << LB)
    return (-x) & 0xFFFFFFFF if neg else x


def inv_model_by(y):
    """inv_wave's Bernstein-Yang form: f = p, g = y; d, e the signed cofactors
    (f = d y, g = e y mod p, both sides divided by 2^15 per batch, the k p step
    keeping the division exact); stop when g = 0, then f = +-1 and
    y^-1 = +-d."""
    f, fs = P_L[:], False
    g, gs = to_limbs(y), False
    d, ds = to_limbs(0), False
    e, es = to_limbs(1), False
    eta = -1
    batches = iters = 0
    while any(g):
        eta, u, v, q, r, it = divsteps_var(eta, low30(f, fs), low30(g, gs))
        iters += it
        batches += 1
        nfs, nf = lincomb(f, fs, u, g, gs, v)
        ngs, ng = lincomb(f, fs, q, g, gs, r)
        ud = -u if ds else u
        ve = -v if es else v
        qd = -q if ds else q
        re = -r if es else r
        kd = (-(d[0] * ud + e[0] * ve)) & LM
        ke = (-(d[0] * qd + e[0] * re)) & LM
        nds, nd = lincomb(d, ds, u, e, es, v, kd)
        nes, ne = lincomb(d, ds, q, e, es, r, ke)
        f, fs, g, gs, d, ds, e, es = nf, nfs, ng, ngs, nd, nds, ne, nes
        assert batches <= 80  # inv_wave.h BY_MAX_BATCHES (73 batches cover the 1091-divstep bound)
    assert from_limbs(f) == 1, from_limbs(f)
    dv = from_limbs(d)
    assert dv < 80 * P
    neg = ds != fs
    return (-dv if neg else dv) % P, batches, iters


def main():
    random.seed(5)
    ys = [1, 2, 3, P - 1, P - 2, (1 << 376) + 12345, P // 2] + [random.randrange(1, P) for _ in range(300)]
    for y in ys:
        r = inv_model(y)
        assert r * y % P == 1, y
    print("inv_wave model ok: %d iterations of %d divsteps" % (ITERS, K))
    nb = ni = mb = 0
    for y in ys:
        r, b, it = inv_model_by(y)
        assert r * y % P == 1, y
        nb += b
        ni += it
        mb = max(mb, b)
    print("Bernstein-Yang variable-time form ok: %.1f batches (max %d), %.1f inner iterations per inverse"
          % (nb / len(ys), mb, ni / len(ys)))


if __name__ == "__main__":
    main()
