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


def main():
    random.seed(5)
    for y in [1, 2, 3, P - 1, P - 2, (1 << 376) + 12345, P // 2] + [random.randrange(1, P) for _ in range(300)]:
        r = inv_model(y)
        assert r * y % P == 1, y
    print("inv_wave model ok: %d iterations of %d divsteps" % (ITERS, K))


if __name__ == "__main__":
    main()
