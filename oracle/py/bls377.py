"""BLS12-377 arithmetic restated in pure Python big integers.

TEST INFRASTRUCTURE ONLY.  This module is the slow, first-principles oracle
used by ``tests/`` and by ``oracle/py/gen_golden.py`` to produce the committed
golden vectors.  The product (``testudo_amd``) never imports it.

What it restates (the arithmetic lives in un-vendored arkworks crates, see
SURVEY.md §8(c)):

* ark-bls12-377 0.4: Fq (377-bit), Fr (253-bit), G1: y^2 = x^3 + 1,
  G2 on the D-type twist y^2 = x^3 + 1/u over Fq2 = Fq[u]/(u^2 + 5),
  Fq6 = Fq2[v]/(v^3 - u), Fq12 = Fq6[w]/(w^2 - v).
* ark-ec 0.4 ``Bls12::multi_pairing``: optimal-ate Miller loop over
  x = 0x8508c00000000001 followed by the final exponentiation of
  eprint 2020/875 (gnark/arkworks chain), whose exponent is
  3 * (p^12 - 1) / r.  Two independent restatements are given:
  ``pairing_textbook`` (affine lines, direct exponentiation by
  3(p^12-1)/r) and ``pairing_ark`` (arkworks' projective line
  coefficients + the 2020/875 addition chain).  Tests check they agree.

Fq12 is held as a polynomial in w of degree < 12 with w^12 = -5
(w^2 = v, w^6 = u), which is the same field as the tower; ``fq12_to_tower``
gives arkworks' coefficient order for serialization.
"""

from __future__ import annotations

P = 0x01AE3A4617C510EAC63B05C06CA1493B1A22D9F300F5138F1EF3622FBA094800170B5D44300000008508C00000000001
R = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001
X = 0x8508C00000000001  # BLS parameter (positive), ark-bls12-377 Config::X

G1_GEN = (
    0x8848DEFE740A67C8FC6225BF87FF5485951E2CAA9D41BB188282C8BD37CB5CD5481512FFCD394EEAB9B16EB21BE9EF,
    0x1914A69C5102EFF1F674F5D30AFEEC4BD7FB348CA3E52D96D182AD44FB82305C2FE3D3634A9591AFD82DE55559C8EA6,
)
G2_GEN = (
    (0x018480BE71C785FEC89630A2A3841D01C565F071203E50317EA501F557DB6B9B71889F52BB53540274E3E48F7C005196,
     0x00EA6040E700403170DC5A51B1B140D5532777EE6651CECBE7223ECE0799C9DE5CF89984BFF76FE6B26BFEFA6EA16AFE),
    (0x00690D665D446F7BD960736BCBB2EFB4DE03ED7274B49A58E458C282F832D204F2CF88886D8C7C2EF094094409FD4DDF,
     0x00F8169FD28355189E549DA3151A70AA61EF11AC3D591BF12463B01ACEE304C24279B83F5E52270BD9A1CDD185EB8F93),
)

# ---------------------------------------------------------------- Fq2 -----
# Fq2 = Fq[u]/(u^2 + 5); elements are (c0, c1) = c0 + c1*u.
NONRES = P - 5


def f2(a, b=0):
    return (a % P, b % P)


F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - 5 * a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_mul_fq(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_inv(a):
    n = (a[0] * a[0] + 5 * a[1] * a[1]) % P
    ni = pow(n, -1, P)
    return (a[0] * ni % P, (-a[1]) * ni % P)


G2_B = (0, (-pow(5, -1, P)) % P)  # b' = 1/u = -u/5  (ark-bls12-377 g2 COEFF_B)


# -------------------------------------------------------------- fields ----
class _FqOps:
    zero, one = 0, 1
    add = staticmethod(lambda a, b: (a + b) % P)
    sub = staticmethod(lambda a, b: (a - b) % P)
    mul = staticmethod(lambda a, b: a * b % P)
    neg = staticmethod(lambda a: (-a) % P)
    inv = staticmethod(lambda a: pow(a, -1, P))
    b = 1


class _Fq2Ops:
    zero, one = F2_ZERO, F2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    neg = staticmethod(f2_neg)
    inv = staticmethod(f2_inv)
    b = G2_B


# -------------------------------------------------------------- curves ----
# Affine points are tuples (x, y); the point at infinity is None.
def _on_curve(F, pt):
    if pt is None:
        return True
    x, y = pt
    return F.sub(F.mul(y, y), F.add(F.mul(F.mul(x, x), x), F.b)) == F.zero


def _add_affine(F, a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if a[1] == b[1] and a[1] != F.zero:
            return _dbl_affine(F, a)
        return None
    lam = F.mul(F.sub(b[1], a[1]), F.inv(F.sub(b[0], a[0])))
    x3 = F.sub(F.sub(F.mul(lam, lam), a[0]), b[0])
    y3 = F.sub(F.mul(lam, F.sub(a[0], x3)), a[1])
    return (x3, y3)


def _dbl_affine(F, a):
    if a is None or a[1] == F.zero:
        return None
    x, y = a
    x2 = F.mul(x, x)
    lam = F.mul(F.add(F.add(x2, x2), x2), F.inv(F.add(y, y)))
    x3 = F.sub(F.mul(lam, lam), F.add(x, x))
    y3 = F.sub(F.mul(lam, F.sub(x, x3)), y)
    return (x3, y3)


# Jacobian (X, Y, Z) for fast scalar multiplication; Z == zero means infinity.
def _jac_dbl(F, p):
    X1, Y1, Z1 = p
    if Z1 == F.zero or Y1 == F.zero:
        return (F.one, F.one, F.zero)
    A = F.mul(X1, X1)
    B = F.mul(Y1, Y1)
    C = F.mul(B, B)
    t = F.add(X1, B)
    D = F.sub(F.sub(F.mul(t, t), A), C)
    D = F.add(D, D)
    E = F.add(F.add(A, A), A)
    Fv = F.mul(E, E)
    X3 = F.sub(Fv, F.add(D, D))
    C8 = F.add(C, C)
    C8 = F.add(C8, C8)
    C8 = F.add(C8, C8)
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
    Z3 = F.mul(Y1, Z1)
    Z3 = F.add(Z3, Z3)
    return (X3, Y3, Z3)


def _jac_add_affine(F, p, q):
    if q is None:
        return p
    X1, Y1, Z1 = p
    if Z1 == F.zero:
        return (q[0], q[1], F.one)
    Z1Z1 = F.mul(Z1, Z1)
    U2 = F.mul(q[0], Z1Z1)
    S2 = F.mul(F.mul(q[1], Z1), Z1Z1)
    H = F.sub(U2, X1)
    rr = F.sub(S2, Y1)
    if H == F.zero:
        if rr == F.zero:
            return _jac_dbl(F, p)
        return (F.one, F.one, F.zero)
    HH = F.mul(H, H)
    HHH = F.mul(H, HH)
    V = F.mul(X1, HH)
    X3 = F.sub(F.sub(F.mul(rr, rr), HHH), F.add(V, V))
    Y3 = F.sub(F.mul(rr, F.sub(V, X3)), F.mul(Y1, HHH))
    Z3 = F.mul(Z1, H)
    return (X3, Y3, Z3)


def _jac_to_affine(F, p):
    X1, Y1, Z1 = p
    if Z1 == F.zero:
        return None
    zi = F.inv(Z1)
    zi2 = F.mul(zi, zi)
    return (F.mul(X1, zi2), F.mul(F.mul(Y1, zi2), zi))


def _mul(F, pt, k):
    k %= R  # callers only multiply points of order r
    if pt is None or k == 0:
        return None
    acc = (F.one, F.one, F.zero)
    for bit in bin(k)[2:]:
        acc = _jac_dbl(F, acc)
        if bit == "1":
            acc = _jac_add_affine(F, acc, pt)
    return _jac_to_affine(F, acc)


def _mul_raw(F, pt, k):
    """Scalar multiplication without reducing k mod r (for subgroup checks)."""
    if pt is None or k == 0:
        return None
    acc = (F.one, F.one, F.zero)
    for bit in bin(k)[2:]:
        acc = _jac_dbl(F, acc)
        if bit == "1":
            acc = _jac_add_affine(F, acc, pt)
    return _jac_to_affine(F, acc)


def _neg(F, pt):
    return None if pt is None else (pt[0], F.neg(pt[1]))


def g1_add(a, b):
    return _add_affine(_FqOps, a, b)


def g1_neg(a):
    return _neg(_FqOps, a)


def g1_mul(a, k):
    return _mul(_FqOps, a, k)


def g1_on_curve(a):
    return _on_curve(_FqOps, a)


def g2_add(a, b):
    return _add_affine(_Fq2Ops, a, b)


def g2_neg(a):
    return _neg(_Fq2Ops, a)


def g2_mul(a, k):
    return _mul(_Fq2Ops, a, k)


def g2_on_curve(a):
    return _on_curve(_Fq2Ops, a)


def g1_in_subgroup(a):
    return _mul_raw(_FqOps, a, R) is None


def g2_in_subgroup(a):
    return _mul_raw(_Fq2Ops, a, R) is None


def _msm(F, bases, scalars):
    """sum_i scalars[i] * bases[i]; truncates to the shorter input like
    ark-ec ``VariableBaseMSM::msm_unchecked``."""
    n = min(len(bases), len(scalars))
    acc = (F.one, F.one, F.zero)
    # simple 4-bit fixed-window Straus over all points (correctness only)
    tables = []
    for i in range(n):
        t = [None, bases[i]]
        for _ in range(14):
            t.append(_add_affine(F, t[-1], bases[i]))
        tables.append(t)
    sc = [scalars[i] % R for i in range(n)]
    for w in range(63, -1, -1):
        for _ in range(4):
            acc = _jac_dbl(F, acc)
        for i in range(n):
            d = (sc[i] >> (4 * w)) & 15
            if d:
                acc = _jac_add_affine(F, acc, tables[i][d])
    return _jac_to_affine(F, acc)


def g1_msm(bases, scalars):
    return _msm(_FqOps, bases, scalars)


def g2_msm(bases, scalars):
    return _msm(_Fq2Ops, bases, scalars)


# --------------------------------------------------------------- Fq12 -----
# Element = list of 12 ints a[k], value sum a[k] w^k, w^12 = -5.
def f12_one():
    return [1] + [0] * 11


def f12_mul(a, b):
    t = [0] * 23
    for i, ai in enumerate(a):
        if ai:
            for j, bj in enumerate(b):
                t[i + j] += ai * bj
    return [(t[k] - 5 * t[k + 12]) % P for k in range(11)] + [t[11] % P]


def f12_sqr(a):
    return f12_mul(a, a)


def f12_inv(a):
    """Inverse by Gaussian elimination on the 12x12 multiplication matrix."""
    cols = []
    for k in range(12):
        e = [0] * 12
        e[k] = 1
        cols.append(f12_mul(a, e))
    # M[row][col] = coefficient row of a*w^col ; solve M x = e0
    M = [[cols[c][r_] for c in range(12)] + [1 if r_ == 0 else 0] for r_ in range(12)]
    for c in range(12):
        piv = next(r_ for r_ in range(c, 12) if M[r_][c] % P)
        M[c], M[piv] = M[piv], M[c]
        iv = pow(M[c][c], -1, P)
        M[c] = [v * iv % P for v in M[c]]
        for r_ in range(12):
            if r_ != c and M[r_][c]:
                fct = M[r_][c]
                M[r_] = [(v - fct * w) % P for v, w in zip(M[r_], M[c])]
    return [M[r_][12] for r_ in range(12)]


def f12_pow(a, e):
    res = f12_one()
    base = a
    while e:
        if e & 1:
            res = f12_mul(res, base)
        e >>= 1
        if e:
            base = f12_sqr(base)
    return res


# Frobenius: (sum a_k w^k)^(p^j) = sum a_k gamma_{j,k} w^k with
# gamma_{j,k} = (-5)^{k (p^j - 1) / 12}  (p = 1 mod 12).
_FROB = {}


def f12_frob(a, j=1):
    j %= 12
    if j not in _FROB:
        e = (P ** j - 1) // 12
        g = pow(P - 5, e, P)
        _FROB[j] = [pow(g, k, P) for k in range(12)]
    gam = _FROB[j]
    return [a[k] * gam[k] % P for k in range(12)]


def f12_conj(a):
    """a^(p^6): the cyclotomic inverse on GT."""
    return f12_frob(a, 6)


def fq2_to_f12(c, k):
    """Place Fq2 element c at w^k (u = w^6)."""
    out = [0] * 12
    out[k] = c[0]
    out[k + 6] = c[1]
    return out


def fq12_to_tower(a):
    """Poly form -> arkworks coefficient order
    (c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1): 12 Fq."""
    out = []
    for half in (0, 1):
        for j in range(3):
            out.append(a[2 * j + half])       # Fq2.c0  at w^(2j+half)
            out.append(a[2 * j + half + 6])   # Fq2.c1  at w^(2j+half+6)
    return out


def fq12_from_tower(t):
    a = [0] * 12
    idx = 0
    for half in (0, 1):
        for j in range(3):
            a[2 * j + half] = t[idx] % P
            a[2 * j + half + 6] = t[idx + 1] % P
            idx += 2
    return a


# ------------------------------------------------------------- pairing ----
FINAL_EXP = 3 * (P ** 12 - 1) // R


def _line_eval(lam, xt, yt, Pg1):
    """Line through T' (on the twist) with slope lam', evaluated at the
    untwisted P: y_P - lam' x_P w + (lam' x_T - y_T) w^3."""
    xp, yp = Pg1
    out = [0] * 12
    out[0] = yp
    c = f2_mul_fq(lam, xp)
    out[1] = (-c[0]) % P
    out[7] = (-c[1]) % P
    d = f2_sub(f2_mul(lam, xt), yt)
    out[3] = d[0]
    out[9] = d[1]
    return out


def miller_textbook(Pg1, Qg2):
    """f_{x,Q}(P) with affine chord/tangent lines (vertical lines omitted:
    they lie in a proper subfield and die in the final exponentiation)."""
    f = f12_one()
    T = Qg2
    for bit in bin(X)[3:]:
        x, y = T
        x2 = f2_sqr(x)
        lam = f2_mul(f2_add(f2_add(x2, x2), x2), f2_inv(f2_add(y, y)))
        f = f12_mul(f12_sqr(f), _line_eval(lam, x, y, Pg1))
        T = g2_add(T, T)
        if bit == "1":
            x, y = T
            lam = f2_mul(f2_sub(Qg2[1], y), f2_inv(f2_sub(Qg2[0], x)))
            f = f12_mul(f, _line_eval(lam, x, y, Pg1))
            T = g2_add(T, Qg2)
    return f


def pairing_textbook(Pg1, Qg2):
    if Pg1 is None or Qg2 is None:
        return f12_one()
    return f12_pow(miller_textbook(Pg1, Qg2), FINAL_EXP)


# arkworks-shaped: projective G2Prepared coefficients (ark-ec bls12/g2.rs
# double_in_place / add_in_place, TwistType::D) and Bls12::ell.
TWO_INV = pow(2, -1, P)


def g2_prepare(Q):
    coeffs = []
    rx, ry, rz = Q[0], Q[1], F2_ONE
    for bit in bin(X)[3:]:
        # doubling step
        a = f2_mul_fq(f2_mul(rx, ry), TWO_INV)
        b = f2_sqr(ry)
        c = f2_sqr(rz)
        e = f2_mul(G2_B, f2_add(f2_add(c, c), c))
        f_ = f2_add(f2_add(e, e), e)
        g = f2_mul_fq(f2_add(b, f_), TWO_INV)
        h = f2_sub(f2_sqr(f2_add(ry, rz)), f2_add(b, c))
        i = f2_sub(e, b)
        j = f2_sqr(rx)
        e2 = f2_sqr(e)
        rx = f2_mul(a, f2_sub(b, f_))
        ry = f2_sub(f2_sqr(g), f2_add(f2_add(e2, e2), e2))
        rz = f2_mul(b, h)
        coeffs.append((f2_neg(h), f2_add(f2_add(j, j), j), i))
        if bit == "1":
            theta = f2_sub(ry, f2_mul(Q[1], rz))
            lam = f2_sub(rx, f2_mul(Q[0], rz))
            c_ = f2_sqr(theta)
            d = f2_sqr(lam)
            e_ = f2_mul(lam, d)
            ff = f2_mul(rz, c_)
            gg = f2_mul(rx, d)
            hh = f2_sub(f2_add(e_, ff), f2_add(gg, gg))
            rx = f2_mul(lam, hh)
            ry = f2_sub(f2_mul(theta, f2_sub(gg, hh)), f2_mul(e_, ry))
            rz = f2_mul(rz, e_)
            jj = f2_sub(f2_mul(theta, Q[0]), f2_mul(lam, Q[1]))
            coeffs.append((lam, f2_neg(theta), jj))
    return coeffs


def _ell(f, coeff, Pg1):
    c0 = f2_mul_fq(coeff[0], Pg1[1])
    c1 = f2_mul_fq(coeff[1], Pg1[0])
    c2 = coeff[2]
    # mul_by_034: sparse element c0 + c1*w + c2*v*w  (v*w = w^3)
    sp = [0] * 12
    sp[0], sp[6] = c0
    sp[1], sp[7] = c1
    sp[3], sp[9] = c2
    return f12_mul(f, sp)


def multi_miller_ark(g1s, g2s):
    pairs = [(p, g2_prepare(q)) for p, q in zip(g1s, g2s) if p is not None and q is not None]
    f = f12_one()
    idx = 0
    for bit in bin(X)[3:]:
        f = f12_sqr(f)
        for p, c in pairs:
            f = _ell(f, c[idx], p)
        idx += 1
        if bit == "1":
            for p, c in pairs:
                f = _ell(f, c[idx], p)
            idx += 1
    return f


def _exp_by_x(f):
    return f12_pow(f, X)


def final_exp_ark(f):
    """eprint 2020/875 chain as in ark-ec Bls12::final_exponentiation."""
    f1 = f12_conj(f)
    f2_ = f12_inv(f)
    r_ = f12_mul(f1, f2_)
    f2_ = r_
    r_ = f12_frob(r_, 2)
    r_ = f12_mul(r_, f2_)
    y0 = f12_sqr(r_)
    y1 = _exp_by_x(r_)
    y2 = f12_conj(r_)
    y1 = f12_mul(y1, y2)
    y2 = _exp_by_x(y1)
    y1 = f12_conj(y1)
    y1 = f12_mul(y1, y2)
    y2 = _exp_by_x(y1)
    y1 = f12_frob(y1, 1)
    y1 = f12_mul(y1, y2)
    r_ = f12_mul(r_, y0)
    y0 = _exp_by_x(y1)
    y2 = _exp_by_x(y0)
    y0 = f12_frob(y1, 2)
    y1 = f12_conj(y1)
    y1 = f12_mul(y1, y2)
    y1 = f12_mul(y1, y0)
    r_ = f12_mul(r_, y1)
    return r_


def final_exp_fast(f):
    """Same value as final_exp_ark (exponent 3(p^12-1)/r) computed as
    easy part by Frobenius + hard part by plain exponentiation."""
    t = f12_mul(f12_conj(f), f12_inv(f))
    t = f12_mul(f12_frob(t, 2), t)
    return f12_pow(t, 3 * (P ** 4 - P ** 2 + 1) // R)


def multi_pairing(g1s, g2s):
    """ark-ec ``Pairing::multi_pairing`` value (PairingOutput.0)."""
    return final_exp_ark(multi_miller_ark(g1s, g2s))


def pairing(p, q):
    return multi_pairing([p], [q])


# --------------------------------------------------------- serialization --
def fq_to_bytes(a):
    return int(a).to_bytes(48, "little")


def fr_to_bytes(a):
    return int(a).to_bytes(32, "little")


def _ge(a, b):
    return a >= b


def g1_to_bytes(pt, compress=False):
    """ark-serialize of G1Affine: x (48 B) [, y (48 B)] with SWFlags in the
    top bits of the last byte (YIsNegative = 0x80 when y > -y,
    PointAtInfinity = 0x40)."""
    if pt is None:
        x, y, flag = 0, 0, 0x40
    else:
        x, y = pt
        flag = 0x80 if y > (P - y) % P else 0
    if compress:
        b = bytearray(fq_to_bytes(x))
    else:
        b = bytearray(fq_to_bytes(x) + fq_to_bytes(y))
    b[-1] |= flag
    return bytes(b)


def _f2_gt(a, b):
    # arkworks QuadExtField Ord: compare c1 first, then c0
    if a[1] != b[1]:
        return a[1] > b[1]
    return a[0] > b[0]


def g2_to_bytes(pt, compress=False):
    if pt is None:
        x, y, flag = F2_ZERO, F2_ZERO, 0x40
    else:
        x, y = pt
        flag = 0x80 if _f2_gt(y, f2_neg(y)) else 0
    xb = fq_to_bytes(x[0]) + fq_to_bytes(x[1])
    b = bytearray(xb if compress else xb + fq_to_bytes(y[0]) + fq_to_bytes(y[1]))
    b[-1] |= flag
    return bytes(b)


def fq12_to_bytes(a):
    return b"".join(fq_to_bytes(c) for c in fq12_to_tower(a))
