"""Generate testudo_amd/csrc/wave_ops.inc: the tables of the wave-cooperative
tower arithmetic (csrc/wave_tower.h).

Why: a lone GPU lane evaluating an Fq12 chain (Miller loop, final
exponentiation) costs one *wave* instruction per limb operation, so the
chain runs at ~1.6 us per Fq multiply whatever the lane count.  Spreading
the independent Fq products of one tower operation over the 64 lanes of a
wave turns an Fq12 multiply (54 Fq products) into one "stage":

  phase 1   lane i < np:  x_i = sum_j cx_ij * in_j,  y_i = sum_j cy_ij * in_j
                          p_i = x_i * y_i (Montgomery)
  phase 2   lane k < no:  out_k = sum_i co_ki * p_i + sum_j cl_kj * in_j  (mod p)

The linear forms (small integer coefficients) are derived here by running
the tower formulas of csrc/field.h / pairing.h symbolically, and every
operation is checked numerically against the pure-Python oracle before the
tables are written.  Operand kinds: A, B (input registers), K (constants),
P (this stage's products); outputs go to C or D.
"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "py"))
import bls377 as O  # noqa: E402

P = O.P
RQ = 1 << 384
OPS = ("A", "B", "K", "P")
OPCODE = {"A": 0, "B": 1, "K": 2, "P": 3}
DSTCODE = {"C": 0, "D": 1}


class L(dict):
    """Linear combination atom -> int coefficient."""

    def __add__(self, o):
        r = L(self)
        for k, v in o.items():
            r[k] = r.get(k, 0) + v
            if r[k] == 0:
                del r[k]
        return r

    def __neg__(self):
        return L({k: -v for k, v in self.items()})

    def __sub__(self, o):
        return self + (-o)

    def sc(self, c):
        return L({k: v * c for k, v in self.items()}) if c else L()

    def weight(self):
        return sum(abs(v) for v in self.values())


def atom(kind, i):
    return L({(kind, i): 1})


class Prog:
    def __init__(self, consts):
        self.products = []
        self.consts = consts  # shared list of Fq constant values

    def mul(self, x, y):
        for f in (x, y):
            for k in f:
                assert k[0] in ("A", "B", "K"), k
        self.products.append((x, y))
        return atom("P", len(self.products) - 1)

    def sqr(self, x):
        """x^2: the same object as both factors marks a square; a stage whose
        products are all squares skips its Y forms and runs the Montgomery
        squaring (78 instead of 144 limb products)."""
        return self.mul(x, x)

    def all_squares(self):
        return bool(self.products) and all(x is y for x, y in self.products)

    def const(self, v):
        v %= P
        if v not in self.consts:
            self.consts.append(v)
        return atom("K", self.consts.index(v))


# ---- symbolic tower (mirrors csrc/field.h) -------------------------------
def f2_add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def f2_sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def f2_neg(a):
    return (-a[0], -a[1])


def f2_sc(a, c):
    return (a[0].sc(c), a[1].sc(c))


def f2_mul(pg, a, b):
    v0 = pg.mul(a[0], b[0])
    v1 = pg.mul(a[1], b[1])
    s = pg.mul(a[0] + a[1], b[0] + b[1])
    return (v0 - v1.sc(5), s - v0 - v1)


def f2_mul_fq(pg, a, s):
    return (pg.mul(a[0], s), pg.mul(a[1], s))


def f2_mul_by_u(a):
    return (a[1].sc(-5), a[0])


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul(pg, a, b):
    v0 = f2_mul(pg, a[0], b[0])
    v1 = f2_mul(pg, a[1], b[1])
    v2 = f2_mul(pg, a[2], b[2])
    c0 = f2_add(f2_mul_by_u(f2_sub(f2_sub(f2_mul(pg, f2_add(a[1], a[2]), f2_add(b[1], b[2])), v1), v2)), v0)
    c1 = f2_add(f2_sub(f2_sub(f2_mul(pg, f2_add(a[0], a[1]), f2_add(b[0], b[1])), v0), v1), f2_mul_by_u(v2))
    c2 = f2_add(f2_sub(f2_sub(f2_mul(pg, f2_add(a[0], a[2]), f2_add(b[0], b[2])), v0), v2), v1)
    return (c0, c1, c2)


def f6_mul_by_v(a):
    return (f2_mul_by_u(a[2]), a[0], a[1])


def f6_mul_by_01(pg, a, b0, b1):
    v0 = f2_mul(pg, a[0], b0)
    v1 = f2_mul(pg, a[1], b1)
    t1 = f2_add(f2_mul_by_u(f2_sub(f2_mul(pg, f2_add(a[1], a[2]), b1), v1)), v0)
    t3 = f2_add(f2_sub(f2_mul(pg, f2_add(a[0], a[2]), b0), v0), v1)
    t2 = f2_sub(f2_sub(f2_mul(pg, f2_add(b0, b1), f2_add(a[0], a[1])), v0), v1)
    return (t1, t2, t3)


def f12_mul(pg, a, b):
    v0 = f6_mul(pg, a[0], b[0])
    v1 = f6_mul(pg, a[1], b[1])
    c1 = f6_sub(f6_sub(f6_mul(pg, f6_add(a[0], a[1]), f6_add(b[0], b[1])), v0), v1)
    return (f6_add(v0, f6_mul_by_v(v1)), c1)


def f12_mul_by_034(pg, f, c0, c3, c4):
    a = tuple(f2_mul(pg, f[0][i], c0) for i in range(3))
    b = f6_mul_by_01(pg, f[1], c3, c4)
    e = f6_mul_by_01(pg, f6_add(f[0], f[1]), f2_add(c0, c3), c4)
    return (f6_add(a, f6_mul_by_v(b)), f6_sub(e, f6_add(a, b)))


def f2_sqr_sq(pg, a):
    """a^2 from three Fq squares: (a0^2 - 5 a1^2, (a0 + a1)^2 - a0^2 - a1^2)."""
    s0 = pg.sqr(a[0])
    s1 = pg.sqr(a[1])
    s01 = pg.sqr(a[0] + a[1])
    return (s0 - s1.sc(5), s01 - s0 - s1)


def cyclotomic_sqr(pg, f):
    r0, r4, r3 = f[0]
    r2, r1, r5 = f[1]

    # Fp4 square of x + y s: t = x^2 + u y^2, 2xy = (x + y)^2 - x^2 - y^2 --
    # the same values as the Karatsuba form (x y, (x + y)(x + u y)), from 27
    # Fq squares instead of 18 products, so the stage is all squares
    def part(x, y):
        x2 = f2_sqr_sq(pg, x)
        y2 = f2_sqr_sq(pg, y)
        s2 = f2_sqr_sq(pg, f2_add(x, y))
        return f2_add(x2, f2_mul_by_u(y2)), f2_sub(f2_sub(s2, x2), y2)
    t0, t1 = part(r0, r1)
    t2, t3 = part(r2, r3)
    t4, t5 = part(r4, r5)
    z00 = f2_sub(f2_sc(t0, 3), f2_sc(r0, 2))
    z11 = f2_add(f2_sc(t1, 3), f2_sc(r1, 2))
    tmp = f2_mul_by_u(t5)
    z10 = f2_add(f2_sc(tmp, 3), f2_sc(r2, 2))
    z02 = f2_sub(f2_sc(t4, 3), f2_sc(r3, 2))
    z01 = f2_sub(f2_sc(t2, 3), f2_sc(r4, 2))
    z12 = f2_add(f2_sc(t3, 3), f2_sc(r5, 2))
    return ((z00, z01, z02), (z10, z11, z12))


def fq2_val(c):
    return (c[0], c[1])


def reg12(kind):
    a = [atom(kind, i) for i in range(12)]
    f2 = [(a[2 * i], a[2 * i + 1]) for i in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def reg_f2(kind, i):
    return (atom(kind, 2 * i), atom(kind, 2 * i + 1))


def flat12(f):
    return [c for f6 in f for f2 in f6 for c in f2]


# ---- ops -------------------------------------------------------------------
def op_f12_mul(pg):
    return {"C": flat12(f12_mul(pg, reg12("A"), reg12("B")))}


def f6_sqr_sq(pg, c):
    """(c0 + c1 v + c2 v^2)^2 from six Fq2 squares (v^3 = u):
    c0^2 + u 2c1c2, 2c0c1 + u c2^2, c1^2 + 2c0c2 with 2xy = (x + y)^2 - x^2 - y^2."""
    c0, c1, c2 = c
    s0, s1, s2 = f2_sqr_sq(pg, c0), f2_sqr_sq(pg, c1), f2_sqr_sq(pg, c2)
    t12 = f2_sub(f2_sub(f2_sqr_sq(pg, f2_add(c1, c2)), s1), s2)
    t01 = f2_sub(f2_sub(f2_sqr_sq(pg, f2_add(c0, c1)), s0), s1)
    t02 = f2_sub(f2_sub(f2_sqr_sq(pg, f2_add(c0, c2)), s0), s2)
    return (f2_add(s0, f2_mul_by_u(t12)), f2_add(t01, f2_mul_by_u(s2)), f2_add(s1, t02))


def f12_sqr_sq(pg, a):
    """(a0 + a1 w)^2 = a0^2 + v a1^2 + ((a0 + a1)^2 - a0^2 - a1^2) w: 54 Fq squares."""
    q0, q1 = f6_sqr_sq(pg, a[0]), f6_sqr_sq(pg, a[1])
    q01 = f6_sqr_sq(pg, f6_add(a[0], a[1]))
    return (f6_add(q0, f6_mul_by_v(q1)), f6_sub(f6_sub(q01, q0), q1))


def op_f12_sqr(pg):
    return {"C": flat12(f12_sqr_sq(pg, reg12("A")))}


def op_f12_sqr_prod(pg):
    return {"C": flat12(f12_mul(pg, reg12("A"), reg12("A")))}


def op_cyc_sqr(pg):
    return {"C": flat12(cyclotomic_sqr(pg, reg12("A")))}


def line_prep(pg, base):
    """B[base..base+8) = line (c0, c1, c2) + (px, py) -> (c0*py, c1*px, c2)."""
    c0, c1, c2 = reg_f2("B", base // 2), reg_f2("B", base // 2 + 1), reg_f2("B", base // 2 + 2)
    px, py = atom("B", base + 6), atom("B", base + 7)
    a = f2_mul_fq(pg, c0, py)
    b = f2_mul_fq(pg, c1, px)
    return [a[0], a[1], b[0], b[1], c2[0], c2[1]]


def op_line_prep(pg):
    return {"D": line_prep(pg, 0)}


def op_sqr_lp1(pg):
    c = op_f12_sqr_prod(pg)["C"]
    return {"C": c, "D": line_prep(pg, 0)}


def op_sqr_lp2(pg):
    c = op_f12_sqr_prod(pg)["C"]
    d0 = line_prep(pg, 0)
    # second line: coefficients at B[8..14), same point (px, py) = B[6], B[7]
    c0, c1, c2 = reg_f2("B", 4), reg_f2("B", 5), reg_f2("B", 6)
    px, py = atom("B", 6), atom("B", 7)
    a = f2_mul_fq(pg, c0, py)
    b = f2_mul_fq(pg, c1, px)
    return {"C": c, "D": d0 + [a[0], a[1], b[0], b[1], c2[0], c2[1]]}


def op_mul034(pg):
    f = reg12("A")
    c0, c3, c4 = reg_f2("B", 0), reg_f2("B", 1), reg_f2("B", 2)
    return {"C": flat12(f12_mul_by_034(pg, f, c0, c3, c4))}


def frob_consts(k):
    u = (0, 1)

    def f2pow(a, e):
        r, b = (1, 0), a
        while e:
            if e & 1:
                r = O.f2_mul(r, b)
            b = O.f2_mul(b, b)
            e >>= 1
        return r
    pk = P ** k
    return f2pow(u, (pk - 1) // 3), f2pow(u, 2 * (pk - 1) // 3), f2pow(u, (pk - 1) // 6)


def op_frob(k):
    def build(pg):
        c61, c62, c12 = frob_consts(k)
        c61_12 = O.f2_mul(c61, c12)
        c62_12 = O.f2_mul(c62, c12)
        f = reg12("A")

        def fr2(a):
            return (a[0], -a[1]) if k & 1 else a

        def kmul(a, c):
            kc = (pg.const(c[0]), pg.const(c[1]))
            return f2_mul(pg, a, kc)
        x0 = (fr2(f[0][0]), kmul(fr2(f[0][1]), c61), kmul(fr2(f[0][2]), c62))
        x1 = (kmul(fr2(f[1][0]), c12), kmul(fr2(f[1][1]), c61_12), kmul(fr2(f[1][2]), c62_12))
        return {"C": flat12((x0, x1))}
    return build


def op_conj(pg):
    f = reg12("A")
    return {"C": flat12((f[0], f6_neg(f[1])))}


def op_copy(pg):
    return {"C": [atom("A", i) for i in range(12)]}


# Fq12 inversion (field.h inv(Fq12) -> inv(Fq6) -> inv(Fq2) -> inv(Fq)), in
# stages: registers hold Fq-slot vectors; A / B are the two inputs.
def op_inv1(pg):
    """A = f (12) -> C[0..6) = t = c0^2 - v c1^2."""
    f = reg12("A")
    t = f6_sub(f6_mul(pg, f[0], f[0]), f6_mul_by_v(f6_mul(pg, f[1], f[1])))
    return {"C": [c for f2 in t for c in f2]}


def reg6(kind, base=0):
    return tuple((atom(kind, base + 2 * i), atom(kind, base + 2 * i + 1)) for i in range(3))


def op_inv2(pg):
    """A = t (6) -> C = (c0', c1', c2') (6)."""
    a = reg6("A")
    c0 = f2_sub(f2_mul(pg, a[0], a[0]), f2_mul_by_u(f2_mul(pg, a[1], a[2])))
    c1 = f2_sub(f2_mul_by_u(f2_mul(pg, a[2], a[2])), f2_mul(pg, a[0], a[1]))
    c2 = f2_sub(f2_mul(pg, a[1], a[1]), f2_mul(pg, a[0], a[2]))
    return {"C": [c for f2 in (c0, c1, c2) for c in f2]}


def op_inv3(pg):
    """A = c' (6), B = t (6) -> C[0..2) = t' = t0 c0' + u (t2 c1' + t1 c2')."""
    c = reg6("A")
    a = reg6("B")
    tp = f2_add(f2_mul(pg, a[0], c[0]), f2_mul_by_u(f2_add(f2_mul(pg, a[2], c[1]), f2_mul(pg, a[1], c[2]))))
    return {"C": [tp[0], tp[1]]}


def op_inv4(pg):
    """A = t' (2) -> C[0] = t0'^2 + 5 t1'^2."""
    a0, a1 = atom("A", 0), atom("A", 1)
    return {"C": [pg.mul(a0, a0) + pg.mul(a1, a1).sc(5)]}


def op_inv5(pg):
    """A = t' (2), B[0] = n^-1 -> C = t'^-1 = (t0' ni, -t1' ni)."""
    ni = atom("B", 0)
    return {"C": [pg.mul(atom("A", 0), ni), -pg.mul(atom("A", 1), ni)]}


def op_inv6(pg):
    """A = c' (6), B = t'^-1 (2) -> C = t^-1 = c' * t'^-1 (6)."""
    c = reg6("A")
    ti = (atom("B", 0), atom("B", 1))
    r = [f2_mul(pg, c[i], ti) for i in range(3)]
    return {"C": [x for f2 in r for x in f2]}


def op_inv7(pg):
    """A = f (12), B = t^-1 (6) -> C = f^-1 = (c0 t^-1, -c1 t^-1)."""
    f = reg12("A")
    ti = reg6("B")
    return {"C": flat12((f6_mul(pg, f[0], ti), f6_neg(f6_mul(pg, f[1], ti))))}


# ---- G2 line preparation (pairing.h g2_double_step / g2_add_step) ---------
# Region ops: every operand is a slot of one per-wave region (atoms ("A", s)),
# outputs {slot: form}.  Layout: R = x 0-1, y 2-3, z 4-5; line c0 6-7, c1 8-9,
# c2 10-11; scratch 12-25; Q = x 26-27, y 28-29; addition scratch 30-43.
def rf2(s):
    return (atom("A", s), atom("A", s + 1))


def put2(d, s, v):
    d[s], d[s + 1] = v[0], v[1]


B1 = (-pow(5, -1, P)) % P  # G2_B = (0, b1) = 1/u
TWO_INV = pow(2, -1, P)


def op_dbl1(pg):
    x, y, z = rf2(0), rf2(2), rf2(4)
    o = {}
    xy = f2_mul(pg, x, y)
    b = f2_mul(pg, y, y)
    c = f2_mul(pg, z, z)
    hh = f2_mul(pg, f2_add(y, z), f2_add(y, z))
    j = f2_mul(pg, x, x)
    put2(o, 12, xy)
    put2(o, 14, b)
    put2(o, 16, c)
    put2(o, 6, f2_sub(f2_add(b, c), hh))  # c0 = -h
    put2(o, 8, f2_sc(j, 3))               # c1 = 3 j
    return {"C": o}


def op_dbl2(pg):
    xy, c = rf2(12), rf2(16)
    ti = pg.const(TWO_INV)
    o = {}
    put2(o, 18, f2_mul_fq(pg, xy, ti))                      # a = xy / 2
    put2(o, 20, (pg.mul(c[1], pg.const(-15 * B1)), pg.mul(c[0], pg.const(3 * B1))))  # e = b' 3c
    return {"C": o}


def op_dbl3(pg):
    nh, b, a, e = rf2(6), rf2(14), rf2(18), rf2(20)
    ti = pg.const(TWO_INV)
    o = {}
    put2(o, 22, f2_mul_fq(pg, f2_add(b, f2_sc(e, 3)), ti))  # g = (b + 3e) / 2
    put2(o, 24, f2_mul(pg, e, e))                           # e^2
    put2(o, 0, f2_mul(pg, a, f2_sub(b, f2_sc(e, 3))))       # x' = a (b - f)
    put2(o, 4, f2_neg(f2_mul(pg, b, nh)))                   # z' = b h
    put2(o, 10, f2_sub(e, b))                               # c2 = i = e - b
    return {"C": o}


def op_dbl4(pg):
    g, e2 = rf2(22), rf2(24)
    o = {}
    put2(o, 2, f2_sub(f2_mul(pg, g, g), f2_sc(e2, 3)))     # y' = g^2 - 3 e^2
    return {"C": o}


def op_add1(pg):
    x, y, z, qx, qy = rf2(0), rf2(2), rf2(4), rf2(26), rf2(28)
    o = {}
    theta = f2_sub(y, f2_mul(pg, qy, z))
    lam = f2_sub(x, f2_mul(pg, qx, z))
    put2(o, 30, theta)
    put2(o, 32, lam)
    put2(o, 6, lam)               # c0 = lambda
    put2(o, 8, f2_neg(theta))     # c1 = -theta
    return {"C": o}


def op_add2(pg):
    theta, lam, qx, qy = rf2(30), rf2(32), rf2(26), rf2(28)
    o = {}
    put2(o, 34, f2_mul(pg, theta, theta))  # c
    put2(o, 36, f2_mul(pg, lam, lam))      # d
    put2(o, 10, f2_sub(f2_mul(pg, theta, qx), f2_mul(pg, lam, qy)))  # c2 = j
    return {"C": o}


def op_add3(pg):
    x, z, lam, c, d = rf2(0), rf2(4), rf2(32), rf2(34), rf2(36)
    o = {}
    e = f2_mul(pg, lam, d)
    f = f2_mul(pg, z, c)
    g = f2_mul(pg, x, d)
    put2(o, 38, e)
    put2(o, 40, g)
    put2(o, 42, f2_sub(f2_add(e, f), f2_sc(g, 2)))  # h
    return {"C": o}


def op_add4(pg):
    y, z, theta, lam, e, g, h = rf2(2), rf2(4), rf2(30), rf2(32), rf2(38), rf2(40), rf2(42)
    o = {}
    put2(o, 0, f2_mul(pg, lam, h))
    put2(o, 2, f2_sub(f2_mul(pg, theta, f2_sub(g, h)), f2_mul(pg, e, y)))
    put2(o, 4, f2_mul(pg, z, e))
    return {"C": o}


OP_LIST = [
    ("F12_MUL", op_f12_mul),
    ("F12_SQR", op_f12_sqr),
    ("CYC_SQR", op_cyc_sqr),
    ("LINE_PREP", op_line_prep),
    ("SQR_LP1", op_sqr_lp1),
    ("SQR_LP2", op_sqr_lp2),
    ("MUL034", op_mul034),
    ("FROB1", op_frob(1)),
    ("FROB2", op_frob(2)),
    ("FROB3", op_frob(3)),
    ("CONJ", op_conj),
    ("COPY", op_copy),
    ("INV1", op_inv1),
    ("INV2", op_inv2),
    ("INV3", op_inv3),
    ("INV4", op_inv4),
    ("INV5", op_inv5),
    ("INV6", op_inv6),
    ("INV7", op_inv7),
    ("G2_DBL1", op_dbl1),
    ("G2_DBL2", op_dbl2),
    ("G2_DBL3", op_dbl3),
    ("G2_DBL4", op_dbl4),
    ("G2_ADD1", op_add1),
    ("G2_ADD2", op_add2),
    ("G2_ADD3", op_add3),
    ("G2_ADD4", op_add4),
]


# ---- numeric evaluation ------------------------------------------------------
def evaluate(pg, outs, env):
    def ev(lin, extra):
        s = 0
        for (kind, i), c in lin.items():
            if kind == "P":
                s += c * extra[i]
            elif kind == "K":
                s += c * pg.consts[i]
            else:
                s += c * env[kind][i]
        return s % P
    prods = [ev(x, None) * ev(y, None) % P for x, y in pg.products]
    return {d: ({k: ev(l, prods) for k, l in lst.items()} if isinstance(lst, dict) else [ev(l, prods) for l in lst])
            for d, lst in outs.items()}


def t2p(t):
    return O.fq12_from_tower(t)


def p2t(a):
    return O.fq12_to_tower(a)


def rnd(n):
    return [random.randrange(P) for _ in range(n)]


def check(name, pg, outs):
    A, B = rnd(16), rnd(16)
    got = evaluate(pg, outs, {"A": A, "B": B})
    if name == "F12_MUL":
        assert got["C"] == p2t(O.f12_mul(t2p(A[:12]), t2p(B[:12])))
    elif name == "F12_SQR":
        assert got["C"] == p2t(O.f12_mul(t2p(A[:12]), t2p(A[:12])))
    elif name == "CYC_SQR":
        f = t2p(A[:12])
        r = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
        r = O.f12_mul(O.f12_frob(r, 2), r)
        got = evaluate(pg, outs, {"A": p2t(r), "B": B})
        assert got["C"] == p2t(O.f12_mul(r, r))
    elif name in ("LINE_PREP", "SQR_LP1", "SQR_LP2"):
        px, py = B[6], B[7]
        exp = [B[0] * py % P, B[1] * py % P, B[2] * px % P, B[3] * px % P, B[4], B[5]]
        if name == "SQR_LP2":
            exp += [B[8] * py % P, B[9] * py % P, B[10] * px % P, B[11] * px % P, B[12], B[13]]
        assert got["D"] == exp
        if name != "LINE_PREP":
            assert got["C"] == p2t(O.f12_mul(t2p(A[:12]), t2p(A[:12])))
    elif name == "MUL034":
        sp = [0] * 12
        sp[0], sp[6] = B[0], B[1]
        sp[1], sp[7] = B[2], B[3]
        sp[3], sp[9] = B[4], B[5]
        assert got["C"] == p2t(O.f12_mul(t2p(A[:12]), sp))
    elif name.startswith("FROB"):
        k = int(name[-1])
        assert got["C"] == p2t(O.f12_frob(t2p(A[:12]), k))
    elif name == "CONJ":
        assert got["C"] == p2t(O.f12_conj(t2p(A[:12])))
    elif name == "COPY":
        assert got["C"] == A[:12]
    return True


def check_prepare_chain(pgs):
    q = O.g2_mul(O.G2_GEN, 0x1234567)
    ref = O.g2_prepare(q)
    reg = {i: 0 for i in range(44)}
    reg[0], reg[1] = q[0]
    reg[2], reg[3] = q[1]
    reg[4], reg[5] = 1, 0
    reg[26], reg[27] = q[0]
    reg[28], reg[29] = q[1]
    idx = 0
    for bit in bin(O.X)[3:]:
        steps = ["G2_DBL1", "G2_DBL2", "G2_DBL3", "G2_DBL4"]
        if bit == "1":
            steps += ["G2_ADD1", "G2_ADD2", "G2_ADD3", "G2_ADD4"]
        for st in steps:
            pg, outs = pgs[st]
            reg.update(evaluate(pg, outs, {"A": reg, "B": reg})["C"])
            if st in ("G2_DBL4", "G2_ADD4"):
                c0, c1, c2 = ref[idx]
                assert (reg[6], reg[7], reg[8], reg[9], reg[10], reg[11]) == (*c0, *c1, *c2), (st, idx)
                idx += 1
    assert idx == len(ref)


def check_inverse_chain(pgs):
    f = rnd(12)
    env = lambda a, b=None: {"A": a, "B": b or [0] * 16}  # noqa: E731
    t = evaluate(*pgs["INV1"], env(f))["C"]
    c = evaluate(*pgs["INV2"], env(t))["C"]
    tp = evaluate(*pgs["INV3"], env(c, t))["C"]
    n = evaluate(*pgs["INV4"], env(tp))["C"]
    ni = [pow(n[0], -1, P)]
    ti2 = evaluate(*pgs["INV5"], env(tp, ni))["C"]
    ti6 = evaluate(*pgs["INV6"], env(c, ti2))["C"]
    fi = evaluate(*pgs["INV7"], env(f, ti6))["C"]
    assert fi == p2t(O.f12_inv(t2p(f)))


# ---- emission ----------------------------------------------------------------
def mont(v):
    return v * RQ % P


def limbs(v):
    return ", ".join("0x%08xu" % ((v >> (32 * k)) & 0xFFFFFFFF) for k in range(12))


def enc_term(kind, i, c):
    assert 0 < abs(c) < 256 and 0 <= i < 256
    return OPCODE[kind] | (i << 8) | ((1 if c < 0 else 0) << 2) | (abs(c) << 24)


def render():
    """Build every op, check it numerically against the oracle, and return
    (text of wave_ops.inc, per-op stats lines)."""
    random.seed(377)
    consts = []
    built = {}
    for name, fn in OP_LIST:
        pg = Prog(consts)
        outs = fn(pg)
        built[name] = (pg, outs)
    for name, (pg, outs) in built.items():
        if not name.startswith(("INV", "G2_")):
            check(name, pg, outs)
    check_inverse_chain(built)
    check_prepare_chain(built)
    blob, offs, lens, stats = [], [], [], []
    lines = ["// Generated by tools/gen_wave_ops.py -- do not edit.", "#pragma once", "#include <stdint.h>",
             "namespace tpst { namespace wave {"]
    lines.append("constexpr int N_CONSTS = %d;" % len(consts))
    lines.append("static TPST_WAVE_CONST uint32_t CONSTS[%d][12] = {%s};" % (
        max(1, len(consts)), ", ".join("{%s}" % limbs(mont(v)) for v in consts) or "{0}"))
    names = []
    for name, (pg, outs) in built.items():
        # block layout: [hdr, x[np], y[np], o[no], dst[no], terms...]; info words are
        # (term index relative to the block << 8) | term count
        np_ = len(pg.products)
        assert np_ <= 64, (name, np_)
        need_red = int(any(x.weight() * y.weight() > 64 for x, y in pg.products))
        if need_red:
            assert all(x.weight() < 1024 and y.weight() < 1024 for x, y in pg.products)
        olist = [(DSTCODE[d] << 8 | k, lin) for d, lst in outs.items()
                 for k, lin in (sorted(lst.items()) if isinstance(lst, dict) else enumerate(lst))]
        no = len(olist)
        assert no <= 64
        # long output forms are split into chunks summed by separate lanes
        # (phase 2a), then combined per output (phase 2b): smallest chunk
        # length that fits all chunks in one wave
        lens_o = [max(1, len(lin)) for _, lin in olist]
        tmax = 4
        while sum(-(-n // tmax) for n in lens_o) > 64:
            tmax += 1
        chunks, info_o = [], []
        for _, lin in olist:
            items = sorted(lin.items())
            nch = max(1, -(-len(items) // tmax))
            info_o.append(len(chunks) << 8 | nch)
            per = -(-len(items) // nch) if items else 0
            for c in range(nch):
                chunks.append(items[c * per:(c + 1) * per])
        nc = len(chunks)
        assert nc <= 64
        # term lists padded to a per-op uniform length (zero words = 0 * A[0])
        # and stored term-major: term j of lane l at [j * lanes + l]
        sq = int(pg.all_squares())
        xs = [sorted(x.items()) for x, _ in pg.products]
        ys = [] if sq else [sorted(y.items()) for _, y in pg.products]
        tx = max((len(v) for v in xs), default=0)
        ty = max((len(v) for v in ys), default=0)
        tc = max((len(v) for v in chunks), default=0)
        assert max(tx, ty, tc) <= 8, (name, tx, ty, tc)

        def major(lists, t):
            out = []
            for j in range(t):
                for items in lists:
                    out.append(enc_term(items[j][0][0], items[j][0][1], items[j][1]) if j < len(items) else 0)
            return out
        maxw = max((lin.weight() for _, lin in olist), default=0)
        assert maxw < 1024, (name, maxw)
        block = ([np_ | no << 8 | need_red << 16 | sq << 17 | nc << 24, tx | ty << 8 | tc << 16] + major(xs, tx) +
                 major(ys, ty) + major(chunks, tc) + info_o + [d for d, _ in olist])
        offs.append(len(blob))
        lens.append(len(block))
        blob += block
        names.append(name)
        stats.append("//   %-10s %s %2d (terms %d x %d)  outputs %2d  chunks %2d (<= %d terms)  max weight %3d  words %4d"
                     % (name, "squares " if sq else "products", np_, tx, ty, no, nc, tc, maxw, len(block)))
    lines += stats
    lines.append("enum OpId {%s, N_OPS};" % ", ".join("OP_" + n for n in names))
    lines.append("static constexpr uint32_t OP_OFF[N_OPS] = {%s};" % ", ".join(map(str, offs)))
    lines.append("static constexpr uint32_t OP_LEN[N_OPS] = {%s};" % ", ".join(map(str, lens)))
    lines.append("static TPST_WAVE_CONST uint32_t BLOB[%d] = {%s};" % (len(blob), ", ".join("0x%08xu" % t for t in blob)))
    lines.append("static constexpr double INV_P320 = %r;  // 2^320 / p" % (2.0 ** 320 / P))
    lines.append("}}  // namespace tpst::wave")
    return "\n".join(lines) + "\n", stats


INC_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "testudo_amd", "csrc",
                        "wave_ops.inc")


def main():
    text, stats = render()
    open(INC_PATH, "w").write(text)
    print("\n".join(stats))
    print("wrote", INC_PATH)


if __name__ == "__main__":
    main()
