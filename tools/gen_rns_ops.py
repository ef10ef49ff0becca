"""Generate testudo_amd/csrc/rns_ops.inc: tables of the residue-number-system
(RNS) Fq12 engine (csrc/rns_engine.h) that runs the final-exponentiation
chains.

Why RNS: the radix engine (wave_tower.h) evaluates one Fq product per lane,
so a serial Fq12 chain costs at least one lone-lane Montgomery product
(~1.9k cycles) plus the linear forms around it per stage.  In RNS an Fq
value is a vector of residues modulo 31 word-sized moduli, one per lane:
products and linear combinations are lane-local, and the only cross-lane
work is the two base extensions of the Montgomery reduction (Bajard /
Kawamura style, exact second extension by Shenoy-Kumaresan with a 2^32
redundant channel).  An Fq12 operation becomes, per output coefficient o,

    t_o = sum_k c_k * x_k * y_k      (monomials in the input slots, lane-local)
    out_o = t_o * M^-1 mod p          (RNS Montgomery, M = prod of base B)

with no intermediate product list: the tower formulas of gen_wave_ops.py are
expanded symbolically into monomials (Fq constants absorb their
coefficients), and every op is checked against the oracle through an exact
model of the device arithmetic (every 64-bit accumulator and every bound).

Channels (lane & 31):  0..14 base B (m_i = 2^28 - c_i prime), 15 the
redundant 2^32 channel, 16..30 base B' (same form), 31 idle; the two halves
of a wave carry two independent chains.  Values are kept in the
"M-domain" (x~ = x M mod p) as integers < 16 p; a slot also stores the
residues of N1 - x~ (N1 = 16 p) so negative coefficients are plain products.
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_wave_ops as W  # noqa: E402

O = W.O
P = W.P
RQ = 1 << 384          # field.h Montgomery radix
NB = 15                # channels per base
LANES = 32
R_CH = NB              # redundant channel (mod 2^32)
BP0 = NB + 1           # first B' channel
M32 = (1 << 32) - 1
N1 = 16 * P            # negation offset; every slot value is < N1
TERM_C_MAX = 15
KLOAD_MAX = 8          # longest chain of raw (unconverted) factors


def is_prime(n):
    if n < 2:
        return False
    for q in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % q == 0:
            return n == q
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


MODS = [m for m in ((1 << 28) - c for c in range(1, 20000, 2)) if is_prime(m)][:2 * NB]
BASE = MODS[:NB]
BASEP = MODS[NB:]
MB = 1
for m in BASE:
    MB *= m
MBP = 1
for m in BASEP:
    MBP *= m
assert MB > (1 << 16) * P * 2 and MBP > N1


def lane_mod(ch):
    if ch < NB:
        return BASE[ch]
    if BP0 <= ch < BP0 + NB:
        return BASEP[ch - BP0]
    return None  # redundant channel (mod 2^32)


# per-lane constant words (rns_engine.h RnsLane)
LANE_FIELDS = ["MOD", "C32", "CC", "NEGK", "K1", "PJ", "MINV", "K3", "MPINV", "MPN", "K5", "ISR"]
LANE_WORDS = 64
ROW1_OFF = 16
ROW2_OFF = 32
POW32_OFF = 48


def lane_consts(ch):
    c = {k: 0 for k in LANE_FIELDS}
    row1 = [0] * NB
    row2 = [0] * NB
    pow32 = [0] * 12
    if ch == 31:
        ch = 0  # idle lane: a copy of channel 0 (its results are never read)
    m = lane_mod(ch)
    if m is None:  # redundant channel, arithmetic mod 2^32
        c["ISR"] = 1
        c["NEGK"] = N1 & M32
        c["PJ"] = P & M32
        c["MINV"] = pow(MB, -1, 1 << 32)
        c["MPINV"] = pow(MBP, -1, 1 << 32)
        row1 = [(MB // mi) & M32 for mi in BASE]
        row2 = [(MBP // mj) & M32 for mj in BASEP]
        pow32 = [1] + [0] * 11
    else:
        c["MOD"] = m
        c["C32"] = (1 << 32) % m
        c["CC"] = (1 << 28) - m
        c["NEGK"] = N1 % m + m
        pow32 = [pow(2, 32 * k, m) for k in range(12)]
        if ch < NB:
            Mi = MB // m
            c["K1"] = (-pow(P, -1, m) * pow(Mi, -1, m)) % m
            c["MPN"] = (m - MBP % m) % m
            c["K5"] = pow(Mi, -1, m)
            row2 = [(MBP // mj) % m for mj in BASEP]
        else:
            Mj = MBP // m
            c["PJ"] = P % m
            c["MINV"] = pow(MB, -1, m)
            c["K3"] = pow(Mj, -1, m)
            row1 = [(MB // mi) % m for mi in BASE]
    words = [0] * LANE_WORDS
    for i, k in enumerate(LANE_FIELDS):
        words[i] = c[k]
    words[ROW1_OFF:ROW1_OFF + NB] = row1
    words[ROW2_OFF:ROW2_OFF + NB] = row2
    words[POW32_OFF:POW32_OFF + 12] = pow32
    return words


LANE_TABLE = [lane_consts(ch) for ch in range(LANES)]


def L_(ch, name):
    return LANE_TABLE[ch][LANE_FIELDS.index(name)]


# ---- exact model of the device arithmetic -----------------------------------
def red64(x, ch):
    """rns_engine.h red64: x (< 2^64) mod the lane's modulus (2^32 on the
    redundant channel), by three folds of the high word."""
    assert 0 <= x < 1 << 64, x
    if L_(ch, "ISR"):
        return x & M32
    m, c32, cc = L_(ch, "MOD"), L_(ch, "C32"), L_(ch, "CC")
    y = (x >> 32) * c32 + (x & M32)
    z = (y >> 32) * c32 + (y & M32)
    assert z < 1 << 33
    w = (z >> 28) * cc + (z & ((1 << 28) - 1))
    if w >= m:
        w -= m
    assert w < m
    return w


def residues(v):
    return [v % lane_mod(ch) if lane_mod(ch) else v & M32 for ch in range(LANES - 1)] + [v % BASE[0]]


def crt(res):
    """integer of B residues (exact, < M), checked against B' and 2^32"""
    v = 0
    for i, m in enumerate(BASE):
        Mi = MB // m
        v += res[i] * pow(Mi, -1, m) % m * Mi
    v %= MB
    for j, m in enumerate(BASEP):
        assert v % m == res[BP0 + j], "B' channel disagrees"
    assert v & M32 == res[R_CH], "redundant channel disagrees"
    return v


def mont(t):
    """RNS Montgomery reduction of the lane residues t -> (t + q p) / M."""
    xi = [red64(t[ch] * L_(ch, "K1"), ch) for ch in range(LANES)]       # B lanes
    out = [0] * LANES
    x2 = [0] * LANES
    for ch in range(LANES):                                             # B' + r lanes
        acc = sum(xi[i] * LANE_TABLE[ch][ROW1_OFF + i] for i in range(NB))
        assert acc < 1 << 64
        q = red64(acc, ch)
        u = red64(q * L_(ch, "PJ") + t[ch], ch)
        rr = red64(u * L_(ch, "MINV"), ch)
        out[ch] = rr
        x2[ch] = rr if L_(ch, "ISR") else red64(rr * L_(ch, "K3"), ch)
    beta = 0
    for ch in range(LANES):                                             # B + r lanes
        acc = sum(x2[BP0 + j] * LANE_TABLE[ch][ROW2_OFF + j] for j in range(NB))
        if L_(ch, "ISR"):
            beta = (((acc & M32) - x2[R_CH]) * L_(ch, "MPINV")) & M32
    assert beta < NB, beta
    for ch in range(NB):
        acc = sum(x2[BP0 + j] * LANE_TABLE[ch][ROW2_OFF + j] for j in range(NB))
        assert acc < 1 << 64
        s = red64(acc, ch)
        v = s + beta * L_(ch, "MPN")
        assert v < 1 << 32
        out[ch] = red64(v, ch)
    out[31] = out[0]
    return out


def store_model(res):
    """rns_engine.h store(): residues of r (< 16 p) -> r mod p through CRT over
    B, alpha from the 2^32 channel, columns of sum_i xi_i M_i in 64 bits"""
    xi = [red64(res[i] * L_(i, "K5"), i) for i in range(NB)]
    acc = sum(xi[i] * LANE_TABLE[R_CH][ROW1_OFF + i] for i in range(NB))
    alpha = (((acc & M32) - res[R_CH]) * L_(R_CH, "MINV")) & M32
    cols = [sum(xi[i] * ((MB // BASE[i]) >> (32 * k) & M32) for i in range(NB)) for k in range(14)]
    assert all(c < 1 << 64 for c in cols)
    v = sum(c << (32 * k) for k, c in enumerate(cols)) - alpha * MB
    assert v == crt(res) and 0 <= v < N1
    for k in (8, 4, 2, 1):
        if v >= k * P:
            v -= k * P
    assert v < P
    return v


# ---- programs ----------------------------------------------------------------
KIND = {"A": 0, "B": 1, "K": 2}


class RnsProg:
    def __init__(self):
        self.consts = []  # Fq values; slot k stores k M mod p

    def const(self, v):
        v %= P
        if v not in self.consts:
            self.consts.append(v)
        return ("K", self.consts.index(v))


def expand(pg, lin, rp):
    """output linear form over products / atoms -> {(atom_a, atom_b): coef}"""
    mono = {}

    def add(a, b, c):
        key = tuple(sorted((a, b)))
        mono[key] = mono.get(key, 0) + c
    for (kind, i), co in lin.items():
        if kind == "P":
            x, y = pg.products[i]
            for ka, cx in x.items():
                for kb, cy in y.items():
                    add(ka, kb, co * cx * cy)
        else:
            add((kind, i), ("ONE", 0), co)
    # constants absorb coefficients: (a, K_k, c) -> (a, K_{c k}, 1)
    terms = {}
    for (a, b), c in mono.items():
        if c == 0:
            continue
        kv = None
        if b[0] in ("K", "ONE"):
            kv = pg.consts[b[1]] if b[0] == "K" else 1
            other = a
        elif a[0] in ("K", "ONE"):
            kv = pg.consts[a[1]] if a[0] == "K" else 1
            other = b
        if kv is not None:
            if other[0] in ("K", "ONE"):   # constant term: K * ONE
                kv2 = pg.consts[other[1]] if other[0] == "K" else 1
                kslot = rp.const(c * kv * kv2)
                terms[(kslot, rp.const(1))] = terms.get((kslot, rp.const(1)), 0) + 1
            else:
                kslot = rp.const(c * kv)
                terms[(other, kslot)] = terms.get((other, kslot), 0) + 1
        else:
            terms[(a, b)] = terms.get((a, b), 0) + c
    out = []
    for (a, b), c in sorted(terms.items()):
        if c == 0:
            continue
        if a[0] == "K":
            a, b = b, a
        neg = c < 0
        c = abs(c)
        while c:
            cc = min(c, TERM_C_MAX)
            out.append((a, b, cc, neg))
            c -= cc
    return out


def enc(a, b, c, neg):
    assert a[0] in KIND and b[0] in KIND and 0 <= a[1] < 256 and 0 <= b[1] < 256
    return a[1] | KIND[a[0]] << 8 | b[1] << 10 | KIND[b[0]] << 18 | int(neg) << 20 | c << 24


OPS = ["F12_MUL", "F12_SQR", "CYC_SQR", "FROB1", "FROB2", "FROB3", "CONJ", "COPY",
       "INV1", "INV2", "INV3", "INV4", "INV5", "INV6", "INV7",
       "G2_DBL1", "G2_DBL2", "G2_DBL3", "G2_DBL4", "G2_ADD1", "G2_ADD2", "G2_ADD3", "G2_ADD4"]


def rw_overlap(progs, name):
    """1 if an output slot of the op is also one of its A inputs (the G2
    region ops run in place, a == c): the stage must then finish every
    wave's reads before any wave writes"""
    reads = {t[k][1] for _, terms in progs[name] for t in terms for k in (0, 1) if t[k][0] == "A"}
    outs = {dst & 0xff for dst, _ in progs[name] if dst >> 8 == 0}
    return int(bool(reads & outs))


def build_ops():
    wconsts = []
    built = {}
    fns = dict(W.OP_LIST)
    for name in OPS:
        pg = W.Prog(wconsts)
        outs = fns[name](pg)
        built[name] = (pg, outs)
    rp = RnsProg()
    rp.const(1)
    progs = {}
    for name in OPS:
        pg, outs = built[name]
        olist = [(W.DSTCODE[d] << 8 | k, lin) for d, lst in outs.items()
                 for k, lin in (sorted(lst.items()) if isinstance(lst, dict) else enumerate(lst))]
        progs[name] = [(dst, expand(pg, lin, rp)) for dst, lin in olist]
    return built, rp, progs


def bound_check(terms):
    # 64-bit accumulator: c x y with x < m, y < 2m (negated) or m, m < 2^28
    s = sum(c * (2 if neg else 1) for _, _, c, neg in terms)
    assert s < 256, s
    return s


def run_op(rp, terms_list, env, regs):
    """exact model of one stage: env kind -> list of slot residue vectors"""
    outs = {}
    for dst, terms in terms_list:
        t = [0] * LANES
        for ch in range(LANES):
            acc = 0
            for a, b, c, neg in terms:
                x = env[a[0]][a[1]][ch]
                y = env[b[0]][b[1]][ch]
                if neg:
                    y = (L_(ch, "NEGK") - y) & M32
                acc += ((c * x) & M32) * y
            if not L_(ch, "ISR"):
                assert acc < 1 << 64
            t[ch] = red64(acc & ((1 << 64) - 1), ch)
        outs[dst] = mont(t)
    return outs


def to_m(v, slack=True):
    """a random M-domain representative (< 16 p) of the field element v"""
    x = v * MB % P
    if slack:
        x += random.randrange(15) * P
    return x


def check_all():
    random.seed(2377)
    built, rp, progs = build_ops()
    kres = [residues(k * MB % P) for k in rp.consts]
    maxw = 0
    for name in OPS:
        for _, terms in progs[name]:
            maxw = max(maxw, bound_check(terms))
    for name in OPS:
        pg, outs = built[name]
        A, B = W.rnd(48), W.rnd(48)
        if name == "CYC_SQR":
            f = W.t2p(A[:12])
            r = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
            r = O.f12_mul(O.f12_frob(r, 2), r)
            A = W.p2t(r) + A[12:]
        exp = W.evaluate(pg, outs, {"A": A, "B": B})
        env = {"A": [residues(to_m(v)) for v in A], "B": [residues(to_m(v)) for v in B], "K": kres}
        got = run_op(rp, progs[name], env, None)
        for d, lst in exp.items():
            items = sorted(lst.items()) if isinstance(lst, dict) else enumerate(lst)
            for k, v in items:
                r = got[W.DSTCODE[d] << 8 | k]
                x = crt(r)
                assert x < N1, (name, k, x // P)
                assert x % P == v * MB % P, (name, d, k)
    # the whole G2Prepared chain (pairing.h g2_double_step / g2_add_step) in
    # place on one 44-slot region, as k_g2_prepare_rns runs it
    q = O.g2_mul(O.G2_GEN, 0x1234567)
    ref = O.g2_prepare(q)
    vals = {i: 0 for i in range(44)}
    vals[0], vals[1] = q[0]
    vals[2], vals[3] = q[1]
    vals[4], vals[5] = 1, 0
    vals[26], vals[27] = q[0]
    vals[28], vals[29] = q[1]
    reg = [residues(to_m(vals[i])) for i in range(44)]
    idx = 0
    for bit in bin(O.X)[3:]:
        steps = ["G2_DBL1", "G2_DBL2", "G2_DBL3", "G2_DBL4"]
        if bit == "1":
            steps += ["G2_ADD1", "G2_ADD2", "G2_ADD3", "G2_ADD4"]
        for st in steps:
            out = run_op(rp, progs[st], {"A": reg, "B": reg, "K": kres}, None)
            for dst, r in out.items():
                reg[dst & 0xff] = r
            if st in ("G2_DBL4", "G2_ADD4"):
                got = [crt(reg[6 + j]) % P * pow(MB, -1, P) % P for j in range(6)]
                c0, c1, c2 = ref[idx]
                assert tuple(got) == (*c0, *c1, *c2), (st, idx)
                assert all(crt(reg[i]) < N1 for i in range(44))
                idx += 1
    assert idx == len(ref)
    # conversions: std Montgomery (v R mod p, < p) -> M-domain and back
    kin = rp.const(MB * pow(RQ, -1, P) % P)                           # k M = M^2 / R
    kout = rp.const(RQ * pow(MB, -1, P) % P)                          # k M = R
    # first factor of a chain of k raw (unconverted) factors: k M = M^(k+1) / R^k
    kload = [rp.const(pow(MB * pow(RQ, -1, P), k, P)) for k in range(1, KLOAD_MAX + 1)]
    assert kload[0] == kin
    kres = [residues(k * MB % P) for k in rp.consts]
    for _ in range(20):
        a = random.randrange(P)
        v = a * RQ % P
        limbs = [(v >> (32 * k)) & M32 for k in range(12)]
        t = []
        for ch in range(LANES):
            acc = sum(limbs[k] * LANE_TABLE[ch][POW32_OFF + k] for k in range(12))
            r0 = red64(acc & ((1 << 64) - 1), ch)
            t.append(red64(r0 * kres[kin[1]][ch], ch))
        x = mont(t)
        xv = crt(x)
        assert xv < N1 and xv % P == a * MB % P
        t = [red64(x[ch] * kres[kout[1]][ch], ch) for ch in range(LANES)]
        y = mont(t)
        yv = crt(y)
        assert yv < N1 and yv % P == a * RQ % P
        assert store_model(y) == a * RQ % P
    # a chain of raw factors: first load with K_LOAD[k], then k - 1 raw loads
    for k in (2, 4, 8):
        vals = [random.randrange(P) for _ in range(k)]
        res = [residues(v * RQ % P) for v in vals]
        kk = kres[kload[k - 1][1]]
        acc = mont([red64(res[0][ch] * kk[ch], ch) for ch in range(LANES)])
        for r in res[1:]:
            acc = mont([red64(acc[ch] * r[ch], ch) for ch in range(LANES)])
        want = 1
        for v in vals:
            want = want * v % P
        assert crt(acc) < N1 and crt(acc) % P == want * MB % P
    return built, rp, progs, kin[1], kout[1], maxw, [k[1] for k in kload]


def limbs32(v, n):
    return [(v >> (32 * k)) & M32 for k in range(n)]


def render():
    built, rp, progs, kin, kout, maxw, kload = check_all()
    lines = ["// Generated by tools/gen_rns_ops.py -- do not edit.", "#pragma once", "#include <stdint.h>",
             "namespace tpst { namespace rns {"]
    lines.append("// base B  = %s" % BASE)
    lines.append("// base B' = %s" % BASEP)
    lines.append("// M = prod B ~ 2^%.2f, M' ~ 2^%.2f, M / p ~ 2^%.1f; max term weight %d (< 256)" % (
        MB.bit_length(), MBP.bit_length(), MB.bit_length() - P.bit_length(), maxw))
    lines.append("constexpr int NB = %d, R_CH = %d, BP0 = %d, LANE_WORDS = %d, ROW1_OFF = %d, ROW2_OFF = %d, "
                 "POW32_OFF = %d;" % (NB, R_CH, BP0, LANE_WORDS, ROW1_OFF, ROW2_OFF, POW32_OFF))
    lines.append("enum LaneField { %s };" % ", ".join("LF_%s = %d" % (k, i) for i, k in enumerate(LANE_FIELDS)))
    lines.append("static TPST_RNS_CONST uint32_t LANE[32][%d] = {%s};" % (
        LANE_WORDS, ", ".join("{%s}" % ", ".join("%du" % w for w in row) for row in LANE_TABLE)))
    lines.append("constexpr int N_CONSTS = %d, K_IN = %d, K_OUT = %d, KLOAD_MAX = %d;" % (
        len(rp.consts), kin, kout, KLOAD_MAX))
    lines.append("static constexpr int K_LOAD[KLOAD_MAX + 1] = {0, %s};  // (M/R)^k: k raw factors" % (
        ", ".join(map(str, kload))))
    lines.append("static TPST_RNS_CONST uint32_t CONST_RES[%d][32] = {%s};" % (
        len(rp.consts), ", ".join("{%s}" % ", ".join("%du" % r for r in residues(k * MB % P)) for k in rp.consts)))
    # CRT output: M_i (13 limbs), M (14 limbs), p (12 limbs)
    lines.append("static TPST_RNS_CONST uint32_t MI_LIMBS[%d][14] = {%s};" % (
        NB, ", ".join("{%s}" % ", ".join("0x%08xu" % w for w in limbs32(MB // m, 14)) for m in BASE)))
    lines.append("static TPST_RNS_CONST uint32_t M_LIMBS[14] = {%s};" % ", ".join("0x%08xu" % w for w in limbs32(MB, 14)))
    # programs: [no | nt << 8] then per output [dst, nt terms]
    blob, offs, stats = [], [], []
    for name in OPS:
        ol = progs[name]
        nt = max(len(t) for _, t in ol)
        offs.append(len(blob))
        blob.append(len(ol) | nt << 8)
        for dst, terms in ol:
            blob.append(dst)
            blob += [enc(*t) for t in terms] + [0] * (nt - len(terms))
        stats.append("//   %-8s outputs %2d  terms <= %2d  (total %d)" % (name, len(ol), nt, sum(len(t) for _, t in ol)))
    lines += stats
    lines.append("enum OpId {%s, N_OPS};" % ", ".join("OP_" + n for n in OPS))
    lines.append("static constexpr int OP_OFF[N_OPS] = {%s};" % ", ".join(map(str, offs)))
    lines.append("static constexpr int OP_NO[N_OPS] = {%s};" % ", ".join(str(blob[o] & 0xff) for o in offs))
    lines.append("static constexpr int OP_NT[N_OPS] = {%s};" % ", ".join(str(blob[o] >> 8) for o in offs))
    lines.append("static constexpr int OP_RW[N_OPS] = {%s};  // outputs overlap A inputs (in place)" % (
        ", ".join(str(rw_overlap(progs, n)) for n in OPS)))
    lines.append("// term word: idx_a | kind_a << 8 | idx_b << 10 | kind_b << 18 | neg_b << 20 | c << 24 "
                 "(kinds A 0, B 1, K 2); per output [dst (D << 8 | k), terms...]")
    lines.append("static constexpr uint32_t PROG[%d] = {%s};" % (len(blob), ", ".join("0x%08xu" % t for t in blob)))
    lines.append("}}  // namespace tpst::rns")
    return "\n".join(lines) + "\n", stats


INC_PATH = os.path.join(os.path.dirname(HERE), "testudo_amd", "csrc", "rns_ops.inc")


def main():
    text, stats = render()
    open(INC_PATH, "w").write(text)
    print("\n".join(stats))
    print("wrote", INC_PATH)


if __name__ == "__main__":
    main()
