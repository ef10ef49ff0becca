// CPU restatement of the reference's sqrt-PST hot path on BLS12-377.
//
// TEST INFRASTRUCTURE ONLY: used by tests/ (as the checker), by
// __graft_entry__.smoke() and by bench.py's cpu_baseline leg.  Never linked
// into or called by the product (testudo_amd/).  Independent of the product
// code: 64-bit limbs with __int128 CIOS here, 32-bit limbs on the GPU.
//
// What it restates (file:line under the reference tree; upstream crates are
// un-vendored):
//  * ark-ec msm_bigint_wnaf: signed-digit Pippenger, c = ln_without_floats(n)+2,
//    windows in parallel, running-sum bucket reduction, Horner over windows
//    (called at sqrt_pst.rs:124/198, mipp.rs:393, commitments.rs:76/85).
//  * ark-ec Bls12::multi_pairing: projective G2Prepared (D-twist), ell /
//    mul_by_034, final exponentiation eprint 2020/875 (sqrt_pst.rs:143,
//    mipp.rs:90-92/397).
//  * sqrt-PST Polynomial::{from_evaluations,get_q,eval,commit,open,verify}
//    (sqrt_pst.rs:32-264), MippProof::{prove,verify} (mipp.rs:31-320),
//    PoseidonTranscript (poseidon_transcript.rs:17-34) with the FR table of
//    parameters.rs:17-153 read into Fq.
//  * MultilinearPC::{commit,open,commit_g2,open_g1,check,check_2}
//    (circuit_verifier.rs:175-314).
// Parity of this restatement is pinned by the golden vectors generated from
// oracle/py (tests/golden) and by the reference's own KAT
// (dense_mlpoly.rs:609-623).
#include <omp.h>

#include <cstdint>
#include <algorithm>
#include <cstring>
#include <vector>

#include "consts.h"

typedef unsigned __int128 u128;
typedef uint64_t u64;

namespace orc {

// ------------------------------------------------------------- fields ---
template <int N, const u64* MOD, const u64* INVP, const u64* R2, const u64* ONE>
struct Fp {
  u64 l[N];
  static Fp zero() { Fp r; memset(r.l, 0, sizeof r.l); return r; }
  static Fp one() { Fp r; memcpy(r.l, ONE, sizeof r.l); return r; }
  bool is_zero() const { for (int i = 0; i < N; i++) if (l[i]) return false; return true; }
  bool operator==(const Fp& o) const { return memcmp(l, o.l, sizeof l) == 0; }
  bool operator!=(const Fp& o) const { return !(*this == o); }
  static bool geq_mod(const u64* a) {
    for (int i = N - 1; i >= 0; i--) {
      if (a[i] > MOD[i]) return true;
      if (a[i] < MOD[i]) return false;
    }
    return true;
  }
  static void sub_mod_raw(u64* a) {
    u64 br = 0;
    for (int i = 0; i < N; i++) {
      u128 d = (u128)a[i] - MOD[i] - br;
      a[i] = (u64)d;
      br = (u64)(d >> 64) & 1;
    }
  }
  Fp operator+(const Fp& b) const {
    Fp r;
    u64 c = 0;
    for (int i = 0; i < N; i++) {
      u128 s = (u128)l[i] + b.l[i] + c;
      r.l[i] = (u64)s;
      c = (u64)(s >> 64);
    }
    if (geq_mod(r.l)) sub_mod_raw(r.l);
    return r;
  }
  Fp operator-(const Fp& b) const {
    Fp r;
    u64 br = 0;
    for (int i = 0; i < N; i++) {
      u128 d = (u128)l[i] - b.l[i] - br;
      r.l[i] = (u64)d;
      br = (u64)(d >> 64) & 1;
    }
    if (br) {
      u64 c = 0;
      for (int i = 0; i < N; i++) {
        u128 s = (u128)r.l[i] + MOD[i] + c;
        r.l[i] = (u64)s;
        c = (u64)(s >> 64);
      }
    }
    return r;
  }
  Fp operator-() const { return zero() - *this; }
  Fp operator*(const Fp& b) const {
    u64 t[N + 2];
    memset(t, 0, sizeof t);
    for (int i = 0; i < N; i++) {
      u64 c = 0;
      for (int j = 0; j < N; j++) {
        u128 s = (u128)l[j] * b.l[i] + t[j] + c;
        t[j] = (u64)s;
        c = (u64)(s >> 64);
      }
      u128 s = (u128)t[N] + c;
      t[N] = (u64)s;
      t[N + 1] = (u64)(s >> 64);
      u64 m = t[0] * INVP[0];
      u128 s2 = (u128)m * MOD[0] + t[0];
      c = (u64)(s2 >> 64);
      for (int j = 1; j < N; j++) {
        s2 = (u128)m * MOD[j] + t[j] + c;
        t[j - 1] = (u64)s2;
        c = (u64)(s2 >> 64);
      }
      s2 = (u128)t[N] + c;
      t[N - 1] = (u64)s2;
      t[N] = t[N + 1] + (u64)(s2 >> 64);
    }
    Fp r;
    memcpy(r.l, t, sizeof r.l);
    if (t[N] || geq_mod(r.l)) sub_mod_raw(r.l);
    return r;
  }
  Fp sq() const { return *this * *this; }
  Fp dbl() const { return *this + *this; }
  static Fp from_canon(const u64* a) {
    Fp x, r2;
    memcpy(x.l, a, sizeof x.l);
    memcpy(r2.l, R2, sizeof r2.l);
    return x * r2;
  }
  void to_canon(u64* out) const {
    Fp one = zero();
    one.l[0] = 1;
    Fp r = *this * one;
    memcpy(out, r.l, sizeof r.l);
  }
  Fp pow(const u64* e, int nlimbs) const {
    Fp r = one();
    for (int i = nlimbs - 1; i >= 0; i--)
      for (int b = 63; b >= 0; b--) {
        r = r.sq();
        if ((e[i] >> b) & 1) r = r * *this;
      }
    return r;
  }
  Fp inv() const {
    u64 e[N];
    memcpy(e, MOD, sizeof e);
    e[0] -= 2;
    return pow(e, N);
  }
};

static const u64 FQ_INVP[1] = {FQ_INV};
static const u64 FR_INVP[1] = {FR_INV};
typedef Fp<6, FQ_MOD, FQ_INVP, FQ_R2, FQ_ONE> Fq;
typedef Fp<4, FR_MOD, FR_INVP, FR_R2, FR_ONE> Fr;

static Fq fq_c(const u64* a) { return Fq::from_canon(a); }

struct Fq2 {
  Fq c0, c1;
  static Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
  static Fq2 one() { return {Fq::one(), Fq::zero()}; }
  bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  bool operator==(const Fq2& o) const { return c0 == o.c0 && c1 == o.c1; }
  Fq2 operator+(const Fq2& b) const { return {c0 + b.c0, c1 + b.c1}; }
  Fq2 operator-(const Fq2& b) const { return {c0 - b.c0, c1 - b.c1}; }
  Fq2 operator-() const { return {-c0, -c1}; }
  static Fq m5(const Fq& a) { Fq t = a.dbl().dbl(); return t + a; }
  Fq2 operator*(const Fq2& b) const {
    Fq v0 = c0 * b.c0, v1 = c1 * b.c1;
    return {v0 - m5(v1), (c0 + c1) * (b.c0 + b.c1) - v0 - v1};
  }
  Fq2 sq() const { return *this * *this; }
  Fq2 dbl() const { return *this + *this; }
  Fq2 mulfq(const Fq& s) const { return {c0 * s, c1 * s}; }
  Fq2 conj() const { return {c0, -c1}; }
  Fq2 inv() const {
    Fq n = c0.sq() + m5(c1.sq());
    Fq ni = n.inv();
    return {c0 * ni, -(c1 * ni)};
  }
  Fq2 mul_nr() const { return {-m5(c1), c0}; }  // * u
};

static Fq2 fq2_c(const u64 (*a)[6]) { return {fq_c(a[0]), fq_c(a[1])}; }

struct Fq6 {
  Fq2 c0, c1, c2;
  static Fq6 zero() { return {Fq2::zero(), Fq2::zero(), Fq2::zero()}; }
  static Fq6 one() { return {Fq2::one(), Fq2::zero(), Fq2::zero()}; }
  Fq6 operator+(const Fq6& b) const { return {c0 + b.c0, c1 + b.c1, c2 + b.c2}; }
  Fq6 operator-(const Fq6& b) const { return {c0 - b.c0, c1 - b.c1, c2 - b.c2}; }
  Fq6 operator-() const { return {-c0, -c1, -c2}; }
  bool operator==(const Fq6& o) const { return c0 == o.c0 && c1 == o.c1 && c2 == o.c2; }
  Fq6 operator*(const Fq6& b) const {
    // schoolbook with v^3 = u
    Fq2 a0b0 = c0 * b.c0, a1b1 = c1 * b.c1, a2b2 = c2 * b.c2;
    Fq2 r0 = a0b0 + (c1 * b.c2 + c2 * b.c1).mul_nr();
    Fq2 r1 = c0 * b.c1 + c1 * b.c0 + a2b2.mul_nr();
    Fq2 r2 = c0 * b.c2 + a1b1 + c2 * b.c0;
    return {r0, r1, r2};
  }
  Fq6 mul_nr() const { return {c2.mul_nr(), c0, c1}; }  // * v
  Fq6 inv() const {
    Fq2 t0 = c0.sq() - (c1 * c2).mul_nr();
    Fq2 t1 = c2.sq().mul_nr() - c0 * c1;
    Fq2 t2 = c1.sq() - c0 * c2;
    Fq2 d = c0 * t0 + (c2 * t1 + c1 * t2).mul_nr();
    Fq2 di = d.inv();
    return {t0 * di, t1 * di, t2 * di};
  }
};

struct Fq12 {
  Fq6 c0, c1;
  static Fq12 one() { return {Fq6::one(), Fq6::zero()}; }
  bool operator==(const Fq12& o) const { return c0 == o.c0 && c1 == o.c1; }
  Fq12 operator*(const Fq12& b) const {
    Fq6 v0 = c0 * b.c0, v1 = c1 * b.c1;
    return {v0 + v1.mul_nr(), c0 * b.c1 + c1 * b.c0};
  }
  Fq12 sq() const { return *this * *this; }
  Fq12 conj() const { return {c0, -c1}; }
  Fq12 inv() const {
    Fq6 t = c0 * c0 - (c1 * c1).mul_nr();
    Fq6 ti = t.inv();
    return {c0 * ti, -(c1 * ti)};
  }
  Fq12 frob(int k) const {
    const u64(*c61)[6] = k == 1 ? F6C1_1 : F6C1_2;
    const u64(*c62)[6] = k == 1 ? F6C2_1 : F6C2_2;
    const u64(*c12)[6] = k == 1 ? F12C1_1 : F12C1_2;
    Fq2 a = fq2_c(c61), b = fq2_c(c62), w = fq2_c(c12);
    auto f2 = [&](const Fq2& x) { return (k & 1) ? x.conj() : x; };
    Fq6 x0 = {f2(c0.c0), f2(c0.c1) * a, f2(c0.c2) * b};
    Fq6 x1 = {f2(c1.c0) * w, f2(c1.c1) * a * w, f2(c1.c2) * b * w};
    return {x0, x1};
  }
  void to_canon(u64* out) const {  // arkworks order, 72 u64
    const Fq* f[12] = {&c0.c0.c0, &c0.c0.c1, &c0.c1.c0, &c0.c1.c1, &c0.c2.c0, &c0.c2.c1,
                       &c1.c0.c0, &c1.c0.c1, &c1.c1.c0, &c1.c1.c1, &c1.c2.c0, &c1.c2.c1};
    for (int i = 0; i < 12; i++) f[i]->to_canon(out + 6 * i);
  }
  static Fq12 from_canon(const u64* in) {
    Fq12 r;
    Fq* f[12] = {&r.c0.c0.c0, &r.c0.c0.c1, &r.c0.c1.c0, &r.c0.c1.c1, &r.c0.c2.c0, &r.c0.c2.c1,
                 &r.c1.c0.c0, &r.c1.c0.c1, &r.c1.c1.c0, &r.c1.c1.c1, &r.c1.c2.c0, &r.c1.c2.c1};
    for (int i = 0; i < 12; i++) *f[i] = Fq::from_canon(in + 6 * i);
    return r;
  }
  Fq12 pow_fr(const Fr& e) const {  // exponent = canonical value of e
    u64 c[4];
    e.to_canon(c);
    Fq12 r = one();
    for (int i = 3; i >= 0; i--)
      for (int b = 63; b >= 0; b--) {
        r = r.sq();
        if ((c[i] >> b) & 1) r = r * *this;
      }
    return r;
  }
};

// -------------------------------------------------------------- curves ---
template <class F> struct CB;
template <> struct CB<Fq> { static Fq b() { return Fq::one(); } };
template <> struct CB<Fq2> { static Fq2 b() { return {Fq::zero(), fq_c(G2B1)}; } };

template <class F>
struct Aff {
  F x, y;
  bool inf;
};

template <class F>
struct Proj {  // Jacobian
  F X, Y, Z;
  static Proj zero() { return {F::one(), F::one(), F::zero()}; }
  bool is_zero() const { return Z.is_zero(); }
};

template <class F>
Proj<F> pdbl(const Proj<F>& p) {
  if (p.is_zero()) return p;
  F A = p.X.sq(), B = p.Y.sq(), C = B.sq();
  F D = ((p.X + B).sq() - A - C).dbl();
  F E = A.dbl() + A;
  F Ff = E.sq();
  F X3 = Ff - D.dbl();
  F C8 = C.dbl().dbl().dbl();
  F Y3 = E * (D - X3) - C8;
  F Z3 = (p.Y * p.Z).dbl();
  return {X3, Y3, Z3};
}

template <class F>
Proj<F> padd_mixed(const Proj<F>& p, const Aff<F>& q) {
  if (q.inf) return p;
  if (p.is_zero()) return {q.x, q.y, F::one()};
  F Z1Z1 = p.Z.sq();
  F U2 = q.x * Z1Z1;
  F S2 = q.y * p.Z * Z1Z1;
  F H = U2 - p.X, rr = S2 - p.Y;
  if (H.is_zero()) {
    if (rr.is_zero()) return pdbl(Proj<F>{q.x, q.y, F::one()});
    return Proj<F>::zero();
  }
  F HH = H.sq(), HHH = H * HH, V = p.X * HH;
  F X3 = rr.sq() - HHH - V.dbl();
  F Y3 = rr * (V - X3) - p.Y * HHH;
  return {X3, Y3, p.Z * H};
}

template <class F>
Proj<F> padd(const Proj<F>& p, const Proj<F>& q) {
  if (p.is_zero()) return q;
  if (q.is_zero()) return p;
  F Z1Z1 = p.Z.sq(), Z2Z2 = q.Z.sq();
  F U1 = p.X * Z2Z2, U2 = q.X * Z1Z1;
  F S1 = p.Y * q.Z * Z2Z2, S2 = q.Y * p.Z * Z1Z1;
  F H = U2 - U1, rr = S2 - S1;
  if (H.is_zero()) {
    if (rr.is_zero()) return pdbl(p);
    return Proj<F>::zero();
  }
  F HH = H.sq(), HHH = H * HH, V = U1 * HH;
  F X3 = rr.sq() - HHH - V.dbl();
  F Y3 = rr * (V - X3) - S1 * HHH;
  return {X3, Y3, p.Z * q.Z * H};
}

template <class F>
Aff<F> to_aff(const Proj<F>& p) {
  if (p.is_zero()) return {F::zero(), F::zero(), true};
  F zi = p.Z.inv(), zi2 = zi.sq();
  return {p.X * zi2, p.Y * zi2 * zi, false};
}

template <class F>
Aff<F> aneg(const Aff<F>& a) { return {a.x, -a.y, a.inf}; }

template <class F>
Proj<F> to_proj(const Aff<F>& a) { return a.inf ? Proj<F>::zero() : Proj<F>{a.x, a.y, F::one()}; }

// canonical Fr -> 4 u64
static void fr_canon(const Fr& a, u64* out) { a.to_canon(out); }

template <class F>
Proj<F> smul(const Aff<F>& a, const u64* k, int nlimbs = 4) {
  Proj<F> acc = Proj<F>::zero();
  for (int i = nlimbs - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      acc = pdbl(acc);
      if ((k[i] >> b) & 1) acc = padd_mixed(acc, a);
    }
  return acc;
}

template <class F>
Proj<F> smul_fr(const Aff<F>& a, const Fr& k) {
  u64 c[4];
  fr_canon(k, c);
  return smul(a, c);
}

template <class F>
Proj<F> smul_proj(const Proj<F>& a, const Fr& k) {
  u64 c[4];
  fr_canon(k, c);
  Proj<F> acc = Proj<F>::zero();
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      acc = pdbl(acc);
      if ((c[i] >> b) & 1) acc = padd(acc, a);
    }
  return acc;
}

// ------------------------------------------------------------- MSM -------
static int ln_without_floats(size_t a) {  // ark_std: log2(a) * 69 / 100
  int lg = 0;
  while ((size_t(1) << (lg + 1)) <= a) lg++;
  if (a && (a & (a - 1))) lg++;  // ceil log2 as ark's log2
  return lg * 69 / 100;
}

// make_digits (ark-ec msm/variable_base/mod.rs)
static void make_digits(const u64* s, int w, int num_bits, int64_t* out) {
  const u64 radix = 1ull << w, mask = radix - 1;
  u64 carry = 0;
  int count = (num_bits + w - 1) / w;
  for (int i = 0; i < count; i++) {
    int off = i * w, ui = off / 64, bi = off % 64;
    u64 buf;
    if (bi < 64 - w || ui == 3)
      buf = s[ui] >> bi;
    else
      buf = (s[ui] >> bi) | (s[ui + 1] << (64 - bi));
    u64 coef = carry + (buf & mask);
    carry = (coef + radix / 2) >> w;
    int64_t d = (int64_t)coef - (int64_t)(carry << w);
    if (i == count - 1) d += (int64_t)(carry << w);
    out[i] = d;
  }
}

// msm_bigint_wnaf; `par` parallelises the windows
template <class F>
Proj<F> msm(const Aff<F>* bases, const u64* scalars /*4 u64 canonical*/, size_t n, bool par) {
  if (n == 0) return Proj<F>::zero();
  const int c = n < 32 ? 3 : ln_without_floats(n) + 2;
  const int num_bits = 253;
  const int W = (num_bits + c - 1) / c;
  std::vector<int64_t> dig(n * W);
  for (size_t i = 0; i < n; i++) make_digits(scalars + 4 * i, c, num_bits, &dig[i * W]);
  std::vector<Proj<F>> wins(W);
#pragma omp parallel for schedule(dynamic, 1) if (par)
  for (int w = 0; w < W; w++) {
    std::vector<Proj<F>> buckets(size_t(1) << c, Proj<F>::zero());
    for (size_t i = 0; i < n; i++) {
      int64_t d = dig[i * W + w];
      if (d > 0) buckets[d - 1] = padd_mixed(buckets[d - 1], bases[i]);
      else if (d < 0) buckets[-d - 1] = padd_mixed(buckets[-d - 1], aneg(bases[i]));
    }
    Proj<F> run = Proj<F>::zero(), res = Proj<F>::zero();
    for (size_t b = buckets.size(); b-- > 0;) {
      run = padd(run, buckets[b]);
      res = padd(res, run);
    }
    wins[w] = res;
  }
  Proj<F> total = Proj<F>::zero();
  for (int w = W - 1; w >= 1; w--) {
    total = padd(total, wins[w]);
    for (int k = 0; k < c; k++) total = pdbl(total);
  }
  return padd(total, wins[0]);
}

// ---------------------------------------------------------- pairing -----
struct Coeff {
  Fq2 a, b, c;
};

static void g2_prepare(const Aff<Fq2>& q, std::vector<Coeff>& out) {
  out.clear();
  if (q.inf) return;
  const Fq two_inv = fq_c(TWO_INV);
  const Fq2 B = CB<Fq2>::b();
  Fq2 rx = q.x, ry = q.y, rz = Fq2::one();
  for (int bit = 62; bit >= 0; bit--) {
    Fq2 a = (rx * ry).mulfq(two_inv);
    Fq2 b = ry.sq(), c = rz.sq();
    Fq2 e = B * (c.dbl() + c);
    Fq2 f = e.dbl() + e;
    Fq2 g = (b + f).mulfq(two_inv);
    Fq2 h = (ry + rz).sq() - (b + c);
    Fq2 i = e - b, j = rx.sq(), e2 = e.sq();
    rx = a * (b - f);
    ry = g.sq() - (e2.dbl() + e2);
    rz = b * h;
    out.push_back({-h, j.dbl() + j, i});
    if ((BLS_X >> bit) & 1) {
      Fq2 th = ry - q.y * rz, la = rx - q.x * rz;
      Fq2 C = th.sq(), D = la.sq(), E = la * D, Fv = rz * C, G = rx * D;
      Fq2 H = E + Fv - G.dbl();
      rx = la * H;
      ry = th * (G - H) - E * ry;
      rz = rz * E;
      Fq2 J = th * q.x - la * q.y;
      out.push_back({la, -th, J});
    }
  }
}

static Fq12 mul_by_034(const Fq12& f, const Fq2& c0, const Fq2& c3, const Fq2& c4) {
  Fq12 sp = {Fq6{c0, Fq2::zero(), Fq2::zero()}, Fq6{c3, c4, Fq2::zero()}};
  return f * sp;
}

static Fq12 miller(const std::vector<Aff<Fq>>& ps, const std::vector<std::vector<Coeff>>& cs) {
  Fq12 f = Fq12::one();
  size_t idx = 0;
  for (int bit = 62; bit >= 0; bit--) {
    f = f.sq();
    for (size_t i = 0; i < ps.size(); i++) {
      const Coeff& k = cs[i][idx];
      f = mul_by_034(f, k.a.mulfq(ps[i].y), k.b.mulfq(ps[i].x), k.c);
    }
    idx++;
    if ((BLS_X >> bit) & 1) {
      for (size_t i = 0; i < ps.size(); i++) {
        const Coeff& k = cs[i][idx];
        f = mul_by_034(f, k.a.mulfq(ps[i].y), k.b.mulfq(ps[i].x), k.c);
      }
      idx++;
    }
  }
  return f;
}

static Fq12 exp_x(const Fq12& f) {
  Fq12 r = f;
  for (int bit = 62; bit >= 0; bit--) {
    r = r.sq();
    if ((BLS_X >> bit) & 1) r = r * f;
  }
  return r;
}

static Fq12 final_exp(const Fq12& f) {
  Fq12 r = f.conj() * f.inv();
  r = r.frob(2) * r;
  Fq12 y0 = r.sq(), y1 = exp_x(r), y2 = r.conj();
  y1 = y1 * y2;
  y2 = exp_x(y1);
  y1 = y1.conj();
  y1 = y1 * y2;
  y2 = exp_x(y1);
  y1 = y1.frob(1);
  y1 = y1 * y2;
  r = r * y0;
  y0 = exp_x(y1);
  y2 = exp_x(y0);
  y0 = y1.frob(2);
  y1 = y1.conj();
  y1 = y1 * y2;
  y1 = y1 * y0;
  return r * y1;
}

static Fq12 miller_product(const Aff<Fq>* g1, const Aff<Fq2>* g2, size_t n) {
  // chunks of 4 pairs share f, chunks run in parallel (bls12/mod.rs)
  std::vector<Aff<Fq>> ps;
  std::vector<Aff<Fq2>> qs;
  for (size_t i = 0; i < n; i++)
    if (!g1[i].inf && !g2[i].inf) {
      ps.push_back(g1[i]);
      qs.push_back(g2[i]);
    }
  size_t m = ps.size();
  size_t nch = (m + 3) / 4;
  std::vector<Fq12> parts(nch, Fq12::one());
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t ch = 0; ch < nch; ch++) {
    std::vector<Aff<Fq>> p;
    std::vector<std::vector<Coeff>> c;
    for (size_t i = ch * 4; i < m && i < ch * 4 + 4; i++) {
      p.push_back(ps[i]);
      c.emplace_back();
      g2_prepare(qs[i], c.back());
    }
    parts[ch] = miller(p, c);
  }
  Fq12 f = Fq12::one();
  for (auto& x : parts) f = f * x;
  return f;
}

static Fq12 multi_pairing(const Aff<Fq>* g1, const Aff<Fq2>* g2, size_t n) {
  return final_exp(miller_product(g1, g2, n));
}

// --------------------------------------------------------- encodings -----
static Aff<Fq> g1_in(const u64* a) {
  bool z = true;
  for (int i = 0; i < 12; i++) z &= a[i] == 0;
  if (z) return {Fq::zero(), Fq::zero(), true};
  return {fq_c(a), fq_c(a + 6), false};
}
static void g1_out(const Aff<Fq>& p, u64* o) {
  if (p.inf) { memset(o, 0, 96); return; }
  p.x.to_canon(o);
  p.y.to_canon(o + 6);
}
static Aff<Fq2> g2_in(const u64* a) {
  bool z = true;
  for (int i = 0; i < 24; i++) z &= a[i] == 0;
  if (z) return {Fq2::zero(), Fq2::zero(), true};
  return {{fq_c(a), fq_c(a + 6)}, {fq_c(a + 12), fq_c(a + 18)}, false};
}
static void g2_out(const Aff<Fq2>& p, u64* o) {
  if (p.inf) { memset(o, 0, 192); return; }
  p.x.c0.to_canon(o);
  p.x.c1.to_canon(o + 6);
  p.y.c0.to_canon(o + 12);
  p.y.c1.to_canon(o + 18);
}
static Fr fr_in(const u64* a) { return Fr::from_canon(a); }

// serialize (Compress::No) for the transcript
static void fq_bytes(const Fq& a, uint8_t* b) {
  u64 c[6];
  a.to_canon(c);
  memcpy(b, c, 48);
}
static bool fq_gt_neg(const Fq& y) {  // y > -y  (canonical compare)
  u64 a[6], b[6];
  y.to_canon(a);
  (-y).to_canon(b);
  for (int i = 5; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return false;
}
static void g1_bytes(const Aff<Fq>& p, uint8_t* b) {  // 96 bytes
  if (p.inf) {
    memset(b, 0, 96);
    b[95] |= 0x40;
    return;
  }
  fq_bytes(p.x, b);
  fq_bytes(p.y, b + 48);
  if (fq_gt_neg(p.y)) b[95] |= 0x80;
}
static void fq12_bytes(const Fq12& f, uint8_t* b) {
  u64 c[72];
  f.to_canon(c);
  memcpy(b, c, 576);
}

// --------------------------------------------------------- Poseidon -----
struct Poseidon {
  Fq ark[39][3], mds[3][3];
  Fq st[3];
  bool squeezing = false;
  int idx = 0;
  void permute() {
    for (int r = 0; r < 39; r++) {
      for (int i = 0; i < 3; i++) st[i] = st[i] + ark[r][i];
      bool full = r < 4 || r >= 35;
      for (int i = 0; i < (full ? 3 : 1); i++) {
        Fq x = st[i], x2 = x.sq(), x4 = x2.sq(), x8 = x4.sq(), x16 = x8.sq();
        st[i] = x16 * x;  // alpha = 17
      }
      Fq ns[3];
      for (int i = 0; i < 3; i++) ns[i] = mds[i][0] * st[0] + mds[i][1] * st[1] + mds[i][2] * st[2];
      for (int i = 0; i < 3; i++) st[i] = ns[i];
    }
  }
  void absorb_elems(const std::vector<Fq>& e) {
    if (e.empty()) return;
    size_t k = 0;
    int i0;
    if (!squeezing) {
      i0 = idx;
      if (i0 == 2) {
        permute();
        i0 = 0;
      }
    } else {
      permute();
      i0 = 0;
    }
    while (true) {
      size_t rem = e.size() - k;
      if (i0 + rem <= 2) {
        for (size_t j = 0; j < rem; j++) st[1 + i0 + j] = st[1 + i0 + j] + e[k + j];
        squeezing = false;
        idx = i0 + (int)rem;
        return;
      }
      int take = 2 - i0;
      for (int j = 0; j < take; j++) st[1 + i0 + j] = st[1 + i0 + j] + e[k + j];
      permute();
      k += take;
      i0 = 0;
    }
  }
  void absorb_bytes(const uint8_t* d, size_t n) {
    std::vector<uint8_t> buf(8 + n);
    u64 len = n;
    memcpy(buf.data(), &len, 8);
    memcpy(buf.data() + 8, d, n);
    std::vector<Fq> e;
    for (size_t o = 0; o < buf.size(); o += 47) {
      u64 l[6] = {0, 0, 0, 0, 0, 0};
      size_t m = buf.size() - o < 47 ? buf.size() - o : 47;
      memcpy(l, buf.data() + o, m);
      e.push_back(Fq::from_canon(l));
    }
    absorb_elems(e);
  }
  Fq squeeze1() {
    int i0;
    if (!squeezing) {
      permute();
      i0 = 0;
    } else {
      i0 = idx;
      if (i0 == 2) {
        permute();
        i0 = 0;
      }
    }
    Fq out = st[1 + i0];
    squeezing = true;
    idx = i0 + 1;
    return out;
  }
  Fr challenge() {
    u64 c[6];
    squeeze1().to_canon(c);
    u64 f[4] = {c[0], c[1], c[2], c[3] & ((1ull << 60) - 1)};  // low 252 bits
    return Fr::from_canon(f);
  }
  void append_g1(const Aff<Fq>& p) {
    uint8_t b[96];
    g1_bytes(p, b);
    absorb_bytes(b, 96);
  }
  void append_gt(const Fq12& f) {
    uint8_t b[576];
    fq12_bytes(f, b);
    absorb_bytes(b, 576);
  }
};

}  // namespace orc

using namespace orc;

// ------------------------------------------------------------------ SRS ---
struct orc_srs {
  int nv;
  Aff<Fq> g;
  Aff<Fq2> h;
  std::vector<std::vector<Aff<Fq>>> pg;   // powers_of_g[i], 2^(nv-i)
  std::vector<std::vector<Aff<Fq2>>> ph;  // powers_of_h[i]
  std::vector<Aff<Fq>> gmask;
  std::vector<Aff<Fq2>> hmask;
  std::vector<std::vector<Coeff>> h_prep;  // unused cache slot
};

static Poseidon make_poseidon(const u64* ark /*39*3*6*/, const u64* mds /*3*3*6*/) {
  Poseidon p;
  for (int r = 0; r < 39; r++)
    for (int i = 0; i < 3; i++) p.ark[r][i] = Fq::from_canon(ark + 6 * (3 * r + i));
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) p.mds[i][j] = Fq::from_canon(mds + 6 * (3 * i + j));
  for (int i = 0; i < 3; i++) p.st[i] = Fq::zero();
  return p;
}

static std::vector<u64> g_ark, g_mds;

static u64 splitmix(u64 seed, u64 i) {
  u64 z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static bool lt_r(const u64* v) {
  for (int i = 3; i >= 0; i--) {
    if (v[i] < FR_MOD[i]) return true;
    if (v[i] > FR_MOD[i]) return false;
  }
  return false;
}

extern "C" {

int orc_threads(void) { return omp_get_max_threads(); }
void orc_set_threads(int n) { omp_set_num_threads(n); }

// n uniform Fr (canonical) from the SplitMix64 stream (oracle/py/pst.py fr_stream)
u64 orc_fr_stream(u64 seed, size_t n, u64 start, u64* out) {
  u64 k = start;
  size_t got = 0;
  while (got < n) {
    u64 v[4];
    for (int j = 0; j < 4; j++) v[j] = splitmix(seed, 4 * k + j);
    v[3] &= (1ull << 61) - 1;
    k++;
    if (lt_r(v)) {
      memcpy(out + 4 * got, v, 32);
      got++;
    }
  }
  return k;
}

void orc_set_poseidon(const u64* ark, const u64* mds) {
  g_ark.assign(ark, ark + 39 * 3 * 6);
  g_mds.assign(mds, mds + 9 * 6);
}

int orc_g1_msm(const u64* bases, const u64* scalars, size_t n, u64* out, int parallel) {
  std::vector<Aff<Fq>> b(n);
  for (size_t i = 0; i < n; i++) b[i] = g1_in(bases + 12 * i);
  g1_out(to_aff(msm(b.data(), scalars, n, parallel != 0)), out);
  return 0;
}

int orc_g2_msm(const u64* bases, const u64* scalars, size_t n, u64* out, int parallel) {
  std::vector<Aff<Fq2>> b(n);
  for (size_t i = 0; i < n; i++) b[i] = g2_in(bases + 24 * i);
  g2_out(to_aff(msm(b.data(), scalars, n, parallel != 0)), out);
  return 0;
}

// rows independent MSMs sharing bases (scalar (r,j) at scalars + 4*(r*rs + j*cs))
int orc_g1_msm_batch(const u64* bases, size_t N, const u64* scalars, size_t rows, size_t rs, size_t cs, u64* out) {
  std::vector<Aff<Fq>> b(N);
  for (size_t i = 0; i < N; i++) b[i] = g1_in(bases + 12 * i);
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t r = 0; r < rows; r++) {
    std::vector<u64> sc(4 * N);
    for (size_t j = 0; j < N; j++) memcpy(&sc[4 * j], scalars + 4 * (r * rs + j * cs), 32);
    g1_out(to_aff(msm(b.data(), sc.data(), N, false)), out + 12 * r);
  }
  return 0;
}

int orc_multi_pairing(const u64* g1, const u64* g2, size_t n, u64* out) {
  std::vector<Aff<Fq>> a(n);
  std::vector<Aff<Fq2>> b(n);
  for (size_t i = 0; i < n; i++) {
    a[i] = g1_in(g1 + 12 * i);
    b[i] = g2_in(g2 + 24 * i);
  }
  multi_pairing(a.data(), b.data(), n).to_canon(out);
  return 0;
}

// prod of the Miller loops of n pairs, before final exponentiation (the
// per-rank IPP partial of the row-sharded commit)
int orc_miller_product(const u64* g1, const u64* g2, size_t n, u64* out) {
  std::vector<Aff<Fq>> a(n);
  std::vector<Aff<Fq2>> b(n);
  for (size_t i = 0; i < n; i++) {
    a[i] = g1_in(g1 + 12 * i);
    b[i] = g2_in(g2 + 24 * i);
  }
  miller_product(a.data(), b.data(), n).to_canon(out);
  return 0;
}

// FE(prod of k canonical Fq12)
int orc_gt_final_exp_product(const u64* parts, size_t k, u64* out) {
  Fq12 f = Fq12::one();
  for (size_t i = 0; i < k; i++) f = f * Fq12::from_canon(parts + 72 * i);
  final_exp(f).to_canon(out);
  return 0;
}

int orc_g1_mul_gen(const u64* scalars, size_t n, u64* out) {
  Aff<Fq> g = {fq_c(G1X), fq_c(G1Y), false};
#pragma omp parallel for
  for (size_t i = 0; i < n; i++) g1_out(to_aff(smul(g, scalars + 4 * i)), out + 12 * i);
  return 0;
}

int orc_g2_mul_gen(const u64* scalars, size_t n, u64* out) {
  Aff<Fq2> g = {{fq_c(G2X0), fq_c(G2X1)}, {fq_c(G2Y0), fq_c(G2Y1)}, false};
#pragma omp parallel for
  for (size_t i = 0; i < n; i++) g2_out(to_aff(smul(g, scalars + 4 * i)), out + 24 * i);
  return 0;
}

// MultilinearPC::setup semantics from the seeded trapdoor (oracle/py/pst.py SRS)
orc_srs* orc_srs_setup(int nv, u64 seed) {
  orc_srs* s = new orc_srs();
  s->nv = nv;
  std::vector<u64> vals(4 * (nv + 2));
  orc_fr_stream(seed, nv + 2, 0, vals.data());
  Aff<Fq> G = {fq_c(G1X), fq_c(G1Y), false};
  Aff<Fq2> H = {{fq_c(G2X0), fq_c(G2X1)}, {fq_c(G2Y0), fq_c(G2Y1)}, false};
  s->g = to_aff(smul(G, &vals[0]));
  s->h = to_aff(smul(H, &vals[4]));
  std::vector<Fr> t(nv);
  for (int i = 0; i < nv; i++) t[i] = fr_in(&vals[4 * (2 + i)]);
  s->pg.resize(nv);
  s->ph.resize(nv);
  for (int i = 0; i < nv; i++) {
    std::vector<Fr> tab(1, Fr::one());
    for (int j = i; j < nv; j++) {
      size_t m = tab.size();
      tab.resize(2 * m);
      for (size_t x = 0; x < m; x++) {
        Fr v = tab[x];
        tab[x] = v * (Fr::one() - t[j]);
        tab[x + m] = v * t[j];
      }
    }
    s->pg[i].resize(tab.size());
    s->ph[i].resize(tab.size());
#pragma omp parallel for
    for (size_t x = 0; x < tab.size(); x++) {
      s->pg[i][x] = to_aff(smul_fr(s->g, tab[x]));
      s->ph[i][x] = to_aff(smul_fr(s->h, tab[x]));
    }
  }
  for (int i = 0; i < nv; i++) {
    s->gmask.push_back(to_aff(smul_fr(s->g, t[i])));
    s->hmask.push_back(to_aff(smul_fr(s->h, t[i])));
  }
  return s;
}

void orc_srs_free(orc_srs* s) { delete s; }

// export layout: g(12) h(24) then for i: pg[i] (2^(nv-i)*12), ph[i] (*24), gmask (nv*12), hmask (nv*24)
size_t orc_srs_export_len(const orc_srs* s) {
  size_t n = 12 + 24;
  for (int i = 0; i < s->nv; i++) n += (size_t(1) << (s->nv - i)) * 36;
  return n + s->nv * 36;
}

void orc_srs_export(const orc_srs* s, u64* out) {
  g1_out(s->g, out);
  g2_out(s->h, out + 12);
  u64* o = out + 36;
  for (int i = 0; i < s->nv; i++) {
    for (auto& p : s->pg[i]) { g1_out(p, o); o += 12; }
    for (auto& p : s->ph[i]) { g2_out(p, o); o += 24; }
  }
  for (auto& p : s->gmask) { g1_out(p, o); o += 12; }
  for (auto& p : s->hmask) { g2_out(p, o); o += 24; }
}

// --------------------------------------------------------------- sqrt-PST --
static Fr chi(const std::vector<Fr>& b, size_t i) {  // sqrt_pst.rs:152-166 MSB-first
  size_t m = b.size();
  Fr prod = Fr::one();
  for (size_t j = 0; j < m; j++) prod = prod * (((i >> (m - j - 1)) & 1) ? b[j] : Fr::one() - b[j]);
  return prod;
}

static std::vector<Fr> chis_msb(const std::vector<Fr>& b) {  // all chi_i(b), i < 2^m
  std::vector<Fr> t(1, Fr::one());
  for (size_t j = 0; j < b.size(); j++) {  // b[0] is the MSB
    std::vector<Fr> n(2 * t.size());
    for (size_t x = 0; x < t.size(); x++) {
      n[2 * x] = t[x] * (Fr::one() - b[j]);
      n[2 * x + 1] = t[x] * b[j];
    }
    t.swap(n);
  }
  return t;
}

struct Dims {
  int n, m_col, m_row, odd;
};
static Dims dims(int n) { return {n, n / 2, n - n / 2, n % 2}; }

static void get_q(const u64* Z, const Dims& d, const std::vector<Fr>& point, std::vector<Fr>& q, std::vector<Fr>& chis) {
  std::vector<Fr> b(point.begin() + d.m_col + d.odd, point.end());
  chis = chis_msb(b);
  size_t C = size_t(1) << d.m_col, Rn = size_t(1) << d.m_row;
  q.assign(Rn, Fr::zero());
#pragma omp parallel for
  for (size_t j = 0; j < Rn; j++) {
    Fr acc = Fr::zero();
    for (size_t i = 0; i < C; i++) acc = acc + fr_in(Z + 4 * ((j << d.m_col) | i)) * chis[i];
    q[j] = acc;
  }
}

// sqrt_pst.rs:105-115
int orc_pst_eval(const u64* Z, int n, const u64* point, u64* out_v) {
  Dims d = dims(n);
  std::vector<Fr> pt(n);
  for (int i = 0; i < n; i++) pt[i] = fr_in(point + 4 * i);
  std::vector<Fr> q, chis;
  get_q(Z, d, pt, q, chis);
  std::vector<Fr> a(pt.begin(), pt.begin() + d.m_row);
  std::vector<Fr> ca = chis_msb(a);
  Fr v = Fr::zero();
  for (size_t j = 0; j < q.size(); j++) v = v + q[j] * ca[j];
  v.to_canon(out_v);
  return 0;
}

// sqrt_pst.rs:117-149
int orc_pst_commit(const orc_srs* s, const u64* Z, int n, u64* comms, u64* T) {
  Dims d = dims(n);
  if (d.m_row != s->nv) return -1;
  size_t C = size_t(1) << d.m_col, Rn = size_t(1) << d.m_row;
  std::vector<Aff<Fq>> cm(C);
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t i = 0; i < C; i++) {
    std::vector<u64> sc(4 * Rn);
    for (size_t j = 0; j < Rn; j++) memcpy(&sc[4 * j], Z + 4 * ((j << d.m_col) | i), 32);
    cm[i] = to_aff(msm(s->pg[0].data(), sc.data(), Rn, false));
  }
  for (size_t i = 0; i < C; i++) g1_out(cm[i], comms + 12 * i);
  multi_pairing(cm.data(), s->ph[d.odd].data(), C).to_canon(T);
  return 0;
}

static void fr_vec_canon(const std::vector<Fr>& v, std::vector<u64>& out) {
  out.resize(4 * v.size());
  for (size_t i = 0; i < v.size(); i++) v[i].to_canon(&out[4 * i]);
}

extern "C++" {
// PST open over powers_of_{g|h}[off + i]
template <class F>
static void pst_open_generic(const std::vector<std::vector<Aff<F>>>& powers, int nv_ck, const std::vector<Fr>& evals,
                             const std::vector<Fr>& point, std::vector<Aff<F>>& proofs) {
  int nv = (int)point.size();
  int off = nv_ck - nv;
  std::vector<Fr> r = evals;
  proofs.assign(nv, Aff<F>{F::zero(), F::zero(), true});
  for (int i = 0; i < nv; i++) {
    size_t half = r.size() / 2;
    std::vector<Fr> q(half), rn(half);
    for (size_t b = 0; b < half; b++) {
      q[b] = r[2 * b + 1] - r[2 * b];
      rn[b] = r[2 * b] * (Fr::one() - point[i]) + r[2 * b + 1] * point[i];
    }
    std::vector<u64> sc(4 * 2 * half);
    for (size_t x = 0; x < 2 * half; x++) q[x >> 1].to_canon(&sc[4 * x]);
    proofs[i] = to_aff(msm(powers[off + i].data(), sc.data(), 2 * half, true));
    r.swap(rn);
  }
}

}  // extern "C++"

// open: outputs U(12), pst_proof (m_row*24), comms_t (m_col*2*72), comms_u (m_col*2*12),
// final_a (12), final_h (24), pst_proof_h (m_col*12)
int orc_pst_open(const orc_srs* s, const u64* Z, int n, const u64* point, const u64* comms, u64* U, u64* pst_proof,
                 u64* comms_t, u64* comms_u, u64* final_a, u64* final_h, u64* pst_proof_h) {
  if (g_ark.empty()) return -2;
  Dims d = dims(n);
  size_t C = size_t(1) << d.m_col;
  std::vector<Fr> pt(n);
  for (int i = 0; i < n; i++) pt[i] = fr_in(point + 4 * i);
  std::vector<Fr> q, chis;
  get_q(Z, d, pt, q, chis);
  std::vector<Aff<Fq>> A(C);
  for (size_t i = 0; i < C; i++) A[i] = g1_in(comms + 12 * i);
  std::vector<u64> chis_c;
  fr_vec_canon(chis, chis_c);
  Aff<Fq> cu = to_aff(msm(A.data(), chis_c.data(), C, true));  // sqrt_pst.rs:198
  g1_out(cu, U);
  // MIPP (mipp.rs:31-153)
  Poseidon tr = make_poseidon(g_ark.data(), g_mds.data());
  tr.append_g1(cu);
  std::vector<Aff<Fq>> ma = A;
  std::vector<Fr> my = chis;
  std::vector<Aff<Fq2>> mh = s->ph[d.odd];
  std::vector<Fr> xs_inv;
  int round = 0;
  while (ma.size() > 1) {
    size_t sp = ma.size() / 2;
    std::vector<u64> yl, yr;
    fr_vec_canon(std::vector<Fr>(my.begin(), my.begin() + sp), yl);
    fr_vec_canon(std::vector<Fr>(my.begin() + sp, my.end()), yr);
    Aff<Fq> ul = to_aff(msm(ma.data(), yr.data(), sp, true));
    Aff<Fq> ur = to_aff(msm(ma.data() + sp, yl.data(), sp, true));
    Fq12 tl = multi_pairing(ma.data(), mh.data() + sp, sp);
    Fq12 trr = multi_pairing(ma.data() + sp, mh.data(), sp);
    tr.append_g1(ul);
    tr.append_g1(ur);
    tr.append_gt(tl);
    tr.append_gt(trr);
    Fr c_inv = tr.challenge();
    Fr c = c_inv.inv();
    std::vector<Aff<Fq>> na(sp);
    std::vector<Aff<Fq2>> nh(sp);
    std::vector<Fr> ny(sp);
#pragma omp parallel for
    for (size_t i = 0; i < sp; i++) {
      na[i] = to_aff(padd_mixed(smul_fr(ma[sp + i], c), ma[i]));
      nh[i] = to_aff(padd_mixed(smul_fr(mh[sp + i], c_inv), mh[i]));
      ny[i] = my[i] + my[sp + i] * c_inv;
    }
    ma.swap(na);
    mh.swap(nh);
    my.swap(ny);
    tl.to_canon(comms_t + 144 * round);
    trr.to_canon(comms_t + 144 * round + 72);
    g1_out(ul, comms_u + 24 * round);
    g1_out(ur, comms_u + 24 * round + 12);
    xs_inv.push_back(c_inv);
    round++;
  }
  g1_out(ma[0], final_a);
  g2_out(mh[0], final_h);
  int m = (int)xs_inv.size();
  std::vector<Fr> poly(size_t(1) << m);
  for (size_t i = 0; i < poly.size(); i++) {  // mipp.rs:159-180
    Fr v = Fr::one();
    for (int j = 0; j < m; j++)
      if ((i >> j) & 1) v = v * xs_inv[m - j - 1];
    poly[i] = v;
  }
  std::vector<Fr> rs(m);
  for (int i = 0; i < m; i++) rs[i] = tr.challenge();
  std::vector<Aff<Fq>> ph;
  pst_open_generic(s->pg, s->nv, poly, rs, ph);  // open_g1
  for (int i = 0; i < m; i++) g1_out(ph[i], pst_proof_h + 12 * i);
  // PST open of q at a_rev (sqrt_pst.rs:218-225)
  std::vector<Fr> a_rev(pt.begin(), pt.begin() + d.m_row);
  std::reverse(a_rev.begin(), a_rev.end());
  std::vector<Aff<Fq2>> pp;
  pst_open_generic(s->ph, s->nv, q, a_rev, pp);
  for (int i = 0; i < d.m_row; i++) g2_out(pp[i], pst_proof + 24 * i);
  return 0;
}

static Fq12 pair1(const Aff<Fq>& p, const Aff<Fq2>& q) { return multi_pairing(&p, &q, 1); }

// Polynomial::verify (sqrt_pst.rs:232-264) + MippProof::verify (mipp.rs:182-320)
int orc_pst_verify(const orc_srs* s, int n, const u64* point, const u64* v_in, const u64* U_in, const u64* pst_proof,
                   const u64* comms_t, const u64* comms_u, const u64* final_a_in, const u64* final_h_in,
                   const u64* pst_proof_h, const u64* T_in) {
  if (g_ark.empty()) return -2;
  Dims d = dims(n);
  std::vector<Fr> pt(n);
  for (int i = 0; i < n; i++) pt[i] = fr_in(point + 4 * i);
  std::vector<Fr> b(pt.begin() + d.m_row, pt.end());
  Aff<Fq> U = g1_in(U_in), final_a = g1_in(final_a_in);
  Aff<Fq2> final_h = g2_in(final_h_in);
  Fq12 T = Fq12::from_canon(T_in);
  Poseidon tr = make_poseidon(g_ark.data(), g_mds.data());
  tr.append_g1(U);
  int m = d.m_col;
  std::vector<Fr> xs, xs_inv;
  Fr final_y = Fr::one();
  Fq12 tc = T;
  Proj<Fq> uc = to_proj(U);
  for (int i = 0; i < m; i++) {
    Aff<Fq> ul = g1_in(comms_u + 24 * i), ur = g1_in(comms_u + 24 * i + 12);
    Fq12 tl = Fq12::from_canon(comms_t + 144 * i), trr = Fq12::from_canon(comms_t + 144 * i + 72);
    tr.append_g1(ul);
    tr.append_g1(ur);
    tr.append_gt(tl);
    tr.append_gt(trr);
    Fr ci = tr.challenge();
    Fr c = ci.inv();
    xs.push_back(c);
    xs_inv.push_back(ci);
    final_y = final_y * (Fr::one() + ci * b[i] - b[i]);
    tc = tc * tl.pow_fr(ci) * trr.pow_fr(c);
    uc = padd(uc, padd(smul_fr(ul, ci), smul_fr(ur, c)));
  }
  std::vector<Fr> rs(m);
  for (int i = 0; i < m; i++) rs[i] = tr.challenge();
  Fr v = Fr::one();
  for (int i = 0; i < m; i++) v = v * (Fr::one() + rs[i] * xs_inv[m - i - 1] - rs[i]);
  // check_2: e(g, C_h - h^v) == prod e(pi_i, h_mask[nv-m+i] - h^{rs_i})
  Aff<Fq2> lh = to_aff(padd_mixed(smul_fr(s->h, v), aneg(final_h)));  // h^v - C_h
  Fq12 left = pair1(s->g, aneg(lh));
  std::vector<Aff<Fq>> pl(m);
  std::vector<Aff<Fq2>> pr(m);
  for (int i = 0; i < m; i++) {
    pl[i] = g1_in(pst_proof_h + 12 * i);
    pr[i] = to_aff(padd_mixed(smul_fr(s->h, rs[i]), aneg(s->hmask[s->nv - m + i])));
    pr[i] = aneg(pr[i]);
  }
  bool ok_h = left == multi_pairing(pl.data(), pr.data(), m);
  Aff<Fq> fu = to_aff(smul_fr(final_a, final_y));
  bool ok_u = (to_aff(uc).inf == fu.inf) && (fu.inf || (to_aff(uc).x == fu.x && to_aff(uc).y == fu.y));
  bool ok_t = tc == pair1(final_a, final_h);
  // MultilinearPC::check: e(U - g^v, h) == prod e(g_mask[i] - g^{a_rev_i}, pi_i)
  Fr vv = fr_in(v_in);
  std::vector<Fr> a_rev(pt.begin(), pt.begin() + d.m_row);
  std::reverse(a_rev.begin(), a_rev.end());
  Aff<Fq> lu = to_aff(padd_mixed(smul_fr(s->g, vv), aneg(U)));
  Fq12 left2 = pair1(aneg(lu), s->h);
  std::vector<Aff<Fq>> ql(d.m_row);
  std::vector<Aff<Fq2>> qr(d.m_row);
  for (int i = 0; i < d.m_row; i++) {
    ql[i] = aneg(to_aff(padd_mixed(smul_fr(s->g, a_rev[i]), aneg(s->gmask[i]))));
    qr[i] = g2_in(pst_proof + 24 * i);
  }
  bool ok_pst = left2 == multi_pairing(ql.data(), qr.data(), d.m_row);
  return (ok_h && ok_u && ok_t && ok_pst) ? 1 : 0;
}

}  // extern "C"

// ----------------------------------------------------------------- R1CS ---
// R1CSProof::prove between the witness commitment and the PST opening
// (r1csproof.rs:248-340): synthetic instance (r1csinstance.rs:166-242 over the
// seeded stream), the transcript from T on, EqPolynomial tables, multiply_vec,
// the phase-one cubic and phase-two quad sum-checks (sumcheck.rs:67-148,
// 387-444), compute_eval_table_sparse; OpenMP over the table loops.  The
// bench's R1CS CPU leg and a checker of csrc/r1cs.hip.
namespace {
std::vector<Fr> eq_table(const std::vector<Fr>& r) {  // dense_mlpoly.rs:231-250
  std::vector<Fr> e(size_t(1) << r.size(), Fr::one());
  size_t size = 1;
  for (size_t j = 0; j < r.size(); j++) {
    size *= 2;
    for (size_t i = size - 1; i >= 1; i -= 2) {
      Fr s = e[i / 2];
      e[i] = s * r[j];
      e[i - 1] = s - e[i];
      if (i == 1) break;
    }
  }
  return e;
}

Fr fr_small(u64 v) {
  u64 l[4] = {v, 0, 0, 0};
  return Fr::from_canon(l);
}

void from_evals(const Fr* e, int n, Fr* cs) {  // unipoly.rs:15-45
  static const Fr i2 = fr_small(2).inv(), i6 = fr_small(6).inv();
  if (n == 3) {
    Fr c = e[0], a = i2 * (e[2] - e[1] - e[1] + c);
    cs[0] = c;
    cs[1] = e[1] - c - a;
    cs[2] = a;
    return;
  }
  Fr d = e[0];
  Fr a = i6 * (e[3] - fr_small(3) * e[2] + fr_small(3) * e[1] - e[0]);
  Fr b = i2 * (e[0] + e[0] - fr_small(5) * e[1] + fr_small(4) * e[2] - e[3]);
  cs[0] = d;
  cs[1] = e[1] - d - a - b;
  cs[2] = b;
  cs[3] = a;
}

Fr uni_eval(const Fr* cs, int n, const Fr& r) {
  Fr out = cs[0], pw = r;
  for (int i = 1; i < n; i++) {
    out = out + pw * cs[i];
    pw = pw * r;
  }
  return out;
}

void append_fr(Poseidon& tr, const Fr& x) {  // append_scalar: one Fq of the same value
  u64 c[4], l[6] = {0, 0, 0, 0, 0, 0};
  x.to_canon(c);
  memcpy(l, c, 32);
  tr.absorb_elems({Fq::from_canon(l)});
}

void reset_fr(Poseidon& tr, const Fr& x) {  // new_from_state2
  tr = make_poseidon(g_ark.data(), g_mds.data());
  u64 c[4];
  x.to_canon(c);
  tr.absorb_bytes((const uint8_t*)c, 32);
}

// K = 4: tau (A B - C); K = 2: A B.  Tables are consumed (bound in place).
template <int K>
void sumcheck(std::vector<Fr>* t, int rounds, Fr e, Poseidon& tr, u64* polys, std::vector<Fr>& rs) {
  const int NC = K == 4 ? 4 : 3;
  for (int j = 0; j < rounds; j++) {
    const size_t n = t[0].size() / 2;
    Fr s0 = Fr::zero(), s2 = Fr::zero(), s3 = Fr::zero();
#pragma omp parallel
    {
      Fr a0 = Fr::zero(), a2 = Fr::zero(), a3 = Fr::zero();
#pragma omp for schedule(static)
      for (long long i = 0; i < (long long)n; i++) {
        Fr lo[K], p[K], q[K];
        for (int k = 0; k < K; k++) {
          lo[k] = t[k][i];
          const Fr d = t[k][n + i] - lo[k];
          p[k] = t[k][n + i] + d;
          q[k] = p[k] + d;
        }
        if (K == 4) {
          a0 = a0 + lo[0] * (lo[1] * lo[2] - lo[3]);
          a2 = a2 + p[0] * (p[1] * p[2] - p[3]);
          a3 = a3 + q[0] * (q[1] * q[2] - q[3]);
        } else {
          a0 = a0 + lo[0] * lo[1];
          a2 = a2 + p[0] * p[1];
        }
      }
#pragma omp critical
      {
        s0 = s0 + a0;
        s2 = s2 + a2;
        s3 = s3 + a3;
      }
    }
    Fr ev[4] = {s0, e - s0, s2, s3}, cs[4];
    from_evals(ev, NC, cs);
    for (int c = 0; c < NC; c++) {
      cs[c].to_canon(polys + 4 * ((size_t)j * NC + c));
      append_fr(tr, cs[c]);
    }
    const Fr r = tr.challenge();
    rs.push_back(r);
    e = uni_eval(cs, NC, r);
    for (int k = 0; k < K; k++) {
#pragma omp parallel for schedule(static)
      for (long long i = 0; i < (long long)n; i++) t[k][i] = t[k][i] + r * (t[k][n + i] - t[k][i]);
      t[k].resize(n);
    }
  }
}
}  // namespace

extern "C" int orc_r1cs_sumchecks(size_t num_cons, size_t num_vars, size_t num_inputs, u64 seed, const u64* T,
                                  u64* sc1, u64* sc2, u64* rx_out, u64* ry_out, u64* claims, u64* sat_state) {
  if (g_ark.empty()) return -2;
  const size_t sz = num_vars + num_inputs + 1;
  std::vector<u64> zc(4 * sz);
  orc_fr_stream(seed, sz, 0, zc.data());
  std::vector<Fr> Z(sz);
  for (size_t i = 0; i < sz; i++) Z[i] = fr_in(&zc[4 * i]);
  Z[num_vars] = Fr::one();
  // C values Z[a] Z[b] / Z[c]: one batch inversion (Montgomery's trick)
  std::vector<Fr> den(num_cons), pre(num_cons);
  Fr acc = Fr::one();
  for (size_t i = 0; i < num_cons; i++) {
    Fr zc3 = Z[(i + 3) % sz];
    den[i] = zc3.is_zero() ? Fr::one() : zc3;
    pre[i] = acc;
    acc = acc * den[i];
  }
  Fr inv = acc.inv();
  std::vector<Fr> cval(num_cons);
  std::vector<size_t> ccol(num_cons);
  for (size_t ii = num_cons; ii-- > 0;) {
    const Fr di = inv * pre[ii];
    inv = inv * den[ii];
    const size_t a = ii % sz, b = (ii + 2) % sz, c = (ii + 3) % sz;
    const Fr ab = Z[a] * Z[b];
    if (Z[c].is_zero()) {
      ccol[ii] = num_vars;
      cval[ii] = ab;
    } else {
      ccol[ii] = c;
      cval[ii] = ab * di;
    }
  }
  // transcript from the witness commitment on (r1csproof.rs:256-283)
  Poseidon tr = make_poseidon(g_ark.data(), g_mds.data());
  tr.absorb_bytes((const uint8_t*)T, 576);
  const Fr init = tr.challenge();
  reset_fr(tr, init);
  for (size_t i = 0; i < num_inputs; i++) append_fr(tr, Z[num_vars + 1 + i]);
  const size_t nz = 2 * num_vars;
  std::vector<Fr> z(nz, Fr::zero());
  for (size_t i = 0; i <= num_vars + num_inputs; i++) z[i] = Z[i];
  int rx_n = 0, ry_n = 0;
  while ((size_t(1) << rx_n) < num_cons) rx_n++;
  while ((size_t(1) << ry_n) < nz) ry_n++;
  std::vector<Fr> tau(rx_n);
  for (int j = 0; j < rx_n; j++) tau[j] = tr.challenge();
  std::vector<Fr> t4[4];
  t4[0] = eq_table(tau);
  for (int k = 1; k < 4; k++) t4[k].resize(num_cons);
#pragma omp parallel for schedule(static)
  for (long long i = 0; i < (long long)num_cons; i++) {
    t4[1][i] = z[i % sz];
    t4[2][i] = z[(i + 2) % sz];
    t4[3][i] = z[ccol[i]] * cval[i];
  }
  std::vector<Fr> rx, ry;
  sumcheck<4>(t4, rx_n, Fr::zero(), tr, sc1, rx);
  const Fr az = t4[1][0], bz = t4[2][0], cz = t4[3][0];
  az.to_canon(claims);
  bz.to_canon(claims + 4);
  cz.to_canon(claims + 8);
  (az * bz).to_canon(claims + 12);
  const Fr rA = tr.challenge(), rB = tr.challenge(), rC = tr.challenge();
  const Fr claim2 = rA * az + rB * bz + rC * cz;
  std::vector<Fr> ex = eq_table(rx);
  std::vector<Fr> t2[2];
  t2[0] = z;
  t2[1].assign(nz, Fr::zero());
  for (size_t i = 0; i < num_cons; i++) {  // compute_eval_table_sparse, combined
    t2[1][i % sz] = t2[1][i % sz] + rA * ex[i];
    t2[1][(i + 2) % sz] = t2[1][(i + 2) % sz] + rB * ex[i];
    t2[1][ccol[i]] = t2[1][ccol[i]] + rC * ex[i] * cval[i];
  }
  sumcheck<2>(t2, ry_n, claim2, tr, sc2, ry);
  for (int j = 0; j < rx_n; j++) rx[j].to_canon(rx_out + 4 * j);
  for (int j = 0; j < ry_n; j++) ry[j].to_canon(ry_out + 4 * j);
  tr.challenge().to_canon(sat_state);
  return 0;
}
