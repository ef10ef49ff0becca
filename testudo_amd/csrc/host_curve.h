// Host-side (x86-64) BLS12-377 G1 / G2 arithmetic on 64-bit limbs, for the
// verifier's short serial chains: subgroup checks ([r] P == O) and the
// two-term combinations of MultilinearPC::check / check_2.  A lone GPU lane
// runs such a chain at ~1.6 us per Fq product (a wave instruction per limb
// operation); here a product is one 6 x 6-word CIOS pass (~0.1 us), and the
// independent chains of one verification run on host threads.
//
// HFq holds exactly the bits of Fq (6 x u64 = 12 x u32 little-endian limbs,
// Montgomery R = 2^384), so values convert by memcpy.  The curve formulas are
// curve.h's templates (Xyzz / Affine / scalar_mul), instantiated on HFq and
// HFq2 through argument-dependent lookup of the functions below.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "curve.h"
#include "field29.h"

namespace tpst {
namespace host {

typedef unsigned __int128 u128;

struct HFq {
  uint64_t v[6];
  static HFq from(const Fq& a) {
    HFq r;
    memcpy(r.v, a.v, 48);
    return r;
  }
  Fq to() const {
    Fq r;
    memcpy(r.v, v, 48);
    return r;
  }
  static HFq zero() { return HFq{{0, 0, 0, 0, 0, 0}}; }
  static HFq one() { return from(Fq::one()); }
};

struct Mod64 {
  uint64_t p[6];
  uint64_t inv;  // -p^-1 mod 2^64
  Mod64() {
    for (int i = 0; i < 6; i++) p[i] = (uint64_t)params::FQ_P[2 * i] | ((uint64_t)params::FQ_P[2 * i + 1] << 32);
    uint64_t x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - p[0] * x;  // Newton: x = p^-1 mod 2^64
    inv = 0 - x;
  }
};
inline const Mod64& mod64() {
  static const Mod64 m;
  return m;
}

// t (6 words + carry word) - p if t >= p
inline HFq cond_sub(const uint64_t* t, uint64_t hi) {
  const Mod64& P = mod64();
  uint64_t r[6];
  u128 br = 0;
  for (int j = 0; j < 6; j++) {
    const u128 d = (u128)t[j] - P.p[j] - (uint64_t)br;
    r[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  HFq out;
  memcpy(out.v, (hi || !br) ? r : t, 48);
  return out;
}

inline HFq add(const HFq& a, const HFq& b) {
  uint64_t t[6];
  u128 c = 0;
  for (int j = 0; j < 6; j++) {
    c += (u128)a.v[j] + b.v[j];
    t[j] = (uint64_t)c;
    c >>= 64;
  }
  return cond_sub(t, (uint64_t)c);
}

inline HFq sub(const HFq& a, const HFq& b) {
  const Mod64& P = mod64();
  uint64_t t[6];
  u128 br = 0;
  for (int j = 0; j < 6; j++) {
    const u128 d = (u128)a.v[j] - b.v[j] - (uint64_t)br;
    t[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  if (br) {  // add p back
    u128 c = 0;
    for (int j = 0; j < 6; j++) {
      c += (u128)t[j] + P.p[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
  }
  HFq r;
  memcpy(r.v, t, 48);
  return r;
}

inline HFq neg(const HFq& a) { return sub(HFq::zero(), a); }
inline HFq dbl(const HFq& a) { return add(a, a); }
inline HFq mul3(const HFq& a) { return add(dbl(a), a); }

inline bool is_zero(const HFq& a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3] | a.v[4] | a.v[5]); }
inline bool eq(const HFq& a, const HFq& b) { return !memcmp(a.v, b.v, 48); }

// CIOS Montgomery product, 64-bit words
inline HFq mul(const HFq& a, const HFq& b) {
  const Mod64& P = mod64();
  uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; i++) {
    u128 c = 0;
    for (int j = 0; j < 6; j++) {
      c += (u128)a.v[j] * b.v[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[6] = (uint64_t)c;
    t[7] = (uint64_t)(c >> 64);
    const uint64_t m = t[0] * P.inv;
    c = ((u128)m * P.p[0] + t[0]) >> 64;
    for (int j = 1; j < 6; j++) {
      c += (u128)m * P.p[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[5] = (uint64_t)c;
    t[6] = t[7] + (uint64_t)(c >> 64);
  }
  return cond_sub(t, t[6]);
}

inline HFq sqr(const HFq& a) { return mul(a, a); }

// a^-1 (0 -> 0): field29.h's binary GCD (batches of 29 divsteps on 13-limb
// values) runs ~6x faster here than the Fermat power by host products
inline HFq inv(const HFq& a) { return HFq::from(tpst::inv(a.to())); }

// Fq2 = Fq[u] / (u^2 + 5)
struct HFq2 {
  HFq c0, c1;
  static HFq2 zero() { return {HFq::zero(), HFq::zero()}; }
  static HFq2 one() { return {HFq::one(), HFq::zero()}; }
  static HFq2 from(const Fq2& a) { return {HFq::from(a.c0), HFq::from(a.c1)}; }
  Fq2 to() const { return {c0.to(), c1.to()}; }
};

inline HFq mul5(const HFq& a) { return add(dbl(dbl(a)), a); }
inline HFq2 add(const HFq2& a, const HFq2& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
inline HFq2 sub(const HFq2& a, const HFq2& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
inline HFq2 neg(const HFq2& a) { return {neg(a.c0), neg(a.c1)}; }
inline HFq2 dbl(const HFq2& a) { return {dbl(a.c0), dbl(a.c1)}; }
inline HFq2 mul3(const HFq2& a) { return {mul3(a.c0), mul3(a.c1)}; }
inline bool is_zero(const HFq2& a) { return is_zero(a.c0) && is_zero(a.c1); }
inline bool eq(const HFq2& a, const HFq2& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
inline HFq2 mul(const HFq2& a, const HFq2& b) {  // Karatsuba, u^2 = -5
  const HFq t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
  const HFq s = mul(add(a.c0, a.c1), add(b.c0, b.c1));
  return {sub(t0, mul5(t1)), sub(sub(s, t0), t1)};
}
inline HFq2 sqr(const HFq2& a) { return mul(a, a); }
inline HFq2 inv(const HFq2& a) {  // conj / norm, norm = c0^2 + 5 c1^2
  const HFq ni = inv(add(sqr(a.c0), mul5(sqr(a.c1))));
  return {mul(a.c0, ni), neg(mul(a.c1, ni))};
}

// canonical u64 coordinates <-> host Montgomery affine points
inline HFq fq_in(const uint64_t* c) {
  Fq a;
  memcpy(a.v, c, 48);
  return HFq::from(to_mont(a));
}
inline void fq_put(const HFq& a, uint64_t* c) {
  const Fq r = from_mont(a.to());
  memcpy(c, r.v, 48);
}

template <class F>
struct HostOf;
template <>
struct HostOf<Fq> {
  using T = HFq;
  static constexpr int NQ = 1;
};
template <>
struct HostOf<Fq2> {
  using T = HFq2;
  static constexpr int NQ = 2;
};

// affine point from canonical limbs (x || y, all-zero = infinity)
template <class H>
inline Affine<H> aff_in(const uint64_t* p);
template <>
inline Affine<HFq> aff_in<HFq>(const uint64_t* p) {
  return {fq_in(p), fq_in(p + 6)};
}
template <>
inline Affine<HFq2> aff_in<HFq2>(const uint64_t* p) {
  return {{fq_in(p), fq_in(p + 6)}, {fq_in(p + 12), fq_in(p + 18)}};
}
inline void aff_put(const Affine<HFq>& a, uint64_t* o) {
  fq_put(a.x, o);
  fq_put(a.y, o + 6);
}
inline void aff_put(const Affine<HFq2>& a, uint64_t* o) {
  fq_put(a.x.c0, o);
  fq_put(a.x.c1, o + 6);
  fq_put(a.y.c0, o + 12);
  fq_put(a.y.c1, o + 18);
}

// independent tasks on up to `threads` host threads (OMP_NUM_THREADS or the
// hardware count, capped at 16: the GPU box gives a job a 16-core share)
inline unsigned pool_threads() {
  static const unsigned n = [] {
    unsigned t = std::thread::hardware_concurrency();
    const char* e = getenv("OMP_NUM_THREADS");
    if (e && atoi(e) > 0) t = (unsigned)atoi(e);
    return std::max(1u, std::min(t ? t : 1u, 16u));
  }();
  return n;
}

template <class Fn>
void parallel_for(size_t n, Fn&& fn) {
  const unsigned T = (unsigned)std::min<size_t>(n, pool_threads());
  if (T <= 1) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<size_t> next(0);
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
  };
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (unsigned t = 1; t < T; t++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

}  // namespace host

template <>
struct CurveB<host::HFq> {
  static host::HFq b() { return host::HFq::one(); }
};
template <>
struct CurveB<host::HFq2> {
  static host::HFq2 b() { return host::HFq2::from(fq2_const(params::G2_B)); }
};

namespace host {

// canonical coordinates < p, on the curve, [r] P == O
template <class F>
bool point_in_subgroup(const uint64_t* p) {
  using H = typename HostOf<F>::T;
  constexpr int NQ = HostOf<F>::NQ;
  const Mod64& M = mod64();
  bool all0 = true;
  for (int k = 0; k < 2 * NQ; k++) {
    const uint64_t* c = p + 6 * k;
    for (int i = 0; i < 6; i++) all0 = all0 && !c[i];
    for (int i = 5; i >= 0; i--) {
      if (c[i] != M.p[i]) {
        if (c[i] > M.p[i]) return false;
        break;
      }
      if (i == 0) return false;  // == p
    }
  }
  if (all0) return true;  // infinity
  const Affine<H> a = aff_in<H>(p);
  if (!eq(sqr(a.y), add(mul(sqr(a.x), a.x), CurveB<H>::b()))) return false;
  return is_inf(scalar_mul(a, params::FR_P, 253));
}

// a P + sign Q (canonical affine in and out; a canonical Fr; sign = +1 / -1):
// the check / check_2 terms C - g^v and g^{t_i} - g_mask_i need one scalar
// multiplication each
template <class F>
void mul_add(const uint64_t* P, const uint64_t* a, const uint64_t* Q, int sign, uint64_t* out) {
  using H = typename HostOf<F>::T;
  Xyzz<H> r = scalar_mul(aff_in<H>(P), reinterpret_cast<const uint32_t*>(a), 253);
  Affine<H> q = aff_in<H>(Q);
  if (sign < 0) q = neg(q);
  r = add_affine(r, q);
  aff_put(to_affine(r), out);
}

}  // namespace host
}  // namespace tpst
