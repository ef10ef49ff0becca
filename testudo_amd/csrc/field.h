// BLS12-377 field tower for CDNA4 (gfx950) and host.
//
//   Fq  : 377-bit prime field, 12 x u32 limbs, Montgomery R = 2^384
//   Fr  : 253-bit scalar field,  8 x u32 limbs, Montgomery R = 2^256
//   Fq2 = Fq[u]/(u^2 + 5), Fq6 = Fq2[v]/(v^3 - u), Fq12 = Fq6[w]/(w^2 - v)
//
// The tower and its non-residues are ark-bls12-377 0.4's;
// the byte layout of an element (12 u32 = 6 u64 little-endian Montgomery
// limbs) is identical to arkworks' in-memory Fp384, so device buffers and
// host buffers are interchangeable.
//
// Multiplication is the "no-carry" CIOS Montgomery product: both moduli have
// a top limb < 2^31 - 1, so the running sum never needs an extra word.  Each
// limb product is one v_mad_u64_u32 on gfx950.  All values are kept fully
// reduced (< modulus), so equality is limb equality.
#pragma once
#include <stdint.h>
#include "bls12_377_params.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TPST_HD __host__ __device__ __forceinline__
#define TPST_NI __host__ __device__ inline __attribute__((noinline))
#else
#define TPST_HD inline
#define TPST_NI inline __attribute__((noinline))
#endif

namespace tpst {

struct FqCfg {
  static constexpr int N = 12;
  static TPST_HD uint32_t p(int i) { return params::FQ_P[i]; }
  static TPST_HD uint32_t one(int i) { return params::FQ_ONE[i]; }
  static TPST_HD uint32_t r2(int i) { return params::FQ_R2[i]; }
  static TPST_HD uint32_t pm2(int i) { return params::FQ_PM2[i]; }
  static TPST_HD uint32_t r3(int i) { return params::FQ_R3[i]; }
  static TPST_HD uint32_t invk(int i) { return params::FQ_INVK[i]; }
  static constexpr int INV_ITERS = params::FQ_INV_ITERS;
  static constexpr uint32_t INV = params::FQ_INV;
  static constexpr bool P0_IS_ONE = true;  // p = 1 mod 2^32 -> m = -t0
};

struct FrCfg {
  static constexpr int N = 8;
  static TPST_HD uint32_t p(int i) { return params::FR_P[i]; }
  static TPST_HD uint32_t one(int i) { return params::FR_ONE[i]; }
  static TPST_HD uint32_t r2(int i) { return params::FR_R2[i]; }
  static TPST_HD uint32_t pm2(int i) { return params::FR_PM2[i]; }
  static TPST_HD uint32_t r3(int i) { return params::FR_R3[i]; }
  static TPST_HD uint32_t invk(int i) { return params::FR_INVK[i]; }
  static constexpr int INV_ITERS = params::FR_INV_ITERS;
  static constexpr uint32_t INV = params::FR_INV;
  static constexpr bool P0_IS_ONE = true;  // r = 1 mod 2^32
};

template <class C>
struct Fp {
  uint32_t v[C::N];
  static TPST_HD Fp zero() {
    Fp r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = 0;
    return r;
  }
  static TPST_HD Fp one() {
    Fp r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = C::one(i);
    return r;
  }
  static TPST_HD Fp from_limbs(const uint32_t* l) {
    Fp r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = l[i];
    return r;
  }
};

using Fq = Fp<FqCfg>;
using Fr = Fp<FrCfg>;

// ------------------------------------------------------------ base field --
template <class C>
TPST_HD bool is_zero(const Fp<C>& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) acc |= a.v[i];
  return acc == 0;
}

template <class C>
TPST_HD bool eq(const Fp<C>& a, const Fp<C>& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

// r = t - p if t >= p else t   (t < 2p)
template <class C>
TPST_HD void reduce_once(Fp<C>& t) {
  uint32_t s[C::N];
  int64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    int64_t d = (int64_t)t.v[i] - C::p(i) + borrow;
    s[i] = (uint32_t)d;
    borrow = d >> 32;  // 0 or -1
  }
  // borrow == 0  <=>  t >= p  -> take s
  const bool take = (borrow == 0);
#pragma unroll
  for (int i = 0; i < C::N; i++) t.v[i] = take ? s[i] : t.v[i];
}

template <class C>
TPST_HD Fp<C> add(const Fp<C>& a, const Fp<C>& b) {
  Fp<C> r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    c += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  reduce_once(r);
  return r;
}

template <class C>
TPST_HD Fp<C> dbl(const Fp<C>& a) { return add(a, a); }

template <class C>
TPST_HD Fp<C> sub(const Fp<C>& a, const Fp<C>& b) {
  Fp<C> r;
  int64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    int64_t d = (int64_t)a.v[i] - b.v[i] + borrow;
    r.v[i] = (uint32_t)d;
    borrow = d >> 32;
  }
  // if negative add p back
  const uint32_t mask = (uint32_t)borrow;  // 0 or 0xffffffff
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    c += (uint64_t)r.v[i] + (C::p(i) & mask);
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}

template <class C>
TPST_HD Fp<C> neg(const Fp<C>& a) { return sub(Fp<C>::zero(), a); }

#if defined(__HIP_DEVICE_COMPILE__)
// acc(64) + hi(32) += a * b, using v_mad_u64_u32's carry-out into an SGPR
// pair and one v_addc: 2 VALU ops per limb product, no zero-extension moves.
__device__ __forceinline__ void mac_vv(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32_e64 %1, %2, 0, %1, %2"
      : "+v"(acc), "+v"(hi), "=&s"(c)
      : "v"(a), "v"(b));
}
__device__ __forceinline__ void mac_vs(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32_e64 %1, %2, 0, %1, %2"
      : "+v"(acc), "+v"(hi), "=&s"(c)
      : "v"(a), "s"(b));
}

#endif  // __HIP_DEVICE_COMPILE__

// Montgomery product a*b*R^-1 mod p.  Device: finely-integrated product
// scanning (column-wise, the reduction word m_k formed as column k
// completes, 2 VALU ops per limb product).  Host: no-carry CIOS.
template <class C>
TPST_HD Fp<C> mul(const Fp<C>& a, const Fp<C>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int N = C::N;
  uint32_t m[N], t[N];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j >= 0 && j < N) mac_vv(acc, hi, a.v[i], b.v[j]);
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N) mac_vs(acc, hi, m[i], C::p(j));
    }
    if (k < N) {
      if constexpr (C::P0_IS_ONE) {
        // p0 = 1: m = -lo, and lo + m*p0 == 0 mod 2^32 with carry-out (lo != 0)
        const uint32_t lo = (uint32_t)acc;
        m[k] = 0u - lo;
        acc = ((acc >> 32) | ((uint64_t)hi << 32)) + (lo != 0u ? 1u : 0u);
        hi = 0;
        continue;
      } else {
        m[k] = (uint32_t)acc * C::INV;
        mac_vs(acc, hi, m[k], C::p(0));
      }
    } else {
      t[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[N - 1] = (uint32_t)acc;
  Fp<C> r;
#pragma unroll
  for (int j = 0; j < N; j++) r.v[j] = t[j];
  reduce_once(r);
  return r;
#else
  constexpr int N = C::N;
  uint32_t t[N];
  for (int j = 0; j < N; j++) t[j] = 0;
  for (int i = 0; i < N; i++) {
    const uint32_t bi = b.v[i];
    uint64_t s = (uint64_t)a.v[0] * bi + t[0];
    uint32_t A = (uint32_t)(s >> 32);
    const uint32_t t0 = (uint32_t)s;
    const uint32_t m = t0 * C::INV;
    uint64_t s2 = (uint64_t)m * C::p(0) + t0;
    uint32_t Cc = (uint32_t)(s2 >> 32);
    for (int j = 1; j < N; j++) {
      s = (uint64_t)a.v[j] * bi + t[j] + A;
      A = (uint32_t)(s >> 32);
      s2 = (uint64_t)m * C::p(j) + (uint32_t)s + Cc;
      Cc = (uint32_t)(s2 >> 32);
      t[j - 1] = (uint32_t)s2;
    }
    t[N - 1] = Cc + A;
  }
  Fp<C> r;
  for (int j = 0; j < N; j++) r.v[j] = t[j];
  reduce_once(r);
  return r;
#endif
}

// Montgomery square: the same product scanning as mul, with each column's
// cross products a_i a_j (i < j) taken once in a side accumulator that is
// doubled before joining the column, plus the diagonal a_i^2 -- N (N + 1) / 2
// limb products instead of N^2 before the reduction (78 of 144 for Fq).
template <class C>
TPST_HD Fp<C> sqr(const Fp<C>& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int N = C::N;
  uint32_t m[N], t[N];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t cacc = 0;
    uint32_t chi = 0;
    bool any = false;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < j && j < N) {
        mac_vv(cacc, chi, a.v[i], a.v[j]);
        any = true;
      }
    }
    if (any) {  // column += 2 * cross (a compile-time branch: loops are unrolled)
      chi = (chi << 1) | (uint32_t)(cacc >> 63);
      cacc <<= 1;
      const uint64_t s2 = acc + cacc;
      hi += chi + (s2 < acc ? 1u : 0u);
      acc = s2;
    }
    if ((k & 1) == 0 && (k >> 1) < N) mac_vv(acc, hi, a.v[k >> 1], a.v[k >> 1]);
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N) mac_vs(acc, hi, m[i], C::p(j));
    }
    if (k < N) {
      if constexpr (C::P0_IS_ONE) {
        const uint32_t lo = (uint32_t)acc;
        m[k] = 0u - lo;
        acc = ((acc >> 32) | ((uint64_t)hi << 32)) + (lo != 0u ? 1u : 0u);
        hi = 0;
        continue;
      } else {
        m[k] = (uint32_t)acc * C::INV;
        mac_vs(acc, hi, m[k], C::p(0));
      }
    } else {
      t[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[N - 1] = (uint32_t)acc;
  Fp<C> r;
#pragma unroll
  for (int j = 0; j < N; j++) r.v[j] = t[j];
  reduce_once(r);
  return r;
#else
  return mul(a, a);
#endif
}

template <class C>
TPST_HD Fp<C> to_mont(const Fp<C>& a) {  // canonical -> Montgomery
  Fp<C> r2;
#pragma unroll
  for (int i = 0; i < C::N; i++) r2.v[i] = C::r2(i);
  return mul(a, r2);
}

template <class C>
TPST_HD Fp<C> from_mont(const Fp<C>& a) {  // Montgomery -> canonical
  Fp<C> one = Fp<C>::zero();
  one.v[0] = 1;
  return mul(a, one);
}

// ---------------------------------------------------------------- inverse --
// Constant-flow modular inverse: Pornin's optimised binary GCD (eprint
// 2020/972, Alg. 2, k = 32).  Each outer iteration runs 31 divsteps on 64-bit
// approximations of (a, b) (low 31 bits + top 33 bits), then applies the
// accumulated 2x2 matrix to the full-width a, b and to the Bezout
// coefficients u, v (mod m).  No data-dependent branches: every lane of a wave
// follows the same path (the previous binary GCD diverged and cost ~1 ms per
// wave of 64 different inputs).  Result v 2^-t is fixed up, together with
// the Montgomery factors, by one product with K = 2^-t R^3.  a == 0 -> 0.
//
// x*|fx| +/- y*|fy| for signed fx, fy (|f| <= 2^31): magnitude in r[N+2], returns sign
template <int N>
TPST_HD bool lincomb(const uint32_t* x, int64_t fx, const uint32_t* y, int64_t fy, uint32_t* r) {
  const bool sx = fx < 0, sy = fy < 0;
  const uint32_t mx = (uint32_t)(sx ? -fx : fx), my = (uint32_t)(sy ? -fy : fy);
  uint32_t p1[N + 1], p2[N + 1];
  uint64_t c1 = 0, c2 = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    c1 += (uint64_t)x[i] * mx;
    p1[i] = (uint32_t)c1;
    c1 >>= 32;
    c2 += (uint64_t)y[i] * my;
    p2[i] = (uint32_t)c2;
    c2 >>= 32;
  }
  p1[N] = (uint32_t)c1;
  p2[N] = (uint32_t)c2;
  // sum and difference, then select
  uint32_t sm[N + 2], df[N + 1];
  uint64_t cs = 0;
  int64_t bd = 0;
#pragma unroll
  for (int i = 0; i <= N; i++) {
    cs += (uint64_t)p1[i] + p2[i];
    sm[i] = (uint32_t)cs;
    cs >>= 32;
    const int64_t d = (int64_t)p1[i] - p2[i] + bd;
    df[i] = (uint32_t)d;
    bd = d >> 32;
  }
  sm[N + 1] = (uint32_t)cs;
  const bool borrow = bd != 0;
  // negate df if it went negative
  const uint32_t nm = borrow ? 0xffffffffu : 0u;
  uint64_t cn = borrow ? 1u : 0u;
#pragma unroll
  for (int i = 0; i <= N; i++) {
    cn += (uint64_t)(df[i] ^ nm);
    df[i] = (uint32_t)cn;
    cn >>= 32;
  }
  const bool same = sx == sy;
#pragma unroll
  for (int i = 0; i <= N; i++) r[i] = same ? sm[i] : df[i];
  r[N + 1] = same ? sm[N + 1] : 0u;
  return same ? sx : (borrow ? sy : sx);
}

template <class C>
TPST_HD void inv_matrix_mod(const uint32_t* u, int64_t fu, const uint32_t* v, int64_t fv, uint32_t* out) {
  constexpr int N = C::N;
  uint32_t m[N + 2];
  const bool neg = lincomb<N>(u, fu, v, fv, m);
  // m < 2^33 p: quotient estimate from the top 4 limbs (error <= 1 either way)
  double top = 0.0, pd = 0.0;
#pragma unroll
  for (int i = N + 1; i >= N - 2; i--) top = top * 4294967296.0 + (double)m[i];
#pragma unroll
  for (int i = N - 1; i >= N - 2; i--) pd = pd * 4294967296.0 + (double)C::p(i);
  double qd = top / pd;  // units: 2^(32 (N-2)) / 2^(32 (N-2))
  if (qd < 0.0) qd = 0.0;
  const uint64_t q = (uint64_t)qd;
  const uint32_t ql = (uint32_t)q, qh = (uint32_t)(q >> 32);
  // r = m - q p  (signed, N+2 limbs)
  int64_t br = 0;
  uint64_t cl = 0, ch = 0;
  uint32_t r[N + 2];
#pragma unroll
  for (int i = 0; i < N + 2; i++) {
    const uint32_t pi = i < N ? C::p(i) : 0u;
    const uint32_t pim1 = (i >= 1 && i - 1 < N) ? C::p(i - 1) : 0u;
    cl += (uint64_t)ql * pi;
    ch += (uint64_t)qh * pim1;
    const uint32_t sub_l = (uint32_t)cl, sub_h = (uint32_t)ch;
    cl >>= 32;
    ch >>= 32;
    const int64_t d = (int64_t)m[i] - sub_l - sub_h + br;
    r[i] = (uint32_t)d;
    br = d >> 32;
  }
  // r in (-p, 2p): fix with one conditional add and one conditional subtract
  const bool negr = (int32_t)r[N + 1] < 0;
  {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      c += (uint64_t)r[i] + (negr ? C::p(i) : 0u);
      r[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  Fp<C> rr;
#pragma unroll
  for (int i = 0; i < N; i++) rr.v[i] = r[i];
  reduce_once(rr);
  // negative combination: p - r (r != 0)
  const bool nz = !is_zero(rr);
  Fp<C> nr = sub(Fp<C>::zero(), rr);
#pragma unroll
  for (int i = 0; i < N; i++) out[i] = (neg && nz) ? nr.v[i] : rr.v[i];
}

template <class C>
TPST_HD bool limbs_is_one(const uint32_t* a) {
  uint32_t acc = a[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < C::N; i++) acc |= a[i];
  return acc == 0;
}

// bits [s, s + 33) of x (s >= 0)
template <class C>
TPST_HD uint64_t bits33(const uint32_t* x, int s) {
  uint64_t w = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    const int sh = 32 * i - s;
    const uint64_t xi = x[i];
    if (sh >= 0 && sh < 64) w |= xi << sh;
    if (sh < 0 && sh > -32) w |= xi >> (-sh);
  }
  return w & ((1ull << 33) - 1);
}

template <class C>
TPST_NI Fp<C> inv(const Fp<C>& y) {
  constexpr int N = C::N;
  uint32_t a[N], b[N], u[N], v[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    a[i] = y.v[i];
    b[i] = C::p(i);
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0;
  }
  for (int it = 0; it < C::INV_ITERS; it++) {
    // n = max(bitlen(a | b), 64); approximations from bits [n - 33, n) and [0, 31)
    int nb = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const uint32_t x = a[i] | b[i];
#if defined(__HIP_DEVICE_COMPILE__)
      const int bl = x ? 32 - __clz((int)x) : 0;
#else
      const int bl = x ? 32 - __builtin_clz(x) : 0;
#endif
      nb = x ? 32 * i + bl : nb;
    }
    const int n = nb > 64 ? nb : 64;
    uint64_t ab = (uint64_t)(a[0] & 0x7fffffffu) | (bits33<C>(a, n - 33) << 31);
    uint64_t bb = (uint64_t)(b[0] & 0x7fffffffu) | (bits33<C>(b, n - 33) << 31);
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 1
    for (int j = 0; j < 31; j++) {
      const uint64_t odd = 0ull - (ab & 1u);
      const uint64_t sw = odd & (0ull - (uint64_t)(ab < bb));
      const uint64_t t = (ab ^ bb) & sw;
      ab ^= t;
      bb ^= t;
      const int64_t tf = (f0 ^ f1) & (int64_t)sw, tg = (g0 ^ g1) & (int64_t)sw;
      f0 ^= tf;
      f1 ^= tf;
      g0 ^= tg;
      g1 ^= tg;
      ab -= bb & odd;
      f0 -= f1 & (int64_t)odd;
      g0 -= g1 & (int64_t)odd;
      ab >>= 1;
      f1 += f1;
      g1 += g1;
    }
    // (a, b) <- ((f0 a + g0 b), (f1 a + g1 b)) / 2^31, signs folded into the matrix
    uint32_t na[N + 2], nbv[N + 2];
    const bool sa = lincomb<N>(a, f0, b, g0, na);
    const bool sb = lincomb<N>(a, f1, b, g1, nbv);
#pragma unroll
    for (int i = 0; i < N; i++) {
      a[i] = (na[i] >> 31) | (na[i + 1] << 1);
      b[i] = (nbv[i] >> 31) | (nbv[i + 1] << 1);
    }
    if (sa) {
      f0 = -f0;
      g0 = -g0;
    }
    if (sb) {
      f1 = -f1;
      g1 = -g1;
    }
    uint32_t nu[N], nv[N];
    inv_matrix_mod<C>(u, f0, v, g0, nu);
    inv_matrix_mod<C>(u, f1, v, g1, nv);
#pragma unroll
    for (int i = 0; i < N; i++) {
      u[i] = nu[i];
      v[i] = nv[i];
    }
  }
  // b == gcd == 1 for invertible inputs
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = v[i];
  Fp<C> k;
#pragma unroll
  for (int i = 0; i < N; i++) k.v[i] = C::invk(i);
  r = mul(r, k);
  return limbs_is_one<C>(b) ? r : Fp<C>::zero();
}

// Fq's inverse: the radix-2^29 binary GCD of field29.h, ~3x fewer
// instructions than the 32-bit-limb template above, which Fr keeps.
// field29.h needs only the base field above and is included here; the
// declaration covers a translation unit that includes field29.h first.
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wattributes"
TPST_NI Fq inv(const Fq& a);
#pragma GCC diagnostic pop

}  // namespace tpst

#include "field29.h"

namespace tpst {

// small constant multiples
template <class C>
TPST_HD Fp<C> mul3(const Fp<C>& a) { return add(dbl(a), a); }

// ------------------------------------------------------------------ Fq2 ---
// Translation units whose G2 code is not on a hot path (msm_g2.hip: the
// verifier's and the C-ABI's variable-base G2 MSMs) define TPST_FQ2_ATTR as
// TPST_NI before including this header: one out-of-line Fq2 product instead of
// three inlined Montgomery products per call site keeps their build in seconds.
#ifndef TPST_FQ2_ATTR
#define TPST_FQ2_ATTR TPST_HD
#endif
struct Fq2 {
  Fq c0, c1;
  static TPST_HD Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
  static TPST_HD Fq2 one() { return {Fq::one(), Fq::zero()}; }
};

TPST_HD bool is_zero(const Fq2& a) { return is_zero(a.c0) && is_zero(a.c1); }
TPST_HD bool eq(const Fq2& a, const Fq2& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
TPST_HD Fq2 add(const Fq2& a, const Fq2& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
TPST_HD Fq2 sub(const Fq2& a, const Fq2& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
TPST_HD Fq2 dbl(const Fq2& a) { return {dbl(a.c0), dbl(a.c1)}; }
TPST_HD Fq2 neg(const Fq2& a) { return {neg(a.c0), neg(a.c1)}; }
TPST_HD Fq2 mul3(const Fq2& a) { return {mul3(a.c0), mul3(a.c1)}; }
TPST_HD Fq mul5(const Fq& a) { return add(dbl(dbl(a)), a); }
TPST_HD Fq2 conj(const Fq2& a) { return {a.c0, neg(a.c1)}; }

TPST_FQ2_ATTR Fq2 mul(const Fq2& a, const Fq2& b) {
  const Fq v0 = mul(a.c0, b.c0);
  const Fq v1 = mul(a.c1, b.c1);
  const Fq s = mul(add(a.c0, a.c1), add(b.c0, b.c1));
  return {sub(v0, mul5(v1)), sub(sub(s, v0), v1)};
}

TPST_FQ2_ATTR Fq2 sqr(const Fq2& a) {
  // (a0 + a1 u)^2 = a0^2 - 5 a1^2 + 2 a0 a1 u
  const Fq v0 = mul(a.c0, a.c1);
  // (a0 + a1)(a0 - 5 a1) = a0^2 - 5a1^2 - 4 a0 a1
  const Fq t = mul(add(a.c0, a.c1), sub(a.c0, mul5(a.c1)));
  const Fq c0 = add(t, dbl(dbl(v0)));
  return {c0, dbl(v0)};
}

TPST_HD Fq2 mul_fq(const Fq2& a, const Fq& s) { return {mul(a.c0, s), mul(a.c1, s)}; }

TPST_NI Fq2 inv(const Fq2& a) {
  const Fq n = add(sqr(a.c0), mul5(sqr(a.c1)));
  const Fq ni = inv(n);
  return {mul(a.c0, ni), neg(mul(a.c1, ni))};
}

// times the Fq6 non-residue u:  (x0 + x1 u) u = -5 x1 + x0 u
TPST_HD Fq2 mul_by_u(const Fq2& a) { return {neg(mul5(a.c1)), a.c0}; }

TPST_HD Fq2 fq2_const(const uint32_t (*c)[12]) {
  return {Fq::from_limbs(c[0]), Fq::from_limbs(c[1])};
}

// ------------------------------------------------------------------ Fq6 ---
struct Fq6 {
  Fq2 c0, c1, c2;
  static TPST_HD Fq6 zero() { return {Fq2::zero(), Fq2::zero(), Fq2::zero()}; }
  static TPST_HD Fq6 one() { return {Fq2::one(), Fq2::zero(), Fq2::zero()}; }
};

TPST_HD Fq6 add(const Fq6& a, const Fq6& b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
TPST_HD Fq6 sub(const Fq6& a, const Fq6& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1), sub(a.c2, b.c2)}; }
TPST_HD Fq6 neg(const Fq6& a) { return {neg(a.c0), neg(a.c1), neg(a.c2)}; }
TPST_HD Fq6 dbl(const Fq6& a) { return {dbl(a.c0), dbl(a.c1), dbl(a.c2)}; }
TPST_HD bool eq(const Fq6& a, const Fq6& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1) && eq(a.c2, b.c2); }
TPST_HD bool is_zero(const Fq6& a) { return is_zero(a.c0) && is_zero(a.c1) && is_zero(a.c2); }

TPST_NI Fq6 mul(const Fq6& a, const Fq6& b) {
  const Fq2 v0 = mul(a.c0, b.c0);
  const Fq2 v1 = mul(a.c1, b.c1);
  const Fq2 v2 = mul(a.c2, b.c2);
  const Fq2 c0 = add(mul_by_u(sub(sub(mul(add(a.c1, a.c2), add(b.c1, b.c2)), v1), v2)), v0);
  const Fq2 c1 = add(sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), v0), v1), mul_by_u(v2));
  const Fq2 c2 = add(sub(sub(mul(add(a.c0, a.c2), add(b.c0, b.c2)), v0), v2), v1);
  return {c0, c1, c2};
}

TPST_HD Fq6 sqr(const Fq6& a) { return mul(a, a); }

// times the Fq12 non-residue v: (x0 + x1 v + x2 v^2) v = u x2 + x0 v + x1 v^2
TPST_HD Fq6 mul_by_v(const Fq6& a) { return {mul_by_u(a.c2), a.c0, a.c1}; }

// (a0 + a1 v + a2 v^2)(b0 + b1 v)      ark Fp6::mul_by_01
TPST_NI Fq6 mul_by_01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
  const Fq2 v0 = mul(a.c0, b0);
  const Fq2 v1 = mul(a.c1, b1);
  const Fq2 t1 = add(mul_by_u(sub(mul(add(a.c1, a.c2), b1), v1)), v0);
  const Fq2 t3 = add(sub(mul(add(a.c0, a.c2), b0), v0), v1);
  const Fq2 t2 = sub(sub(mul(add(b0, b1), add(a.c0, a.c1)), v0), v1);
  return {t1, t2, t3};
}

TPST_NI Fq6 inv(const Fq6& a) {
  // standard: c0 = a0^2 - u a1 a2, c1 = u a2^2 - a0 a1, c2 = a1^2 - a0 a2
  const Fq2 c0 = sub(sqr(a.c0), mul_by_u(mul(a.c1, a.c2)));
  const Fq2 c1 = sub(mul_by_u(sqr(a.c2)), mul(a.c0, a.c1));
  const Fq2 c2 = sub(sqr(a.c1), mul(a.c0, a.c2));
  const Fq2 t = add(mul(a.c0, c0), mul_by_u(add(mul(a.c2, c1), mul(a.c1, c2))));
  const Fq2 ti = inv(t);
  return {mul(c0, ti), mul(c1, ti), mul(c2, ti)};
}

// ----------------------------------------------------------------- Fq12 ---
struct Fq12 {
  Fq6 c0, c1;
  static TPST_HD Fq12 one() { return {Fq6::one(), Fq6::zero()}; }
};

TPST_HD bool eq(const Fq12& a, const Fq12& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }

TPST_NI Fq12 mul(const Fq12& a, const Fq12& b) {
  const Fq6 v0 = mul(a.c0, b.c0);
  const Fq6 v1 = mul(a.c1, b.c1);
  const Fq6 c1 = sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), v0), v1);
  return {add(v0, mul_by_v(v1)), c1};
}

TPST_NI Fq12 sqr(const Fq12& a) {
  // complex squaring
  const Fq6 ab = mul(a.c0, a.c1);
  const Fq6 t = mul(add(a.c0, a.c1), add(a.c0, mul_by_v(a.c1)));
  const Fq6 c0 = sub(sub(t, ab), mul_by_v(ab));
  return {c0, dbl(ab)};
}

TPST_HD Fq12 conj(const Fq12& a) { return {a.c0, neg(a.c1)}; }

TPST_NI Fq12 inv(const Fq12& a) {
  const Fq6 t = sub(sqr(a.c0), mul_by_v(sqr(a.c1)));
  const Fq6 ti = inv(t);
  return {mul(a.c0, ti), neg(mul(a.c1, ti))};
}

// f *= (c0 + c3 w + c4 v w)                 ark Fp12::mul_by_034
TPST_NI Fq12 mul_by_034(const Fq12& f, const Fq2& c0, const Fq2& c3, const Fq2& c4) {
  const Fq6 a = {mul(f.c0.c0, c0), mul(f.c0.c1, c0), mul(f.c0.c2, c0)};
  const Fq6 b = mul_by_01(f.c1, c3, c4);
  const Fq6 e = mul_by_01(add(f.c0, f.c1), add(c0, c3), c4);
  return {add(a, mul_by_v(b)), sub(e, add(a, b))};
}

TPST_HD Fq2 frob2(const Fq2& a, int k) { return (k & 1) ? conj(a) : a; }

// Frobenius x -> x^(p^k), k in {1,2,3}
TPST_NI Fq12 frobenius(const Fq12& a, int k) {
  Fq2 c61, c62, c12;
  if (k == 1) {
    c61 = fq2_const(params::FROB6_C1_1); c62 = fq2_const(params::FROB6_C2_1); c12 = fq2_const(params::FROB12_C1_1);
  } else if (k == 2) {
    c61 = fq2_const(params::FROB6_C1_2); c62 = fq2_const(params::FROB6_C2_2); c12 = fq2_const(params::FROB12_C1_2);
  } else {
    c61 = fq2_const(params::FROB6_C1_3); c62 = fq2_const(params::FROB6_C2_3); c12 = fq2_const(params::FROB12_C1_3);
  }
  Fq6 x0 = {frob2(a.c0.c0, k), mul(frob2(a.c0.c1, k), c61), mul(frob2(a.c0.c2, k), c62)};
  Fq6 x1 = {frob2(a.c1.c0, k), mul(frob2(a.c1.c1, k), c61), mul(frob2(a.c1.c2, k), c62)};
  x1 = {mul(x1.c0, c12), mul(x1.c1, c12), mul(x1.c2, c12)};
  return {x0, x1};
}

}  // namespace tpst

