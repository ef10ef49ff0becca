// Reduced-radix Fq for the throughput kernels (MSM bucket accumulation):
// 13 limbs of 29 bits (377 bits), Montgomery R = 2^377, values canonical
// (< p) in every limb representation handed between functions.
//
// Why: field.h's Fq product spends one v_mad_u64_u32 AND one v_addc per limb
// product (a 32 x 32-bit product into a 64-bit column needs the carry-out),
// 276 of each for 12 x 32-bit limbs.  With 29-bit limbs a limb product is
// < 2^58 and a column of up to 26 of them stays below 2^63, so each limb
// product is a single v_mad_u64_u32 into a 64-bit accumulator and the carry
// moves once per column: 169 + 156 multiply-adds (p_0 = 1: the reduction
// word of a column is m = -t mod 2^29 and m * p_0 is an add), no v_addc.
// Chip issue, measured (profiles/r02/s11/mb_wave.log): v_mad_u64_u32 takes
// two issue slots of a v_add_u32, so the product drops from ~993 to ~790
// slots.
//
// Conversions: field.h keeps arkworks' layout (12 x u32, R = 2^384).
//   from_std: V = x 2^384 -> x 2^377 = (V + k p) / 2^7, k = -V mod 2^7
//             (p = 1 mod 2^46), then the bits regrouped -- no product;
//   to_std:   Y = x 2^377 -> Montgomery product by 2^384 mod p (one product;
//             used only where a bucket or piece leaves the kernel).
#pragma once
#include "field.h"

namespace tpst {

namespace r29 {
constexpr int N = 13;
constexpr uint32_t M = (1u << 29) - 1;
// p in radix 2^29 (p_0 = 1)
static constexpr uint32_t P[N] = {0x00000001u, 0x08460000u, 0x00000021u, 0x16ba8860u, 0x14800170u,
                                  0x1117dd04u, 0x0e3c7bcdu, 0x1e601ea2u, 0x1b1a22d9u, 0x03650a49u,
                                  0x118ec170u, 0x0f8a21d5u, 0x1ae3a461u};
// 2^377 mod p (Montgomery one)
static constexpr uint32_t ONE[N] = {0x1fffffffu, 0x17b9ffffu, 0x1fffffdeu, 0x0945779fu, 0x0b7ffe8fu,
                                    0x0ee822fbu, 0x11c38432u, 0x019fe15du, 0x04e5dd26u, 0x1c9af5b6u,
                                    0x0e713e8fu, 0x1075de2au, 0x051c5b9eu};
// 2^384 mod p in radix 2^29, plain (the to_std multiplier: Y * C / 2^377 = Y 2^7)
static constexpr uint32_t TO_STD[N] = {0x1fffff68u, 0x166fffffu, 0x1fffec40u, 0x013f06ffu, 0x13ff2514u,
                                       0x19d4c53eu, 0x0c167df6u, 0x16edcf8cu, 0x087b4e97u, 0x1c01e427u,
                                       0x133d256fu, 0x05fbe934u, 0x08d6661eu};
// (2^377)^3 mod p (the inverse's Montgomery fix-up)
static constexpr uint32_t R3[N] = {0x1a997c41u, 0x165dd821u, 0x0e457c6fu, 0x0922ab08u, 0x196758efu,
                                   0x01d99018u, 0x1f324cf9u, 0x0a3fa669u, 0x19c6215au, 0x165a2cf1u,
                                   0x0159dd10u, 0x14ecc9dbu, 0x08839adcu};
constexpr int INV_ITERS = 26;  // ceil((2 * 377 - 1) / 29) iterations of 29 divsteps
}  // namespace r29

struct Fq29 {
  uint32_t v[r29::N];
  static TPST_HD Fq29 zero() {
    Fq29 r;
#pragma unroll
    for (int i = 0; i < r29::N; i++) r.v[i] = 0;
    return r;
  }
  static TPST_HD Fq29 one() {
    Fq29 r;
#pragma unroll
    for (int i = 0; i < r29::N; i++) r.v[i] = r29::ONE[i];
    return r;
  }
};

TPST_HD bool is_zero(const Fq29& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) acc |= a.v[i];
  return acc == 0;
}

TPST_HD bool eq(const Fq29& a, const Fq29& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

// t - p if t >= p (limbs normalised except the top one, < 2^30; the top
// limb of t - p is kept whole, so t < 2.7 p takes two calls)
TPST_HD void reduce_once(Fq29& t) {
  uint32_t s[r29::N];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < r29::N - 1; i++) {
    const int32_t d = (int32_t)t.v[i] - (int32_t)r29::P[i] + br;
    s[i] = (uint32_t)d & r29::M;
    br = d >> 29;  // 0 or -1
  }
  const int32_t dt = (int32_t)t.v[r29::N - 1] - (int32_t)r29::P[r29::N - 1] + br;
  s[r29::N - 1] = (uint32_t)dt;
  const bool take = dt >= 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) t.v[i] = take ? s[i] : t.v[i];
}

TPST_HD Fq29 add(const Fq29& a, const Fq29& b) {
  Fq29 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) {
    const uint32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = i < r29::N - 1 ? (s & r29::M) : s;
    c = s >> 29;
  }
  reduce_once(r);
  return r;
}

TPST_HD Fq29 dbl(const Fq29& a) { return add(a, a); }

TPST_HD Fq29 sub(const Fq29& a, const Fq29& b) {
  Fq29 r;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) {
    const int32_t d = (int32_t)a.v[i] - (int32_t)b.v[i] + br;
    r.v[i] = (uint32_t)d & r29::M;
    br = d >> 29;
  }
  const uint32_t mask = (uint32_t)br;  // all ones if a < b: add p back
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) {
    const uint32_t s = r.v[i] + (r29::P[i] & mask) + c;
    r.v[i] = s & r29::M;
    c = s >> 29;
  }
  return r;
}

TPST_HD Fq29 neg(const Fq29& a) { return sub(Fq29::zero(), a); }

// c ? -a : a for canonical a: p - a in one borrow pass (a = 0 stays 0) -- the
// sign of a gathered point in the accumulation loops, where neg's second pass
// (the conditional add of p) is dead weight
TPST_HD Fq29 cneg(const Fq29& a, bool c) {
  Fq29 r;
  int32_t br = 0;
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) {
    const int32_t d = (int32_t)r29::P[i] - (int32_t)a.v[i] + br;
    r.v[i] = (uint32_t)d & r29::M;
    br = d >> 29;
    nz |= a.v[i];
  }
  const bool take = c && nz != 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) r.v[i] = take ? r.v[i] : a.v[i];
  return r;
}
TPST_HD Fq29 mul3(const Fq29& a) { return add(dbl(a), a); }

// Montgomery product a b 2^-377 mod p, product scanning: column k gathers its
// a_i b_j and m_i p_j (i < k) in one 64-bit accumulator (<= 26 terms < 2^58
// each), then the reduction word m_k = -acc mod 2^29 (p_0 = 1) for k < 13 or
// the output limb, and the carry acc >> 29 moves to the next column.
// (Two accumulators per column -- the a_i b_j and the m_i p_j terms as two
// dependency chains -- measured neutral: 2^20 MSM 219.6 vs 218.7 Mscalar/s,
// product latency 0.91 us either way; a lone wave is issue-bound, not
// latency-bound, profiles/r05/ab1.)
TPST_HD Fq29 mul(const Fq29& a, const Fq29& b) {
  constexpr int N = r29::N;
  uint32_t m[N], t[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j >= 0 && j < N) acc += (uint64_t)a.v[i] * b.v[j];
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N) acc += (uint64_t)m[i] * r29::P[j];
    }
    if (k < N) {
      m[k] = (0u - (uint32_t)acc) & r29::M;
      acc = (acc + r29::M) >> 29;  // = (acc + m_k) / 2^29 = ceil(acc / 2^29): independent of m_k
    } else {
      t[k - N] = (uint32_t)acc & r29::M;
      acc >>= 29;
    }
  }
  t[N - 1] = (uint32_t)acc;  // < 2^30: t < 2p
  Fq29 r;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = t[i];
  reduce_once(r);
  return r;
}

// a b + c d (Montgomery) with ONE reduction for both products: column k
// gathers the a_i b_j, the c_i d_j and the m_i p_j (<= 38 terms < 2^58, with
// the carry < 2^64); canonical inputs (< p) only -- the sum is < (2 p^2 +
// R p) / R < 2.7 p, so two conditional subtractions.  A point addition's
// Y3 = R (Q - X3) - S PPP is one such sum (with p - PPP): one Montgomery
// reduction (156 multiply-adds) fewer per mixed add.
TPST_HD Fq29 mul_sum(const Fq29& a, const Fq29& b, const Fq29& c, const Fq29& d) {
  constexpr int N = r29::N;
  uint32_t m[N], t[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j >= 0 && j < N) acc += (uint64_t)a.v[i] * b.v[j] + (uint64_t)c.v[i] * d.v[j];
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N) acc += (uint64_t)m[i] * r29::P[j];
    }
    if (k < N) {
      m[k] = (0u - (uint32_t)acc) & r29::M;
      acc = (acc + r29::M) >> 29;  // = (acc + m_k) / 2^29 = ceil(acc / 2^29): independent of m_k
    } else {
      t[k - N] = (uint32_t)acc & r29::M;
      acc >>= 29;
    }
  }
  t[N - 1] = (uint32_t)acc;  // < 2^31: t < 2.7 p
  Fq29 r;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = t[i];
  reduce_once(r);
  reduce_once(r);
  return r;
}

// p - a in one borrow pass for a <= p (p - 0 = p is fine as a mul_sum
// operand: its limbs are 29-bit and p = 0 mod p)
TPST_HD Fq29 p_minus(const Fq29& a) {
  Fq29 r;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < r29::N; i++) {
    const int32_t d = (int32_t)r29::P[i] - (int32_t)a.v[i] + br;
    r.v[i] = (uint32_t)d & r29::M;
    br = d >> 29;
  }
  return r;
}

// a b - c d for canonical operands: one reduction (mul_sum with p - d; the
// sum stays < 2.7 p with d = p too)
TPST_HD Fq29 mul_sub(const Fq29& a, const Fq29& b, const Fq29& c, const Fq29& d) {
  return mul_sum(a, b, c, p_minus(d));
}

// square: cross products a_i a_j (i < j) once, doubled per column
TPST_HD Fq29 sqr(const Fq29& a) {
  constexpr int N = r29::N;
  uint32_t m[N], t[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t cr = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < j && j < N) cr += (uint64_t)a.v[i] * a.v[j];
    }
    acc += cr << 1;  // <= 13 cross terms < 2^58: doubled < 2^63
    if ((k & 1) == 0 && (k >> 1) < N) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N) acc += (uint64_t)m[i] * r29::P[j];
    }
    if (k < N) {
      m[k] = (0u - (uint32_t)acc) & r29::M;
      acc = (acc + r29::M) >> 29;  // = (acc + m_k) / 2^29 = ceil(acc / 2^29): independent of m_k
    } else {
      t[k - N] = (uint32_t)acc & r29::M;
      acc >>= 29;
    }
  }
  t[N - 1] = (uint32_t)acc;
  Fq29 r;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = t[i];
  reduce_once(r);
  return r;
}

// bits [s, s + 29) of a 13-word little-endian value (s + 29 <= 416)
TPST_HD uint32_t bits29(const uint32_t* w, int s) {
  const int q = s >> 5, o = s & 31;
  const uint32_t lo = q < 13 ? w[q] : 0u;
  const uint32_t hi = q + 1 < 13 ? w[q + 1] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
  // a funnel shift of two words: composing (hi << 32) | lo made the compiler
  // read w[q], w[q + 1] as one unaligned 64-bit word from a private-memory
  // copy of w (64 B/lane scratch in every accumulation kernel)
  return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)o) & r29::M;
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> o) & r29::M;
#endif
}

// The accumulation kernels' internal bucket / piece format: the radix-2^29
// Montgomery value itself (x 2^377, canonical, < p < 2^377) with its 377 bits
// regrouped into 12 u32 words -- field.h's footprint, but no modular
// conversion either way (to_std / from_std cost a quotient estimate, 12 limb
// products and a conditional subtraction per coordinate; this is ~2 bit
// operations per word)
TPST_HD void pack377(const Fq29& a, uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const int s = 32 * i, j = s / 29, o = s % 29;
    uint32_t v = a.v[j] >> o;
    if (j + 1 < r29::N) v |= a.v[j + 1] << (29 - o);
    if (j + 2 < r29::N && 58 - o < 32) v |= a.v[j + 2] << (58 - o);
    w[i] = v;
  }
}

TPST_HD Fq29 unpack377(const uint32_t* w) {
  Fq29 r;
#pragma unroll
  for (int j = 0; j < r29::N; j++) {
    const int s = 29 * j, q = s >> 5, o = s & 31;
    const uint32_t lo = w[q];
    const uint32_t hi = q + 1 < 12 ? w[q + 1] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
    r.v[j] = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)o) & r29::M;
#else
    r.v[j] = (uint32_t)((((uint64_t)hi << 32) | lo) >> o) & r29::M;
#endif
  }
  return r;
}

// field.h Montgomery (x 2^384, 12 x u32) -> x 2^377 in radix 2^29:
// (a + k p) / 2^7 < p for a < p; for an unreduced a < 64 p (a wave-engine
// form) the sum carries into a 13th word and the result is < 1.5 p < 2^377
TPST_HD Fq29 from_std(const Fq& a) {
  const uint32_t k = (0u - a.v[0]) & 127u;  // (a + k p) = 0 mod 2^7
  uint32_t w[13];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    c += (uint64_t)k * params::FQ_P[i] + a.v[i];
    w[i] = (uint32_t)c;
    c >>= 32;
  }
  w[12] = (uint32_t)c;
  Fq29 r;
#pragma unroll
  for (int j = 0; j < r29::N - 1; j++) r.v[j] = bits29(w, 29 * j + 7);
  // the top limb keeps every remaining bit: (a + k p) / 2^7 may reach 2^377
  // for a wide operand (< 1.5 p); mul's columns stay below 2^63 with a 30-bit top limb
  r.v[r29::N - 1] = (w[11] >> 3) | (w[12] << 29);  // bits 355.. (29 * 12 + 7)
  return r;
}

// x 2^377 (radix 2^29, < p) -> field.h Montgomery x 2^384 = Y 2^7 mod p
// without a product: W = Y 2^7 < 128 p < 2^384 in 32-bit words, q from a
// floating-point estimate of W / p biased low (q or q - 1), W - q p < 2p,
// one conditional subtraction
TPST_HD Fq to_std(const Fq29& a) {
  uint32_t w[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    // bits [32 i - 7, 32 i + 25) of the 29-bit limbs
    const int s = 32 * i - 7;
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < r29::N; j++) {
      const int sh = 29 * j - s;  // position of limb j relative to bit s
      if (sh > -29 && sh < 32) v |= sh >= 0 ? ((uint64_t)a.v[j] << sh) : ((uint64_t)a.v[j] >> (-sh));
    }
    w[i] = (uint32_t)v;
  }
  const double top = (double)w[11] * 4294967296.0 + (double)w[10];
  const double pt = (double)params::FQ_P[11] * 4294967296.0 + (double)params::FQ_P[10];
  const double qd = top / pt - 1e-6;
  const uint32_t q = qd > 0.0 ? (uint32_t)qd : 0u;
  Fq r;
  uint64_t c = 0;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint64_t t = (uint64_t)q * params::FQ_P[i] + c;
    c = t >> 32;
    const int64_t d = (int64_t)w[i] - (int64_t)(uint32_t)t + br;
    r.v[i] = (uint32_t)d;
    br = d >> 32;
  }
  reduce_once(r);
  return r;
}

// the same conversion as one Montgomery product by 2^384 mod p (reference
// form of to_std, kept for the host tests)
TPST_HD Fq to_std_mul(const Fq29& a) {
  Fq29 c;
#pragma unroll
  for (int i = 0; i < r29::N; i++) c.v[i] = r29::TO_STD[i];
  const Fq29 y = mul(a, c);  // a 2^384 / 2^377 = a 2^7, canonical
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    // bits [32 i, 32 i + 32) of the 29-bit limbs
    const int s = 32 * i, j = s / 29, o = s % 29;
    uint64_t v = (uint64_t)y.v[j] >> o;
    if (j + 1 < r29::N) v |= (uint64_t)y.v[j + 1] << (29 - o);
    if (j + 2 < r29::N) v |= (uint64_t)y.v[j + 2] << (58 - o);
    r.v[i] = (uint32_t)v;
  }
  return r;
}

}  // namespace tpst

namespace tpst {

// ------------------------------------------------------------ inversion --
// Pornin's optimised binary GCD (eprint 2020/972, Alg. 2) with k - 1 = 29
// divsteps per iteration, laid out for radix 2^29: each iteration runs the 29
// divsteps on 60-bit approximations (low 29 bits + top 31 bits of a and b),
// then applies the 2x2 matrix (|f| + |g| <= 2^29) to the full values, where
// the exact division by 2^29 is dropping limb 0, and to the Bezout
// coefficients u, v mod p, where the division by 2^29 is a Montgomery step:
// p = 1 mod 2^29, so adding k p with k = -t_0 mod 2^29 clears limb 0.  No
// quotient estimates, no final 2^-t correction: u, v track a, b exactly
// (a = u y, b = v y mod p).  Three times fewer instructions than field.h's
// 32-bit-limb version, which reduces u, v mod p with a quotient estimate in
// every iteration.
namespace r29 {

// (x f + y g) / 2^29 for signed 29-bit-or-less factors; x, y nonneg < 2^377
// in 13 limbs; the exact quotient (low limb zero) in 13 limbs, returns its sign
// (true: negative, r holds the magnitude)
TPST_HD bool lincomb_shift(const uint32_t* x, int32_t f, const uint32_t* y, int32_t g, uint32_t* r) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    c += (int64_t)x[i] * f + (int64_t)y[i] * g;
    if (i) r[i - 1] = (uint32_t)c & M;
    c >>= 29;  // arithmetic: floor
  }
  r[N - 1] = (uint32_t)c & M;
  const bool neg = c < 0;  // top carry: the sign of the whole value
  // two's complement negation over the 13 limbs when negative
  uint32_t cr = neg ? 1u : 0u;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t t = (neg ? (~r[i] & M) : r[i]) + cr;
    r[i] = t & M;
    cr = t >> 29;
  }
  return neg;
}

// (u f + v g) / 2^29 mod p for u, v in [0, p), |f| + |g| <= 2^29 -> [0, p)
TPST_HD void lincomb_mod(const uint32_t* u, int32_t f, const uint32_t* v, int32_t g, uint32_t* r) {
  const int64_t t0 = (int64_t)u[0] * f + (int64_t)v[0] * g;
  const uint32_t k = (0u - (uint32_t)t0) & M;  // t + k p = 0 mod 2^29 (p_0 = 1)
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    c += (int64_t)u[i] * f + (int64_t)v[i] * g + (int64_t)k * P[i];
    if (i) r[i - 1] = (uint32_t)c & M;
    c >>= 29;
  }
  // value = c 2^(29*12) + r[0..11], in (-p, 2p): one add or one subtract of p
  // (c < 2^30 when nonnegative: the value may reach 2^377)
  const bool neg = c < 0;
  r[N - 1] = neg ? ((uint32_t)c & M) : (uint32_t)c;
  if (neg) {
    uint32_t cr = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const uint32_t t = r[i] + P[i] + cr;
      r[i] = t & M;
      cr = t >> 29;
    }
  } else {
    Fq29 w;
#pragma unroll
    for (int i = 0; i < N; i++) w.v[i] = r[i];
    reduce_once(w);
#pragma unroll
    for (int i = 0; i < N; i++) r[i] = w.v[i];
  }
}

// bits [s, s + 31) of a 13-limb radix-2^29 value (s >= 0)
TPST_HD uint64_t top31(const uint32_t* x, int s) {
  uint64_t w = 0;
#pragma unroll
  for (int j = 0; j < N; j++) {
    const int sh = 29 * j - s;
    if (sh > -29 && sh < 31) w |= sh >= 0 ? ((uint64_t)x[j] << sh) : ((uint64_t)x[j] >> (-sh));
  }
  return w & ((1ull << 31) - 1);
}

}  // namespace r29

// a^-1 in Montgomery form (a = x 2^377 -> x^-1 2^377); 0 -> 0
TPST_HD Fq29 inv(const Fq29& y) {
  using namespace r29;
  uint32_t a[N], b[N], u[N], v[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    a[i] = y.v[i];
    b[i] = P[i];
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0;
  }
  for (int it = 0; it < INV_ITERS; it++) {
    int nb = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const uint32_t x = a[i] | b[i];
#if defined(__HIP_DEVICE_COMPILE__)
      const int bl = x ? 32 - __clz((int)x) : 0;
#else
      const int bl = x ? 32 - __builtin_clz(x) : 0;
#endif
      nb = x ? 29 * i + bl : nb;
    }
    const int n = nb > 60 ? nb : 60;
    uint64_t ab = (uint64_t)(a[0] & M) | (top31(a, n - 31) << 29);
    uint64_t bb = (uint64_t)(b[0] & M) | (top31(b, n - 31) << 29);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 1
    for (int j = 0; j < 29; j++) {
      const uint64_t odd = 0ull - (ab & 1u);
      const uint64_t sw = odd & (0ull - (uint64_t)(ab < bb));
      const uint64_t t = (ab ^ bb) & sw;
      ab ^= t;
      bb ^= t;
      const int32_t sw32 = (int32_t)sw;
      const int32_t tf = (f0 ^ f1) & sw32, tg = (g0 ^ g1) & sw32;
      f0 ^= tf;
      f1 ^= tf;
      g0 ^= tg;
      g1 ^= tg;
      const int32_t o32 = (int32_t)odd;
      ab -= bb & odd;
      f0 -= f1 & o32;
      g0 -= g1 & o32;
      ab >>= 1;
      f1 += f1;
      g1 += g1;
    }
    uint32_t na[N], nbv[N];
    const bool sa = lincomb_shift(a, f0, b, g0, na);
    const bool sb = lincomb_shift(a, f1, b, g1, nbv);
    if (sa) {
      f0 = -f0;
      g0 = -g0;
    }
    if (sb) {
      f1 = -f1;
      g1 = -g1;
    }
    uint32_t nu[N], nv[N];
    lincomb_mod(u, f0, v, g0, nu);
    lincomb_mod(u, f1, v, g1, nv);
#pragma unroll
    for (int i = 0; i < N; i++) {
      a[i] = na[i];
      b[i] = nbv[i];
      u[i] = nu[i];
      v[i] = nv[i];
    }
  }
  // b = gcd = 1 for invertible inputs; v = y^-1 (plain) = x^-1 2^-377
  uint32_t one_chk = b[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < N; i++) one_chk |= b[i];
  Fq29 r, k;
#pragma unroll
  for (int i = 0; i < N; i++) {
    r.v[i] = v[i];
    k.v[i] = R3[i];
  }
  r = mul(r, k);  // x^-1 2^-377 2^(3 377) / 2^377
  return one_chk == 0 ? r : Fq29::zero();
}

// field.h's Fq inverse (declared there): Montgomery in and out, radix 2^29 inside
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wattributes"
TPST_NI Fq inv(const Fq& a) { return to_std(inv(from_std(a))); }
#pragma GCC diagnostic pop

}  // namespace tpst
