// One Fq inversion by a whole wave (device only).
//
// Why: the lone-lane inverse (field29.h inv: 26 batches of 29 divsteps on
// 13-limb values) is a ~0.13 ms serial chain.  Where only one or two values
// are inverted -- the open's per-round cross commitments, an MSM's single
// output point, the final-exponentiation chain -- that chain sits on the
// critical path with 63 lanes idle.  Here the wave shares the work: the
// Bernstein-Yang GCD in batches of K = 15 divsteps, variable time (the
// libsecp256k1 modinv shape: each inner step skips g's trailing zeros and
// cancels up to eta + 1 low bits with one multiple of f), run on wave-uniform
// low bits, i.e. on the scalar unit -- 5 inner steps per batch on average
// against 15 branch-free divsteps of Pornin's form -- and the big values f, g
// (the GCD pair) and d, e (the cofactors, signed) as NL = 28 limbs of 15 bits,
// one limb per lane.  A batch's four updates
//     (x u + y v + k p) / 2^15
// are one limb product per lane plus a carry normalisation: a bias makes every
// limb sum nonnegative, two local carry passes (DPP shift by one lane) leave
// limbs <= 2^15 + 4, and one ballot pass resolves the remaining +1 ripples
// (carry-lookahead on the 64-bit lane masks); the division by 2^15 is a shift
// down by one lane.  Exact model, every step as computed here:
// tools/inv_wave_model.py (inv_model_by; 52.6 batches on average, at most 55).
//
// Bounds (checked by the model): |u| + |v| <= 2^15 and limbs < 2^15, so a
// limb sum stays below 2^31 in magnitude; the cofactors grow by at most p per
// batch (below 80 p < 2^384).
#pragma once
#include "field29.h"
#include "curve.h"

namespace tpst {
namespace invw {

constexpr int NL = 28;
constexpr int K = 15;
constexpr uint32_t LM = (1u << 15) - 1;
constexpr uint64_t NLMASK = (1ull << NL) - 1;

// p in radix 2^15
__device__ static constexpr uint32_t P15[32] = {
    0x0001u, 0x0000u, 0x0000u, 0x2846u, 0x0008u, 0x0000u, 0x510cu, 0x05aeu, 0x0017u, 0x1290u, 0x3ee8u,
    0x1b11u, 0x71efu, 0x2271u, 0x403du, 0x6cf9u, 0x1a22u, 0x1276u, 0x3285u, 0x2e03u, 0x63b0u, 0x1d58u,
    0x7144u, 0x230bu, 0x2e3au, 0x0003u, 0x0000u, 0x0000u, 0, 0, 0, 0};

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// lane i receives lane i-1's value, lane 0 receives 0
__device__ __forceinline__ uint32_t shift_up(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
}
// lane i receives lane i+1's value, lane 63 receives 0
__device__ __forceinline__ uint32_t shift_down(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t rl(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }

// one-bit lane carries of a 64-bit lane mask -> this lane's bit
__device__ __forceinline__ uint32_t lane_bit(uint64_t m, uint32_t lane) { return (uint32_t)(m >> lane) & 1u; }

// limb sums t (|t| < 2^31) -> (value / 2^15) as sign + magnitude limbs;
// the value is a multiple of 2^15 by construction
__device__ __forceinline__ uint32_t div_signed(int32_t t, uint32_t lane, bool& neg) {
  const bool live = lane < (uint32_t)NL;
  uint32_t x = (uint32_t)t + 0x80000000u - (lane ? 0x10000u : 0u);
  x = live ? x : 0u;
#pragma unroll
  for (int pass = 0; pass < 2; pass++) x = (x & LM) + shift_up(x >> 15);
  const uint64_t g = __ballot(live && x > LM);
  uint32_t base = x & LM;
  uint64_t pr = __ballot(live && base == LM);
  uint32_t limb = (base + lane_bit(((g << 1) + pr) ^ pr, lane)) & LM;
  limb = live ? limb : 0u;
  neg = (rl(limb, NL - 1) >> 14) & 1u;
  if (neg) {  // wave-uniform: magnitude = ~limbs + 1
    const uint32_t iv = live ? LM - limb : 0u;
    pr = __ballot(live && iv == LM);
    limb = (iv + lane_bit((1ull + pr) ^ pr, lane)) & LM;
    limb = live ? limb : 0u;
  }
  return shift_down(limb);  // limb 0 is zero: / 2^15
}

// (49 d + 80) / 17 = 1091 divsteps bound the GCD for d = 377 bits
// (Bernstein-Yang), i.e. 73 batches of 15; the loop stops at g = 0 (52.6
// batches on average in the model), so the cap costs nothing
constexpr int BY_MAX_BATCHES = 80;

// low 30 bits of a signed sign-magnitude value (limbs 0 and 1), two's complement
__device__ __forceinline__ uint32_t low30(uint32_t mag, bool neg) {
  const uint32_t x = rl(mag, 0) | (rl(mag, 1) << 15);
  return neg ? 0u - x : x;
}

// K divsteps of Bernstein-Yang on the low bits, variable time (scalar unit):
// each step skips g's trailing zeros, then cancels min(eta + 1, i) low bits
// of g with one multiple of f (f^-1 mod 2^32 by Newton).  Returns eta and the
// transition matrix, |u| + |v| <= 2^K.  tools/inv_wave_model.py divsteps_var.
__device__ __forceinline__ int divsteps_var(int eta, uint32_t f, uint32_t g, int32_t& mu, int32_t& mv, int32_t& mq,
                                            int32_t& mr) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = K;
#pragma unroll 1
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xFFFFFFFFu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {
      eta = -eta;
      const uint32_t tf = f, tu = u, tv = v;
      f = g;
      g = 0u - tf;
      u = q;
      q = 0u - tu;
      v = r;
      r = 0u - tv;
    }
    const int limit = eta + 1 < i ? eta + 1 : i;
    const uint32_t m = (1u << limit) - 1u;
    uint32_t x = f;
    x *= 2u - f * x;
    x *= 2u - f * x;
    x *= 2u - f * x;
    const uint32_t w = ((0u - g) * x) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  mu = (int32_t)u;
  mv = (int32_t)v;
  mq = (int32_t)q;
  mr = (int32_t)r;
  return eta;
}

}  // namespace invw

// y^-1 for a Montgomery-form y (x 2^377 -> x^-1 2^377), 0 -> 0.  Every lane of
// the wave must call it with the same y (wave-uniform); every lane gets the
// result.
__device__ inline __attribute__((noinline)) Fq29 inv_wave(const Fq29& y) {
  using namespace invw;
  const uint32_t lane = lane_id();
  // lane i: bits [15 i, 15 i + 15) of y
  uint32_t a;
  {
    const uint32_t bit = 15u * lane, j = bit / 29u, sh = bit % 29u;
    uint32_t w0 = 0, w1 = 0;
#pragma unroll
    for (int jj = 0; jj < r29::N; jj++) {
      w0 = (uint32_t)jj == j ? y.v[jj] : w0;
      w1 = (uint32_t)jj == j + 1 ? y.v[jj] : w1;
    }
    a = ((w0 >> sh) | (sh ? w1 << (29u - sh) : 0u)) & LM;
    a = lane < (uint32_t)NL ? a : 0u;
  }
  const uint32_t pl = P15[lane & 31];
  // Bernstein-Yang, variable time: f = p, g = y; d, e the signed cofactors
  // (f = d y, g = e y mod p; each batch divides both sides by 2^15, the k p
  // term keeping the cofactor division exact); stops when g = 0, f = +-1
  uint32_t f = lane < (uint32_t)NL ? pl : 0u, g = a;
  uint32_t d = 0, e = lane == 0 ? 1u : 0u;
  bool fs = false, gs = false, ds = false, es = false;
  int eta = -1;
#pragma unroll 1
  for (int it = 0; it < BY_MAX_BATCHES && (__ballot(g != 0u) != 0); it++) {
    int32_t u, v, q, r;
    eta = divsteps_var(eta, low30(f, fs), low30(g, gs), u, v, q, r);
    bool nfs, ngs;
    const uint32_t nf = div_signed((int32_t)f * (fs ? -u : u) + (int32_t)g * (gs ? -v : v), lane, nfs);
    const uint32_t ng = div_signed((int32_t)f * (fs ? -q : q) + (int32_t)g * (gs ? -r : r), lane, ngs);
    const int32_t ud = ds ? -u : u, ve = es ? -v : v, qd = ds ? -q : q, re = es ? -r : r;
    const int32_t d0 = (int32_t)rl(d, 0), e0 = (int32_t)rl(e, 0);
    const int32_t kd = (int32_t)((uint32_t)(-(d0 * ud + e0 * ve)) & LM);
    const int32_t ke = (int32_t)((uint32_t)(-(d0 * qd + e0 * re)) & LM);
    bool nds, nes;
    const uint32_t nd = div_signed((int32_t)d * ud + (int32_t)e * ve + kd * (int32_t)pl, lane, nds);
    const uint32_t ne = div_signed((int32_t)d * qd + (int32_t)e * re + ke * (int32_t)pl, lane, nes);
    f = nf;
    g = ng;
    d = nd;
    e = ne;
    fs = nfs;
    gs = ngs;
    ds = nds;
    es = nes;
  }
  // f = +-1 for y != 0; then y^-1 = +-d (plain), |d| < 80 p
  const bool ok = (__ballot(f != (lane == 0 ? 1u : 0u)) & NLMASK) == 0;
  const uint32_t v = d;
  const bool vs = ds != fs;
  uint32_t vl[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) vl[i] = rl(v, i);
  // radix 2^15 -> 14 limbs of 2^29
  uint32_t r[14];
#pragma unroll
  for (int j = 0; j < 14; j++) {
    uint64_t w = 0;
#pragma unroll
    for (int i = 0; i < NL; i++) {
      const int sh = 15 * i - 29 * j;
      if (sh > -15 && sh < 29) w |= sh >= 0 ? ((uint64_t)vl[i] << sh) : ((uint64_t)vl[i] >> (-sh));
    }
    r[j] = (uint32_t)w & r29::M;
  }
  // r mod p: a quotient estimate from the top limbs (q < 80, low by at most
  // one), then one conditional subtraction
  {
    const double dv = (double)r[13] * 536870912.0 + (double)r[12] + (double)r[11] * (1.0 / 536870912.0);
    const double dp = (double)r29::P[12] + (double)r29::P[11] * (1.0 / 536870912.0);
    const int64_t q = (int64_t)(dv / dp * (1.0 - 1e-12));
    int64_t c = 0;
#pragma unroll
    for (int j = 0; j < 14; j++) {
      const int64_t w = (int64_t)r[j] - q * (int64_t)(j < r29::N ? r29::P[j] : 0u) + c;
      r[j] = (uint32_t)w & r29::M;
      c = w >> 29;
    }
    uint32_t s[14];
    int64_t bw = 0;
#pragma unroll
    for (int j = 0; j < 14; j++) {
      const int64_t w = (int64_t)r[j] - (int64_t)(j < r29::N ? r29::P[j] : 0u) + bw;
      s[j] = (uint32_t)w & r29::M;
      bw = w >> 29;
    }
#pragma unroll
    for (int j = 0; j < 14; j++) r[j] = bw == 0 ? s[j] : r[j];
  }
  Fq29 x, k;
  uint32_t nzv = 0;
#pragma unroll
  for (int j = 0; j < r29::N; j++) {
    x.v[j] = r[j];
    nzv |= r[j];
    k.v[j] = r29::R3[j];
  }
  if (vs && nzv) {  // -r mod p
    int64_t bw = 0;
#pragma unroll
    for (int j = 0; j < r29::N; j++) {
      const int64_t w = (int64_t)r29::P[j] - (int64_t)x.v[j] + bw;
      x.v[j] = (uint32_t)w & r29::M;
      bw = w >> 29;
    }
  }
  x = mul(x, k);  // x^-1 2^-377 -> x^-1 2^377
  return ok ? x : Fq29::zero();
}

// field.h layout wrappers
__device__ __forceinline__ Fq inv_w(const Fq& a) { return to_std(inv_wave(from_std(a))); }
__device__ __forceinline__ Fq2 inv_w(const Fq2& a) {
  const Fq n = add(sqr(a.c0), mul5(sqr(a.c1)));
  const Fq ni = inv_w(n);
  return {mul(a.c0, ni), neg(mul(a.c1, ni))};
}

// curve.h to_affine with the wave inverse (wave-uniform point)
template <class F>
__device__ Affine<F> to_affine_w(const Xyzz<F>& p) {
  if (is_zero(p.ZZ)) return Affine<F>::inf();
  const F t = inv_w(mul(p.ZZ, p.ZZZ));
  return {mul(p.X, mul(t, p.ZZZ)), mul(p.Y, mul(t, p.ZZ))};
}

}  // namespace tpst
