// Host-side Poseidon sponge of the Fiat-Shamir transcript
// (poseidon_transcript.rs; ark-crypto-primitives PoseidonSponge<Fq>) and the
// 64-bit-limb Montgomery arithmetic it runs on.  Host only: included by
// pst_api.hip (the transcript C-ABI and the MIPP prover/verifier loops) and by
// tools/host_poseidon_bench.cpp.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/tpst.h"
#include "field.h"

namespace tpst {
#include "poseidon_constants.inc"

namespace {

Fq fq_canon(const uint64_t* c) {  // canonical u64 limbs -> Montgomery
  Fq a;
  memcpy(a.v, c, 48);
  return to_mont(a);
}
void fq_out(const Fq& a, uint64_t* c) {
  Fq r = from_mont(a);
  memcpy(c, r.v, 48);
}

// 64-bit-limb host Montgomery product (CIOS, unsigned __int128) on the same
// bits as Fq (6 x u64 = 12 x u32, R = 2^384 either way): the transcript's
// Poseidon permutations run ~17 per MIPP round on the host, between device
// phases, so their multiplications sit on the open's critical path.
struct HostP64 {
  uint64_t p[6];
  uint64_t inv;  // -p^-1 mod 2^64
  HostP64() {
    for (int i = 0; i < 6; i++) p[i] = (uint64_t)params::FQ_P[2 * i] | ((uint64_t)params::FQ_P[2 * i + 1] << 32);
    uint64_t x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - p[0] * x;  // Newton: x = p^-1 mod 2^64
    inv = 0 - x;
  }
};
const HostP64& hp64() {
  static HostP64 h;
  return h;
}

// (host pass only: a HIP device pass defines __x86_64__ too)
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#define TPST_HOST_ADX 1
#include "host_mont_adx.inc"
#else
#define TPST_HOST_ADX 0
#endif

// no-carry CIOS (p's top word < 2^62: the running value fits 6 words + the
// carry word of each row), fully unrolled over the 6 words of b
template <bool LAZY = false>
Fq hmul_cxx(const Fq& a, const Fq& b) {
  typedef unsigned __int128 u128;
  const HostP64& P = hp64();
  uint64_t x[6], y[6];
  memcpy(x, a.v, 48);
  memcpy(y, b.v, 48);
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
#define TPST_HMUL_ROW(i)                                                              \
  {                                                                                   \
    const uint64_t yi = y[i];                                                         \
    u128 c = (u128)x[0] * yi + t0;                                                    \
    const uint64_t a0 = (uint64_t)c;                                                  \
    uint64_t A = (uint64_t)(c >> 64);                                                 \
    const uint64_t m = a0 * P.inv;                                                    \
    u128 d = (u128)m * P.p[0] + a0;                                                   \
    uint64_t C = (uint64_t)(d >> 64);                                                 \
    c = (u128)x[1] * yi + t1 + A;                                                     \
    A = (uint64_t)(c >> 64);                                                          \
    d = (u128)m * P.p[1] + (uint64_t)c + C;                                           \
    C = (uint64_t)(d >> 64);                                                          \
    t0 = (uint64_t)d;                                                                 \
    c = (u128)x[2] * yi + t2 + A;                                                     \
    A = (uint64_t)(c >> 64);                                                          \
    d = (u128)m * P.p[2] + (uint64_t)c + C;                                           \
    C = (uint64_t)(d >> 64);                                                          \
    t1 = (uint64_t)d;                                                                 \
    c = (u128)x[3] * yi + t3 + A;                                                     \
    A = (uint64_t)(c >> 64);                                                          \
    d = (u128)m * P.p[3] + (uint64_t)c + C;                                           \
    C = (uint64_t)(d >> 64);                                                          \
    t2 = (uint64_t)d;                                                                 \
    c = (u128)x[4] * yi + t4 + A;                                                     \
    A = (uint64_t)(c >> 64);                                                          \
    d = (u128)m * P.p[4] + (uint64_t)c + C;                                           \
    C = (uint64_t)(d >> 64);                                                          \
    t3 = (uint64_t)d;                                                                 \
    c = (u128)x[5] * yi + t5 + A;                                                     \
    A = (uint64_t)(c >> 64);                                                          \
    d = (u128)m * P.p[5] + (uint64_t)c + C;                                           \
    C = (uint64_t)(d >> 64);                                                          \
    t4 = (uint64_t)d;                                                                 \
    t5 = C + A;                                                                       \
  }
  TPST_HMUL_ROW(0) TPST_HMUL_ROW(1) TPST_HMUL_ROW(2) TPST_HMUL_ROW(3) TPST_HMUL_ROW(4) TPST_HMUL_ROW(5)
#undef TPST_HMUL_ROW
  // t < 2p: one conditional subtraction (LAZY: left < 2p for a product)
  const uint64_t t[6] = {t0, t1, t2, t3, t4, t5};
  if (LAZY) {
    Fq out;
    memcpy(out.v, t, 48);
    return out;
  }
  uint64_t r[6];
  u128 br = 0;
  for (int j = 0; j < 6; j++) {
    const u128 dd = (u128)t[j] - P.p[j] - (uint64_t)br;
    r[j] = (uint64_t)dd;
    br = (dd >> 64) & 1;
  }
  Fq out;
  memcpy(out.v, br ? t : r, 48);
  return out;
}

// word-by-word Montgomery reduction of a 12-word t (t < p R): t R^-1 mod p,
// one conditional subtraction (t R^-1 < 2p).  Carries out of each row go to
// the next row's top word (c2) -- no data-dependent branches.
template <bool LAZY = false>
__attribute__((always_inline)) inline Fq redc12(uint64_t* t) {
  typedef unsigned __int128 u128;
  const HostP64& P = hp64();
  uint64_t c2 = 0;
  #pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint64_t m = t[i] * P.inv;
    u128 c = 0;
    #pragma unroll
    for (int j = 0; j < 6; j++) {
      c += (u128)m * P.p[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    const u128 s2 = (u128)t[i + 6] + (uint64_t)c + c2;
    t[i + 6] = (uint64_t)s2;
    c2 = (uint64_t)(s2 >> 64);
  }
  if (LAZY) {  // t < 12 p^2 (three products of inputs < 2p): t R^-1 < 1.1 p, c2 = 0
    Fq out;
    memcpy(out.v, t + 6, 48);
    return out;
  }
  uint64_t r[6];
  u128 br = 0;
  #pragma unroll
  for (int j = 0; j < 6; j++) {
    const u128 d = (u128)t[6 + j] - P.p[j] - (uint64_t)br;
    r[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  const bool ge = c2 || !br;
  Fq out;
  memcpy(out.v, ge ? r : t + 6, 48);
  return out;
}

// t += x y (12 words; the running sum stays below 2^768)
__attribute__((always_inline)) inline void mac12(uint64_t* t, const uint64_t* x, const uint64_t* y) {
  typedef unsigned __int128 u128;
  uint64_t c2 = 0;
  #pragma unroll
  for (int i = 0; i < 6; i++) {
    u128 c = 0;
    #pragma unroll
    for (int j = 0; j < 6; j++) {
      c += (u128)x[j] * y[i] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    const u128 s2 = (u128)t[i + 6] + (uint64_t)c + c2;
    t[i + 6] = (uint64_t)s2;
    c2 = (uint64_t)(s2 >> 64);
  }
}

// sum of three Montgomery products with one reduction: the 768-bit products
// are added unreduced (3 p^2 < p R) and reduced once, so an MDS row costs
// three multiplications and one REDC instead of three of each
template <bool LAZY = false>
Fq hmul3_cxx(const Fq& a0, const Fq& b0, const Fq& a1, const Fq& b1, const Fq& a2, const Fq& b2) {
  uint64_t t[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, x[6], y[6];
  memcpy(x, a0.v, 48);
  memcpy(y, b0.v, 48);
  mac12(t, x, y);
  memcpy(x, a1.v, 48);
  memcpy(y, b1.v, 48);
  mac12(t, x, y);
  memcpy(x, a2.v, 48);
  memcpy(y, b2.v, 48);
  mac12(t, x, y);
  return redc12<LAZY>(t);
}

// Montgomery square: the 15 cross products once, doubled, plus the 6
// squares, then the REDC -- the S-box's x^2, x^4, x^8, x^16
template <bool LAZY = false>
Fq hsqr_cxx(const Fq& a) {
  typedef unsigned __int128 u128;
  uint64_t x[6];
  memcpy(x, a.v, 48);
  uint64_t t[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  #pragma unroll
  for (int i = 0; i < 5; i++) {
    u128 c = 0;
    #pragma unroll
    for (int j = i + 1; j < 6; j++) {
      c += (u128)x[i] * x[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 6] = (uint64_t)c;
  }
  #pragma unroll
  for (int i = 11; i > 0; i--) t[i] = (t[i] << 1) | (t[i - 1] >> 63);
  t[0] <<= 1;
  u128 c = 0;
  #pragma unroll
  for (int i = 0; i < 6; i++) {
    const u128 sq = (u128)x[i] * x[i];
    c += (u128)t[2 * i] + (uint64_t)sq;
    t[2 * i] = (uint64_t)c;
    c >>= 64;
    c += (u128)t[2 * i + 1] + (uint64_t)(sq >> 64);
    t[2 * i + 1] = (uint64_t)c;
    c >>= 64;
  }
  return redc12<LAZY>(t);
}

// a + b mod p on 64-bit words (a, b < p)
inline Fq hadd(const Fq& a, const Fq& b) {
  typedef unsigned __int128 u128;
  const HostP64& P = hp64();
  uint64_t x[6], y[6], t[6], r[6];
  memcpy(x, a.v, 48);
  memcpy(y, b.v, 48);
  u128 c = 0;
  for (int j = 0; j < 6; j++) {
    c += (u128)x[j] + y[j];
    t[j] = (uint64_t)c;
    c >>= 64;
  }
  u128 br = 0;
  for (int j = 0; j < 6; j++) {
    const u128 d = (u128)t[j] - P.p[j] - (uint64_t)br;
    r[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  Fq out;
  memcpy(out.v, br ? t : r, 48);  // a + b < 2p < 2^384: no carry out of t
  return out;
}

// a + b for a, b < 2p, left < 2p (the permutation's lazy form: every value
// inside it stays below 2p, products and REDCs skip the final subtraction)
inline Fq hadd_lazy(const Fq& a, const Fq& b) {
  typedef unsigned __int128 u128;
  const HostP64& P = hp64();
  uint64_t x[6], y[6], t[6], r[6], p2[6];
  memcpy(x, a.v, 48);
  memcpy(y, b.v, 48);
  u128 c = 0;
  for (int j = 0; j < 6; j++) {
    c += (u128)x[j] + y[j];
    t[j] = (uint64_t)c;
    c >>= 64;
    p2[j] = (P.p[j] << 1) | (j ? P.p[j - 1] >> 63 : 0);
  }
  u128 br = 0;
  for (int j = 0; j < 6; j++) {
    const u128 d = (u128)t[j] - p2[j] - (uint64_t)br;
    r[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  Fq out;
  memcpy(out.v, br ? t : r, 48);  // a + b < 4p < 2^379
  return out;
}

// a + b without reduction (the sum < 2^384)
inline Fq hadd_raw(const Fq& a, const Fq& b) {
  typedef unsigned __int128 u128;
  uint64_t x[6], y[6], t[6];
  memcpy(x, a.v, 48);
  memcpy(y, b.v, 48);
  u128 c = 0;
  for (int j = 0; j < 6; j++) {
    c += (u128)x[j] + y[j];
    t[j] = (uint64_t)c;
    c >>= 64;
  }
  Fq out;
  memcpy(out.v, t, 48);
  return out;
}

// x < 2p -> canonical
inline Fq hcanon(const Fq& a) {
  typedef unsigned __int128 u128;
  const HostP64& P = hp64();
  uint64_t t[6], r[6];
  memcpy(t, a.v, 48);
  u128 br = 0;
  for (int j = 0; j < 6; j++) {
    const u128 d = (u128)t[j] - P.p[j] - (uint64_t)br;
    r[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  Fq out;
  memcpy(out.v, br ? t : r, 48);
  return out;
}

// t - m if t >= m (6 words; t < 2^384)
inline Fq sub_if_ge(const Fq& a, const uint64_t* m) {
  typedef unsigned __int128 u128;
  uint64_t t[6], r[6];
  memcpy(t, a.v, 48);
  u128 br = 0;
  for (int j = 0; j < 6; j++) {
    const u128 d = (u128)t[j] - m[j] - (uint64_t)br;
    r[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  Fq out;
  memcpy(out.v, br ? t : r, 48);
  return out;
}

// The products the transcript's permutations run on: MULX / ADCX / ADOX
// assembly (host_mont_adx.inc, generated by tools/gen_mont_adx.py) where the
// host CPU has BMI2 + ADX -- 2.3x faster than the __int128 CIOS above
// (tests/cpp/test_mont_adx.cpp: 58 vs 136 ns on the build container) -- else
// the C++ forms.  Every MIPP round's Poseidon absorption of t_l / t_r sits on
// the opening's critical path (~13 permutations of ~500 products).
inline bool host_adx() {
#if TPST_HOST_ADX
  // (__builtin_cpu_init first: a shared library's code may run before the
  // runtime's own CPU-model constructor has)
  static const bool ok = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("adx") && __builtin_cpu_supports("bmi2");
  }();
  return ok;
#else
  return false;
#endif
}

template <bool LAZY = false>
Fq hmul(const Fq& a, const Fq& b) {
#if TPST_HOST_ADX
  if (host_adx()) {  // < a b / R + p < 1.03 p for a, b < 2p
    Fq r;
    mont_mul_adx(reinterpret_cast<uint64_t*>(r.v), reinterpret_cast<const uint64_t*>(a.v),
                 reinterpret_cast<const uint64_t*>(b.v), hp64().p, hp64().inv);
    return LAZY ? r : hcanon(r);
  }
#endif
  return hmul_cxx<LAZY>(a, b);
}

template <bool LAZY = false>
Fq hsqr(const Fq& a) {
  if (host_adx()) return hmul<LAZY>(a, a);
  return hsqr_cxx<LAZY>(a);
}

// the sum of the three products: each < 1.03 p from the ADX product, the sum
// < 3.1 p, brought below 2p (LAZY) or below p
template <bool LAZY = false>
Fq hmul3(const Fq& a0, const Fq& b0, const Fq& a1, const Fq& b1, const Fq& a2, const Fq& b2) {
  if (host_adx()) {
    const Fq s = hadd_raw(hadd_raw(hmul<true>(a0, b0), hmul<true>(a1, b1)), hmul<true>(a2, b2));
    uint64_t p2[6];
    const HostP64& P = hp64();
    for (int j = 0; j < 6; j++) p2[j] = (P.p[j] << 1) | (j ? P.p[j - 1] >> 63 : 0);
    const Fq r = sub_if_ge(s, p2);  // < 2p
    return LAZY ? r : hcanon(r);
  }
  return hmul3_cxx<LAZY>(a0, b0, a1, b1, a2, b2);
}

// x^17 (alpha = 17), lazy: x < 2p in, < 2p out
Fq sbox17(const Fq& x) { return hmul<true>(hsqr<true>(hsqr<true>(hsqr<true>(hsqr<true>(x)))), x); }

// ------------------------------------------------------------ Poseidon ----
// The permutation is evaluated in the equivalent form of the Poseidon paper's
// appendix B (same outputs, fewer products), derived once from the sponge's
// parameters:
//  - partial-round constants: a partial round's S-box touches only element 0,
//    so M S(x + c) = M S(x + c_0 e_0) + M (0, c_1, c_2): the second term is
//    carried into the next round's constants; after the last partial round it
//    lands in the first closing full round's;
//  - sparse partial-round matrices: the round matrix M_r = M' M'' with
//    M'' = [[a, b^T], [D^-1 c, I]] and M' = diag(1, D); M' leaves element 0
//    alone, so it commutes with the next partial S-box and its e_0 constant
//    and is folded into the next round's matrix (M_{r+1} = M M').  30 partial
//    rounds apply a 5-product M''; the last applies its dense M_r.
struct PoseidonParams {
  static constexpr int RF0 = 4, RP = 31, RN = 39;  // full rounds 0..3 and 35..38
  Fq ark[RN][3];
  Fq mds[3][3];
  Fq sp[RP - 1][5];  // sparse rounds: a, b1, b2, w1, w2
  Fq last[3][3];     // dense matrix of the last partial round
  static Fq finv(const Fq& a) {  // a^(p-2), one-time
    const HostP64& P = hp64();
    uint64_t e[6];
    memcpy(e, P.p, 48);
    e[0] -= 2;
    Fq r = Fq::one(), b = a;
    for (int i = 0; i < 377; i++) {
      if ((e[i >> 6] >> (i & 63)) & 1) r = hmul(r, b);
      b = hsqr(b);
    }
    return r;
  }
  static void mat_mul(const Fq (*x)[3], const Fq (*y)[3], Fq (*z)[3]) {
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) z[i][j] = hmul3(x[i][0], y[0][j], x[i][1], y[1][j], x[i][2], y[2][j]);
  }
  PoseidonParams() {
    for (int r = 0; r < RN; r++)
      for (int i = 0; i < 3; i++) ark[r][i] = fq_canon(POSEIDON_ARK[r][i]);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) mds[i][j] = fq_canon(POSEIDON_MDS[i][j]);
    const Fq z = Fq::zero();
    for (int r = RF0; r < RF0 + RP; r++) {  // constants 1, 2 of partial rounds -> next round
      for (int i = 0; i < 3; i++)
        ark[r + 1][i] = add(ark[r + 1][i], hmul3(mds[i][0], z, mds[i][1], ark[r][1], mds[i][2], ark[r][2]));
      ark[r][1] = ark[r][2] = z;
    }
    Fq cur[3][3];
    memcpy(cur, mds, sizeof(cur));
    for (int k = 0; k < RP - 1; k++) {
      // cur = [[a, b^T], [c, D]]: w = D^-1 c
      const Fq det = sub(hmul(cur[1][1], cur[2][2]), hmul(cur[1][2], cur[2][1]));
      const Fq di = finv(det);
      const Fq w1 = hmul(di, sub(hmul(cur[2][2], cur[1][0]), hmul(cur[1][2], cur[2][0])));
      const Fq w2 = hmul(di, sub(hmul(cur[1][1], cur[2][0]), hmul(cur[2][1], cur[1][0])));
      sp[k][0] = cur[0][0];
      sp[k][1] = cur[0][1];
      sp[k][2] = cur[0][2];
      sp[k][3] = w1;
      sp[k][4] = w2;
      Fq mp[3][3] = {{Fq::one(), z, z}, {z, cur[1][1], cur[1][2]}, {z, cur[2][1], cur[2][2]}};
      Fq nx[3][3];
      mat_mul(mds, mp, nx);
      memcpy(cur, nx, sizeof(cur));
    }
    memcpy(last, cur, sizeof(last));
  }
};
const PoseidonParams& pparams() {
  static PoseidonParams p;
  return p;
}

// ark-crypto-primitives PoseidonSponge<Fq>: rate 2, capacity 1, alpha 17,
// 8 full + 31 partial rounds (parameters.rs:309-338)
struct Sponge {
  Fq st[3];
  bool squeezing;
  int idx;
  void load(const tpst_transcript* t) {
    for (int i = 0; i < 3; i++) st[i] = fq_canon(t->state[i]);
    squeezing = t->squeezing != 0;
    idx = (int)t->index;
  }
  void store(tpst_transcript* t) const {
    for (int i = 0; i < 3; i++) fq_out(st[i], t->state[i]);
    t->squeezing = squeezing ? 1 : 0;
    t->index = (uint32_t)idx;
  }
  void full_round(const PoseidonParams& P, int r) {
    Fq x[3];
    for (int i = 0; i < 3; i++) x[i] = sbox17(hadd_lazy(st[i], P.ark[r][i]));
    for (int i = 0; i < 3; i++) st[i] = hmul3<true>(P.mds[i][0], x[0], P.mds[i][1], x[1], P.mds[i][2], x[2]);
  }
  // lazy throughout (values < 2p), canonical state in and out
  void permute() {
    const PoseidonParams& P = pparams();
    for (int r = 0; r < P.RF0; r++) full_round(P, r);
    for (int k = 0; k < P.RP - 1; k++) {
      const Fq* m = P.sp[k];
      const Fq x0 = sbox17(hadd_lazy(st[0], P.ark[P.RF0 + k][0]));
      const Fq n0 = hmul3<true>(m[0], x0, m[1], st[1], m[2], st[2]);
      st[1] = hadd_lazy(st[1], hmul<true>(m[3], x0));
      st[2] = hadd_lazy(st[2], hmul<true>(m[4], x0));
      st[0] = n0;
    }
    {
      const Fq x0 = sbox17(hadd_lazy(st[0], P.ark[P.RF0 + P.RP - 1][0]));
      Fq ns[3];
      for (int i = 0; i < 3; i++)
        ns[i] = hmul3<true>(P.last[i][0], x0, P.last[i][1], st[1], P.last[i][2], st[2]);
      for (int i = 0; i < 3; i++) st[i] = ns[i];
    }
    for (int r = P.RF0 + P.RP; r < P.RN; r++) full_round(P, r);
    for (int i = 0; i < 3; i++) st[i] = hcanon(st[i]);
  }
  void absorb(const std::vector<Fq>& e) {
    if (e.empty()) return;
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
    size_t k = 0;
    for (;;) {
      const size_t rem = e.size() - k;
      if (i0 + rem <= 2) {
        for (size_t j = 0; j < rem; j++) st[1 + i0 + j] = hadd(st[1 + i0 + j], e[k + j]);
        squeezing = false;
        idx = i0 + (int)rem;
        return;
      }
      const int take = 2 - i0;
      for (int j = 0; j < take; j++) st[1 + i0 + j] = hadd(st[1 + i0 + j], e[k + j]);
      permute();
      k += take;
      i0 = 0;
    }
  }
  // Absorb for Vec<u8>: u64 LE length prefix, 47-byte chunks -> Fq
  void absorb_bytes(const uint8_t* d, size_t n) {
    std::vector<uint8_t> buf(8 + n);
    const uint64_t len = n;
    memcpy(buf.data(), &len, 8);
    if (n) memcpy(buf.data() + 8, d, n);
    std::vector<Fq> e;
    for (size_t o = 0; o < buf.size(); o += 47) {
      uint64_t l[6] = {0, 0, 0, 0, 0, 0};
      const size_t m = buf.size() - o < 47 ? buf.size() - o : 47;
      memcpy(l, buf.data() + o, m);
      e.push_back(fq_canon(l));
    }
    absorb(e);
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
    const Fq out = st[1 + i0];
    squeezing = true;
    idx = i0 + 1;
    return out;
  }
  // non-native squeeze_field_elements::<Fr>(1): low 252 bits of one Fq
  void challenge(uint64_t* fr_canon_out) {
    uint64_t c[6];
    fq_out(squeeze1(), c);
    fr_canon_out[0] = c[0];
    fr_canon_out[1] = c[1];
    fr_canon_out[2] = c[2];
    fr_canon_out[3] = c[3] & ((1ull << 60) - 1);
  }
};

}  // namespace
}  // namespace tpst
