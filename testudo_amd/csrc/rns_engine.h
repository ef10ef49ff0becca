// Residue-number-system Fq12 engine for the serial pairing chains (Horner
// over the Miller block multipliers + final exponentiation, k_chain_final).
//
// wave_tower.h evaluates one Fq product per lane, so each stage of a serial
// chain is bounded by one lone-lane Montgomery product (~1.9k cycles) plus
// the linear forms around it.  Here an Fq value is a vector of residues,
// one per lane (tools/gen_rns_ops.py picks the moduli and checks every
// bound through an exact model of this file's arithmetic):
//
//   lane & 31 :  0..14  base B  (m_i = 2^28 - c_i, prime)
//                15     redundant channel, arithmetic mod 2^32
//                16..30 base B'
//                31     idle (a copy of channel 0)
//   lane >> 5 :  which of the workgroup's two chains
//
// Values are kept in the "M-domain" (x~ = x M mod p, M = prod B) as integers
// below 16 p.  One stage evaluates an Fq12 operation with one wave per
// output coefficient o:
//
//   t_o   = sum_k c_k x_k y_k                 lane-local monomials of the
//                                             input slots (c_k <= 15)
//   out_o = (t_o + q p) / M                   RNS Montgomery reduction:
//     B lanes   xi_i = t_i (-p^-1 M_i^-1)      q^ = sum xi_i M_i = q + alpha M
//     B', 2^32  q^ by fast base extension,  r = (t + q^ p) M^-1
//     B lanes   r by an exact extension back (Shenoy-Kumaresan: the 2^32
//               channel gives beta = floor(sum xi'_j M'_j / M'))
//
// so the cross-lane work per output is two 15-term base extensions through
// the wave's exchange words, and a stage costs about one wave-issue of
// ~150 VALU slots per output instead of a lone-lane product chain.
#pragma once
#include "field.h"

#if defined(__HIPCC__)
#define TPST_RNS_CONST __constant__ const
#else
#define TPST_RNS_CONST const
#endif
#include "rns_ops.inc"

namespace tpst {
namespace rns {

typedef __attribute__((address_space(3))) uint32_t lds_t;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u lds4_t;

constexpr int SLOT = 64;  // u32 per slot: residue of lane l at [l]
constexpr int XCH = 192;  // u32 exchange words per wave

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// this lane's channel constants (gen_rns_ops.py lane_consts)
struct Lane {
  uint32_t m, c32, cc, mask, negk, k1, pj, minv, k3, mpinv, mpn, k5;
  uint32_t row1[NB], row2[NB];
  __device__ __forceinline__ uint32_t r1(int i) const { return row1[i]; }
  __device__ __forceinline__ uint32_t r2(int j) const { return row2[j]; }
};

// the same constants with the two 15-entry extension rows in LDS (a
// [2 NB][32] table, conflict-free reads): ~30 fewer VGPRs, so two 12-wave
// workgroups fit a CU -- for the throughput kernels (tree levels, tables)
struct LaneL {
  uint32_t m, c32, cc, mask, negk, k1, pj, minv, k3, mpinv, mpn, k5;
  const __attribute__((address_space(3))) uint32_t* rows;
  int ch;
  __device__ __forceinline__ uint32_t r1(int i) const { return rows[i * 32 + ch]; }
  __device__ __forceinline__ uint32_t r2(int j) const { return rows[(NB + j) * 32 + ch]; }
};

__device__ __forceinline__ Lane load_lane() {
  const uint32_t* w = LANE[threadIdx.x & 31];
  Lane L;
  L.m = w[LF_MOD];
  L.c32 = w[LF_C32];
  L.cc = w[LF_CC];
  L.mask = w[LF_ISR] ? 0xffffffffu : 0x0fffffffu;
  L.negk = w[LF_NEGK];
  L.k1 = w[LF_K1];
  L.pj = w[LF_PJ];
  L.minv = w[LF_MINV];
  L.k3 = w[LF_K3];
  L.mpinv = w[LF_MPINV];
  L.mpn = w[LF_MPN];
  L.k5 = w[LF_K5];
#pragma unroll
  for (int i = 0; i < NB; i++) {
    L.row1[i] = w[ROW1_OFF + i];
    L.row2[i] = w[ROW2_OFF + i];
  }
  return L;
}

// rows: 2 NB x 32 u32 of LDS, filled here (the caller's __syncthreads
// publishes them)
__device__ __forceinline__ LaneL load_lane_lds(__attribute__((address_space(3))) uint32_t* rows) {
  for (int i = threadIdx.x; i < 2 * NB * 32; i += blockDim.x) {
    const int r = i >> 5, c = i & 31;
    rows[i] = LANE[c][(r < NB ? ROW1_OFF : ROW2_OFF - NB) + r];
  }
  const uint32_t* w = LANE[threadIdx.x & 31];
  LaneL L;
  L.m = w[LF_MOD];
  L.c32 = w[LF_C32];
  L.cc = w[LF_CC];
  L.mask = w[LF_ISR] ? 0xffffffffu : 0x0fffffffu;
  L.negk = w[LF_NEGK];
  L.k1 = w[LF_K1];
  L.pj = w[LF_PJ];
  L.minv = w[LF_MINV];
  L.k3 = w[LF_K3];
  L.mpinv = w[LF_MPINV];
  L.mpn = w[LF_MPN];
  L.k5 = w[LF_K5];
  L.rows = rows;
  L.ch = threadIdx.x & 31;
  return L;
}

// x mod m (m = 2^28 - c) by folding 2^32 = 16 c twice and 2^28 = c once;
// on the 2^32 channel c32 = cc = m = 0 and mask = ~0, so the same
// instructions return the low word
template <class LT>
__device__ __forceinline__ uint32_t red64(uint64_t x, const LT& L) {
  const uint64_t y = (uint64_t)(uint32_t)(x >> 32) * L.c32 + (uint32_t)x;
  const uint64_t z = (uint64_t)(uint32_t)(y >> 32) * L.c32 + (uint32_t)y;  // < 2^33
  const uint32_t zh = (uint32_t)(z >> 28);
  const uint32_t w = __umul24(zh, L.cc) + ((uint32_t)z & L.mask);
  return w >= L.m ? w - L.m : w;
}

template <class LT>
__device__ __forceinline__ uint32_t red32(uint32_t v, const LT& L) {
  const uint32_t w = __umul24(v >> 28, L.cc) + (v & L.mask);
  return w >= L.m ? w - L.m : w;
}

struct Eng {
  lds_t* slots;  // slot s at slots[s * SLOT + lane]
  lds_t* xch;    // this wave's exchange words
  int kon;       // first constant slot
};

__device__ __forceinline__ void read15(const lds_t* p, uint32_t (&x)[NB]) {
  const lds4_t* q = reinterpret_cast<const lds4_t*>(p);
  const v4u a = q[0], b = q[1], c = q[2], d = q[3];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w;
  x[12] = d.x; x[13] = d.y; x[14] = d.z;
}

// RNS Montgomery reduction of this lane's residue t of T (< 2^16 p^2 * 2):
// returns its residue of (T + q p) / M (< 16 p, = T M^-1 mod p)
template <class LT>
__device__ __forceinline__ uint32_t mont(const Eng& e, const LT& L, uint32_t t) {
  const int lane = threadIdx.x & 63, hb = lane & 32, ch = lane & 31;
  e.xch[lane] = red64((uint64_t)t * L.k1, L);  // B: xi_i
  wave_sync();
  uint32_t xs[NB];
  read15(e.xch + hb, xs);
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NB; i++) acc += (uint64_t)xs[i] * L.r1(i);
  const uint32_t q = red64(acc, L);                      // B', 2^32: q^
  const uint32_t u = red64((uint64_t)q * L.pj + t, L);
  const uint32_t r = red64((uint64_t)u * L.minv, L);     // (t + q^ p) / M
  e.xch[64 + lane] = ch == R_CH ? r : red64((uint64_t)r * L.k3, L);
  wave_sync();
  read15(e.xch + 64 + hb + BP0, xs);
  acc = 0;
#pragma unroll
  for (int j = 0; j < NB; j++) acc += (uint64_t)xs[j] * L.r2(j);
  // 2^32 channel: beta = (sum xi'_j M'_j - r) / M' exactly (< 15)
  if (ch == R_CH) e.xch[128 + (hb >> 5)] = ((uint32_t)acc - r) * L.mpinv;
  const uint32_t s = red64(acc, L);
  wave_sync();
  const uint32_t beta = e.xch[128 + (hb >> 5)];
  const uint32_t rb = red32(s + beta * L.mpn, L);        // s - beta M' (mod m_i)
  return ch < NB ? rb : r;
}

// ---- stages -----------------------------------------------------------------
// output O of op OP: sum of its monomials (term words folded at compile time)
template <int OP, int O, class LT>
__device__ __forceinline__ uint64_t out_terms(const LT& L, const lds_t* pa, const lds_t* pb, const lds_t* pk,
                                              int& dst) {
  constexpr int NT = OP_NT[OP];
  constexpr int BLK = OP_OFF[OP] + 1 + O * (1 + NT);
  dst = (int)PROG[BLK];
  uint64_t acc = 0;
#pragma unroll
  for (int j = 0; j < NT; j++) {
    const uint32_t tw = PROG[BLK + 1 + j];
    if (tw == 0) continue;
    const uint32_t ka = (tw >> 8) & 3, kb = (tw >> 18) & 3;
    const lds_t* sa = ka == 0 ? pa : (ka == 1 ? pb : pk);
    const lds_t* sb = kb == 0 ? pa : (kb == 1 ? pb : pk);
    uint32_t x = sa[(tw & 0xff) * SLOT];
    uint32_t y = sb[((tw >> 10) & 0xff) * SLOT];
    if ((tw >> 20) & 1) y = L.negk - y;
    const uint32_t c = tw >> 24;
    if (c != 1) x *= c;
    acc += (uint64_t)x * y;
  }
  return acc;
}

template <int OP, int O = 0, class LT>
__device__ __forceinline__ uint64_t terms(int w, const LT& L, const lds_t* pa, const lds_t* pb, const lds_t* pk,
                                          int& dst) {
  if constexpr (O + 1 < OP_NO[OP]) {
    if (w != O) return terms<OP, O + 1>(w, L, pa, pb, pk, dst);
  }
  return out_terms<OP, O>(L, pa, pb, pk, dst);
}

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// C/D = OP(A, B): wave w < OP_NO evaluates output coefficient w of both chains;
// the destination registers must not overlap the inputs
// INPLACE: outputs may overwrite inputs (the G2 region ops, a == c): every
// wave finishes its reads before any wave writes
template <int OP, bool INPLACE = false, class LT>
__device__ __forceinline__ void stage(const Eng& e, const LT& L, int a, int b, int c, int d = 0) {
  const int w = wave_id(), lane = threadIdx.x & 63;
  int dst = 0;
  uint64_t acc = 0;
  if (w < OP_NO[OP])
    acc = terms<OP>(w, L, e.slots + a * SLOT + lane, e.slots + b * SLOT + lane, e.slots + e.kon * SLOT + lane, dst);
  if (INPLACE) __syncthreads();
  if (w < OP_NO[OP]) {
    const uint32_t r = mont(e, L, red64(acc, L));
    e.slots[(((dst >> 8) ? d : c) + (dst & 0xff)) * SLOT + lane] = r;
  }
  __syncthreads();
}

// this lane's residue of a field.h Montgomery Fq (12 limbs) as an integer
template <class LT>
__device__ __forceinline__ uint32_t residue(const LT& L, const uint32_t* s) {
  const uint32_t* pw = LANE[threadIdx.x & 31] + POW32_OFF;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) acc += (uint64_t)s[k] * pw[k];
  return red64(acc, L);
}

// slots c .. c+n-1 <- src_h[0 .. n): field.h Montgomery Fq (v = a R < p) into
// the M-domain, times (M/R)^(k-1) for the first of k raw factors: the slot
// gets mont(v * K_LOAD[k]) = a (M/R)^(k-1) M (chain h = lane >> 5 reads src_h)
template <class LT>
__device__ __forceinline__ void load(const Eng& e, const LT& L, const Fq* src0, const Fq* src1, int c, int n,
                                     int k = 1) {
  const int w = wave_id(), lane = threadIdx.x & 63;
  if (w < n) {
    const uint32_t v = residue(L, ((lane & 32) ? src1 : src0)[w].v);
    const uint32_t kin = e.slots[(e.kon + K_LOAD[k]) * SLOT + lane];
    e.slots[(c + w) * SLOT + lane] = mont(e, L, red64((uint64_t)v * kin, L));
  }
  __syncthreads();
}

// raw factor: slots c .. c+n-1 <- the residues of v = a R itself (the
// M-domain element a R / M), no reduction; src_h == nullptr loads field.h's
// one (R mod p) for that chain
template <class LT>
__device__ __forceinline__ void load_raw(const Eng& e, const LT& L, const Fq* src0, const Fq* src1, int c, int n) {
  const int w = wave_id(), lane = threadIdx.x & 63;
  if (w < n) {
    const Fq* src = (lane & 32) ? src1 : src0;
    uint32_t v;
    if (src) {
      v = residue(L, src[w].v);
    } else {
      uint32_t one[12];
#pragma unroll
      for (int k = 0; k < 12; k++) one[k] = w == 0 ? params::FQ_ONE[k] : 0u;
      v = residue(L, one);
    }
    e.slots[(c + w) * SLOT + lane] = v;
  }
  __syncthreads();
}

// r (12 limbs, < 16 p) mod p: a quotient estimate from the top two limbs
// (scaled down so it never exceeds floor(r / p) and is at most one below),
// one q p subtraction, one conditional subtraction
__device__ __forceinline__ void reduce16p(uint32_t (&r)[12]) {
  constexpr double PTOP = (double)params::FQ_P[11] * 4294967296.0 + (double)params::FQ_P[10];
  const double num = (double)r[11] * 4294967296.0 + (double)r[10];
  const uint32_t q = (uint32_t)(num / PTOP * (1.0 - 1e-9));
  uint64_t cp = 0;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint64_t qp = (uint64_t)params::FQ_P[i] * q + cp;
    cp = qp >> 32;
    const int64_t t = (int64_t)r[i] - (int64_t)(uint32_t)qp + br;
    r[i] = (uint32_t)t;
    br = t >> 32;
  }
  uint32_t d[12];
  br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const int64_t t = (int64_t)r[i] - (int64_t)params::FQ_P[i] + br;
    d[i] = (uint32_t)t;
    br = t >> 32;
  }
  if (br == 0) {
#pragma unroll
    for (int i = 0; i < 12; i++) r[i] = d[i];
  }
}

// this wave's two values (one per half, residue x of lane) from the M-domain
// to field.h Montgomery form, canonical (< p), through CRT over base B;
// lane 0 of each half writes its half's dst (no workgroup barrier)
template <class LT>
__device__ __forceinline__ void to_fq_wave(const Eng& e, const LT& L, uint32_t x, Fq* dst0, Fq* dst1) {
  const int lane = threadIdx.x & 63, hb = lane & 32, ch = lane & 31;
  const uint32_t kout = e.slots[(e.kon + K_OUT) * SLOT + lane];
  const uint32_t r = mont(e, L, red64((uint64_t)x * kout, L));  // value R, < 16 p
  // r = sum_i xi_i M_i - alpha M, xi_i = r_i M_i^-1 mod m_i
  e.xch[lane] = red64((uint64_t)r * L.k5, L);
  wave_sync();
  uint32_t xs[NB];
  read15(e.xch + hb, xs);
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NB; i++) acc += (uint64_t)xs[i] * L.r1(i);
  if (ch == R_CH) e.xch[128 + (hb >> 5)] = ((uint32_t)acc - r) * L.minv;  // alpha
  if (ch < 14) {  // column ch of sum_i xi_i M_i
    uint64_t col = 0;
#pragma unroll
    for (int i = 0; i < NB; i++) col += (uint64_t)xs[i] * MI_LIMBS[i][ch];
    e.xch[64 + hb + 2 * ch] = (uint32_t)col;
    e.xch[64 + hb + 2 * ch + 1] = (uint32_t)(col >> 32);
  }
  wave_sync();
  if (ch == 0) {
    const uint32_t alpha = e.xch[128 + (hb >> 5)];
    uint32_t s[15];
    uint64_t cy = 0;
#pragma unroll
    for (int k = 0; k < 14; k++) {
      cy += (uint64_t)e.xch[64 + hb + 2 * k] | ((uint64_t)e.xch[64 + hb + 2 * k + 1] << 32);
      s[k] = (uint32_t)cy;
      cy >>= 32;
    }
    s[14] = (uint32_t)cy;
    uint32_t v[12];
    uint64_t cm = 0;
    int64_t br = 0;
#pragma unroll
    for (int k = 0; k < 14; k++) {
      const uint64_t am = (uint64_t)alpha * M_LIMBS[k] + cm;
      cm = am >> 32;
      const int64_t t = (int64_t)s[k] - (int64_t)(uint32_t)am + br;
      if (k < 12) v[k] = (uint32_t)t;
      br = t >> 32;
    }
    reduce16p(v);
    Fq* d = hb ? dst1 : dst0;
#pragma unroll
    for (int k = 0; k < 12; k++) d->v[k] = v[k];
  }
  wave_sync();  // the exchange words are reused by the next call
}

// dst_h[0 .. n) <- slots a .. a+n-1: M-domain to field.h Montgomery form
template <class LT>
__device__ __forceinline__ void store(const Eng& e, const LT& L, int a, Fq* dst0, Fq* dst1, int n) {
  const int w = wave_id(), lane = threadIdx.x & 63;
  if (w < n) to_fq_wave(e, L, e.slots[(a + w) * SLOT + lane], dst0 + w, dst1 + w);
  __syncthreads();
}

// An Fq12 kept in RNS form between kernels: 12 coefficients x 32 channels of
// one chain (u32), 1.5 KB.  load_res / store_res move slots c .. c+n-1.
constexpr int RES_WORDS = 12 * 32;

// (src_h == nullptr: the M-domain one, constant slot 0)
__device__ __forceinline__ void load_res(const Eng& e, const uint32_t* src0, const uint32_t* src1, int c, int n) {
  const int w = wave_id(), lane = threadIdx.x & 63;
  if (w < n) {
    const uint32_t* src = (lane & 32) ? src1 : src0;
    e.slots[(c + w) * SLOT + lane] =
        src ? src[w * 32 + (lane & 31)] : (w == 0 ? e.slots[e.kon * SLOT + lane] : 0u);
  }
  __syncthreads();
}

__device__ __forceinline__ void store_res(const Eng& e, int a, uint32_t* dst0, uint32_t* dst1, int n) {
  const int w = wave_id(), lane = threadIdx.x & 63;
  if (w < n) ((lane & 32) ? dst1 : dst0)[w * 32 + (lane & 31)] = e.slots[(a + w) * SLOT + lane];
}

// first constant slot count: the chain kernels place the constants at slot 0
__device__ __forceinline__ void load_consts(lds_t* slots) {
  for (int i = threadIdx.x; i < N_CONSTS * SLOT; i += blockDim.x) slots[i] = CONST_RES[i / SLOT][i & 31];
}

}  // namespace rns
}  // namespace tpst
