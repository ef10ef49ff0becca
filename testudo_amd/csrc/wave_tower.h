// Wave-cooperative Fq12 arithmetic for the latency-bound pairing chains.
//
// A lone lane running an Fq12 chain pays a full wave instruction for every
// limb operation (~1.6 us per Fq product on gfx950, whatever the number of
// active lanes).  Here one wave evaluates one tower operation as a "stage"
// whose independent Fq products run one per lane (tools/gen_wave_ops.py
// derives the linear forms from the field.h formulas and checks them against
// the oracle):
//
//   phase 1  lane i < np : x_i, y_i = small-integer combinations of the input
//                          slots, p_i = x_i * y_i (Montgomery)  -> PROD[i]
//   phase 2  lane k < no : out_k = combination of PROD and input slots,
//                          reduced mod p                       -> C / D slot
//
// Values live in LDS "slots" of 24 u32: the element (< p) and its negation,
// so negative coefficients are plain additions.  Linear forms accumulate in
// 64-bit limbs with one v_mad_u64_u32 per limb and term; the final value
// (< 1024 p) is reduced with a floating-point quotient estimate and a single
// q*p subtraction.  Operands: A, B (input registers), K (constants), P.
#pragma once
#include "field.h"

#if defined(__HIPCC__)
#define TPST_WAVE_CONST __constant__ const
#else
#define TPST_WAVE_CONST const
#endif
#include "wave_ops.inc"

namespace tpst {
namespace wave {

constexpr int SLOT = 24;  // u32 per slot: x, then p - x

// explicit LDS address space: the engine's helpers are not all inlined into
// the kernels, and a generic pointer would turn every slot access into a
// flat (vector-memory) access
typedef __attribute__((address_space(3))) uint32_t lds_t;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u lds4_t;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void put_slot(lds_t* lds, int slot, const Fq& v) {
  const Fq n = neg(v);
  lds4_t* d = reinterpret_cast<lds4_t*>(lds + slot * SLOT);
  d[0] = v4u{v.v[0], v.v[1], v.v[2], v.v[3]};
  d[1] = v4u{v.v[4], v.v[5], v.v[6], v.v[7]};
  d[2] = v4u{v.v[8], v.v[9], v.v[10], v.v[11]};
  d[3] = v4u{n.v[0], n.v[1], n.v[2], n.v[3]};
  d[4] = v4u{n.v[4], n.v[5], n.v[6], n.v[7]};
  d[5] = v4u{n.v[8], n.v[9], n.v[10], n.v[11]};
}

__device__ __forceinline__ Fq get_slot(const lds_t* lds, int slot) {
  const lds4_t* s = reinterpret_cast<const lds4_t*>(lds + slot * SLOT);
  const v4u a = s[0], b = s[1], c = s[2];
  Fq r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  r.v[8] = c.x; r.v[9] = c.y; r.v[10] = c.z; r.v[11] = c.w;
  return r;
}

// Engine state of one wave: LDS value slots, its product area, constants.
struct Eng {
  lds_t* lds;
  int prod;  // 64 slots
  int kon;   // N_CONSTS slots (shared, read-only)
};

// operand bases of a stage packed as 4 x 16 bits (A, B, K, P) so the term
// decode is a shift, not a divergent branch
__device__ __forceinline__ uint64_t pack_bases(const Eng& e, int a, int b) {
  return (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 16) | ((uint64_t)(uint32_t)e.kon << 32) |
         ((uint64_t)(uint32_t)e.prod << 48);
}

__device__ __forceinline__ void fetch_term(const Eng& e, uint32_t term, uint64_t bases, v4u& q0, v4u& q1, v4u& q2,
                                           uint32_t& c) {
  const uint32_t base = (uint32_t)(bases >> (16 * (term & 3))) & 0xffffu;
  const lds4_t* src = reinterpret_cast<const lds4_t*>(e.lds + (base + ((term >> 8) & 0xff)) * SLOT + (term & 4) * 3);
  q0 = src[0];
  q1 = src[1];
  q2 = src[2];
  c = term >> 24;
}

// sum of coef * slot over the `cnt` terms of one linear form -> 13 limbs.
// Term j of this lane is t[j * stride]; cnt is wave-uniform (lists padded
// with zero terms), so the term words and then every term's slot are
// fetched up front.  One v_mad_u64_u32 per limb and term (coefficients < 256).
__device__ __forceinline__ void form(const Eng& e, const lds_t* t, int stride, int cnt, uint64_t bases,
                                     uint32_t out[13]) {
  uint32_t tw[8];
#pragma unroll
  for (int j = 0; j < 8; j++) tw[j] = j < cnt ? t[j * stride] : 0u;
  uint64_t acc[12];
#pragma unroll
  for (int i = 0; i < 12; i++) acc[i] = 0;
  // every term's slot is read before the first multiply-add: the engine runs
  // one wave per chain, so the LDS reads overlap each other instead of each
  // term waiting out a full LDS round trip (the VGPRs are free at this
  // occupancy)
  v4u q0[8], q1[8], q2[8];
  uint32_t c[8];
#pragma unroll
  for (int j = 0; j < 8; j++)
    if (j < cnt) fetch_term(e, tw[j], bases, q0[j], q1[j], q2[j], c[j]);
#pragma unroll
  for (int j = 0; j < 8; j++) {
    if (j < cnt) {
      const uint32_t cj = c[j];
      acc[0] += (uint64_t)cj * q0[j].x; acc[1] += (uint64_t)cj * q0[j].y;
      acc[2] += (uint64_t)cj * q0[j].z; acc[3] += (uint64_t)cj * q0[j].w;
      acc[4] += (uint64_t)cj * q1[j].x; acc[5] += (uint64_t)cj * q1[j].y;
      acc[6] += (uint64_t)cj * q1[j].z; acc[7] += (uint64_t)cj * q1[j].w;
      acc[8] += (uint64_t)cj * q2[j].x; acc[9] += (uint64_t)cj * q2[j].y;
      acc[10] += (uint64_t)cj * q2[j].z; acc[11] += (uint64_t)cj * q2[j].w;
    }
  }
  uint64_t cr = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    cr += acc[i];
    out[i] = (uint32_t)cr;
    cr >>= 32;
  }
  out[12] = (uint32_t)cr;
}

// v (< 1024 p, 13 limbs) mod p
__device__ __forceinline__ Fq reduce_wide(const uint32_t v[13]) {
  const double top = (double)v[12] * 18446744073709551616.0 + (double)v[11] * 4294967296.0 + (double)v[10];
  const double qd = top * INV_P320 - 1e-6;
  const uint32_t q = qd > 0.0 ? (uint32_t)qd : 0u;
  Fq r;
  uint64_t c = 0;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint64_t t = (uint64_t)q * params::FQ_P[i] + c;
    c = t >> 32;
    const int64_t d = (int64_t)v[i] - (int64_t)(uint32_t)t + br;
    r.v[i] = (uint32_t)d;
    br = d >> 32;
  }
  reduce_once(r);
  return r;
}

// The stage's Fq product runs in field29.h's radix 2^29 (0.91 vs 1.65 us
// lone-wave latency): operands converted on the way in -- a form left
// unreduced is < 64 p, so (x + k p) / 2^7 < 1.5 p stays in 13 x 29 bits --
// and the product (reduced below p) back to
// field.h's canonical form on the way out.  TPST_WAVE29=0 keeps field.h's
// product (A/B).
#ifndef TPST_WAVE29
#define TPST_WAVE29 1
#endif
__device__ __forceinline__ Fq stage_mul(const Fq& x, const Fq& y) {
#if TPST_WAVE29
  // one operand up to 64 p (the other < p): the product is < 2.26 p before
  // mul's conditional subtraction, so one more brings it below p for to_std
  Fq29 r = mul(from_std(x), from_std(y));
  reduce_once(r);
  return to_std(r);
#else
  return mul(x, y);
#endif
}
__device__ __forceinline__ Fq stage_sqr(const Fq& x) {
#if TPST_WAVE29
  return to_std(sqr(from_std(x)));
#else
  return sqr(x);
#endif
}

// one stage: C/D = op(A, B).
// block: [hdr0 = np | no << 8 | red << 16 | sq << 17 | nc << 24, hdr1 = TX | TY << 8 | TC << 16,
//         X terms (TX x np, term-major), Y terms (TY x np), chunk terms (TC x nc),
//         out[no] = first chunk << 8 | chunks, dst[no]]
// Output forms longer than a few terms are split into chunks summed by
// separate lanes (their 13-limb partials parked in the product area, which
// phase 2a has finished reading), then combined and reduced per output.
__device__ __forceinline__ void run(const Eng& e, const lds_t* blk, int a, int b, int c, int d = 0) {
  const int lane = threadIdx.x & 63;
  const uint32_t hdr = __builtin_amdgcn_readfirstlane(blk[0]);
  const uint32_t hdr1 = __builtin_amdgcn_readfirstlane(blk[1]);
  const int np = hdr & 0xff, no = (hdr >> 8) & 0xff, nc = hdr >> 24;
  const int tx = hdr1 & 0xff, ty = (hdr1 >> 8) & 0xff, tc = (hdr1 >> 16) & 0xff;
  const bool red = (hdr >> 16) & 1;
  const bool sq = (hdr >> 17) & 1;  // every product a square: no Y forms (wave-uniform)
  const uint64_t bases = pack_bases(e, a, b);
  const lds_t* X = blk + 2;
  const lds_t* Y = X + tx * np;
  const lds_t* CH = Y + ty * np;
  const lds_t* O = CH + tc * nc;
  const lds_t* DST = O + no;
  if (lane < np) {
    uint32_t xw[13];
    form(e, X + lane, np, tx, bases, xw);
    Fq x;
    if (red) {
      x = reduce_wide(xw);
    } else {
#pragma unroll
      for (int i = 0; i < 12; i++) x.v[i] = xw[i];
    }
    if (sq) {
      put_slot(e.lds, e.prod + lane, stage_sqr(x));
    } else {
      uint32_t yw[13];
      form(e, Y + lane, np, ty, bases, yw);
      Fq y;
      if (red) {
        y = reduce_wide(yw);
      } else {
#pragma unroll
        for (int i = 0; i < 12; i++) y.v[i] = yw[i];
      }
      put_slot(e.lds, e.prod + lane, stage_mul(x, y));
    }
  }
  wave_sync();
  if (nc == no) {
    if (lane < no) {
      uint32_t w[13];
      form(e, CH + lane, nc, tc, bases, w);
      const uint32_t dst = DST[lane];
      put_slot(e.lds, ((dst >> 8) ? d : c) + (dst & 0xff), reduce_wide(w));
    }
  } else {
    uint32_t w[13];
    if (lane < nc) form(e, CH + lane, nc, tc, bases, w);
    wave_sync();
    lds4_t* part = reinterpret_cast<lds4_t*>(e.lds + e.prod * SLOT);  // 16 u32 per chunk
    if (lane < nc) {
      part[4 * lane + 0] = v4u{w[0], w[1], w[2], w[3]};
      part[4 * lane + 1] = v4u{w[4], w[5], w[6], w[7]};
      part[4 * lane + 2] = v4u{w[8], w[9], w[10], w[11]};
      part[4 * lane + 3] = v4u{w[12], 0, 0, 0};
    }
    wave_sync();
    if (lane < no) {
      const uint32_t o = O[lane];
      const int first = o >> 8, n = o & 0xff;
      uint32_t v[13];
#pragma unroll
      for (int i = 0; i < 13; i++) v[i] = 0;
      for (int j = 0; j < n; j++) {
        const lds4_t* q = part + 4 * (first + j);
        const v4u q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
        const uint32_t s[13] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x};
        uint64_t cr = 0;
#pragma unroll
        for (int i = 0; i < 13; i++) {
          cr += (uint64_t)v[i] + s[i];
          v[i] = (uint32_t)cr;
          cr >>= 32;
        }
      }
      const uint32_t dst = DST[lane];
      put_slot(e.lds, ((dst >> 8) ? d : c) + (dst & 0xff), reduce_wide(v));
    }
  }
  wave_sync();
}

// A fixed list of ops copied to LDS, offsets known at compile time.
template <int N>
struct OpSet {
  int op[N];
  uint32_t off[N];
  int words;
  constexpr OpSet(const int (&ops)[N]) : op(), off(), words(0) {
    for (int i = 0; i < N; i++) {
      op[i] = ops[i];
      off[i] = (uint32_t)words;
      words += (int)OP_LEN[ops[i]];
    }
    words = (words + 3) & ~3;
  }
};

template <int N>
__device__ __forceinline__ void load_set(lds_t* dst, const OpSet<N>& set) {
#pragma unroll
  for (int k = 0; k < N; k++)
    for (uint32_t i = threadIdx.x; i < OP_LEN[set.op[k]]; i += blockDim.x)
      dst[set.off[k] + i] = BLOB[OP_OFF[set.op[k]] + i];
}

__device__ __forceinline__ void load_consts(lds_t* lds, int kon) {
  for (int i = threadIdx.x; i < N_CONSTS; i += blockDim.x) put_slot(lds, kon + i, Fq::from_limbs(CONSTS[i]));
}

// register of 12 slots <- global Fq12 (Montgomery, tower order); lanes 0..11
__device__ __forceinline__ void load_f12(lds_t* lds, int reg, const Fq12* src) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) put_slot(lds, reg + lane, reinterpret_cast<const Fq*>(src)[lane]);
  wave_sync();
}

__device__ __forceinline__ void store_f12(const lds_t* lds, int reg, Fq12* dst) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) reinterpret_cast<Fq*>(dst)[lane] = get_slot(lds, reg + lane);
}

__device__ __forceinline__ void set_one(lds_t* lds, int reg) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) put_slot(lds, reg + lane, lane == 0 ? Fq::one() : Fq::zero());
  wave_sync();
}

}  // namespace wave
}  // namespace tpst
