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

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void put_slot(uint32_t* lds, int slot, const Fq& v) {
  const Fq n = neg(v);
  uint4* d = reinterpret_cast<uint4*>(lds + slot * SLOT);
  d[0] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
  d[1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
  d[2] = make_uint4(v.v[8], v.v[9], v.v[10], v.v[11]);
  d[3] = make_uint4(n.v[0], n.v[1], n.v[2], n.v[3]);
  d[4] = make_uint4(n.v[4], n.v[5], n.v[6], n.v[7]);
  d[5] = make_uint4(n.v[8], n.v[9], n.v[10], n.v[11]);
}

__device__ __forceinline__ Fq get_slot(const uint32_t* lds, int slot) {
  const uint4* s = reinterpret_cast<const uint4*>(lds + slot * SLOT);
  const uint4 a = s[0], b = s[1], c = s[2];
  Fq r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  r.v[8] = c.x; r.v[9] = c.y; r.v[10] = c.z; r.v[11] = c.w;
  return r;
}

// Engine state of one wave: LDS value slots, its product area, constants.
struct Eng {
  uint32_t* lds;
  int prod;  // 64 slots
  int kon;   // N_CONSTS slots (shared, read-only)
};

// sum of coef * slot over the terms of one linear form -> 13 limbs
__device__ __forceinline__ void form(const Eng& e, const uint32_t* blk, uint32_t info, int a, int b,
                                     uint32_t out[13]) {
  uint64_t acc[12];
#pragma unroll
  for (int i = 0; i < 12; i++) acc[i] = 0;
  const uint32_t* t = blk + (info >> 8);
  const int cnt = info & 0xff;
  for (int j = 0; j < cnt; j++) {
    const uint32_t term = t[j];
    const int kind = term & 3;
    const int base = kind == 0 ? a : kind == 1 ? b : kind == 2 ? e.kon : e.prod;
    const uint4* src = reinterpret_cast<const uint4*>(e.lds + (base + ((term >> 8) & 0xff)) * SLOT +
                                                      ((term >> 2) & 1) * 12);
    const uint64_t c = term >> 24;
    const uint4 q0 = src[0], q1 = src[1], q2 = src[2];
    acc[0] += c * q0.x; acc[1] += c * q0.y; acc[2] += c * q0.z; acc[3] += c * q0.w;
    acc[4] += c * q1.x; acc[5] += c * q1.y; acc[6] += c * q1.z; acc[7] += c * q1.w;
    acc[8] += c * q2.x; acc[9] += c * q2.y; acc[10] += c * q2.z; acc[11] += c * q2.w;
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

// one stage: C/D = op(A, B).  C and D must not alias A or B.
__device__ __forceinline__ void run(const Eng& e, const uint32_t* blk, int a, int b, int c, int d = 0) {
  const int lane = threadIdx.x & 63;
  const uint32_t hdr = blk[0];
  const int np = hdr & 0xff, no = (hdr >> 8) & 0xff;
  const bool red = (hdr >> 16) & 1;
  if (lane < np) {
    uint32_t xw[13], yw[13];
    form(e, blk, blk[1 + lane], a, b, xw);
    form(e, blk, blk[1 + np + lane], a, b, yw);
    Fq x, y;
    if (red) {
      x = reduce_wide(xw);
      y = reduce_wide(yw);
    } else {
#pragma unroll
      for (int i = 0; i < 12; i++) {
        x.v[i] = xw[i];
        y.v[i] = yw[i];
      }
    }
    put_slot(e.lds, e.prod + lane, mul(x, y));
  }
  wave_sync();
  if (lane < no) {
    uint32_t w[13];
    form(e, blk, blk[1 + 2 * np + lane], a, b, w);
    const uint32_t dst = blk[1 + 2 * np + no + lane];
    put_slot(e.lds, ((dst >> 8) ? d : c) + (dst & 0xff), reduce_wide(w));
  }
  wave_sync();
}

// cooperative copy of op blocks BLOB[OP_OFF[op] ..) into LDS; returns words used
__device__ __forceinline__ int load_ops(uint32_t* dst, const int* ops, int nops, uint32_t* offs) {
  int o = 0;
  for (int k = 0; k < nops; k++) {
    const int op = ops[k];
    offs[k] = o;
    for (uint32_t i = threadIdx.x; i < OP_LEN[op]; i += blockDim.x) dst[o + i] = BLOB[OP_OFF[op] + i];
    o += OP_LEN[op];
  }
  return o;
}

__device__ __forceinline__ void load_consts(uint32_t* lds, int kon) {
  for (int i = threadIdx.x; i < N_CONSTS; i += blockDim.x) put_slot(lds, kon + i, Fq::from_limbs(CONSTS[i]));
}

// register of 12 slots <- global Fq12 (Montgomery, tower order); lanes 0..11
__device__ __forceinline__ void load_f12(uint32_t* lds, int reg, const Fq12* src) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) put_slot(lds, reg + lane, reinterpret_cast<const Fq*>(src)[lane]);
  wave_sync();
}

__device__ __forceinline__ void store_f12(const uint32_t* lds, int reg, Fq12* dst) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) reinterpret_cast<Fq*>(dst)[lane] = get_slot(lds, reg + lane);
}

__device__ __forceinline__ void set_one(uint32_t* lds, int reg) {
  const int lane = threadIdx.x & 63;
  if (lane < 12) put_slot(lds, reg + lane, lane == 0 ? Fq::one() : Fq::zero());
  wave_sync();
}

}  // namespace wave
}  // namespace tpst
