// Pair-distributed Fq2 for the G2 bucket accumulation.
//
// A lane-level Fq2 mixed addition (8 Fq2 products + 2 squares, 30 Fq
// products) keeps ~400 VGPRs of limbs live and runs at one wave per SIMD with
// its Fq2 products out of line and spilled to scratch.  Here the two lanes of
// a pair (2i, 2i+1) hold the two coordinates of every Fq2 value: lane 2i the
// c0 parts, lane 2i+1 the c1 parts of X, Y, ZZ, ZZZ and of the affine input.
// Additions are lane-local; a product exchanges the operands with the partner
// lane (one DPP quad_perm move per limb, no LDS) and each lane forms its own
// coordinate with two Fq products (schoolbook, u^2 = -5):
//   c0 = a0 b0 - 5 a1 b1      (even lane: own x own, partner x partner)
//   c1 = a0 b1 + a1 b0        (odd lane:  own x partner', partner x own')
// so a madd costs 20 Fq products per lane at G1-like register pressure.
// Control flow is pair-uniform (both lanes of a pair follow the same bucket
// chain); is_zero combines the two coordinates' flags.
#pragma once
#include "curve.h"
#include "device_util.h"

namespace tpst {

__device__ __forceinline__ uint32_t pair_swap_u32(uint32_t v) {
  // quad_perm [1, 0, 3, 2]: each lane reads its pair partner
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

__device__ __forceinline__ bool pair_odd() { return (threadIdx.x & 1) != 0; }

struct Fq2P {
  Fq v;  // this lane's coordinate: c0 on even lanes, c1 on odd lanes
  static __device__ __forceinline__ Fq2P zero() { return {Fq::zero()}; }
  static __device__ __forceinline__ Fq2P one() { return {pair_odd() ? Fq::zero() : Fq::one()}; }
};

__device__ __forceinline__ Fq partner(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = pair_swap_u32(a.v[i]);
  return r;
}

__device__ __forceinline__ Fq2P add(const Fq2P& a, const Fq2P& b) { return {add(a.v, b.v)}; }
__device__ __forceinline__ Fq2P sub(const Fq2P& a, const Fq2P& b) { return {sub(a.v, b.v)}; }
__device__ __forceinline__ Fq2P dbl(const Fq2P& a) { return {dbl(a.v)}; }
__device__ __forceinline__ Fq2P neg(const Fq2P& a) { return {neg(a.v)}; }
__device__ __forceinline__ Fq2P mul3(const Fq2P& a) { return {mul3(a.v)}; }

__device__ __forceinline__ Fq2P mul(const Fq2P& a, const Fq2P& b) {
  const bool odd = pair_odd();
  const Fq pa = partner(a.v), pb = partner(b.v);
  const Fq t1 = mul(a.v, odd ? pb : b.v);
  const Fq t2 = mul(pa, odd ? b.v : pb);
  return {odd ? add(t1, t2) : sub(t1, mul5(t2))};
}

__device__ __forceinline__ Fq2P sqr(const Fq2P& a) { return mul(a, a); }

__device__ __forceinline__ bool is_zero(const Fq2P& a) {
  const uint32_t z = is_zero(a.v) ? 1u : 0u;
  return (z & pair_swap_u32(z)) != 0;
}

__device__ __forceinline__ bool eq(const Fq2P& a, const Fq2P& b) {
  const uint32_t e = eq(a.v, b.v) ? 1u : 0u;
  return (e & pair_swap_u32(e)) != 0;
}

// this lane's coordinates of an affine G2 point (Affine<Fq2> layout: x.c0 x.c1 y.c0 y.c1)
__device__ __forceinline__ Affine<Fq2P> load_affine_pair(const uint32_t* base, size_t idx) {
  const uint32_t* p = base + 48 * idx + 12 * (threadIdx.x & 1);
  return {{load_f<Fq>(p)}, {load_f<Fq>(p + 24)}};
}

// Xyzz<Fq2> layout: X.c0 X.c1 Y.c0 Y.c1 ZZ.c0 ZZ.c1 ZZZ.c0 ZZZ.c1
__device__ __forceinline__ Xyzz<Fq2P> load_xyzz_pair(const Xyzz<Fq2>* base, size_t idx) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(base + idx) + 12 * (threadIdx.x & 1);
  return {{load_f<Fq>(p)}, {load_f<Fq>(p + 24)}, {load_f<Fq>(p + 48)}, {load_f<Fq>(p + 72)}};
}

__device__ __forceinline__ void store_xyzz_pair(Xyzz<Fq2>* base, size_t idx, const Xyzz<Fq2P>& v) {
  uint32_t* p = reinterpret_cast<uint32_t*>(base + idx) + 12 * (threadIdx.x & 1);
  store_f<Fq>(p, v.X.v);
  store_f<Fq>(p + 24, v.Y.v);
  store_f<Fq>(p + 48, v.ZZ.v);
  store_f<Fq>(p + 72, v.ZZZ.v);
}

}  // namespace tpst
