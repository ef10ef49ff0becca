// The field the G1 point arithmetic of the throughput and latency kernels
// computes in: field29.h's radix-2^29 Fq (one v_mad_u64_u32 per limb product:
// 66.7 vs 48.3 G products/s chip-wide, 0.91 vs 1.65 us lone-wave latency,
// tools/mb_fq29.py).  Points and XYZZ values stay in memory in field.h's
// layout (arkworks' Montgomery bytes); AccField<F>::in / out convert them as
// a kernel loads and stores them.  G2 (Fq2) accumulates in Fq2 over the same
// radix-2^29 Fq (Fq2x29).
// TPST_ACC29=0 selects field.h everywhere (A/B builds).
#pragma once
#include "curve.h"
#include "device_util.h"
#include "field29.h"

namespace tpst {

template <>
struct Words<Fq29> {
  static constexpr int n = 13;
};

// Fq2 = Fq[u]/(u^2 + 5) over field29.h's Fq: the G2 accumulation field
// (the opening's h folds, the G2 MSMs), same formulas as field.h's Fq2
struct Fq2x29 {
  Fq29 c0, c1;
  static TPST_HD Fq2x29 zero() { return {Fq29::zero(), Fq29::zero()}; }
  static TPST_HD Fq2x29 one() { return {Fq29::one(), Fq29::zero()}; }
};
template <>
struct Words<Fq2x29> {
  static constexpr int n = 26;
};
TPST_HD bool is_zero(const Fq2x29& a) { return is_zero(a.c0) && is_zero(a.c1); }
TPST_HD bool eq(const Fq2x29& a, const Fq2x29& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
TPST_HD Fq2x29 add(const Fq2x29& a, const Fq2x29& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
TPST_HD Fq2x29 sub(const Fq2x29& a, const Fq2x29& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
TPST_HD Fq2x29 dbl(const Fq2x29& a) { return {dbl(a.c0), dbl(a.c1)}; }
TPST_HD Fq2x29 neg(const Fq2x29& a) { return {neg(a.c0), neg(a.c1)}; }
TPST_HD Fq2x29 mul3(const Fq2x29& a) { return {mul3(a.c0), mul3(a.c1)}; }
TPST_HD Fq29 mul5(const Fq29& a) { return add(dbl(dbl(a)), a); }
TPST_FQ2_ATTR Fq2x29 mul(const Fq2x29& a, const Fq2x29& b) {
  const Fq29 v0 = mul(a.c0, b.c0);
  const Fq29 v1 = mul(a.c1, b.c1);
  const Fq29 s = mul(add(a.c0, a.c1), add(b.c0, b.c1));
  return {sub(v0, mul5(v1)), sub(sub(s, v0), v1)};
}
TPST_FQ2_ATTR Fq2x29 sqr(const Fq2x29& a) {
  const Fq29 v0 = mul(a.c0, a.c1);
  const Fq29 t = mul(add(a.c0, a.c1), sub(a.c0, mul5(a.c1)));
  return {add(t, dbl(dbl(v0))), dbl(v0)};
}
TPST_HD Fq2x29 from_std(const Fq2& a) { return {from_std(a.c0), from_std(a.c1)}; }
TPST_HD Fq2 to_std(const Fq2x29& a) { return {to_std(a.c0), to_std(a.c1)}; }

// Compute field of the G1 bucket accumulation: the radix-2^29 Fq of
// field29.h (one v_mad_u64_u32 per limb product, no carry chain); points are
// converted as they are gathered and bucket pieces as they are stored, so
// everything outside the accumulation kernels keeps field.h's layout.
// TPST_ACC29=0 selects field.h for A/B.
template <class F>
struct AccField {
  using T = F;
  static __device__ __forceinline__ Affine<T> in(const Affine<F>& a) { return a; }
  static __device__ __forceinline__ Xyzz<T> in(const Xyzz<F>& a) { return a; }
  static __device__ __forceinline__ Xyzz<F> out(const Xyzz<T>& a) { return a; }
};
#ifndef TPST_ACC29
#define TPST_ACC29 1
#endif
#if TPST_ACC29
template <>
struct AccField<Fq> {
  using T = Fq29;
  static __device__ __forceinline__ Affine<T> in(const Affine<Fq>& a) { return {from_std(a.x), from_std(a.y)}; }
  static __device__ __forceinline__ Xyzz<T> in(const Xyzz<Fq>& a) {
    return {from_std(a.X), from_std(a.Y), from_std(a.ZZ), from_std(a.ZZZ)};
  }
  static __device__ __forceinline__ Xyzz<Fq> out(const Xyzz<T>& a) {
    return {to_std(a.X), to_std(a.Y), to_std(a.ZZ), to_std(a.ZZZ)};
  }
};
template <>
struct AccField<Fq2> {
  using T = Fq2x29;
  static __device__ __forceinline__ Affine<T> in(const Affine<Fq2>& a) { return {from_std(a.x), from_std(a.y)}; }
  static __device__ __forceinline__ Xyzz<T> in(const Xyzz<Fq2>& a) {
    return {from_std(a.X), from_std(a.Y), from_std(a.ZZ), from_std(a.ZZZ)};
  }
  static __device__ __forceinline__ Xyzz<Fq2> out(const Xyzz<T>& a) {
    return {to_std(a.X), to_std(a.Y), to_std(a.ZZ), to_std(a.ZZZ)};
  }
};
#endif

// bucket / piece / segment values live in memory in field.h's layout; the
// tail kernels (fixups, weighted reductions, window chains) compute in the
// accumulation field too: 45 % lower lone-lane product latency (0.91 vs
// 1.65 us, tools/mb_fq29.py) on their serial chains
template <class F>
__device__ __forceinline__ Xyzz<typename AccField<F>::T> load_acc(const Xyzz<F>* p, size_t i) {
  return AccField<F>::in(load_xyzz(p, i));
}
template <class F>
__device__ __forceinline__ void store_acc(Xyzz<F>* p, size_t i, const Xyzz<typename AccField<F>::T>& v) {
  store_xyzz(p, i, AccField<F>::out(v));
}

// Buckets, parked pieces and block partials of the accumulation kernels
// (written and read only by msm.hip's accumulation / fixup / first reduction
// kernels): for G1 the accumulation field's own Montgomery values packed bit
// for bit (field29.h pack377; 12 words per coordinate like field.h, so buffer
// sizes and the all-zero infinity are unchanged).  The accumulation loops
// store a bucket every few mixed adds, and the conversion to field.h
// (to_std: ~190 VALU per coordinate, run by the whole wave whenever one lane
// ends a bucket) was ~6 % of K2's and ~10 % of K1's issue slots.  G2 keeps
// field.h's layout.
template <class F>
__device__ __forceinline__ Xyzz<typename AccField<F>::T> load_pk(const Xyzz<F>* p, size_t i) {
  return load_acc(p, i);
}
template <class F>
__device__ __forceinline__ void store_pk(Xyzz<F>* p, size_t i, const Xyzz<typename AccField<F>::T>& v) {
  store_acc(p, i, v);
}
#if TPST_ACC29
template <>
__device__ __forceinline__ Xyzz<Fq29> load_pk<Fq>(const Xyzz<Fq>* p, size_t i) {
  const Xyzz<Fq> w = load_xyzz(p, i);
  return {unpack377(w.X.v), unpack377(w.Y.v), unpack377(w.ZZ.v), unpack377(w.ZZZ.v)};
}
template <>
__device__ __forceinline__ void store_pk<Fq>(Xyzz<Fq>* p, size_t i, const Xyzz<Fq29>& v) {
  Xyzz<Fq> w;
  pack377(v.X, w.X.v);
  pack377(v.Y, w.Y.v);
  pack377(v.ZZ, w.ZZ.v);
  pack377(v.ZZZ, w.ZZZ.v);
  store_xyzz(p, i, w);
}
#endif

}  // namespace tpst
