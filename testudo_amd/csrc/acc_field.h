// The field the G1 point arithmetic of the throughput and latency kernels
// computes in: field29.h's radix-2^29 Fq (one v_mad_u64_u32 per limb product:
// 66.7 vs 48.3 G products/s chip-wide, 0.91 vs 1.65 us lone-wave latency,
// tools/mb_fq29.py).  Points and XYZZ values stay in memory in field.h's
// layout (arkworks' Montgomery bytes); AccField<F>::in / out convert them as
// a kernel loads and stores them.  G2 (Fq2) computes in its own field.
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

// Compute field of the G1 bucket accumulation: the radix-2^29 Fq of
// field29.h (one v_mad_u64_u32 per limb product, no carry chain); points are
// converted as they are gathered and bucket pieces as they are stored, so
// everything outside the accumulation kernels keeps field.h's layout.  G2
// (Fq2) accumulates in its own field.  TPST_ACC29=0 selects field.h for A/B.
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

}  // namespace tpst
