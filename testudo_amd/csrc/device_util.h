// Small device/host helpers shared by the HIP translation units: typed
// load/store of field elements and points from flat u32 buffers, error
// plumbing for the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include "curve.h"

namespace tpst {

// number of u32 words of a field element / affine point
template <class F> struct Words;
template <> struct Words<Fq> { static constexpr int n = 12; };
template <> struct Words<Fq2> { static constexpr int n = 24; };
template <> struct Words<Fr> { static constexpr int n = 8; };

template <class F>
__host__ __device__ __forceinline__ F load_f(const uint32_t* p) {
  F r;
  uint32_t* d = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int i = 0; i < Words<F>::n; i++) d[i] = p[i];
  return r;
}

template <class F>
__host__ __device__ __forceinline__ void store_f(uint32_t* p, const F& v) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int i = 0; i < Words<F>::n; i++) p[i] = s[i];
}

// 16-byte vector loads for 96/192-byte affine points (4-dword aligned)
template <class F>
__device__ __forceinline__ Affine<F> load_affine(const uint32_t* base, size_t idx) {
  constexpr int W = 2 * Words<F>::n;
  const uint4* p = reinterpret_cast<const uint4*>(base + idx * W);
  Affine<F> r;
  uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
  for (int i = 0; i < W / 4; i++) d[i] = p[i];
  return r;
}

template <class F>
__device__ __forceinline__ void store_affine(uint32_t* base, size_t idx, const Affine<F>& a) {
  constexpr int W = 2 * Words<F>::n;
  uint4* p = reinterpret_cast<uint4*>(base + idx * W);
  const uint4* s = reinterpret_cast<const uint4*>(&a);
#pragma unroll
  for (int i = 0; i < W / 4; i++) p[i] = s[i];
}

template <class F>
__device__ __forceinline__ Xyzz<F> load_xyzz(const Xyzz<F>* base, size_t idx) {
  constexpr int W = 4 * Words<F>::n;
  const uint4* p = reinterpret_cast<const uint4*>(base + idx);
  Xyzz<F> r;
  uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
  for (int i = 0; i < W / 4; i++) d[i] = p[i];
  return r;
}

template <class F>
__device__ __forceinline__ void store_xyzz(Xyzz<F>* base, size_t idx, const Xyzz<F>& v) {
  constexpr int W = 4 * Words<F>::n;
  uint4* p = reinterpret_cast<uint4*>(base + idx);
  const uint4* s = reinterpret_cast<const uint4*>(&v);
#pragma unroll
  for (int i = 0; i < W / 4; i++) p[i] = s[i];
}

}  // namespace tpst
