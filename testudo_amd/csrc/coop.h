// Quad-cooperative XYZZ doubling for the latency-bound doubling chains
// (window combination of a variable-base MSM, fixed-base table powers).
//
// A lone lane pays one wave instruction per limb operation, so a doubling's
// 9 serial Fq products cost ~9 product latencies.  Here the 4 lanes of a quad
// all hold the point; dbl-2008-s-1 (a = 0) is evaluated in three product
// levels with one product per lane per level, and each product is broadcast
// to the quad with a DPP quad_perm move (VALU, no LDS round trip):
//   L1: V = U^2, XX = X^2                      (U = 2Y, M = 3XX)
//   L2: W = U V, S = X V, ZZ' = V ZZ, MM = M^2  (X' = MM - 2S)
//   L3: W Y, ZZZ' = W ZZZ, M (S - X')           (Y' = M (S - X') - W Y)
// 16 independent chains fit one wave.  Additions get the same treatment:
// add-2008-s in four product levels, madd-2008-s in four.
#pragma once
#include "device_util.h"

namespace tpst {

template <int S>
__device__ __forceinline__ uint32_t quad_bcast_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, S | (S << 2) | (S << 4) | (S << 6), 0xF, 0xF, false);
}

// lane S's value of the quad, in every lane of the quad
template <int S, class F>
__device__ __forceinline__ F quad_bcast(const F& v) {
  F r;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* d = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int i = 0; i < Words<F>::n; i++) d[i] = quad_bcast_u32<S>(s[i]);
  return r;
}

// every lane of the quad holds p (quad-uniform control flow); qi = lane & 3
template <class F>
__device__ __forceinline__ Xyzz<F> dbl_quad(const Xyzz<F>& p, int qi) {
  if (is_zero(p.ZZ)) return p;
  const F U = dbl(p.Y);
  const F a1 = qi == 0 ? U : p.X;
  F r = mul(a1, a1);
  const F V = quad_bcast<0>(r), XX = quad_bcast<1>(r);
  const F M = mul3(XX);
  r = mul(qi == 0 ? U : qi == 1 ? p.X : qi == 2 ? p.ZZ : M, qi == 3 ? M : V);
  const F W = quad_bcast<0>(r), S = quad_bcast<1>(r), ZZ3 = quad_bcast<2>(r), MM = quad_bcast<3>(r);
  Xyzz<F> q;
  q.X = sub(MM, dbl(S));
  r = mul(qi == 2 ? M : W, qi == 0 ? p.Y : qi == 1 ? p.ZZZ : sub(S, q.X));
  q.Y = sub(quad_bcast<2>(r), quad_bcast<0>(r));
  q.ZZ = ZZ3;
  q.ZZZ = quad_bcast<1>(r);
  return q;
}

// p + q (add-2008-s), both XYZZ, every lane of the quad holding both
template <class F>
__device__ __forceinline__ Xyzz<F> add_quad(const Xyzz<F>& p, const Xyzz<F>& q, int qi) {
  if (is_zero(q.ZZ)) return p;
  if (is_zero(p.ZZ)) return q;
  // L1: U1 = X1 ZZ2, U2 = X2 ZZ1, S1 = Y1 ZZZ2, S2 = Y2 ZZZ1
  F r = mul(qi == 0 ? p.X : qi == 1 ? q.X : qi == 2 ? p.Y : q.Y,
            qi == 0 ? q.ZZ : qi == 1 ? p.ZZ : qi == 2 ? q.ZZZ : p.ZZZ);
  const F U1 = quad_bcast<0>(r), U2 = quad_bcast<1>(r), S1 = quad_bcast<2>(r), S2 = quad_bcast<3>(r);
  const F P = sub(U2, U1), R = sub(S2, S1);
  if (is_zero(P)) {
    if (is_zero(R)) return dbl_quad(p, qi);
    return Xyzz<F>::inf();
  }
  // L2: PP = P^2, RR = R^2, Z12 = ZZ1 ZZ2, T12 = ZZZ1 ZZZ2
  r = mul(qi == 0 ? P : qi == 1 ? R : qi == 2 ? p.ZZ : p.ZZZ, qi == 0 ? P : qi == 1 ? R : qi == 2 ? q.ZZ : q.ZZZ);
  const F PP = quad_bcast<0>(r), RR = quad_bcast<1>(r), Z12 = quad_bcast<2>(r), T12 = quad_bcast<3>(r);
  // L3: PPP = P PP, Q = U1 PP, ZZ' = Z12 PP
  r = mul(qi == 0 ? P : qi == 1 ? U1 : Z12, PP);
  const F PPP = quad_bcast<0>(r), Q = quad_bcast<1>(r);
  Xyzz<F> o;
  o.ZZ = quad_bcast<2>(r);
  o.X = sub(sub(RR, PPP), dbl(Q));
  // L4: R (Q - X'), S1 PPP, ZZZ' = T12 PPP
  r = mul(qi == 0 ? R : qi == 1 ? S1 : T12, qi == 0 ? sub(Q, o.X) : PPP);
  o.Y = sub(quad_bcast<0>(r), quad_bcast<1>(r));
  o.ZZZ = quad_bcast<2>(r);
  return o;
}

// p + q (madd-2008-s), q affine
template <class F>
__device__ __forceinline__ Xyzz<F> add_affine_quad(const Xyzz<F>& p, const Affine<F>& q, int qi) {
  if (is_inf(q)) return p;
  if (is_zero(p.ZZ)) return {q.x, q.y, F::one(), F::one()};
  // L1: U2 = x2 ZZ1, S2 = y2 ZZZ1
  F r = mul(qi == 0 ? q.x : q.y, qi == 0 ? p.ZZ : p.ZZZ);
  const F P = sub(quad_bcast<0>(r), p.X), R = sub(quad_bcast<1>(r), p.Y);
  if (is_zero(P)) {
    if (is_zero(R)) return dbl_quad(to_xyzz(q), qi);
    return Xyzz<F>::inf();
  }
  // L2: PP = P^2, RR = R^2
  r = mul(qi == 0 ? P : R, qi == 0 ? P : R);
  const F PP = quad_bcast<0>(r), RR = quad_bcast<1>(r);
  // L3: PPP = P PP, Q = X1 PP, ZZ' = ZZ1 PP
  r = mul(qi == 0 ? P : qi == 1 ? p.X : p.ZZ, PP);
  const F PPP = quad_bcast<0>(r), Q = quad_bcast<1>(r);
  Xyzz<F> o;
  o.ZZ = quad_bcast<2>(r);
  o.X = sub(sub(RR, PPP), dbl(Q));
  // L4: R (Q - X'), Y1 PPP, ZZZ' = ZZZ1 PPP
  r = mul(qi == 0 ? R : qi == 1 ? p.Y : p.ZZZ, qi == 0 ? sub(Q, o.X) : PPP);
  o.Y = sub(quad_bcast<0>(r), quad_bcast<1>(r));
  o.ZZZ = quad_bcast<2>(r);
  return o;
}

// double-and-add by a short scalar (k < 2^nbits), quad-cooperative
template <class F>
__device__ __forceinline__ Xyzz<F> scalar_mul_quad(const Xyzz<F>& a, uint32_t k, int nbits, int qi) {
  Xyzz<F> acc = Xyzz<F>::inf();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = dbl_quad(acc, qi);
    if ((k >> i) & 1) acc = add_quad(acc, a, qi);
  }
  return acc;
}

}  // namespace tpst
