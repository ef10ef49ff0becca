// Quad-cooperative elliptic-curve arithmetic for the latency-bound chains of
// the MSM (bucket reduction, window combination) on gfx950.
//
// One XYZZ point operation is spread over the 4 lanes of a DPP quad: every
// lane of the quad holds the same operands, and each "round" runs ONE field
// multiply per lane (lane q of the quad picks its operands), after which the
// four products are exchanged with quad_perm DPP moves (register to register,
// no LDS).  An XYZZ addition (12M + 2S, multiply depth 4) becomes 4 rounds and
// a doubling (7M + 2S, depth 3) 3 rounds, so a lone chain runs ~3x faster than
// on one lane, at the same multiplies per lane-slot.  The additions and
// subtractions between rounds are replicated on the 4 lanes (cheap).
//
// Contract: all 4 lanes of a quad are active and hold identical inputs; the
// results are identical on the 4 lanes.  Special cases (infinity, P == Q,
// P == -Q) branch uniformly within the quad because the data is replicated.
#pragma once
#include "curve.h"

namespace tpst {
namespace quad {

__device__ __forceinline__ int qlane() { return (int)(threadIdx.x & 3); }

// value of lane K of this lane's quad (DPP quad_perm [K,K,K,K])
template <int K>
__device__ __forceinline__ uint32_t bcast_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xf, 0xf, false);
}

template <int K, class C>
__device__ __forceinline__ Fp<C> bcast(const Fp<C>& a) {
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = bcast_u32<K>(a.v[i]);
  return r;
}

template <int K>
__device__ __forceinline__ Fq2 bcast(const Fq2& a) {
  return {bcast<K>(a.c0), bcast<K>(a.c1)};
}

template <class C>
__device__ __forceinline__ Fp<C> sel(int q, const Fp<C>& a0, const Fp<C>& a1, const Fp<C>& a2, const Fp<C>& a3) {
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = q == 0 ? a0.v[i] : q == 1 ? a1.v[i] : q == 2 ? a2.v[i] : a3.v[i];
  return r;
}

__device__ __forceinline__ Fq2 sel(int q, const Fq2& a0, const Fq2& a1, const Fq2& a2, const Fq2& a3) {
  return {sel(q, a0.c0, a1.c0, a2.c0, a3.c0), sel(q, a0.c1, a1.c1, a2.c1, a3.c1)};
}

// one round: lane q computes x_q * y_q; every lane gets all four products
template <class F>
__device__ __forceinline__ void round4(const F& x0, const F& y0, const F& x1, const F& y1, const F& x2, const F& y2,
                                       const F& x3, const F& y3, F& r0, F& r1, F& r2, F& r3) {
  const int q = qlane();
  const F p = mul(sel(q, x0, x1, x2, x3), sel(q, y0, y1, y2, y3));
  r0 = bcast<0>(p);
  r1 = bcast<1>(p);
  r2 = bcast<2>(p);
  r3 = bcast<3>(p);
}

// three products (lane 3 duplicates lane 2)
template <class F>
__device__ __forceinline__ void round3(const F& x0, const F& y0, const F& x1, const F& y1, const F& x2, const F& y2,
                                       F& r0, F& r1, F& r2) {
  F d;
  round4(x0, y0, x1, y1, x2, y2, x2, y2, r0, r1, r2, d);
}

// dbl-2008-s-1 (a = 0): 3 rounds
template <class F>
__device__ __forceinline__ Xyzz<F> dbl(const Xyzz<F>& p) {
  if (is_zero(p.ZZ)) return p;
  const F U = tpst::dbl(p.Y);
  F V, XX, d0, d1;
  round4(U, U, p.X, p.X, U, U, p.X, p.X, V, XX, d0, d1);  // V = U^2, XX = X^2
  const F M = mul3(XX);
  F W, S, ZZ3, MM;
  round4(U, V, p.X, V, V, p.ZZ, M, M, W, S, ZZ3, MM);
  Xyzz<F> r;
  r.X = sub(MM, tpst::dbl(S));
  F t, u, ZZZ3;
  round3(M, sub(S, r.X), W, p.Y, W, p.ZZZ, t, u, ZZZ3);
  r.Y = sub(t, u);
  r.ZZ = ZZ3;
  r.ZZZ = ZZZ3;
  return r;
}

// add-2008-s: 4 rounds
template <class F>
__device__ __forceinline__ Xyzz<F> add(const Xyzz<F>& p, const Xyzz<F>& q) {
  if (is_zero(q.ZZ)) return p;
  if (is_zero(p.ZZ)) return q;
  F U1, U2, S1, S2;
  round4(p.X, q.ZZ, q.X, p.ZZ, p.Y, q.ZZZ, q.Y, p.ZZZ, U1, U2, S1, S2);
  const F P = sub(U2, U1);
  const F R = sub(S2, S1);
  if (is_zero(P)) {
    if (is_zero(R)) return dbl(p);
    return Xyzz<F>::inf();
  }
  F PP, RR, ZZ12, ZZZ12;
  round4(P, P, R, R, p.ZZ, q.ZZ, p.ZZZ, q.ZZZ, PP, RR, ZZ12, ZZZ12);
  F PPP, Q, ZZ3;
  round3(P, PP, U1, PP, ZZ12, PP, PPP, Q, ZZ3);
  Xyzz<F> r;
  r.X = sub(sub(RR, PPP), tpst::dbl(Q));
  F t, u, ZZZ3;
  round3(R, sub(Q, r.X), S1, PPP, ZZZ12, PPP, t, u, ZZZ3);
  r.Y = sub(t, u);
  r.ZZ = ZZ3;
  r.ZZZ = ZZZ3;
  return r;
}

// k * a for a small canonical scalar of nbits bits (double-and-add)
template <class F>
__device__ __forceinline__ Xyzz<F> scalar_mul(const Xyzz<F>& a, uint32_t k, int nbits) {
  Xyzz<F> acc = Xyzz<F>::inf();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = dbl(acc);
    if ((k >> i) & 1) acc = add(acc, a);
  }
  return acc;
}

}  // namespace quad
}  // namespace tpst
