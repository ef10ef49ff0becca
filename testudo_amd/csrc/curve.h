// BLS12-377 G1 (over Fq, y^2 = x^3 + 1) and G2 (over Fq2, D-twist
// y^2 = x^3 + 1/u) point arithmetic, shared by host and device code.
//
// Representations:
//   Affine<F>  : (x, y); the point at infinity is x = y = 0 (not on either
//                curve), which is also what the C-ABI uses (include/tpst.h).
//   Xyzz<F>    : (X, Y, ZZ, ZZZ) with x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2;
//                infinity iff ZZ == 0.  Used by every bucket accumulator:
//                mixed add = 8M + 2S, no inversion.
//   Jac<F>     : Jacobian (X, Y, Z), used by scalar multiplication chains.
#pragma once
#include "field.h"

namespace tpst {

template <class F> struct CurveB;
template <> struct CurveB<Fq> {
  static TPST_HD Fq b() { return Fq::one(); }
  static TPST_HD Fq b3() { return mul3(Fq::one()); }
};
template <> struct CurveB<Fq2> {
  static TPST_HD Fq2 b() { return fq2_const(params::G2_B); }
  static TPST_HD Fq2 b3() { return fq2_const(params::G2_B3); }
};

template <class F>
struct Affine {
  F x, y;
  static TPST_HD Affine inf() { return {F::zero(), F::zero()}; }
};

template <class F>
TPST_HD bool is_inf(const Affine<F>& a) { return is_zero(a.x) && is_zero(a.y); }

template <class F>
struct Xyzz {
  F X, Y, ZZ, ZZZ;
  static TPST_HD Xyzz inf() { return {F::one(), F::one(), F::zero(), F::zero()}; }
};

template <class F>
TPST_HD bool is_inf(const Xyzz<F>& a) { return is_zero(a.ZZ); }

template <class F>
struct Jac {
  F X, Y, Z;
  static TPST_HD Jac inf() { return {F::one(), F::one(), F::zero()}; }
};

template <class F>
TPST_HD bool is_inf(const Jac<F>& a) { return is_zero(a.Z); }

using G1A = Affine<Fq>;
using G2A = Affine<Fq2>;

template <class F>
TPST_HD Affine<F> neg(const Affine<F>& a) {
  if (is_inf(a)) return a;
  return {a.x, neg(a.y)};
}

template <class F>
TPST_NI bool on_curve(const Affine<F>& a) {
  if (is_inf(a)) return true;
  return eq(sqr(a.y), add(mul(sqr(a.x), a.x), CurveB<F>::b()));
}

// --------------------------------------------------------------- XYZZ ----
// a b - c d; field29.h overloads it for Fq29 with one Montgomery reduction
template <class F>
TPST_HD F mul_sub(const F& a, const F& b, const F& c, const F& d) {
  return sub(mul(a, b), mul(c, d));
}

// dbl-2008-s-1 (a = 0)
template <class F>
TPST_HD Xyzz<F> dbl(const Xyzz<F>& p) {
  if (is_zero(p.ZZ)) return p;
  const F U = dbl(p.Y);
  const F V = sqr(U);
  const F W = mul(U, V);
  const F S = mul(p.X, V);
  const F M = mul3(sqr(p.X));
  Xyzz<F> r;
  r.X = sub(sqr(M), dbl(S));
  r.Y = mul_sub(M, sub(S, r.X), W, p.Y);
  r.ZZ = mul(V, p.ZZ);
  r.ZZZ = mul(W, p.ZZZ);
  return r;
}

// mdbl-2008-s-1: double an affine point into XYZZ
template <class F>
TPST_HD Xyzz<F> dbl_affine(const Affine<F>& q) {
  if (is_inf(q)) return Xyzz<F>::inf();
  const F U = dbl(q.y);
  const F V = sqr(U);
  const F W = mul(U, V);
  const F S = mul(q.x, V);
  const F M = mul3(sqr(q.x));
  Xyzz<F> r;
  r.X = sub(sqr(M), dbl(S));
  r.Y = mul_sub(M, sub(S, r.X), W, q.y);
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// madd-2008-s: p + q (q affine)
template <class F>
TPST_HD Xyzz<F> add_affine(const Xyzz<F>& p, const Affine<F>& q) {
  if (is_inf(q)) return p;
  if (is_zero(p.ZZ)) return {q.x, q.y, F::one(), F::one()};
  const F U2 = mul(q.x, p.ZZ);
  const F S2 = mul(q.y, p.ZZZ);
  const F P = sub(U2, p.X);
  const F R = sub(S2, p.Y);
  if (is_zero(P)) {
    if (is_zero(R)) return dbl_affine(q);
    return Xyzz<F>::inf();
  }
  const F PP = sqr(P);
  const F PPP = mul(P, PP);
  const F Q = mul(p.X, PP);
  Xyzz<F> r;
  r.X = sub(sub(sqr(R), PPP), dbl(Q));
  r.Y = mul_sub(R, sub(Q, r.X), p.Y, PPP);
  r.ZZ = mul(p.ZZ, PP);
  r.ZZZ = mul(p.ZZZ, PPP);
  return r;
}

template <class F>
TPST_HD Xyzz<F> sub_affine(const Xyzz<F>& p, const Affine<F>& q) { return add_affine(p, neg(q)); }

// add-2008-s: p + q (both XYZZ)
template <class F>
TPST_HD Xyzz<F> add(const Xyzz<F>& p, const Xyzz<F>& q) {
  if (is_zero(q.ZZ)) return p;
  if (is_zero(p.ZZ)) return q;
  const F U1 = mul(p.X, q.ZZ);
  const F U2 = mul(q.X, p.ZZ);
  const F S1 = mul(p.Y, q.ZZZ);
  const F S2 = mul(q.Y, p.ZZZ);
  const F P = sub(U2, U1);
  const F R = sub(S2, S1);
  if (is_zero(P)) {
    if (is_zero(R)) return dbl(p);
    return Xyzz<F>::inf();
  }
  const F PP = sqr(P);
  const F PPP = mul(P, PP);
  const F Q = mul(U1, PP);
  Xyzz<F> r;
  r.X = sub(sub(sqr(R), PPP), dbl(Q));
  r.Y = mul_sub(R, sub(Q, r.X), S1, PPP);
  r.ZZ = mul(mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = mul(mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}

template <class F>
TPST_HD Xyzz<F> neg(const Xyzz<F>& p) { return {p.X, neg(p.Y), p.ZZ, p.ZZZ}; }

template <class F>
TPST_HD Affine<F> to_affine(const Xyzz<F>& p) {
  if (is_zero(p.ZZ)) return Affine<F>::inf();
  const F t = inv(mul(p.ZZ, p.ZZZ));
  const F izz = mul(t, p.ZZZ);   // 1/ZZ
  const F izzz = mul(t, p.ZZ);   // 1/ZZZ
  return {mul(p.X, izz), mul(p.Y, izzz)};
}

template <class F>
TPST_HD Xyzz<F> to_xyzz(const Affine<F>& a) {
  if (is_inf(a)) return Xyzz<F>::inf();
  return {a.x, a.y, F::one(), F::one()};
}

template <class F>
TPST_NI bool eq(const Xyzz<F>& a, const Xyzz<F>& b) {
  if (is_zero(a.ZZ) || is_zero(b.ZZ)) return is_zero(a.ZZ) && is_zero(b.ZZ);
  return eq(mul(a.X, b.ZZ), mul(b.X, a.ZZ)) && eq(mul(a.Y, b.ZZZ), mul(b.Y, a.ZZZ));
}

// Double-and-add scalar multiplication by a canonical little-endian scalar of
// `nbits` bits held in 32-bit words.  Used for the small per-element products
// (MIPP compress, SRS setup, verifier), not for MSMs.
template <class F>
TPST_HD Xyzz<F> scalar_mul(const Affine<F>& a, const uint32_t* k, int nbits) {
  Xyzz<F> acc = Xyzz<F>::inf();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1) acc = add_affine(acc, a);
  }
  return acc;
}

template <class F>
TPST_HD Xyzz<F> scalar_mul_xyzz(const Xyzz<F>& a, const uint32_t* k, int nbits) {
  Xyzz<F> acc = Xyzz<F>::inf();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1) acc = add(acc, a);
  }
  return acc;
}

}  // namespace tpst
