// Optimal-ate pairing on BLS12-377, host/device.
//
// Follows ark-ec 0.4 `Bls12::multi_pairing`:
//  * G2Prepared: homogeneous-projective doubling / addition steps on the
//    D-twist that emit line coefficients (c0, c1, c2); ell() multiplies f by
//    the sparse element (c0*py) + (c1*px) w + c2 v w  (mul_by_034).
//  * Miller loop over the bits of x = 0x8508c00000000001 (MSB skipped),
//    63 doubling lines + 6 addition lines = 69 coefficients per G2 point.
//  * Final exponentiation: easy part (p^6-1)(p^2+1), hard part by the
//    eprint 2020/875 chain; total exponent 3(p^12-1)/r (checked against a
//    direct exponentiation in oracle/py/bls377.py).
#pragma once
#include "curve.h"

namespace tpst {

struct LineCoeff {
  Fq2 c0, c1, c2;
};

constexpr int N_LINE_COEFFS = 69;
constexpr int X_BITS = 64;  // bit length of BLS_X

// homogeneous projective point on the twist
struct G2Proj {
  Fq2 x, y, z;
};

TPST_NI LineCoeff g2_double_step(G2Proj& r) {
  const Fq two_inv = Fq::from_limbs(params::FQ_TWO_INV);
  const Fq2 a = mul_fq(mul(r.x, r.y), two_inv);
  const Fq2 b = sqr(r.y);
  const Fq2 c = sqr(r.z);
  const Fq2 e = mul(CurveB<Fq2>::b(), mul3(c));
  const Fq2 f = mul3(e);
  const Fq2 g = mul_fq(add(b, f), two_inv);
  const Fq2 h = sub(sqr(add(r.y, r.z)), add(b, c));
  const Fq2 i = sub(e, b);
  const Fq2 j = sqr(r.x);
  const Fq2 e2 = sqr(e);
  r.x = mul(a, sub(b, f));
  r.y = sub(sqr(g), mul3(e2));
  r.z = mul(b, h);
  return {neg(h), mul3(j), i};
}

TPST_NI LineCoeff g2_add_step(G2Proj& r, const G2A& q) {
  const Fq2 theta = sub(r.y, mul(q.y, r.z));
  const Fq2 lambda = sub(r.x, mul(q.x, r.z));
  const Fq2 c = sqr(theta);
  const Fq2 d = sqr(lambda);
  const Fq2 e = mul(lambda, d);
  const Fq2 f = mul(r.z, c);
  const Fq2 g = mul(r.x, d);
  const Fq2 h = sub(add(e, f), dbl(g));
  r.x = mul(lambda, h);
  r.y = sub(mul(theta, sub(g, h)), mul(e, r.y));
  r.z = mul(r.z, e);
  const Fq2 j = sub(mul(theta, q.x), mul(lambda, q.y));
  return {lambda, neg(theta), j};
}

// Fill out[0..69) with q's line coefficients (stride `stride` LineCoeffs
// between consecutive coefficients, so device code can store them
// coefficient-major).  q must not be infinity.
TPST_NI void g2_prepare(const G2A& q, LineCoeff* out, long stride) {
  G2Proj r = {q.x, q.y, Fq2::one()};
  int idx = 0;
  for (int b = X_BITS - 2; b >= 0; b--) {
    out[(long)idx++ * stride] = g2_double_step(r);
    if ((params::BLS_X >> b) & 1) out[(long)idx++ * stride] = g2_add_step(r, q);
  }
}

TPST_NI Fq12 ell(const Fq12& f, const LineCoeff& c, const G1A& p) {
  return mul_by_034(f, mul_fq(c.c0, p.y), mul_fq(c.c1, p.x), c.c2);
}

// Granger-Scott squaring in the cyclotomic subgroup (valid after the easy
// part of the final exponentiation), as ark-ff Fp12::cyclotomic_square:
// 6 Fq2 products instead of the 12 of a generic Fq12 squaring.
TPST_NI Fq12 cyclotomic_sqr(const Fq12& f) {
  const Fq2 &r0 = f.c0.c0, &r4 = f.c0.c1, &r3 = f.c0.c2, &r2 = f.c1.c0, &r1 = f.c1.c1, &r5 = f.c1.c2;
  Fq2 tmp = mul(r0, r1);
  const Fq2 t0 = sub(sub(mul(add(r0, r1), add(mul_by_u(r1), r0)), tmp), mul_by_u(tmp));
  const Fq2 t1 = dbl(tmp);
  tmp = mul(r2, r3);
  const Fq2 t2 = sub(sub(mul(add(r2, r3), add(mul_by_u(r3), r2)), tmp), mul_by_u(tmp));
  const Fq2 t3 = dbl(tmp);
  tmp = mul(r4, r5);
  const Fq2 t4 = sub(sub(mul(add(r4, r5), add(mul_by_u(r5), r4)), tmp), mul_by_u(tmp));
  const Fq2 t5 = dbl(tmp);
  Fq12 z;
  z.c0.c0 = add(dbl(sub(t0, r0)), t0);  // 3 t0 - 2 r0
  z.c1.c1 = add(dbl(add(t1, r1)), t1);  // 3 t1 + 2 r1
  tmp = mul_by_u(t5);
  z.c1.c0 = add(dbl(add(r2, tmp)), tmp);  // 3 nr(t5) + 2 r2
  z.c0.c2 = add(dbl(sub(t4, r3)), t4);  // 3 t4 - 2 r3
  z.c0.c1 = add(dbl(sub(t2, r4)), t2);  // 3 t2 - 2 r4
  z.c1.c2 = add(dbl(add(t3, r5)), t3);  // 3 t3 + 2 r5
  return z;
}

// f^x for f in the cyclotomic subgroup (x = BLS parameter, positive)
TPST_NI Fq12 exp_by_x(const Fq12& f) {
  Fq12 res = f;
  for (int b = X_BITS - 2; b >= 0; b--) {
    res = cyclotomic_sqr(res);
    if ((params::BLS_X >> b) & 1) res = mul(res, f);
  }
  return res;
}

TPST_NI Fq12 final_exponentiation(const Fq12& f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  Fq12 r = mul(conj(f), inv(f));
  r = mul(frobenius(r, 2), r);
  // hard part, eprint 2020/875 (ark-ec Bls12::final_exponentiation)
  Fq12 y0 = cyclotomic_sqr(r);
  Fq12 y1 = exp_by_x(r);
  Fq12 y2 = conj(r);
  y1 = mul(y1, y2);
  y2 = exp_by_x(y1);
  y1 = conj(y1);
  y1 = mul(y1, y2);
  y2 = exp_by_x(y1);
  y1 = frobenius(y1, 1);
  y1 = mul(y1, y2);
  r = mul(r, y0);
  y0 = exp_by_x(y1);
  y2 = exp_by_x(y0);
  y0 = frobenius(y1, 2);
  y1 = conj(y1);
  y1 = mul(y1, y2);
  y1 = mul(y1, y0);
  r = mul(r, y1);
  return r;
}

// Miller loop for one pair with on-the-fly line coefficients.
TPST_NI Fq12 miller_loop_single(const G1A& p, const G2A& q) {
  if (is_inf(p) || is_inf(q)) return Fq12::one();
  G2Proj r = {q.x, q.y, Fq2::one()};
  Fq12 f = Fq12::one();
  for (int b = X_BITS - 2; b >= 0; b--) {
    f = sqr(f);
    f = ell(f, g2_double_step(r), p);
    if ((params::BLS_X >> b) & 1) f = ell(f, g2_add_step(r, q), p);
  }
  return f;
}

}  // namespace tpst
