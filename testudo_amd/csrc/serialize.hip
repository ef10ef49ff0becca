// arkworks wire format (ark-serialize 0.4, Compress::Yes) of the sqrt-PST
// objects: Commitment, Proof, MippProof (mipp.rs:21-28, derive
// CanonicalSerialize), CommitterKey -- the byte strings whose lengths are the
// proof_size / commiter_key_size columns of benches/pst.rs:43-46,64-74.
// Host-only code (no device work): the proof is a few KB.
//
// Restated encoding rules (ark-serialize / ark-ff / ark-ec 0.4):
//  * Fp: canonical value, little-endian, buffer_byte_size(MODULUS_BIT_SIZE +
//    flag bits) bytes (Fq: 48, Fr: 32); flags OR-ed into the top bits of the
//    last byte.  Fq2 = c0 || c1 with the flags on c1; Fq12 = its 12 Fq
//    coefficients in tower order (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...), no flags.
//  * short-Weierstrass affine, compressed: x with SWFlags -- bit 7 =
//    YIsNegative (y > -y in the field order; Fq2 orders by c1, then c0),
//    bit 6 = PointAtInfinity (x = 0), both set is invalid.  Deserialisation
//    takes y = the smaller square root of x^3 + b when the sign bit is clear,
//    then checks on-curve and the prime-order subgroup (Validate::Yes).
//  * usize as u64 LE; Vec<T> = u64 LE length || elements; tuples and structs
//    field by field in declaration order.
// Parity: restated from the published crates (not vendored here, no Rust
// toolchain), cross-checked against the independent Python restatement in
// oracle/py/serialize.py -- parity unpinned against arkworks itself.
#include <cstring>
#include <vector>

#include "../../include/tpst.h"
#include "curve.h"

using namespace tpst;

namespace {

typedef unsigned __int128 u128;

bool lt_p(const uint64_t* a) {  // a < p (canonical Fq)
  for (int i = 5; i >= 0; i--) {
    const uint64_t pi = (uint64_t)params::FQ_P[2 * i] | ((uint64_t)params::FQ_P[2 * i + 1] << 32);
    if (a[i] != pi) return a[i] < pi;
  }
  return false;
}

Fq fq_in(const uint64_t* c) {
  Fq a;
  memcpy(a.v, c, 48);
  return to_mont(a);
}
void fq_out(const Fq& a, uint64_t* c) {
  const Fq r = from_mont(a);
  memcpy(c, r.v, 48);
}

// canonical compare of two Fq (Montgomery in)
int fq_cmp(const Fq& a, const Fq& b) {
  uint64_t x[6], y[6];
  fq_out(a, x);
  fq_out(b, y);
  for (int i = 5; i >= 0; i--)
    if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
  return 0;
}
bool neg_flag(const Fq& y) { return fq_cmp(y, neg(y)) > 0; }
bool neg_flag(const Fq2& y) {  // QuadExtField Ord: c1 first, then c0
  const Fq2 n = neg(y);
  const int c = fq_cmp(y.c1, n.c1);
  return c != 0 ? c > 0 : fq_cmp(y.c0, n.c0) > 0;
}

// ---- exponentiation and square roots over Fq (p - 1 = 2^46 q) ----
struct BigE {
  uint64_t w[6];
};
BigE p_minus(uint64_t k) {
  BigE e;
  for (int i = 0; i < 6; i++) e.w[i] = (uint64_t)params::FQ_P[2 * i] | ((uint64_t)params::FQ_P[2 * i + 1] << 32);
  e.w[0] -= k;  // p's low limb is 1: no borrow for k <= 1
  return e;
}
BigE shr(BigE e, int s) {
  for (int k = 0; k < s; k++)
    for (int i = 0; i < 6; i++) e.w[i] = (e.w[i] >> 1) | (i < 5 ? e.w[i + 1] << 63 : 0);
  return e;
}
Fq fq_pow(const Fq& a, const BigE& e) {
  Fq r = Fq::one();
  for (int i = 5; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = sqr(r);
      if ((e.w[i] >> b) & 1) r = mul(r, a);
    }
  return r;
}
constexpr int TWO_ADICITY = 46;
struct SqrtConst {
  BigE q, q1h, legendre;  // q = (p-1)/2^46, (q+1)/2, (p-1)/2
  Fq z_q;                 // z^q for a non-residue z
  SqrtConst() {
    legendre = shr(p_minus(1), 1);
    q = shr(p_minus(1), TWO_ADICITY);
    q1h = q;
    q1h.w[0] += 1;  // q odd: q + 1 has no carry beyond limb 0 unless all ones (not the case)
    q1h = shr(q1h, 1);
    Fq z = Fq::one();
    for (;;) {
      z = add(z, Fq::one());
      if (eq(fq_pow(z, legendre), neg(Fq::one()))) break;
    }
    z_q = fq_pow(z, q);
  }
};
const SqrtConst& sqc() {
  static SqrtConst c;
  return c;
}
bool is_square(const Fq& a) { return is_zero(a) || eq(fq_pow(a, sqc().legendre), Fq::one()); }

// Tonelli-Shanks; false if a is a non-residue
bool fq_sqrt(const Fq& a, Fq& out) {
  if (is_zero(a)) {
    out = a;
    return true;
  }
  if (!is_square(a)) return false;
  const SqrtConst& C = sqc();
  int m = TWO_ADICITY;
  Fq c = C.z_q, t = fq_pow(a, C.q), r = fq_pow(a, C.q1h);
  while (!eq(t, Fq::one())) {
    int i = 0;
    Fq t2 = t;
    while (!eq(t2, Fq::one())) {
      t2 = sqr(t2);
      i++;
    }
    Fq b = c;
    for (int k = 0; k < m - i - 1; k++) b = sqr(b);
    m = i;
    c = sqr(b);
    t = mul(t, c);
    r = mul(r, b);
  }
  out = r;
  return true;
}

// Fq2 = Fq[u]/(u^2 + 5): complex method
bool fq2_sqrt(const Fq2& a, Fq2& out) {
  const Fq five = mul5(Fq::one());
  if (is_zero(a.c1)) {
    Fq s;
    if (fq_sqrt(a.c0, s)) {
      out = {s, Fq::zero()};
      return true;
    }
    // a0 = c^2 u^2 = -5 c^2  ->  c = sqrt(-a0 / 5)
    if (!fq_sqrt(neg(mul(a.c0, inv(five))), s)) return false;
    out = {Fq::zero(), s};
    return true;
  }
  Fq delta;
  if (!fq_sqrt(add(sqr(a.c0), mul5(sqr(a.c1))), delta)) return false;  // norm
  const Fq half = inv(dbl(Fq::one()));
  Fq x0 = mul(add(a.c0, delta), half), c0;
  if (!fq_sqrt(x0, c0)) {
    x0 = mul(sub(a.c0, delta), half);
    if (!fq_sqrt(x0, c0)) return false;
  }
  const Fq c1 = mul(a.c1, inv(dbl(c0)));
  out = {c0, c1};
  return eq(sqr(out), a);
}

template <class F>
struct Ser;
template <>
struct Ser<Fq> {
  static constexpr int BYTES = 48, LIMBS = 12;
  static void put_x(const Fq& x, uint8_t* b) { fq_out(x, (uint64_t*)(void*)b); }
  static bool get_x(const uint8_t* b, uint8_t flags_mask, Fq& x) {
    uint64_t l[6];
    memcpy(l, b, 48);
    reinterpret_cast<uint8_t*>(l)[47] &= (uint8_t)~flags_mask;
    if (!lt_p(l)) return false;
    x = fq_in(l);
    return true;
  }
  static bool sqrt(const Fq& a, Fq& r) { return fq_sqrt(a, r); }
};
template <>
struct Ser<Fq2> {
  static constexpr int BYTES = 96, LIMBS = 24;
  static void put_x(const Fq2& x, uint8_t* b) {
    fq_out(x.c0, (uint64_t*)(void*)b);
    fq_out(x.c1, (uint64_t*)(void*)(b + 48));
  }
  static bool get_x(const uint8_t* b, uint8_t flags_mask, Fq2& x) {
    uint64_t l0[6], l1[6];
    memcpy(l0, b, 48);
    memcpy(l1, b + 48, 48);
    reinterpret_cast<uint8_t*>(l1)[47] &= (uint8_t)~flags_mask;
    if (!lt_p(l0) || !lt_p(l1)) return false;
    x = {fq_in(l0), fq_in(l1)};
    return true;
  }
  static bool sqrt(const Fq2& a, Fq2& r) { return fq2_sqrt(a, r); }
};

// canonical limbs (x || y, all-zero = infinity) -> compressed bytes
template <class F>
bool put_point(const uint64_t* p, uint8_t* b) {
  constexpr int NQ = Ser<F>::LIMBS / 12;
  bool inf = true;
  for (int i = 0; i < Ser<F>::LIMBS; i++) inf &= p[i] == 0;
  if (inf) {
    memset(b, 0, Ser<F>::BYTES);
    b[Ser<F>::BYTES - 1] = 0x40;
    return true;
  }
  for (int k = 0; k < 2 * NQ; k++)
    if (!lt_p(p + 6 * k)) return false;
  Affine<F> a;
  Fq* c = reinterpret_cast<Fq*>(&a);
  for (int k = 0; k < 2 * NQ; k++) c[k] = fq_in(p + 6 * k);
  Ser<F>::put_x(a.x, b);
  if (neg_flag(a.y)) b[Ser<F>::BYTES - 1] |= 0x80;
  return true;
}

// compressed bytes -> canonical limbs; Validate::Yes
template <class F>
bool get_point(const uint8_t* b, uint64_t* p) {
  const uint8_t fl = b[Ser<F>::BYTES - 1] & 0xC0;
  if (fl == 0xC0) return false;
  memset(p, 0, Ser<F>::LIMBS * 8);
  Affine<F> a;
  if (!Ser<F>::get_x(b, 0xC0, a.x)) return false;
  if (fl == 0x40) return true;  // PointAtInfinity
  F y;
  if (!Ser<F>::sqrt(add(mul(sqr(a.x), a.x), CurveB<F>::b()), y)) return false;
  const bool y_neg = neg_flag(y);  // y is the larger root iff its flag would be negative
  a.y = (y_neg == (fl == 0x80)) ? y : neg(y);
  if (!on_curve(a) || !is_inf(scalar_mul(a, params::FR_P, 253))) return false;
  const Fq* c = reinterpret_cast<const Fq*>(&a);
  for (int k = 0; k < Ser<F>::LIMBS / 6; k++) fq_out(c[k], p + 6 * k);
  return true;
}

struct Writer {
  uint8_t* out;
  size_t cap, n = 0;
  bool ok = true;
  void bytes(const void* d, size_t k) {
    if (out && n + k <= cap) memcpy(out + n, d, k);
    n += k;
  }
  void u64(uint64_t v) { bytes(&v, 8); }
  template <class F>
  void point(const uint64_t* p) {
    uint8_t b[Ser<F>::BYTES];
    if (!put_point<F>(p, b)) ok = false;
    bytes(b, sizeof(b));
  }
  void gt(const uint64_t* f) {
    for (int k = 0; k < 12; k++)
      if (!lt_p(f + 6 * k)) ok = false;
    bytes(f, 576);
  }
};

int finish(const Writer& w, size_t* len) {
  if (len) *len = w.n;
  if (!w.ok) return TPST_E_ARG;
  if (w.out && w.n > w.cap) return TPST_E_ARG;
  return TPST_OK;
}

struct Reader {
  const uint8_t* in;
  size_t len, n = 0;
  bool ok = true;
  const uint8_t* take(size_t k) {
    if (n + k > len) {
      ok = false;
      return nullptr;
    }
    const uint8_t* p = in + n;
    n += k;
    return p;
  }
  uint64_t u64() {
    const uint8_t* p = take(8);
    uint64_t v = 0;
    if (p) memcpy(&v, p, 8);
    return v;
  }
  template <class F>
  void point(uint64_t* out) {
    const uint8_t* p = take(Ser<F>::BYTES);
    if (!p || !get_point<F>(p, out)) ok = false;
  }
  void gt(uint64_t* out) {
    const uint8_t* p = take(576);
    if (!p) return;
    memcpy(out, p, 576);
    for (int k = 0; k < 12; k++)
      if (!lt_p(out + 6 * k)) ok = false;
  }
};

bool proof_dims_ok(const tpst_open_proof* p) {
  return p && p->m_col >= 0 && p->m_row >= 0 && p->m_col <= TPST_MAX_VARS && p->m_row <= TPST_MAX_VARS;
}

}  // namespace

extern "C" int tpst_ser_g1(const uint64_t* p, uint8_t* out48) {
  if (!p || !out48) return TPST_E_ARG;
  return put_point<Fq>(p, out48) ? TPST_OK : TPST_E_ARG;
}
extern "C" int tpst_ser_g2(const uint64_t* p, uint8_t* out96) {
  if (!p || !out96) return TPST_E_ARG;
  return put_point<Fq2>(p, out96) ? TPST_OK : TPST_E_ARG;
}
extern "C" int tpst_de_g1(const uint8_t* in48, uint64_t* p) {
  if (!p || !in48) return TPST_E_ARG;
  return get_point<Fq>(in48, p) ? TPST_OK : TPST_E_ARG;
}
extern "C" int tpst_de_g2(const uint8_t* in96, uint64_t* p) {
  if (!p || !in96) return TPST_E_ARG;
  return get_point<Fq2>(in96, p) ? TPST_OK : TPST_E_ARG;
}

// Commitment { nv: usize, g_product: G1Affine }
extern "C" int tpst_ser_commitment(int nv, const uint64_t* g1, uint8_t* out, size_t cap, size_t* len) {
  if (!g1 || nv < 0) return TPST_E_ARG;
  Writer w{out, cap};
  w.u64((uint64_t)nv);
  w.point<Fq>(g1);
  return finish(w, len);
}

// Proof { proofs: Vec<G2Affine> } (m_row entries): sqrt_pst.rs:225
extern "C" int tpst_ser_pst_proof(const tpst_open_proof* p, uint8_t* out, size_t cap, size_t* len) {
  if (!proof_dims_ok(p)) return TPST_E_ARG;
  Writer w{out, cap};
  w.u64((uint64_t)p->m_row);
  for (int i = 0; i < p->m_row; i++) w.point<Fq2>(p->pst_proof[i]);
  return finish(w, len);
}

// MippProof { comms_t: Vec<(Fq12, Fq12)>, comms_u: Vec<(G1, G1)>, final_a: G1,
//             final_h: G2, pst_proof_h: ProofG1 { proofs: Vec<G1> } }  (mipp.rs:21-28)
extern "C" int tpst_ser_mipp_proof(const tpst_open_proof* p, uint8_t* out, size_t cap, size_t* len) {
  if (!proof_dims_ok(p)) return TPST_E_ARG;
  Writer w{out, cap};
  w.u64((uint64_t)p->m_col);
  for (int i = 0; i < p->m_col; i++) {
    w.gt(p->comms_t[i][0]);
    w.gt(p->comms_t[i][1]);
  }
  w.u64((uint64_t)p->m_col);
  for (int i = 0; i < p->m_col; i++) {
    w.point<Fq>(p->comms_u[i][0]);
    w.point<Fq>(p->comms_u[i][1]);
  }
  w.point<Fq>(p->final_a);
  w.point<Fq2>(p->final_h);
  w.u64((uint64_t)p->m_col);
  for (int i = 0; i < p->m_col; i++) w.point<Fq>(p->pst_proof_h[i]);
  return finish(w, len);
}

// inverse of the two above (U is serialised separately as a Commitment):
// fills m_row / m_col and every element, validating each point
extern "C" int tpst_de_open_proof(const uint8_t* pst, size_t pst_len, const uint8_t* mipp, size_t mipp_len,
                                  tpst_open_proof* out) {
  if (!pst || !mipp || !out) return TPST_E_ARG;
  memset(out, 0, sizeof(*out));
  Reader a{pst, pst_len};
  const uint64_t m_row = a.u64();
  if (!a.ok || m_row > TPST_MAX_VARS) return TPST_E_ARG;
  out->m_row = (int32_t)m_row;
  for (uint64_t i = 0; i < m_row; i++) a.point<Fq2>(out->pst_proof[i]);
  if (!a.ok || a.n != pst_len) return TPST_E_ARG;
  Reader b{mipp, mipp_len};
  const uint64_t m_col = b.u64();
  if (!b.ok || m_col > TPST_MAX_VARS) return TPST_E_ARG;
  out->m_col = (int32_t)m_col;
  for (uint64_t i = 0; i < m_col; i++) {
    b.gt(out->comms_t[i][0]);
    b.gt(out->comms_t[i][1]);
  }
  if (b.u64() != m_col) return TPST_E_ARG;
  for (uint64_t i = 0; i < m_col; i++) {
    b.point<Fq>(out->comms_u[i][0]);
    b.point<Fq>(out->comms_u[i][1]);
  }
  b.point<Fq>(out->final_a);
  b.point<Fq2>(out->final_h);
  if (b.u64() != m_col) return TPST_E_ARG;
  for (uint64_t i = 0; i < m_col; i++) b.point<Fq>(out->pst_proof_h[i]);
  if (!b.ok || b.n != mipp_len) return TPST_E_ARG;
  return TPST_OK;
}

// CommitterKey { nv: usize, powers_of_g: Vec<Vec<G1>>, powers_of_h: Vec<Vec<G2>>,
// g: G1, h: G2 } (ark-poly-commit multilinear_pc data_structures, after trim)
// from the flat SRS layout of tpst_srs_export
extern "C" int tpst_ser_committer_key(int nv, const uint64_t* flat, size_t flat_len, uint8_t* out, size_t cap,
                                      size_t* len) {
  if (!flat || nv < 1 || nv > TPST_MAX_VARS || flat_len != tpst_srs_flat_len(nv)) return TPST_E_ARG;
  const uint64_t* g = flat;
  const uint64_t* h = flat + 12;
  std::vector<const uint64_t*> pg(nv), ph(nv);
  size_t off = 36;
  for (int i = 0; i < nv; i++) {
    pg[i] = flat + off;
    off += ((size_t)1 << (nv - i)) * 12;
    ph[i] = flat + off;
    off += ((size_t)1 << (nv - i)) * 24;
  }
  Writer w{out, cap};
  w.u64((uint64_t)nv);
  w.u64((uint64_t)nv);
  for (int i = 0; i < nv; i++) {
    const size_t k = (size_t)1 << (nv - i);
    w.u64(k);
    for (size_t j = 0; j < k; j++) w.point<Fq>(pg[i] + 12 * j);
  }
  w.u64((uint64_t)nv);
  for (int i = 0; i < nv; i++) {
    const size_t k = (size_t)1 << (nv - i);
    w.u64(k);
    for (size_t j = 0; j < k; j++) w.point<Fq2>(ph[i] + 24 * j);
  }
  w.point<Fq>(g);
  w.point<Fq2>(h);
  return finish(w, len);
}
