// sqrt-PST protocol layer of libtpst (include/tpst.h): SRS (MultilinearPC
// keys), the Polynomial handle (sqrt_pst.rs:14-265), MIPP prover/verifier
// (mipp.rs:31-320) and the Poseidon transcript (poseidon_transcript.rs).
//
// Everything heavy runs on the device (K1 row MSMs, K2 MSMs, K3 G2 MSMs, K4
// pairings, MIPP folds, Fr kernels); the host keeps the Fiat-Shamir
// transcript, which is inherently sequential and only absorbs a few KB per
// round.
#include <cstring>
#include <memory>
#include <vector>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "../../include/tpst.h"
#include "ctx.h"
#include "fbt.h"
#include "host_curve.h"
#include "device_util.h"
#include "pst_kernels.h"
#include "trace.h"
#include "poseidon_host.h"

using namespace tpst;

// =================================================================== host ==
namespace {

Fr fr_canon(const uint64_t* c) {
  Fr a;
  memcpy(a.v, c, 32);
  return to_mont(a);
}
void fr_out(const Fr& a, uint64_t* c) {
  Fr r = from_mont(a);
  memcpy(c, r.v, 32);
}

// TPST_OPEN_TRACE=1: per-round host timings of tpst_poly_open on stderr
static double host_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static bool open_trace() {
  static const bool on = getenv("TPST_OPEN_TRACE") != nullptr;
  return on;
}

// y > -y on canonical limbs  <=>  2y > p
bool y_is_negative(const uint64_t* y) {
  // compare y with p - y
  uint64_t ny[6];
  unsigned __int128 br = 0;
  const uint32_t* p32 = params::FQ_P;
  for (int i = 0; i < 6; i++) {
    const uint64_t pi = (uint64_t)p32[2 * i] | ((uint64_t)p32[2 * i + 1] << 32);
    unsigned __int128 d = (unsigned __int128)pi - y[i] - (uint64_t)br;
    ny[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  for (int i = 5; i >= 0; i--)
    if (y[i] != ny[i]) return y[i] > ny[i];
  return false;
}

void g1_bytes(const uint64_t* p, uint8_t* b) {  // ark serialize Compress::No
  bool inf = true;
  for (int i = 0; i < 12; i++) inf &= p[i] == 0;
  memcpy(b, p, 96);
  if (inf)
    b[95] |= 0x40;
  else if (y_is_negative(p + 6))
    b[95] |= 0x80;
}

// host Fr helpers
Fr fr_inv(const Fr& a) { return inv(a); }

// device XYZZ points (field.h Montgomery limbs, the same bits as host::HFq)
// -> canonical affine on the host: the open's few-point outputs (a round's
// u_l / u_r, U, final_a, final_h) need one inversion each, ~15 us here
// against a ~0.1 ms single-point kernel on the round's critical stream
template <class F>
void xyzz_to_canonical_host(const uint8_t* raw, size_t n, uint64_t* out) {
  using H = typename host::HostOf<F>::T;
  constexpr size_t PT = sizeof(Xyzz<F>), NQ = host::HostOf<F>::NQ;
  static_assert(sizeof(Xyzz<H>) == PT, "host and device XYZZ layouts differ");
  for (size_t i = 0; i < n; i++) {
    Xyzz<H> x;
    memcpy(&x, raw + i * PT, PT);
    host::aff_put(to_affine(x), out + i * 12 * NQ);
  }
}

// base-x digits of a canonical Fr e (e < r < x^4): e = sum_j out[j] x^j, for
// the GT exponentiations by Frobenius splitting (pairing.hip k_gt_pow_wave)
void base_x_digits(const uint64_t* e, uint64_t* out) {
  uint64_t q[4] = {e[0], e[1], e[2], e[3]};
  for (int t = 0; t < 4; t++) {
    unsigned __int128 rem = 0;
    for (int l = 3; l >= 0; l--) {
      const unsigned __int128 cur = (rem << 64) | q[l];
      q[l] = (uint64_t)(cur / params::BLS_X);
      rem = cur % params::BLS_X;
    }
    out[t] = (uint64_t)rem;
  }
}

// ---- proof-element validation (the reference's elements are typed arkworks
// values, validated when deserialized; here they arrive as raw limbs) ----
bool limbs_lt(const uint64_t* a, const uint32_t* mod32, int n64) {
  for (int i = n64 - 1; i >= 0; i--) {
    const uint64_t mi = (uint64_t)mod32[2 * i] | ((uint64_t)mod32[2 * i + 1] << 32);
    if (a[i] != mi) return a[i] < mi;
  }
  return false;
}
bool fq_ok(const uint64_t* a) { return limbs_lt(a, params::FQ_P, 6); }
bool fr_ok(const uint64_t* a) { return limbs_lt(a, params::FR_P, 4); }
bool all_zero(const uint64_t* a, int n) {
  for (int i = 0; i < n; i++)
    if (a[i]) return false;
  return true;
}
// canonical coordinates, on the curve, and r * P == O (prime-order subgroup),
// on 64-bit host arithmetic (host_curve.h)
template <class F>
bool point_valid(const uint64_t* p) {
  return host::point_in_subgroup<F>(p);
}
bool gt_ok(const uint64_t* f) {
  for (int k = 0; k < 12; k++)
    if (!fq_ok(f + 6 * k)) return false;
  return true;
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t b) {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = b;
    return b ? hipMalloc(&p, b) : hipSuccess;
  }
  uint32_t* u() const { return (uint32_t*)p; }
  // grow-only: keep the buffer when it is large enough
  hipError_t grow(size_t b) { return (p && bytes >= b) ? hipSuccess : alloc(b); }
};

// the opening's device buffers, kept across openings (grow-only): ~40
// hipMalloc / hipFree pairs per call cost the host ~0.4 ms
struct OpenBufs {
  DevBuf up, A, P, Y, chiC, ScA, ScB, ScC, ScD[2], xa, xb, xd, xh, xp, xl[2], LAo[2], Hb[3], Lb[3], gts, canA, canC,
      canD, pstA, pstB, Wall, Wiall, SqT[2], SqG[2], SqM, chis_own, tLoc, A1x, A1, tA1, Hbl[3], Lbl[3];
};

}  // namespace

// ================================================================ state ==
struct SrsState {
  int nv = 0;
  DevBuf g, h;                    // affine Montgomery
  std::vector<std::unique_ptr<DevBuf>> pg, ph, pg_pair, ph_pair;
  DevBuf gmask, hmask;
  BatchTables tables;             // K1 tables over powers_of_g[0]
  DevBuf hprep[2];                // G2Prepared of powers_of_h[odd], odd = 0/1
  DevBuf prep_scratch;            // residue lines of the RNS G2 preparation (g2_prepare_scratch)
  // fixed-base tables (fbt.h), built on first open
  DevBuf t_pg0;                   // powers_of_g[0]            (U = commit(q))
  DevBuf t_h[2];                  // powers_of_h[odd]           (MIPP h folds)
  DevBuf t_pgp, t_php;            // concatenated pg_pair / ph_pair levels (PST level proofs)
  DevBuf seg;                     // u32 level offsets into the concatenation
  std::vector<size_t> lvl_off;
  bool fbt_ready = false, t_h_ready[2] = {false, false};
  DevBuf t_A;                     // per-opening table over the row commitments
  size_t t_A_n = 0;
  // a rank's share of the SRS side for the row-sharded opening (every W-th
  // point of powers_of_h[odd] from `rank`, its prepared lines and table)
  struct Local {
    int W = 0, rank = -1;
    DevBuf H0, L0, tH;
  } local[2];
  // t_A prebuilt by tpst_poly_commit (beside its IPP) for exactly these
  // canonical row commitments; consumed by the next opening of them
  std::vector<uint64_t> t_A_key;
  std::vector<uint64_t> flat;     // canonical export
  OpenBufs ob;                    // the opening's device buffers (grow-only)
  ~SrsState() { batch_tables_free(tables); }
};

struct tpst_poly {
  tpst_ctx* ctx;
  int n, m_col, m_row, odd;
  DevBuf Zown;
  const uint32_t* d_Z = nullptr;  // canonical Fr
  // column slice (multi-GPU shard): only columns [col0,
  // col0 + ncols) of the strided view are resident, as an N x ncols block;
  // ncols == 0 means the whole polynomial
  size_t col0 = 0, ncols = 0;
  DevBuf q, chis;                 // Montgomery
  bool has_q = false;
  // opening-only handle (row-sharded commit): q combined from
  // the ranks' shares, no evaluations resident; optionally c_u combined too
  bool q_only = false;
  bool has_u = false;
  uint64_t U[12] = {};
};

static int srs_fbt(tpst_ctx* ctx, SrsState* st, int odd);

static std::unique_ptr<SrsState>& srs_slot(tpst_ctx* ctx) {
  static std::mutex mu;
  static std::vector<std::pair<tpst_ctx*, std::unique_ptr<SrsState>>> slots;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& s : slots)
    if (s.first == ctx) return s.second;
  slots.emplace_back(ctx, nullptr);
  return slots.back().second;
}

void tpst_release_pst_state(tpst_ctx* ctx) { srs_slot(ctx).reset(); }

extern "C" size_t tpst_srs_flat_len(int nv) {
  size_t n = 12 + 24;
  for (int i = 0; i < nv; i++) n += ((size_t)1 << (nv - i)) * 36;
  return n + (size_t)nv * 36;
}

// upload the flat canonical SRS and build every derived device table
static int srs_install(tpst_ctx* ctx, int nv, const uint64_t* flat) {
  auto st = std::make_unique<SrsState>();
  st->nv = nv;
  st->flat.assign(flat, flat + tpst_srs_flat_len(nv));
  hipStream_t s = ctx->stream;
  DevBuf stage;
  TPST_HIP(ctx, stage.alloc(st->flat.size() * 8));
  TPST_HIP(ctx, hipMemcpyAsync(stage.p, flat, st->flat.size() * 8, hipMemcpyHostToDevice, s));
  const uint32_t* src = stage.u();
  auto take = [&](DevBuf& dst, size_t npts, int words) -> hipError_t {
    hipError_t e = dst.alloc(npts * words * 4);
    if (e != hipSuccess) return e;
    e = words == 24 ? points_to_mont<Fq>(s, src, dst.u(), npts) : points_to_mont<Fq2>(s, src, dst.u(), npts);
    src += npts * words;
    return e;
  };
  TPST_HIP(ctx, take(st->g, 1, 24));
  TPST_HIP(ctx, take(st->h, 1, 48));
  for (int i = 0; i < nv; i++) {
    const size_t m = (size_t)1 << (nv - i);
    st->pg.emplace_back(new DevBuf());
    st->ph.emplace_back(new DevBuf());
    TPST_HIP(ctx, take(*st->pg.back(), m, 24));
    TPST_HIP(ctx, take(*st->ph.back(), m, 48));
    st->pg_pair.emplace_back(new DevBuf());
    st->ph_pair.emplace_back(new DevBuf());
    TPST_HIP(ctx, st->pg_pair.back()->alloc(m / 2 * 96));
    TPST_HIP(ctx, st->ph_pair.back()->alloc(m / 2 * 192));
    TPST_HIP(ctx, pair_sum<Fq>(s, st->pg.back()->u(), m / 2, st->pg_pair.back()->u()));
    TPST_HIP(ctx, pair_sum<Fq2>(s, st->ph.back()->u(), m / 2, st->ph_pair.back()->u()));
  }
  TPST_HIP(ctx, take(st->gmask, nv, 24));
  TPST_HIP(ctx, take(st->hmask, nv, 48));
  const size_t N = (size_t)1 << nv;
  TPST_HIP(ctx, batch_tables_build(s, st->pg[0]->u(), N, batch_window_bits(N), st->tables));
  TPST_HIP(ctx, st->prep_scratch.alloc(g2_prepare_scratch((size_t)1 << nv)));  // released below
  for (int odd = 0; odd < 2 && odd < nv; odd++) {
    const size_t m = (size_t)1 << (nv - odd);
    TPST_HIP(ctx, st->hprep[odd].alloc(m * N_LINE_COEFFS * sizeof(LineCoeff)));
    TPST_HIP(ctx, g2_prepare_batch(s, st->ph[odd]->u(), m, (LineCoeff*)st->hprep[odd].p, st->prep_scratch.u()));
  }
  // fixed-base tables of the opening (a function of the key only, like the
  // cached G2Prepared above): built here so that no open pays for them
  for (int odd = 0; odd < 2 && odd < nv; odd++) {
    int rc = srs_fbt(ctx, st.get(), odd);
    if (rc) return rc;
  }
  TPST_HIP(ctx, hipStreamSynchronize(s));
  TPST_HIP(ctx, st->prep_scratch.alloc(0));
  srs_slot(ctx) = std::move(st);
  return TPST_OK;
}

static SrsState* srs_of(tpst_ctx* ctx) { return srs_slot(ctx).get(); }

// scratch of the RNS G2 preparation (g2_prepare_scratch(n) bytes: residue
// lines, ~53 KB per point) sized for the largest batch prepared since the
// SRS was installed -- the install's 2^nv batch is released right after it
// (217 MB at nv = 12); callers size it before enqueueing any stream work
static int prep_scratch_for(tpst_ctx* ctx, SrsState* st, size_t n) {
  const size_t b = g2_prepare_scratch(n);
  if (st->prep_scratch.p && st->prep_scratch.bytes >= b) return TPST_OK;
  TPST_HIP(ctx, st->prep_scratch.alloc(b));  // hipFree of a smaller one waits for its users
  return TPST_OK;
}

// SplitMix64 Fr stream (same definition as the bench / oracle generators)
static uint64_t splitmix(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

extern "C" uint64_t tpst_fr_stream(uint64_t seed, size_t n, uint64_t start, uint64_t* out) {
  const uint32_t* r = params::FR_P;
  uint64_t k = start;
  size_t got = 0;
  while (got < n) {
    uint64_t v[4];
    for (int j = 0; j < 4; j++) v[j] = splitmix(seed, 4 * k + j);
    v[3] &= (1ull << 61) - 1;
    k++;
    bool lt = false;
    for (int i = 3; i >= 0; i--) {
      const uint64_t ri = (uint64_t)r[2 * i] | ((uint64_t)r[2 * i + 1] << 32);
      if (v[i] != ri) {
        lt = v[i] < ri;
        break;
      }
    }
    if (lt) {
      memcpy(out + 4 * got, v, 32);
      got++;
    }
  }
  return k;
}

// MultilinearPC::setup semantics from a seeded trapdoor: g = k_g G1, h = k_h G2,
// powers_of_g[i][x] = g^{eq(t[i..], x)} (LSB-first), g_mask[i] = g^{t_i}
extern "C" int tpst_srs_setup(tpst_ctx* ctx, int nv, uint64_t seed) {
  if (!ctx || nv <= 0 || nv > 28) return fail(ctx, TPST_E_ARG, "bad nv");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  std::vector<uint64_t> vals(4 * (nv + 2));
  tpst_fr_stream(seed, nv + 2, 0, vals.data());
  std::vector<Fr> t(nv);
  for (int i = 0; i < nv; i++) t[i] = fr_canon(&vals[4 * (2 + i)]);
  // all scalars: [k_g], [k_h] handled by generator muls; then eq tables and t
  std::vector<uint64_t> sc;  // canonical: for i: eq(t[i..]) ; then t
  for (int i = 0; i < nv; i++) {
    std::vector<Fr> tab(1, Fr::one());
    for (int j = i; j < nv; j++) {
      const size_t m = tab.size();
      tab.resize(2 * m);
      for (size_t x = 0; x < m; x++) {
        const Fr v = tab[x];
        tab[x] = mul(v, sub(Fr::one(), t[j]));
        tab[x + m] = mul(v, t[j]);
      }
    }
    for (auto& v : tab) {
      uint64_t c[4];
      fr_out(v, c);
      sc.insert(sc.end(), c, c + 4);
    }
  }
  for (int i = 0; i < nv; i++) sc.insert(sc.end(), &vals[4 * (2 + i)], &vals[4 * (2 + i)] + 4);
  const size_t ns = sc.size() / 4;
  hipStream_t s = ctx->stream;
  DevBuf d_sc, d_gh_sc, d_g, d_h, d_og, d_oh;
  TPST_HIP(ctx, d_sc.alloc(ns * 32));
  TPST_HIP(ctx, d_gh_sc.alloc(64));
  TPST_HIP(ctx, d_g.alloc(96));
  TPST_HIP(ctx, d_h.alloc(192));
  TPST_HIP(ctx, d_og.alloc(ns * 96));
  TPST_HIP(ctx, d_oh.alloc(ns * 192));
  TPST_HIP(ctx, hipMemcpyAsync(d_sc.p, sc.data(), ns * 32, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, hipMemcpyAsync(d_gh_sc.p, vals.data(), 64, hipMemcpyHostToDevice, s));
  // g, h from the standard generators
  {
    const uint32_t* gs = params::G1_GEN_X;
    std::vector<uint32_t> gen1(24), gen2(48);
    memcpy(gen1.data(), params::G1_GEN_X, 48);
    memcpy(gen1.data() + 12, params::G1_GEN_Y, 48);
    memcpy(gen2.data(), params::G2_GEN_X, 96);
    memcpy(gen2.data() + 24, params::G2_GEN_Y, 96);
    (void)gs;
    DevBuf dg1, dg2;
    TPST_HIP(ctx, dg1.alloc(96));
    TPST_HIP(ctx, dg2.alloc(192));
    TPST_HIP(ctx, hipMemcpyAsync(dg1.p, gen1.data(), 96, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, hipMemcpyAsync(dg2.p, gen2.data(), 192, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, fixed_base_mul<Fq>(s, dg1.u(), d_gh_sc.u(), 1, d_g.u()));
    TPST_HIP(ctx, fixed_base_mul<Fq2>(s, dg2.u(), d_gh_sc.u() + 8, 1, d_h.u()));
    TPST_HIP(ctx, fixed_base_mul<Fq>(s, d_g.u(), d_sc.u(), ns, d_og.u()));
    TPST_HIP(ctx, fixed_base_mul<Fq2>(s, d_h.u(), d_sc.u(), ns, d_oh.u()));
    TPST_HIP(ctx, affine_from_mont<Fq>(s, d_g.u(), d_g.u(), 1));
    TPST_HIP(ctx, affine_from_mont<Fq2>(s, d_h.u(), d_h.u(), 1));
    TPST_HIP(ctx, affine_from_mont<Fq>(s, d_og.u(), d_og.u(), ns));
    TPST_HIP(ctx, affine_from_mont<Fq2>(s, d_oh.u(), d_oh.u(), ns));
    TPST_HIP(ctx, hipStreamSynchronize(s));
  }
  std::vector<uint64_t> og(ns * 12), oh(ns * 24), flat(tpst_srs_flat_len(nv));
  TPST_HIP(ctx, hipMemcpy(og.data(), d_og.p, ns * 96, hipMemcpyDeviceToHost));
  TPST_HIP(ctx, hipMemcpy(oh.data(), d_oh.p, ns * 192, hipMemcpyDeviceToHost));
  TPST_HIP(ctx, hipMemcpy(flat.data(), d_g.p, 96, hipMemcpyDeviceToHost));
  TPST_HIP(ctx, hipMemcpy(flat.data() + 12, d_h.p, 192, hipMemcpyDeviceToHost));
  uint64_t* o = flat.data() + 36;
  size_t off = 0;
  for (int i = 0; i < nv; i++) {
    const size_t m = (size_t)1 << (nv - i);
    memcpy(o, &og[12 * off], m * 96);
    o += 12 * m;
    memcpy(o, &oh[24 * off], m * 192);
    o += 24 * m;
    off += m;
  }
  memcpy(o, &og[12 * off], nv * 96);
  o += 12 * nv;
  memcpy(o, &oh[24 * off], nv * 192);
  return srs_install(ctx, nv, flat.data());
}

extern "C" int tpst_srs_load(tpst_ctx* ctx, int nv, const uint64_t* flat) {
  if (!ctx || !flat || nv <= 0 || nv > 28) return fail(ctx, TPST_E_ARG, "bad argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  return srs_install(ctx, nv, flat);
}

extern "C" int tpst_srs_export(tpst_ctx* ctx, uint64_t* flat) {
  if (!ctx || !flat) return fail(ctx, TPST_E_ARG, "null argument");
  SrsState* st = srs_of(ctx);
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  memcpy(flat, st->flat.data(), st->flat.size() * 8);
  return TPST_OK;
}

// Valid::check of an affine point (what Validate::Yes deserialisation runs):
// canonical coordinates, on the curve, in the r-torsion subgroup.  Host only.
extern "C" int tpst_g1_check(const uint64_t* p) { return p && point_valid<Fq>(p) ? TPST_OK : TPST_E_VERIFY; }
extern "C" int tpst_g2_check(const uint64_t* p) { return p && point_valid<Fq2>(p) ? TPST_OK : TPST_E_VERIFY; }

// internal (groth16.hip): the same element validation as the PST verifier
bool tpst_internal_g1_valid(const uint64_t* p) { return point_valid<Fq>(p); }
bool tpst_internal_g2_valid(const uint64_t* p) { return point_valid<Fq2>(p); }

// ============================================================ transcript ==
// internal (r1cs.hip): the device copy of a whole polynomial's evaluations
// (canonical Fr, original order), or nullptr for a column shard
const uint32_t* tpst_internal_poly_evals(const tpst_poly* p) { return p && !p->ncols ? p->d_Z : nullptr; }

extern "C" void tpst_transcript_init(tpst_transcript* t) {
  if (!t) return;
  memset(t, 0, sizeof *t);
}

extern "C" int tpst_transcript_append_g1(tpst_transcript* t, const uint64_t* p) {
  if (!t || !p) return TPST_E_ARG;
  Sponge sp;
  sp.load(t);
  uint8_t b[96];
  g1_bytes(p, b);
  sp.absorb_bytes(b, 96);
  sp.store(t);
  return TPST_OK;
}

extern "C" int tpst_transcript_append_gt(tpst_transcript* t, const uint64_t* gt) {
  if (!t || !gt) return TPST_E_ARG;
  Sponge sp;
  sp.load(t);
  sp.absorb_bytes((const uint8_t*)gt, 576);
  sp.store(t);
  return TPST_OK;
}

// append_bytes (poseidon_transcript.rs:67-69): Absorb of a Vec<u8> (u64 length
// prefix, 47-byte chunks); `append` of any CanonicalSerialize value is this
// over its Compress::No bytes (poseidon_transcript.rs:22-28)
extern "C" int tpst_transcript_append_bytes(tpst_transcript* t, const uint8_t* b, size_t n) {
  if (!t || (n && !b)) return TPST_E_ARG;
  Sponge sp;
  sp.load(t);
  sp.absorb_bytes(b, n);
  sp.store(t);
  return TPST_OK;
}

// append_scalar (poseidon_transcript.rs:83-85): Absorb of an Fr into the Fq
// sponge = one Fq element with the same integer value (r < p)
extern "C" int tpst_transcript_append_fr(tpst_transcript* t, const uint64_t* fr) {
  if (!t || !fr || !fr_ok(fr)) return TPST_E_ARG;
  Sponge sp;
  sp.load(t);
  const uint64_t l[6] = {fr[0], fr[1], fr[2], fr[3], 0, 0};
  sp.absorb(std::vector<Fq>{fq_canon(l)});
  sp.store(t);
  return TPST_OK;
}

// new_from_state2 (poseidon_transcript.rs:55-60): a fresh sponge, then
// append(Fr) = absorb of its 32-byte uncompressed serialisation
extern "C" int tpst_transcript_reset_fr(tpst_transcript* t, const uint64_t* fr) {
  if (!t || !fr || !fr_ok(fr)) return TPST_E_ARG;
  memset(t, 0, sizeof *t);
  Sponge sp;
  sp.load(t);
  sp.absorb_bytes((const uint8_t*)fr, 32);
  sp.store(t);
  return TPST_OK;
}

extern "C" int tpst_transcript_challenge(tpst_transcript* t, uint64_t* out) {
  if (!t || !out) return TPST_E_ARG;
  Sponge sp;
  sp.load(t);
  sp.challenge(out);
  sp.store(t);
  return TPST_OK;
}

// ================================================================ poly ===
static int poly_dims(int n, int& m_col, int& m_row, int& odd) {
  if (n < 2 || n > 40) return -1;
  m_col = n / 2;
  m_row = n - m_col;
  odd = n % 2;
  return 0;
}

extern "C" int tpst_poly_from_evaluations(tpst_ctx* ctx, const uint64_t* Z, int n, tpst_poly** out) {
  if (!ctx || !Z || !out) return fail(ctx, TPST_E_ARG, "null argument");
  auto p = std::make_unique<tpst_poly>();
  if (poly_dims(n, p->m_col, p->m_row, p->odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  p->ctx = ctx;
  p->n = n;
  TPST_HIP(ctx, p->Zown.alloc(((size_t)1 << n) * 32));
  TPST_HIP(ctx, hipMemcpy(p->Zown.p, Z, ((size_t)1 << n) * 32, hipMemcpyHostToDevice));
  p->d_Z = p->Zown.u();
  *out = p.release();
  return TPST_OK;
}

// rank-local upload of the columns [c0, c1) of the strided view: for every
// j < 2^m_row the run Z[j 2^m_col + c0 .. j 2^m_col + c1) -- one 2D copy, no
// host transpose, (c1 - c0) / 2^m_col of the bytes
extern "C" int tpst_poly_from_evaluations_cols(tpst_ctx* ctx, const uint64_t* Z, int n, size_t c0, size_t c1,
                                               tpst_poly** out) {
  if (!ctx || !Z || !out) return fail(ctx, TPST_E_ARG, "null argument");
  auto p = std::make_unique<tpst_poly>();
  if (poly_dims(n, p->m_col, p->m_row, p->odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  const size_t C = (size_t)1 << p->m_col, N = (size_t)1 << p->m_row;
  if (c0 >= c1 || c1 > C) return fail(ctx, TPST_E_ARG, "bad column range");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  p->ctx = ctx;
  p->n = n;
  p->col0 = c0;
  p->ncols = c1 - c0;
  TPST_HIP(ctx, p->Zown.alloc(N * p->ncols * 32));
  TPST_HIP(ctx, hipMemcpy2DAsync(p->Zown.p, p->ncols * 32, Z + 4 * c0, C * 32, p->ncols * 32, N,
                                 hipMemcpyHostToDevice, ctx->stream));
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  p->d_Z = p->Zown.u();
  *out = p.release();
  return TPST_OK;
}

// base pointer and column stride of rows [r0, r1) in the resident block
static int poly_rows_view(tpst_ctx* ctx, const tpst_poly* p, size_t r0, size_t r1, const uint32_t** base,
                          size_t* cs) {
  const size_t C = (size_t)1 << p->m_col;
  if (!p->ncols) {
    if (r1 > C) return fail(ctx, TPST_E_ARG, "row range out of bounds");
    *base = p->d_Z + 8 * r0;
    *cs = C;
    return TPST_OK;
  }
  if (r0 < p->col0 || r1 > p->col0 + p->ncols) return fail(ctx, TPST_E_ARG, "rows outside the resident column slice");
  *base = p->d_Z + 8 * (r0 - p->col0);
  *cs = p->ncols;
  return TPST_OK;
}

static int poly_need_full(tpst_ctx* ctx, const tpst_poly* p) {
  if (p->q_only) return fail(ctx, TPST_E_STATE, "operation needs the evaluations (this handle holds q only)");
  return p->ncols ? fail(ctx, TPST_E_STATE, "operation needs the whole polynomial (this handle holds a column slice)")
                  : TPST_OK;
}

// eval / open need q and chi(b): a whole polynomial computes them, an
// opening-only handle carries them
static int poly_need_q_source(tpst_ctx* ctx, const tpst_poly* p) {
  return p->q_only ? TPST_OK : poly_need_full(ctx, p);
}

extern "C" int tpst_poly_from_evaluations_dev(tpst_ctx* ctx, const void* d_Z, int n, tpst_poly** out) {
  if (!ctx || !d_Z || !out) return fail(ctx, TPST_E_ARG, "null argument");
  auto p = std::make_unique<tpst_poly>();
  if (poly_dims(n, p->m_col, p->m_row, p->odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  p->ctx = ctx;
  p->n = n;
  p->d_Z = (const uint32_t*)d_Z;
  *out = p.release();
  return TPST_OK;
}

extern "C" void tpst_poly_free(tpst_poly* p) { delete p; }

// get_q (sqrt_pst.rs:81-101): chis over b = point[m_row..], q = Z^T chis
static int poly_get_q(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point) {
  TraceRange tr("build_q");
  hipStream_t s = ctx->stream;
  ctx->prof.begin(ST_BUILD_Q, s);
  DevBuf b;
  TPST_HIP(ctx, b.alloc((size_t)(p->m_col ? p->m_col : 1) * 32));
  if (p->m_col) {
    TPST_HIP(ctx, hipMemcpyAsync(b.p, point + 4 * p->m_row, p->m_col * 32, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, fr_to_mont(s, b.u(), b.u(), p->m_col));
  }
  TPST_HIP(ctx, p->chis.alloc(((size_t)1 << p->m_col) * 32));
  TPST_HIP(ctx, p->q.alloc(((size_t)1 << p->m_row) * 32));
  TPST_HIP(ctx, chi_table(s, b.u(), p->m_col, p->chis.u()));
  TPST_HIP(ctx, get_q(s, p->d_Z, p->m_col, p->m_row, p->chis.u(), p->q.u()));
  ctx->prof.end(ST_BUILD_Q, s);
  TPST_HIP(ctx, hipStreamSynchronize(s));
  p->has_q = true;
  return TPST_OK;
}

extern "C" int tpst_poly_eval(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point, uint64_t* out_v) {
  if (!ctx || !p || !point || !out_v) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  if (int rc = poly_need_q_source(ctx, p)) return rc;
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  if (!p->has_q) {
    int rc = poly_get_q(ctx, p, point);
    if (rc) return rc;
  }
  hipStream_t s = ctx->stream;
  DevBuf a, ca, v;
  TPST_HIP(ctx, a.alloc(p->m_row * 32));
  TPST_HIP(ctx, ca.alloc(((size_t)1 << p->m_row) * 32));
  TPST_HIP(ctx, v.alloc(32));
  TPST_HIP(ctx, hipMemcpyAsync(a.p, point, p->m_row * 32, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, fr_to_mont(s, a.u(), a.u(), p->m_row));
  TPST_HIP(ctx, chi_table(s, a.u(), p->m_row, ca.u()));
  TPST_HIP(ctx, fr_dot(s, p->q.u(), ca.u(), (size_t)1 << p->m_row, v.u()));
  TPST_HIP(ctx, fr_from_mont(s, v.u(), v.u(), 1));
  TPST_HIP(ctx, hipMemcpyAsync(out_v, v.p, 32, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

// commit (sqrt_pst.rs:117-149): K1 row MSMs + IPP T = prod e(C_i, h_i)
static int open_streams(tpst_ctx* ctx, size_t n_events, size_t pinned_bytes, bool comm = false);

// the context's pinned host staging (grow-only; the opening's per-round
// transfers, the commit's outputs)
static int ensure_pinned(tpst_ctx* ctx, size_t bytes) {
  if (ctx->pinned_cap >= bytes) return TPST_OK;
  if (ctx->pinned) TPST_HIP(ctx, hipHostFree(ctx->pinned));
  ctx->pinned = nullptr;
  ctx->pinned_cap = 0;
  TPST_HIP(ctx, hipHostMalloc(&ctx->pinned, bytes, hipHostMallocDefault));
  ctx->pinned_cap = bytes;
  return TPST_OK;
}

// prebuild (tpst_poly_commit): also build the opening's fold table over the
// row commitments on a side stream while the IPP runs (TPST_COMMIT_TABLE=0 /
// 1 forces it off / on)
static int poly_commit_dev(tpst_ctx* ctx, tpst_poly* p, uint32_t* d_comms_mont, Fq12* d_T, bool prebuild = false) {
  SrsState* st = srs_of(ctx);
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  if (st->nv != p->m_row) return fail(ctx, TPST_E_ARG, "SRS num_vars != ceil(n/2)");
  hipStream_t s = ctx->stream;
  const size_t C = (size_t)1 << p->m_col;
  ctx->arena2.reset();
  TPST_HIP(ctx, ctx->arena2.reserve(Arena::need(C, sizeof(Xyzz<Fq>)) + 256));
  Xyzz<Fq>* rows = ctx->arena2.take<Xyzz<Fq>>(C);
  Profiler& pf = ctx->prof;
  pf.begin(ST_SQRT_COMMIT, s);
  {
    TraceRange tr("comm_list");  // sqrt_pst.rs:119-126
    pf.begin(ST_COMM_LIST, s);
    TPST_HIP(ctx, msm_batch(ctx->arena, s, st->tables, p->d_Z, C, 1, C, rows));
    TPST_HIP(ctx, xyzz_to_affine_mont<Fq>(s, rows, d_comms_mont, C));
    pf.end(ST_COMM_LIST, s);
  }
  if (prebuild) {  // the opening's GLV fold table over comm_list, beside the IPP
    if (int rc = open_streams(ctx, 8, 0)) return rc;
    if (st->t_A_n < C) {
      TPST_HIP(ctx, st->t_A.alloc(fbt_words<Fq>(C) * 4));
      st->t_A_n = C;
    }
    st->t_A_key.clear();
    hipEvent_t* ev = ctx->events.data();
    TPST_HIP(ctx, hipEventRecord(ev[0], s));
    TPST_HIP(ctx, hipStreamWaitEvent(ctx->side[1], ev[0], 0));
    TPST_HIP(ctx, fbt_build<Fq>(ctx->arena_side[1], ctx->side[1], d_comms_mont, C, st->t_A.u(), true));
    TPST_HIP(ctx, hipEventRecord(ev[1], ctx->side[1]));
  }
  {
    TraceRange tr("ipp");  // sqrt_pst.rs:131-144
    pf.begin(ST_IPP, s);
    const LineCoeff* hp = (const LineCoeff*)st->hprep[p->odd].p;
    ctx->arena.reset();
    TPST_HIP(ctx, ctx->arena.reserve(multi_pairing_scratch(1, C)));
    TPST_HIP(ctx, multi_pairing_prepared(ctx->arena, s, d_comms_mont, st->ph[p->odd]->u(), hp, 1, C, d_T));
    pf.end(ST_IPP, s);
  }
  if (prebuild) TPST_HIP(ctx, hipStreamWaitEvent(s, ctx->events[1], 0));
  pf.end(ST_SQRT_COMMIT, s);
  return TPST_OK;
}

extern "C" int tpst_poly_commit(tpst_ctx* ctx, tpst_poly* p, uint64_t* comms, uint64_t* T) {
  if (!ctx || !p || !comms || !T) return fail(ctx, TPST_E_ARG, "null argument");
  TraceRange tr("sqrt_commit");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  if (int rc = poly_need_full(ctx, p)) return rc;
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  const size_t C = (size_t)1 << p->m_col;
  ctx->io.reset();  // (grow-only: no per-call hipMalloc / hipFree)
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(C * 24, 4) + Arena::need(1, sizeof(Fq12)) +
                                Arena::need(C * 24 + 144, 4) + 512));
  uint32_t* cm = ctx->io.take<uint32_t>(C * 24);
  Fq12* tt = ctx->io.take<Fq12>(1);
  uint32_t* out = ctx->io.take<uint32_t>(C * 24 + 144);
  // the table build runs beside the IPP (2^20: commit + open 21.7 -> 21.2
  // ms); at C = 4096 it outlasts the IPP by ~2 ms but leaves the opening's
  // first round free of it.  TPST_COMMIT_TABLE=0: the opening builds it
  static const int table_env = [] {
    const char* e = getenv("TPST_COMMIT_TABLE");
    return e ? atoi(e) : -1;
  }();
  const bool prebuild = table_env != 0;
  int rc = poly_commit_dev(ctx, p, cm, tt, prebuild);
  if (rc) return rc;
  hipStream_t s = ctx->stream;
  TPST_HIP(ctx, affine_from_mont<Fq>(s, cm, out, C));
  TPST_HIP(ctx, fq12_from_mont(s, tt, out + 24 * C, 1));
  // one asynchronous copy into pinned staging (not two pageable ones)
  if (int rc2 = ensure_pinned(ctx, C * 96 + 576)) return rc2;
  TPST_HIP(ctx, hipMemcpyAsync(ctx->pinned, out, C * 96 + 576, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  memcpy(comms, ctx->pinned, C * 96);
  memcpy(T, (const uint8_t*)ctx->pinned + C * 96, 576);
  if (prebuild) srs_of(ctx)->t_A_key.assign(comms, comms + 12 * C);
  return TPST_OK;
}

// device-resident commit: d_comms canonical affine (C*96 B), d_T canonical GT
extern "C" int tpst_poly_commit_dev(tpst_ctx* ctx, tpst_poly* p, void* d_comms, void* d_T) {
  if (!ctx || !p || !d_comms || !d_T) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  if (int rc = poly_need_full(ctx, p)) return rc;
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  const size_t C = (size_t)1 << p->m_col;
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(C * 24, 4) + Arena::need(1, sizeof(Fq12)) + 512));
  uint32_t* cm = ctx->io.take<uint32_t>(C * 24);
  Fq12* tt = ctx->io.take<Fq12>(1);
  int rc = poly_commit_dev(ctx, p, cm, tt);
  if (rc) return rc;
  TPST_HIP(ctx, affine_from_mont<Fq>(ctx->stream, cm, (uint32_t*)d_comms, C));
  TPST_HIP(ctx, fq12_from_mont(ctx->stream, tt, (uint32_t*)d_T, 1));
  return TPST_OK;
}

// row-sharded commit: rows [r0, r1) of the strided view,
// i.e. this rank's block of columns of Z.  comms: (r1-r0) canonical affine G1.
extern "C" int tpst_poly_commit_rows(tpst_ctx* ctx, tpst_poly* p, size_t r0, size_t r1, uint64_t* comms) {
  if (!ctx || !p || !comms || r1 < r0) return fail(ctx, TPST_E_ARG, "bad argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  if (st->nv != p->m_row) return fail(ctx, TPST_E_ARG, "SRS num_vars != ceil(n/2)");
  const uint32_t* zb;
  size_t cs;
  if (int rc = poly_rows_view(ctx, p, r0, r1, &zb, &cs)) return rc;
  const size_t R = r1 - r0;
  if (R == 0) return TPST_OK;
  hipStream_t s = ctx->stream;
  DevBuf rows, out;
  TPST_HIP(ctx, rows.alloc(R * sizeof(Xyzz<Fq>)));
  TPST_HIP(ctx, out.alloc(R * 96));
  TPST_HIP(ctx, msm_batch(ctx->arena, s, st->tables, zb, R, 1, cs, (Xyzz<Fq>*)rows.p));
  TPST_HIP(ctx, xyzz_to_affine_canonical<Fq>(s, (Xyzz<Fq>*)rows.p, out.u(), R));
  TPST_HIP(ctx, hipMemcpyAsync(comms, out.p, R * 96, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

// IPP of a full commitment list: T = prod_i e(comms[i], powers_of_h[odd][i])
// (sqrt_pst.rs:128-143), for a list gathered from the ranks
extern "C" int tpst_poly_ipp(tpst_ctx* ctx, int n, const uint64_t* comms, uint64_t* T) {
  if (!ctx || !comms || !T) return fail(ctx, TPST_E_ARG, "null argument");
  int m_col, m_row, odd;
  if (poly_dims(n, m_col, m_row, odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  if (st->nv != m_row) return fail(ctx, TPST_E_ARG, "SRS num_vars != ceil(n/2)");
  const size_t C = (size_t)1 << m_col;
  hipStream_t s = ctx->stream;
  DevBuf up, cm, tt, out;
  TPST_HIP(ctx, up.alloc(C * 96));
  TPST_HIP(ctx, cm.alloc(C * 96));
  TPST_HIP(ctx, tt.alloc(sizeof(Fq12)));
  TPST_HIP(ctx, out.alloc(576));
  TPST_HIP(ctx, hipMemcpyAsync(up.p, comms, C * 96, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, points_to_mont<Fq>(s, up.u(), cm.u(), C));
  ctx->arena.reset();
  TPST_HIP(ctx, ctx->arena.reserve(multi_pairing_scratch(1, C)));
  TPST_HIP(ctx, multi_pairing_prepared(ctx->arena, s, cm.u(), st->ph[odd]->u(), (const LineCoeff*)st->hprep[odd].p, 1,
                                       C, (Fq12*)tt.p));
  TPST_HIP(ctx, fq12_from_mont(s, (Fq12*)tt.p, out.u(), 1));
  TPST_HIP(ctx, hipMemcpyAsync(T, out.p, 576, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

// Row-sharded commit with the IPP split across ranks: the
// MSMs of rows [r0, r1) AND the Miller-loop product of their pairs
// prod_{r0 <= i < r1} ml(C_i, h_i) before final exponentiation (canonical
// Fq12, 72 u64).  Rank 0 finishes T = FE(prod over ranks) with
// tpst_gt_final_exp_product, so no rank runs more than its share of Miller loops.
static int commit_rows_partial(tpst_ctx* ctx, tpst_poly* p, size_t r0, size_t r1, uint64_t* comms, uint64_t* miller,
                               void* d_out) {
  if (!ctx || !p || ((!comms || !miller) && !d_out) || r1 < r0) return fail(ctx, TPST_E_ARG, "bad argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  if (st->nv != p->m_row) return fail(ctx, TPST_E_ARG, "SRS num_vars != ceil(n/2)");
  const uint32_t* zb;
  size_t cs;
  if (int rc = poly_rows_view(ctx, p, r0, r1, &zb, &cs)) return rc;
  const size_t R = r1 - r0;
  hipStream_t s = ctx->stream;
  if (R == 0) {  // empty share: comms untouched, partial = 1
    uint64_t one[72] = {1};
    if (d_out) {
      TPST_HIP(ctx, hipMemcpyAsync(d_out, one, 576, hipMemcpyHostToDevice, s));
      TPST_HIP(ctx, hipStreamSynchronize(s));
    } else {
      memcpy(miller, one, 576);
    }
    return TPST_OK;
  }
  if (int rc = prep_scratch_for(ctx, st, R)) return rc;
  DevBuf rows, cm, out, hsub, tt;
  TPST_HIP(ctx, rows.alloc(R * sizeof(Xyzz<Fq>)));
  TPST_HIP(ctx, cm.alloc(R * 96));
  TPST_HIP(ctx, out.alloc(R * 96 + 576));
  TPST_HIP(ctx, tt.alloc(sizeof(Fq12)));
  TPST_HIP(ctx, msm_batch(ctx->arena, s, st->tables, zb, R, 1, cs, (Xyzz<Fq>*)rows.p));
  TPST_HIP(ctx, xyzz_to_affine_mont<Fq>(s, (Xyzz<Fq>*)rows.p, cm.u(), R));
  // this rank's h_i and their prepared lines: the coefficient-major cache has
  // row length C, so the R-pair slice is re-prepared (R G2 points, one launch)
  const uint32_t* h = st->ph[p->odd]->u() + 48 * r0;
  const size_t need = Arena::need(R * N_LINE_COEFFS, sizeof(LineCoeff)) + multi_pairing_scratch(1, R) + 4096;
  ctx->arena.reset();
  TPST_HIP(ctx, ctx->arena.reserve(need));
  LineCoeff* lc = ctx->arena.take<LineCoeff>(R * N_LINE_COEFFS);
  TPST_HIP(ctx, g2_prepare_batch(s, h, R, lc, st->prep_scratch.u()));
  TPST_HIP(ctx, multi_pairing_prepared(ctx->arena, s, cm.u(), h, lc, 1, R, (Fq12*)tt.p, false));
  TPST_HIP(ctx, affine_from_mont<Fq>(s, cm.u(), out.u(), R));
  TPST_HIP(ctx, fq12_from_mont(s, (Fq12*)tt.p, out.u() + 24 * R, 1));
  if (d_out) {  // [comms | partial] straight into the caller's (all-gather) buffer
    TPST_HIP(ctx, hipMemcpyAsync(d_out, out.p, R * 96 + 576, hipMemcpyDeviceToDevice, s));
  } else {
    TPST_HIP(ctx, hipMemcpyAsync(comms, out.p, R * 96, hipMemcpyDeviceToHost, s));
    TPST_HIP(ctx, hipMemcpyAsync(miller, out.u() + 24 * R, 576, hipMemcpyDeviceToHost, s));
  }
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_poly_commit_rows_partial(tpst_ctx* ctx, tpst_poly* p, size_t r0, size_t r1, uint64_t* comms,
                                             uint64_t* miller) {
  return commit_rows_partial(ctx, p, r0, r1, comms, miller, nullptr);
}

extern "C" int tpst_poly_commit_rows_partial_dev(tpst_ctx* ctx, tpst_poly* p, size_t r0, size_t r1, void* d_out) {
  return commit_rows_partial(ctx, p, r0, r1, nullptr, nullptr, d_out);
}

// T = FE(prod_k partials[k]) for k Miller-loop partials (canonical Fq12 each;
// host, or device with a byte stride between consecutive partials)
static int final_exp_product(tpst_ctx* ctx, const uint64_t* partials, const void* d_partials, size_t stride,
                             size_t k, uint64_t* T) {
  if (!ctx || (!partials && !d_partials && k) || !T) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  DevBuf up, out;
  const size_t kk = k ? k : 1;
  TPST_HIP(ctx, up.alloc(kk * sizeof(Fq12)));
  TPST_HIP(ctx, out.alloc(sizeof(Fq12) + 576));
  if (k) {
    if (d_partials)
      TPST_HIP(ctx, hipMemcpy2DAsync(up.p, 576, d_partials, stride, 576, k, hipMemcpyDeviceToDevice, s));
    else
      TPST_HIP(ctx, hipMemcpyAsync(up.p, partials, k * 576, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, points_to_mont<Fq>(s, up.u(), up.u(), 6 * k));  // 12 Fq = 6 "points"
  }
  ctx->arena.reset();
  TPST_HIP(ctx, ctx->arena.reserve(multi_pairing_scratch(1, k)));
  TPST_HIP(ctx, gt_product_final(ctx->arena, s, (const Fq12*)up.p, 1, k, (Fq12*)out.p));
  TPST_HIP(ctx, fq12_from_mont(s, (Fq12*)out.p, out.u() + sizeof(Fq12) / 4, 1));
  TPST_HIP(ctx, hipMemcpyAsync(T, out.u() + sizeof(Fq12) / 4, 576, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_gt_final_exp_product(tpst_ctx* ctx, const uint64_t* partials, size_t k, uint64_t* T) {
  return final_exp_product(ctx, partials, nullptr, 0, k, T);
}

extern "C" int tpst_gt_final_exp_product_dev(tpst_ctx* ctx, const void* d_partials, size_t stride_bytes, size_t k,
                                             uint64_t* T) {
  if (stride_bytes < 576) return fail(ctx, TPST_E_ARG, "stride below one Fq12");
  return final_exp_product(ctx, nullptr, d_partials, stride_bytes, k, T);
}

// ------------------------------------------------ row-sharded opening -----
// rank g holds rows [r0, r1) of the strided view (a
// column-slice handle), so it computes its share of get_q's mat-vec
//   zq_g[j] = sum_{r0 <= i < r1} Z_i[j] chi_i(b)            (sqrt_pst.rs:92-95)
// and of c_u = MSM(comm_list, chi(b))                      (sqrt_pst.rs:198);
// the shares are gathered as bytes (RCCL has no mod-r or elliptic-curve
// reduction) and summed on rank 0, which then opens from q alone.
static int chi_b_table(tpst_ctx* ctx, int m_col, int m_row, const uint64_t* point, DevBuf& chis) {
  hipStream_t s = ctx->stream;
  DevBuf b;
  TPST_HIP(ctx, b.alloc((size_t)(m_col ? m_col : 1) * 32));
  if (m_col) {
    TPST_HIP(ctx, hipMemcpyAsync(b.p, point + 4 * m_row, m_col * 32, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, fr_to_mont(s, b.u(), b.u(), m_col));
  }
  TPST_HIP(ctx, chis.alloc(((size_t)1 << m_col) * 32));
  TPST_HIP(ctx, chi_table(s, b.u(), m_col, chis.u()));
  return hipStreamSynchronize(s) == hipSuccess ? TPST_OK : fail(ctx, TPST_E_HIP, "chi table");
}

static int poly_q_partial(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point, size_t r0, size_t r1, void* d_out,
                          uint64_t* h_out) {
  if (!ctx || !p || !point || (!d_out && !h_out) || r1 < r0) return fail(ctx, TPST_E_ARG, "bad argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  if (p->q_only) return fail(ctx, TPST_E_STATE, "opening-only handle holds no evaluations");
  for (int i = 0; i < p->n; i++)
    if (!fr_ok(point + 4 * i)) return fail(ctx, TPST_E_ARG, "point coordinate >= r");
  const uint32_t* zb;
  size_t cs;
  if (int rc = poly_rows_view(ctx, p, r0, r1, &zb, &cs)) return rc;
  DevBuf chis, tmp;
  if (int rc = chi_b_table(ctx, p->m_col, p->m_row, point, chis)) return rc;
  hipStream_t s = ctx->stream;
  const size_t N = (size_t)1 << p->m_row;
  uint32_t* dst = (uint32_t*)d_out;
  if (!dst) {
    TPST_HIP(ctx, tmp.alloc(N * 32));
    dst = tmp.u();
  }
  if (r1 > r0) {
    TPST_HIP(ctx, get_q_rows(s, zb, cs, r1 - r0, p->m_row, chis.u() + 8 * r0, dst));
  } else {
    TPST_HIP(ctx, hipMemsetAsync(dst, 0, N * 32, s));
  }
  if (h_out) TPST_HIP(ctx, hipMemcpyAsync(h_out, dst, N * 32, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_poly_get_q_partial(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point, size_t r0, size_t r1,
                                       uint64_t* zq) {
  return poly_q_partial(ctx, p, point, r0, r1, nullptr, zq);
}

extern "C" int tpst_poly_get_q_partial_dev(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point, size_t r0, size_t r1,
                                           void* d_zq) {
  return poly_q_partial(ctx, p, point, r0, r1, d_zq, nullptr);
}

extern "C" int tpst_fr_sum_dev(tpst_ctx* ctx, const void* d_parts, size_t k, size_t n, void* d_out) {
  if (!ctx || (n && (!d_parts || !d_out))) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  TPST_HIP(ctx, fr_sum_parts(ctx->stream, (const uint32_t*)d_parts, k, n, (uint32_t*)d_out));
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return TPST_OK;
}

// c_u's share: sum_{r0 <= i < r1} chi_i(b) C_i over this rank's row commitments
extern "C" int tpst_poly_cu_partial(tpst_ctx* ctx, int n, const uint64_t* point, size_t r0, size_t r1,
                                    const uint64_t* comms, uint64_t* out) {
  if (!ctx || !point || (!comms && r1 > r0) || !out || r1 < r0) return fail(ctx, TPST_E_ARG, "bad argument");
  int m_col, m_row, odd;
  if (poly_dims(n, m_col, m_row, odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  if (r1 > ((size_t)1 << m_col)) return fail(ctx, TPST_E_ARG, "row range out of bounds");
  for (int i = 0; i < n; i++)
    if (!fr_ok(point + 4 * i)) return fail(ctx, TPST_E_ARG, "point coordinate >= r");
  std::vector<uint64_t> sc((r1 - r0) * 4 + 4);
  {
    std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
    TPST_HIP(ctx, hipSetDevice(ctx->device));
    DevBuf chis;
    if (int rc = chi_b_table(ctx, m_col, m_row, point, chis)) return rc;
    if (r1 > r0) {
      TPST_HIP(ctx, fr_from_mont(ctx->stream, chis.u() + 8 * r0, chis.u() + 8 * r0, r1 - r0));
      TPST_HIP(ctx, hipMemcpyAsync(sc.data(), chis.u() + 8 * r0, (r1 - r0) * 32, hipMemcpyDeviceToHost, ctx->stream));
      TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
  }
  if (r1 == r0) {
    memset(out, 0, 96);
    return TPST_OK;
  }
  return tpst_g1_msm(ctx, comms, r1 - r0, sc.data(), r1 - r0, out);
}

// opening-only Polynomial from the combined q (2^m_row canonical Fr, device)
// and, optionally, the combined c_u (canonical affine; NULL = the opening
// computes U = MSM(comm_list, chi(b)) itself)
extern "C" int tpst_poly_from_q_dev(tpst_ctx* ctx, int n, const uint64_t* point, const void* d_zq,
                                    const uint64_t* U, tpst_poly** out) {
  if (!ctx || !point || !d_zq || !out) return fail(ctx, TPST_E_ARG, "null argument");
  auto p = std::make_unique<tpst_poly>();
  if (poly_dims(n, p->m_col, p->m_row, p->odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  for (int i = 0; i < n; i++)
    if (!fr_ok(point + 4 * i)) return fail(ctx, TPST_E_ARG, "point coordinate >= r");
  if (U && !point_valid<Fq>(U)) return fail(ctx, TPST_E_ARG, "c_u is not a valid G1 point");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  p->ctx = ctx;
  p->n = n;
  p->q_only = true;
  if (int rc = chi_b_table(ctx, p->m_col, p->m_row, point, p->chis)) return rc;
  const size_t N = (size_t)1 << p->m_row;
  TPST_HIP(ctx, p->q.alloc(N * 32));
  TPST_HIP(ctx, fr_to_mont(ctx->stream, (const uint32_t*)d_zq, p->q.u(), N));
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  p->has_q = true;
  if (U) {
    memcpy(p->U, U, 96);
    p->has_u = true;
  }
  *out = p.release();
  return TPST_OK;
}

// --------------------------------------------------------------- open ----
// The opening is latency-bound (transcript rounds of small MSMs and pairings),
// so every MSM of it runs on fixed-base lookup tables (fbt.h): the SRS sides
// are tabulated once per SRS, the row commitments once per opening, and each
// MIPP round's folds / cross terms are grouped MSMs over the ORIGINAL bases
// with scalars that are products of the challenges so far.

// tabulate the SRS (fbt.h) for opening polynomials of parity `odd` (at SRS
// install; the open path re-checks and is a no-op then)
static int srs_fbt(tpst_ctx* ctx, SrsState* st, int odd) {
  hipStream_t s = ctx->stream;
  const int nv = st->nv;
  if (!st->fbt_ready) {
    const size_t N = (size_t)1 << nv;
    TPST_HIP(ctx, st->t_pg0.alloc(fbt_words<Fq>(N) * 4));
    TPST_HIP(ctx, fbt_build<Fq>(ctx->arena, s, st->pg[0]->u(), N, st->t_pg0.u()));
    st->lvl_off.assign(nv + 1, 0);
    for (int i = 0; i < nv; i++) st->lvl_off[i + 1] = st->lvl_off[i] + ((size_t)1 << (nv - i - 1));
    const size_t tot = st->lvl_off[nv];
    TPST_HIP(ctx, st->t_pgp.alloc(fbt_words<Fq>(tot) * 4));
    TPST_HIP(ctx, st->t_php.alloc(fbt_words<Fq2>(tot) * 4));
    for (int i = 0; i < nv; i++) {
      const size_t m = (size_t)1 << (nv - i - 1);
      TPST_HIP(ctx, fbt_build<Fq>(ctx->arena, s, st->pg_pair[i]->u(), m, st->t_pgp.u() + fbt_words<Fq>(st->lvl_off[i])));
      TPST_HIP(ctx,
               fbt_build<Fq2>(ctx->arena, s, st->ph_pair[i]->u(), m, st->t_php.u() + fbt_words<Fq2>(st->lvl_off[i])));
    }
    std::vector<uint32_t> off32(st->lvl_off.begin(), st->lvl_off.end());
    TPST_HIP(ctx, st->seg.alloc(off32.size() * 4));
    TPST_HIP(ctx, hipMemcpyAsync(st->seg.p, off32.data(), off32.size() * 4, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, hipStreamSynchronize(s));
    st->fbt_ready = true;
  }
  if (!st->t_h_ready[odd]) {
    const size_t C = (size_t)1 << (nv - odd);
    TPST_HIP(ctx, st->t_h[odd].alloc(fbt_words<Fq2>(C) * 4));
    TPST_HIP(ctx, fbt_build<Fq2>(ctx->arena, s, st->ph[odd]->u(), C, st->t_h[odd].u()));
    TPST_HIP(ctx, hipStreamSynchronize(s));
    st->t_h_ready[odd] = true;
  }
  return TPST_OK;
}

// PST open of 2^k evals (Montgomery) at k Montgomery
// scalars d_pt over the pair levels off..off+k-1: the k quotient scalar
// vectors first (cheap Fr recurrence), then ONE grouped table MSM with a
// group per level.  Writes k XYZZ points.  Stream-ordered on `s` with the
// caller's scratch (pst_open_scratch_words u32), so it can run beside the MIPP.
static size_t pst_open_scratch_words(const SrsState* st, int k) {
  return ((size_t)2 << k) * 8 + st->lvl_off[st->nv] * 8;
}

template <class F>
static hipError_t pst_open_fbt_s(hipStream_t s, Arena& ar, const SrsState* st, const uint32_t* table, int off,
                                 const uint32_t* d_evals, int k, const uint32_t* d_pt, Xyzz<F>* d_out,
                                 uint32_t* scratch) {
  const size_t full = (size_t)1 << k;
  uint32_t* cur = scratch;
  uint32_t* nxt = scratch + full * 8;
  uint32_t* sc = scratch + 2 * full * 8;
  hipError_t e = hipMemcpyAsync(cur, d_evals, full * 32, hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return e;
  for (int i = 0; i < k; i++) {
    const size_t half = (size_t)1 << (k - i - 1);
    e = pst_step(s, cur, half, d_pt + 8 * i, sc + 8 * st->lvl_off[off + i], nxt);
    if (e != hipSuccess) return e;
    std::swap(cur, nxt);
  }
  FbGroups g;
  g.groups = k;
  g.members = (size_t)1 << (k - 1);
  g.d_seg = st->seg.u() + off;
  return fbt_msm<F>(ar, s, table, sc, g, d_out);
}

template <class F>
static int pst_open_fbt(tpst_ctx* ctx, SrsState* st, const uint32_t* table, int off, const uint32_t* d_evals, int k,
                        const uint32_t* d_pt, Xyzz<F>* d_out) {
  DevBuf scratch;
  TPST_HIP(ctx, scratch.alloc(pst_open_scratch_words(st, k) * 4));
  TPST_HIP(ctx, pst_open_fbt_s<F>(ctx->stream, ctx->arena, st, table, off, d_evals, k, d_pt, d_out, scratch.u()));
  return TPST_OK;
}

// ---------------------------------------------------------------- open ----
// Streams of the opening (created once per context) and a pool of events.
static int open_streams(tpst_ctx* ctx, size_t n_events, size_t pinned_bytes, bool comm) {
  int least = 0, greatest = 0;
  TPST_HIP(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
  // side streams at the least priority (the look-ahead streams at the
  // greatest won an open-only sweep, 14.2 -> 13.8 ms, but lost in the commit +
  // open bench: 2^20 open 12.3 -> 13.9 ms; profiles/r04/late/prio6_bench*.json)
  for (int i = 0; i < 3; i++)
    if (!ctx->side[i]) TPST_HIP(ctx, hipStreamCreateWithPriority(&ctx->side[i], hipStreamNonBlocking, least));
  // the row-sharded opening's collectives, in one issue order on every rank
  if (comm && !ctx->comm) TPST_HIP(ctx, hipStreamCreateWithPriority(&ctx->comm, hipStreamNonBlocking, greatest));
  // the per-round h preparation of the opening (its own hardware queue: on
  // stream A it delayed the next round's t; 2^20 open 13.0 -> 11.4 ms; at
  // the least priority 11.05 -> 11.30 ms, profiles/r06/ab/ab_open_c_prio.txt)
  if (!ctx->side_c) TPST_HIP(ctx, hipStreamCreateWithPriority(&ctx->side_c, hipStreamNonBlocking, greatest));
  while (ctx->events.size() < n_events) {
    hipEvent_t e;
    TPST_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->events.push_back(e);
  }
  return ensure_pinned(ctx, pinned_bytes);
}

// Polynomial::open (sqrt_pst.rs:168-230) with MippProof::prove (mipp.rs:31-153).
//
// Critical path = the transcript: each MIPP round's challenge needs that
// round's comms_u and comms_t, and the next round's folds need the challenge.
// Per round r (len = C >> r, s = len / 2, s' = s / 2) the work is spread
// over 4 streams (one hardware queue each; A at the highest priority):
//   A (critical): t^(r) = (t_l, t_r).  Round 0 pairs the row commitments
//     directly.  From round 1 on, t^(r) comes out of the LOOK-AHEAD of round
//     r-1 (stream D): with a' = a_L + c a_R, h' = h_L + c^-1 h_R (mipp.rs:101-
//     120) bilinearity splits round r's cross products into eight pairing
//     products of round r-1's vectors that do not involve c = c_{r-1},
//       t_l = A0 A3 A1^(c^-1) A2^c,  t_r = B0 B3 B1^(c^-1) B2^c
//     (pairing.hip, mipp_lookahead), so once c is known the critical path is
//     four GT exponentiations (base-x Frobenius splitting, ~0.7 ms) and two
//     products instead of fold + Miller loops + final exponentiations
//     (~3.3 ms); comms_t -> host.
//   D: the look-ahead of round r for round r+1: a^(r) and c'a^(r) as ONE
//     grouped table MSM over the original row commitments (scalar sets W,
//     c'W: a^(r)_i = sum_t W_t a_{i+t len}, c' = the previous challenge
//     inverse), then the 8 products against the PREVIOUS round's prepared h:
//       e(a_i, h^(r)_k) = e(a_i, h^(r-1)_k) e(c' a_i, h^(r-1)_{k+len})
//     -> Miller loops + 8 final exponentiations, overlapping round r's own
//     transcript work.
//   B: y fold (compress_field, mipp.rs:124-136) and the cross MSMs u_l, u_r
//     (mipp.rs:66-75) -> canonical -> host; in round 0 first U =
//     MSM(comm_list, chi(b)) (sqrt_pst.rs:198) and after it the PST proof of
//     q (sqrt_pst.rs:218-225), which needs nothing from the MIPP.
//   C: in round 0 the fold table over comm_list (fbt.h); then h^(r) =
//     sum_t Wi_t h_{i + t len} (table MSM over powers_of_h) -> affine ->
//     G2Prepared, consumed by the look-ahead of round r+1.
// The host waits only for the round's comms (pinned staging), absorbs them
// (mipp.rs:97-101) and squeezes the challenge; no stream is drained mid-open.
//
// Row-sharded form (sh != nullptr, tpst_poly_open_sharded):
// rank g of W owns the rows i = g mod W of comm_list, h and y.  While
// len >= 4W every fold group (a^(r)_i = sum_t W_t a_{i + t len}) lies on one
// rank (i + t len = i mod W), and so does every look-ahead pair (positions
// i + j s' share i's residue), so each rank runs the round on its own rows
// with every size divided by W: its own table over its C / W commitments,
// the look-ahead's folds and pairings over len / W positions, the h folds and
// preparations of its positions, and the cross MSMs as partial sums over its
// rows.  ONE all-gather per product combines them on every rank: the cross
// partials summed (XYZZ), the Miller partials multiplied before the single
// final exponentiation (gt_prod_final); every rank then combines t^(r) and
// replays the transcript itself (no broadcast).  At the first round with
// len < 4W the ranks gather the folded a^(r1) (len = 2W points) to rank 0,
// which tabulates it and finishes the remaining rounds with the a-side
// rebased on it (a^(r)_i = sum_{t < 2^(r - r1)} W_r[t] a^(r1)_{i + t len}:
// the first weights of the same W_r) and the epilogue alone.  The exchange is
// the caller's (tpst_exchange: RCCL, gloo, ...), ordered on a dedicated comm
// stream so that every rank issues the same collectives in the same order.
namespace {
struct Shard {
  int W = 1, rank = 0;
  const tpst_exchange* x = nullptr;
  const uint64_t* U = nullptr;  // c_u (canonical affine), every rank
};

size_t xch_align(size_t v) { return (v + 255) & ~(size_t)255; }
size_t xch_slot(size_t bytes, int W) { return xch_align(bytes) + xch_align((size_t)W * bytes); }
// first round whose look-ahead cannot be split over W ranks (len < 4W)
int shard_rounds(int m, int W) {
  int r1 = 0;
  while (r1 < m && (((size_t)1 << m) >> r1) >= (size_t)4 * W) r1++;
  return r1;
}
}  // namespace

extern "C" size_t tpst_open_sharded_arena_bytes(int n, int world) {
  if (n < 1 || n > 2 * TPST_MAX_VARS || world < 1 || (world & (world - 1))) return 0;
  const int m = n / 2, r1 = shard_rounds(m, world);
  if (r1 == 0) return 0;
  constexpr size_t X1 = sizeof(Xyzz<Fq>), T12 = sizeof(Fq12);
  return (size_t)r1 * (xch_slot(2 * X1, world) + xch_slot(8 * T12, world)) + xch_slot(2 * T12, world) +
         xch_slot(2 * X1, world);
}

static int poly_open(tpst_ctx* ctx, tpst_poly* p, tpst_transcript* tr, int n, const uint64_t* comms,
                     const uint64_t* point, tpst_open_proof* proof, const Shard* sh) {
  const bool shd = sh != nullptr;
  const int W = shd ? sh->W : 1, rho = shd ? sh->rank : 0;
  const bool lead = rho == 0;  // produces the proof (and the PST proof of q)
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  if (lead)
    if (int rc = poly_need_q_source(ctx, p)) return rc;
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  int m, k, odd;
  if (poly_dims(n, m, k, odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  if (st->nv != k) return fail(ctx, TPST_E_ARG, "SRS num_vars != ceil(n/2)");
  for (size_t i = 0; i < ((size_t)2 << m); i++)
    if (!fq_ok(comms + 6 * i)) return fail(ctx, TPST_E_ARG, "comm_list coordinate >= p");
  if (lead && !p->has_q) {  // before the reference's open timer (sqrt_pst.rs:177-183)
    int rc = poly_get_q(ctx, p, point);
    if (rc) return rc;
  }
  TraceRange trace_open("sqrt_open");
  Profiler& pf = ctx->prof;
  pf.begin(ST_SQRT_OPEN, ctx->stream);
  {
    int rc = srs_fbt(ctx, st, odd);
    if (rc) return rc;
  }
  const size_t C = (size_t)1 << m;
  // the rounds split across the ranks: [0, r1); rank 0 alone from r1 on
  const int r1 = shd ? shard_rounds(m, W) : 0;
  const size_t Cl = C / W;  // a rank's rows (i = rho mod W)
  std::unique_ptr<tpst_open_proof> own_proof;
  if (!proof) {  // a rank other than 0 fills nothing the caller reads
    own_proof.reset(new tpst_open_proof);
    proof = own_proof.get();
  }
  memset(proof, 0, sizeof *proof);
  proof->m_col = m;
  proof->m_row = k;
  Sponge sp;
  sp.load(tr);

  // ---- host staging layout (bytes): per-round uploads, final upload, downloads
  std::vector<size_t> up_off(m + 2);
  size_t off = 0;
  // per round: c_{r-1}, c_{r-1}^-1, f_0..f_7 (Montgomery Fr), base-x digits of
  // (c^-1, c, c^-1, c); the fold weights themselves are formed on the device
  constexpr size_t UP_ROUND = 10 * 32 + 128;
  for (int r = 0; r < m; r++) {
    up_off[r] = off;
    off += UP_ROUND;
  }
  up_off[m] = off;  // final: c_{m-1}, c_{m-1}^-1, rs (Montgomery Fr), a_rev (canonical Fr)
  off += (2 + m + k) * 32;
  const size_t up_bytes = off;
  // downloads: U, each round's u_l / u_r as raw XYZZ (converted on the host)
  // and t_l / t_r; final_a, final_h raw; pst_proof_h, pst_proof canonical
  constexpr size_t X1 = sizeof(Xyzz<Fq>), X2 = sizeof(Xyzz<Fq2>), DN_ROUND = 2 * X1 + 1152;
  const size_t dn_U = up_bytes, dn_round = dn_U + X1, dn_final = dn_round + (size_t)m * DN_ROUND;
  const size_t dn_fh = dn_final + X1, dn_ph = dn_fh + X2, dn_pst = dn_ph + (size_t)m * 96;
  const size_t dn_bytes = X1 + (size_t)m * DN_ROUND + X1 + X2 + (size_t)m * 96 + (size_t)k * 192;
  const size_t n_ev = 9 + 6 * (size_t)m + (shd ? 8 * (size_t)m + 8 : 0);
  // unsharded rebase: in round rb = 4, a^(4) (C / 16 points) is tabulated
  // (as the sharded hand-over does) on the otherwise idle comm stream, and the
  // later rounds fold 2^(r - 4) of its points instead of C / len row
  // commitments (2^24 open 24.4 -> 23.0 ms, 2^20 10.4 -> 10.2 ms; rebasing at
  // len 16 / 64 at 2^24 gained less: profiles/r06/ab/ab_open_rebase.txt)
  const int rb = !shd && m >= 8 ? 4 : -1;
  const size_t cm_off = up_bytes + dn_bytes;  // comm_list staging (unsharded form)
  if (int rc = open_streams(ctx, n_ev, cm_off + (shd ? 0 : C * 96), shd || rb >= 0)) return rc;
  uint8_t* pin = (uint8_t*)ctx->pinned;
  // five streams: A (critical), B (cross terms), two look-ahead streams for
  // alternating rounds (consecutive look-aheads overlap, each taking longer
  // than a round) and C, the h preparation, at the greatest priority.  h^(r)
  // (G2 fold + G2Prepared lines) is prepared in every round r >= 1 that a
  // look-ahead needs: look-ahead r pairs E = 2^(r - s) fold sets of a^(r)
  // against the prepared h^(s), s = r - 1 (prepared one round earlier: E = 2;
  // in round 1 itself for r = 1: E = 1), s = 0 for r = 0.  Preparing at odd rounds only (s = r - 2 / r - 3, E =
  // 4 / 8) paired two to four times as many pairs; C on stream A delayed the
  // next round's t (2^24 open 26.6 -> 25.5 ms, 2^20 13.0 -> 11.4 ms with both,
  // profiles/r05/i).  The epilogue's final h fold runs on the first look-ahead
  // stream (idle by then), beside final_a (A) and pst_proof_h (B)
  const hipStream_t sA = ctx->stream, sB = ctx->side[0], sC = ctx->side_c;
  const hipStream_t sCe = ctx->side[1];
  hipStream_t sLA[2] = {ctx->side[1], ctx->side[2]};
  Arena &arA = ctx->arena, &arB = ctx->arena_side[0], &arC = ctx->arena2;
  Arena* arLA[2] = {&ctx->arena_side[1], &ctx->arena_side[2]};
  hipEvent_t* ev = ctx->events.data();
  enum { EV_PRE, EV_TABLE, EV_U, EV_FINAL_UP, EV_B_DONE, EV_C_DONE, EV_D_DONE, EV_A_DONE, EV_REBASE };
  auto ev_up = [&](int r) { return ev[9 + 6 * r]; };
  auto ev_a = [&](int r) { return ev[9 + 6 * r + 1]; };
  auto ev_b = [&](int r) { return ev[9 + 6 * r + 2]; };
  auto ev_c = [&](int r) { return ev[9 + 6 * r + 3]; };
  auto ev_la = [&](int r) { return ev[9 + 6 * r + 4]; };
  auto ev_cl = [&](int r) { return ev[9 + 6 * r + 5]; };  // the rank's own h positions prepared
  hipEvent_t* xev = ev + 9 + 6 * m;                         // exchange events (sharded form)
  int last_c = -1;  // the last odd round that issued h work "C"
  // the prepared h the look-ahead of round r pairs against (see above)
  // look-ahead 1 pairs h^(1), prepared by C in round 1 (enqueued before D
  // there), with E = 1 instead of h^(0) with E = 2: half the pairs (2^24 open
  // 22.9 -> 22.5 ms, profiles/r06/ab/ab_open_la1.txt)
  auto la_src = [](int r) { return r == 0 ? 0 : r - 1; };
  // which odd rounds prepare h: for a look-ahead on the rank's own positions
  // (local, sharded rounds) or on every position (global)
  std::vector<char> need_loc(m + 1, 0), need_glob(m + 1, 0);
  for (int r = 1; r < m; r++) {
    if ((C >> r) < 4 || la_src(r) == 0) continue;
    if (shd && r < r1)
      need_loc[la_src(r)] = 1;
    else if (lead)
      need_glob[la_src(r)] = 1;
  }

  // ---- exchange (sharded form): slots in the caller's arena, one comm stream
  size_t x_off = 0;
  int x_n = 0;
  struct Slot {
    uint8_t* send;
    uint8_t* recv;
    size_t send_off, recv_off;
  };
  auto slot = [&](size_t bytes) {
    Slot sl;
    sl.send_off = x_off;
    sl.recv_off = x_off + xch_align(bytes);
    x_off += xch_slot(bytes, W);
    sl.send = (uint8_t*)sh->x->d_arena + sl.send_off;
    sl.recv = (uint8_t*)sh->x->d_arena + sl.recv_off;
    return sl;
  };
  // every rank's `bytes` at its slot's send -> recv (rank-major), ordered
  // after the work queued on `s` so far; `s` then waits for the result
  auto gather = [&](hipStream_t s, const Slot& sl, size_t bytes) -> int {
    hipEvent_t e0 = xev[2 * x_n], e1 = xev[2 * x_n + 1];
    x_n++;
    TPST_HIP(ctx, hipEventRecord(e0, s));
    TPST_HIP(ctx, hipStreamWaitEvent(ctx->comm, e0, 0));
    if (sh->x->allgather(sh->x->user, sl.send_off, sl.recv_off, bytes, (void*)ctx->comm))
      return fail(ctx, TPST_E_STATE, "exchange all-gather failed");
    TPST_HIP(ctx, hipEventRecord(e1, ctx->comm));
    TPST_HIP(ctx, hipStreamWaitEvent(s, e1, 0));
    return TPST_OK;
  };
  if (shd && (sh->x->arena_bytes < tpst_open_sharded_arena_bytes(n, W) || !sh->x->d_arena || !sh->x->allgather))
    return fail(ctx, TPST_E_ARG, "exchange arena smaller than tpst_open_sharded_arena_bytes");

  // ---- device buffers (allocated before any stream runs: no hipFree mid-open)
  const size_t Ch = C > 1 ? C / 2 : 1;
  const size_t Ca0 = shd ? Cl : C;  // a-side bases resident: own rows or all
  auto& [up, A, P, Y, chiC, ScA, ScB, ScC, ScD, xa, xb, xd, xh, xp, xl, LAo, Hb, Lb, gts, canA, canC, canD, pstA, pstB,
         Wall, Wiall, SqT, SqG, SqM, chis_own, tLoc, A1x, A1, tA1, Hbl, Lbl] = st->ob;
  TPST_HIP(ctx, up.grow(up_bytes));
  TPST_HIP(ctx, Wall.grow(2 * C * 32));  // round r's 2^r fold weights at offset 2^r - 1
  TPST_HIP(ctx, Wiall.grow(2 * C * 32));
  TPST_HIP(ctx, A.grow(Ca0 * 96));
  TPST_HIP(ctx, P.grow(Ca0 * 96));
  TPST_HIP(ctx, Y.grow(C * 32));
  TPST_HIP(ctx, chiC.grow(C * 32));
  TPST_HIP(ctx, ScA.grow(2 * C * 32));
  TPST_HIP(ctx, ScB.grow(C * 32));
  TPST_HIP(ctx, ScC.grow(C * 32));
  TPST_HIP(ctx, xa.grow(C * sizeof(Xyzz<Fq>)));
  TPST_HIP(ctx, xb.grow(2 * sizeof(Xyzz<Fq>)));
  TPST_HIP(ctx, xd.grow((k + 1) * sizeof(Xyzz<Fq2>)));
  TPST_HIP(ctx, xh.grow(C * sizeof(Xyzz<Fq2>)));
  TPST_HIP(ctx, xp.grow(((size_t)m + 1) * sizeof(Xyzz<Fq>)));
  for (int i = 0; i < 3; i++) {  // prepared h^(r) in slot r % 3
    TPST_HIP(ctx, Hb[i].grow(Ch * 192));
    TPST_HIP(ctx, Lb[i].grow(Ch * N_LINE_COEFFS * sizeof(LineCoeff)));
    if (shd) {
      TPST_HIP(ctx, Hbl[i].grow((Ch / W ? Ch / W : 1) * 192));
      TPST_HIP(ctx, Lbl[i].grow((Ch / W ? Ch / W : 1) * N_LINE_COEFFS * sizeof(LineCoeff)));
    }
  }
  TPST_HIP(ctx, gts.grow(2 * sizeof(Fq12)));
  for (int i = 0; i < 2; i++) {
    TPST_HIP(ctx, ScD[i].grow(8 * C * 32));
    TPST_HIP(ctx, xl[i].grow(C * sizeof(Xyzz<Fq>)));
    TPST_HIP(ctx, LAo[i].grow(8 * sizeof(Fq12)));
    // sized for either engine (RNS form: rns::RES_WORDS u32 per Fq12)
    TPST_HIP(ctx, SqT[i].grow(4 * 64 * MIPP_TAB_F12_BYTES));
    TPST_HIP(ctx, SqG[i].grow(2 * 10 * MIPP_TAB_F12_BYTES));
  }
  TPST_HIP(ctx, SqM.grow(128 * MIPP_TAB_F12_BYTES));
  TPST_HIP(ctx, canA.grow(2 * 576));
  TPST_HIP(ctx, canC.grow((size_t)(m + 1) * 192));
  TPST_HIP(ctx, canD.grow(96 + (size_t)k * 192));
  TPST_HIP(ctx, pstA.grow(pst_open_scratch_words(st, m) * 4));
  TPST_HIP(ctx, pstB.grow(pst_open_scratch_words(st, k) * 4));
  if (!shd && st->t_A_n < C) {
    TPST_HIP(ctx, st->t_A.alloc(fbt_words<Fq>(C) * 4));
    st->t_A_n = C;
  }
  if (shd) TPST_HIP(ctx, tLoc.grow(fbt_words<Fq>(Cl) * 4));
  if (shd || rb >= 0) {
    const size_t len1 = C >> (shd ? r1 : rb);
    TPST_HIP(ctx, A1x.grow(len1 * X1));
    TPST_HIP(ctx, A1.grow(len1 * 96));
    TPST_HIP(ctx, tA1.grow(fbt_words<Fq>(len1) * 4));
  }
  {  // G2 preparation scratch: the prepared h^(r) (global: <= C / 2 points, a rank's: <= C / 2W)
    size_t mx = 0;
    for (int r = 1; r <= m; r++) {
      if (need_glob[r]) mx = std::max(mx, C >> r);
      if (need_loc[r]) mx = std::max(mx, (C >> r) / W);
    }
    if (mx)
      if (int rc = prep_scratch_for(ctx, st, mx)) return rc;
  }
  const uint32_t* H0 = st->ph[odd]->u();
  const LineCoeff* L0 = (const LineCoeff*)st->hprep[odd].p;
  const uint32_t* tH = st->t_h[odd].u();
  // a rank's own positions of the SRS side (every W-th of h, its prepared
  // lines and its table), cached per (W, rank, parity)
  const uint32_t *H0l = H0, *tHl = tH;
  const LineCoeff* L0l = L0;
  if (shd) {
    SrsState::Local& lc = st->local[odd];
    if (lc.W != W || lc.rank != rho) {
      const size_t tb = fbt_words<Fq2>(1) * 4;  // one point's table block
      const size_t lb = sizeof(LineCoeff);
      TPST_HIP(ctx, lc.H0.alloc(Cl * 192));
      TPST_HIP(ctx, lc.L0.alloc(Cl * N_LINE_COEFFS * lb));
      TPST_HIP(ctx, lc.tH.alloc(Cl * tb));
      TPST_HIP(ctx, hipMemcpy2DAsync(lc.H0.p, 192, (const uint8_t*)H0 + 192 * rho, 192 * W, 192, Cl,
                                     hipMemcpyDeviceToDevice, sA));
      // coefficient-major [idx][pair]: row idx * Cl + j of the copy is column
      // W (idx * Cl + j) + rho of the cache (C = W Cl)
      TPST_HIP(ctx, hipMemcpy2DAsync(lc.L0.p, lb, (const uint8_t*)L0 + lb * rho, lb * W, lb, Cl * N_LINE_COEFFS,
                                     hipMemcpyDeviceToDevice, sA));
      TPST_HIP(ctx, hipMemcpy2DAsync(lc.tH.p, tb, (const uint8_t*)tH + tb * rho, tb * W, tb, Cl,
                                     hipMemcpyDeviceToDevice, sA));
      lc.W = W;
      lc.rank = rho;
    }
    H0l = lc.H0.u();
    L0l = (const LineCoeff*)lc.L0.p;
    tHl = lc.tH.u();
  }
  const uint32_t* tA = shd ? tLoc.u() : st->t_A.u();  // the a-side table (rebased at the hand-over)
  size_t Ca = Ca0;                                    // its base count
  auto dup = [&](size_t byte_off) { return (uint32_t*)((uint8_t*)up.p + byte_off); };

  // ---- prologue (stream A): this rank's comm_list rows -> Montgomery, y = chi(b), canonical chi
  {
    uint8_t* a_stage = pin + up_off[m] + (2 + m) * 32;  // a_rev (canonical) -> D
    for (int i = 0; i < k; i++) memcpy(a_stage + 32 * i, point + 4 * (k - 1 - i), 32);
  }
  if (shd) {
    std::vector<uint64_t> own(Cl * 12);
    for (size_t j = 0; j < Cl; j++) memcpy(&own[12 * j], comms + 12 * (W * j + rho), 96);
    TPST_HIP(ctx, hipMemcpyAsync(A.p, own.data(), Cl * 96, hipMemcpyHostToDevice, sA));
    TPST_HIP(ctx, hipStreamSynchronize(sA));  // `own` is pageable and local
  } else {
    memcpy(pin + cm_off, comms, C * 96);  // pinned: an asynchronous copy, not HIP's pageable staging
    TPST_HIP(ctx, hipMemcpyAsync(A.p, pin + cm_off, C * 96, hipMemcpyHostToDevice, sA));
  }
  TPST_HIP(ctx, points_to_mont<Fq>(sA, A.u(), A.u(), Ca0));
  const uint32_t* chis = nullptr;
  if (lead) {
    chis = p->chis.u();
  } else {
    if (int rc = chi_b_table(ctx, m, k, point, chis_own)) return rc;
    chis = chis_own.u();
  }
  TPST_HIP(ctx, hipMemcpyAsync(Y.p, chis, C * 32, hipMemcpyDeviceToDevice, sA));
  TPST_HIP(ctx, fr_from_mont(sA, chis, chiC.u(), C));
  TPST_HIP(ctx, hipEventRecord(ev[EV_PRE], sA));
  for (hipStream_t s2 : {sB, sLA[0], sLA[1]}) TPST_HIP(ctx, hipStreamWaitEvent(s2, ev[EV_PRE], 0));
  pf.begin(ST_MIPP_PROVE, sA);  // mipp.rs:38-149 (sqrt_pst.rs:211-214)
  TraceRange trace_mipp("mipp_prove");

  // ---- look-ahead stream 1 (idle until round 1): the fold table over comm_list
  // (prebuilt by the commit of exactly these row commitments: used once), or
  // over this rank's rows
  if (shd) {
    TPST_HIP(ctx, fbt_build<Fq>(*arLA[1], sLA[1], A.u(), Cl, tLoc.u(), true));
  } else {
    const bool prebuilt = st->t_A_key.size() == 12 * C && !memcmp(st->t_A_key.data(), comms, C * 96);
    st->t_A_key.clear();
    if (!prebuilt) TPST_HIP(ctx, fbt_build<Fq>(*arLA[1], sLA[1], A.u(), C, st->t_A.u(), true));
  }
  TPST_HIP(ctx, hipEventRecord(ev[EV_TABLE], sLA[1]));
  // ---- stream B: U = MSM(comm_list, chi(b)) on that table, or the c_u the
  // ranks combined
  const uint64_t* U_given = shd ? sh->U : (p->has_u ? p->U : nullptr);
  if (U_given) {
    TPST_HIP(ctx, hipEventRecord(ev[EV_U], sB));
  } else {
    TPST_HIP(ctx, hipStreamWaitEvent(sB, ev[EV_TABLE], 0));
    TraceRange trace_msm("msm");  // sqrt_pst.rs:188-199
    pf.begin(ST_MSM_U, sB);
    FbGroups gu;
    gu.members = C;
    gu.L = gu.D = C;
    gu.glv = true;
    TPST_HIP(ctx, fbt_msm<Fq>(arB, sB, tA, chiC.u(), gu, (Xyzz<Fq>*)xd.p));
    pf.end(ST_MSM_U, sB);
    TPST_HIP(ctx, hipMemcpyAsync(pin + dn_U, xd.p, X1, hipMemcpyDeviceToHost, sB));
    TPST_HIP(ctx, hipEventRecord(ev[EV_U], sB));
  }
  // PST proof of q at a_rev (stream B, after round 0's cross terms)
  auto pst_q = [&]() -> int {
    TraceRange trace_pst("pst_open");  // sqrt_pst.rs:216-226
    pf.begin(ST_PST_OPEN, sB);
    const size_t a_off = up_off[m] + (2 + m) * 32;
    TPST_HIP(ctx, hipMemcpyAsync(dup(a_off), pin + a_off, (size_t)k * 32, hipMemcpyHostToDevice, sB));
    TPST_HIP(ctx, fr_to_mont(sB, dup(a_off), dup(a_off), k));
    Xyzz<Fq2>* x2 = (Xyzz<Fq2>*)xd.p + 1;
    TPST_HIP(ctx, pst_open_fbt_s<Fq2>(sB, arB, st, st->t_php.u(), st->nv - k, p->q.u(), k, dup(a_off), x2, pstB.u()));
    TPST_HIP(ctx, xyzz_to_affine_canonical<Fq2>(sB, x2, canD.u() + 24, k));
    TPST_HIP(ctx, hipMemcpyAsync(pin + dn_pst, canD.u() + 24, (size_t)k * 192, hipMemcpyDeviceToHost, sB));
    pf.end(ST_PST_OPEN, sB);
    return TPST_OK;
  };
  if (m == 0 && lead)
    if (int rc = pst_q()) return rc;

  // W_r[t] / Wi_r[t] (device, mipp_weights): products of the challenges
  // (inverses) folded so far, so that a^(r)_i = sum_t W_r[t] a_{i + t len},
  // h^(r)_i = sum_t Wi_r[t] h_{i + t len}
  std::vector<Fr> xs_inv;
  Fr cprev = Fr::one(), cprev_c = Fr::one();
  uint64_t la_digits[16] = {};
  bool have_U = false;
  hipEvent_t ev_t1 = nullptr;  // the table over the gathered a^(r1) (rank 0, sharded form)
  for (int r = 0; r < m; r++) {  // mipp.rs:58-120
    const double hq = open_trace() ? host_us() : 0.0;
    const size_t len = C >> r, s = len / 2, nW = (size_t)1 << r;
    const bool loc = shd && r < r1;  // this round on the rank's own rows
    // stage c_{r-1}, c_{r-1}^-1, the look-ahead factors and digits; upload
    // once (stream B, whose previous work -- the round's comms_u -- is
    // already done when the challenge exists: on A the upload queued behind
    // A's wait for the look-ahead), form this round's weights there; A, C, D
    // wait on it
    uint8_t* stg = pin + up_off[r];
    // look-ahead fold factors of h^(r) over h^(s), s = la_src(r): f_j = product
    // of c'_{r-1-b} over the set bits b of j (offset j len of h^(s)'s row)
    const int E = r == 0 ? 1 : 1 << (r - la_src(r));
    Fr f[8];
    f[0] = Fr::one();
    for (int j = 1; j < E; j++) {
      const int b = 31 - __builtin_clz((unsigned)j);
      f[j] = mul(f[j ^ (1 << b)], xs_inv[r - 1 - b]);
    }
    memcpy(stg, cprev_c.v, 32);
    memcpy(stg + 32, cprev.v, 32);
    for (int j = 0; j < E; j++) memcpy(stg + 64 + 32 * j, f[j].v, 32);
    memcpy(stg + 320, la_digits, 128);
    uint32_t* dup_r = dup(up_off[r]);
    uint32_t* dcp = dup_r + 8;   // c' = c_{r-1}^-1 (the y fold)
    uint32_t* dfs = dup_r + 16;  // f_0..f_{E-1}
    const uint64_t* ddig = (const uint64_t*)(dup_r + 80);
    TPST_HIP(ctx, hipMemcpyAsync(dup_r, stg, UP_ROUND, hipMemcpyHostToDevice, sB));
    TPST_HIP(ctx, mipp_weights(sB, Wall.u(), Wiall.u(), r, dup_r, dcp));
    uint32_t* dW = Wall.u() + 8 * (nW - 1);
    uint32_t* dWi = Wiall.u() + 8 * (nW - 1);
    TPST_HIP(ctx, hipEventRecord(ev_up(r), sB));
    // (round 0's A and D work -- the direct t and the first look-ahead --
    // needs no upload: they do not wait behind B's U MSM)
    if (r > 0) TPST_HIP(ctx, hipStreamWaitEvent(sA, ev_up(r), 0));

    if (rb >= 0 && r == rb + 1) {  // the rebase table from here on (B waits for it; D, A do below)
      tA = tA1.u();
      Ca = C >> rb;
      TPST_HIP(ctx, hipStreamWaitEvent(sB, ev_t1, 0));
    }
    if (shd && r == r1) {
      // -- hand-over: a^(r1) (len = 2W positions) folded by the owners of its
      // positions, gathered; rank 0 tabulates it and continues alone
      const size_t per = len / W;
      TPST_HIP(ctx, hipStreamWaitEvent(sB, ev[EV_TABLE], 0));
      TPST_HIP(ctx, mipp_scalars(sB, dW, nullptr, len, 0, Cl, ScB.u(), W, rho));
      FbGroups g;
      g.groups = per;
      g.members = C / len;
      g.L = per;
      g.D = 1;
      g.glv = true;
      const Slot sl = slot(per * X1);
      TPST_HIP(ctx, fbt_msm<Fq>(arB, sB, tA, ScB.u(), g, (Xyzz<Fq>*)sl.send));
      if (int rc = gather(sB, sl, per * X1)) return rc;
      if (!lead) {  // this rank's part is done (its transcript stops here: tpst.h)
        pf.end(ST_MIPP_PROVE, sA);
        pf.end(ST_SQRT_OPEN, sA);
        for (hipStream_t s2 : {sA, sB, sLA[0], sLA[1], sC, ctx->comm}) TPST_HIP(ctx, hipStreamSynchronize(s2));
        sp.store(tr);
        return TPST_OK;
      }
      // recv[w][j] = a^(r1) at position W j + w
      for (int w = 0; w < W; w++)
        TPST_HIP(ctx, hipMemcpy2DAsync((uint8_t*)A1x.p + w * X1, W * X1, sl.recv + (size_t)w * per * X1, X1, X1, per,
                                       hipMemcpyDeviceToDevice, sB));
      TPST_HIP(ctx, xyzz_to_affine_mont<Fq>(sB, (const Xyzz<Fq>*)A1x.p, A1.u(), len));
      TPST_HIP(ctx, fbt_build<Fq>(arB, sB, A1.u(), len, tA1.u(), true));
      ev_t1 = xev[2 * x_n];  // past the gathers' events
      TPST_HIP(ctx, hipEventRecord(ev_t1, sB));
      tA = tA1.u();
      Ca = len;
    }

    uint8_t* dn_r = pin + dn_round + (size_t)r * DN_ROUND;
    // -- A: t_l / t_r of this round, enqueued before B from round 1 on (the
    // combination gates the odd rounds and needs only the upload, while B's
    // table MSM costs the host tens of microseconds to enqueue; 2^20 open
    // 11.40 -> 11.25 ms, 2^24 25.5 -> 24.9 ms, profiles/r06/ab/ab_open_order_prio.txt)
    auto enqueue_a = [&]() -> int {
      if (r == 0) {  // direct: the rotated comm_list (affine) against h^(0)
        if (loc) {  // this rank's pairs (a_i, h_{s+i}), (a_{s+i}, h_i), i = rho mod W
          TPST_HIP(ctx, affine_rot(sA, A.u(), P.u(), Cl, 24));
          arA.reset();
          TPST_HIP(ctx, arA.reserve(multi_pairing_scratch(2, s / W)));
          const Slot sl = slot(2 * sizeof(Fq12));
          TPST_HIP(ctx, multi_pairing_prepared(arA, sA, P.u(), H0l, L0l, 2, s / W, (Fq12*)sl.send, false, s / W, 0));
          if (int rc = gather(sA, sl, 2 * sizeof(Fq12))) return rc;
          TPST_HIP(ctx, gt_prod_final(sA, (const Fq12*)sl.recv, W, 2, (Fq12*)gts.p));
        } else {
          TPST_HIP(ctx, affine_rot(sA, A.u(), P.u(), C, 24));
          arA.reset();
          TPST_HIP(ctx, arA.reserve(multi_pairing_scratch(2, s)));
          TPST_HIP(ctx, multi_pairing_prepared(arA, sA, P.u(), H0, L0, 2, s, (Fq12*)gts.p, true, s, 0));
        }
      } else {  // round r-1's look-ahead products, combined with c_{r-1}
        TPST_HIP(ctx, hipStreamWaitEvent(sA, ev_la(r - 1), 0));
        TPST_HIP(ctx, mipp_combine_tab(sA, (Fq12*)SqT[(r - 1) & 1].p, ddig, (Fq12*)SqG[(r - 1) & 1].p,
                                       (Fq12*)SqM.p, (Fq12*)gts.p));
      }
      TPST_HIP(ctx, fq12_from_mont(sA, (Fq12*)gts.p, canA.u(), 2));
      TPST_HIP(ctx, hipMemcpyAsync(dn_r + 2 * X1, canA.p, 1152, hipMemcpyDeviceToHost, sA));
      TPST_HIP(ctx, hipEventRecord(ev_a(r), sA));
      return TPST_OK;
    };
    const bool a_first = r > 0;
    if (a_first)
      if (int rc = enqueue_a()) return rc;
    // -- B: y fold by the previous challenge, cross MSMs u_l / u_r
    // (u_l = a[:s]^y[s:], u_r = a[s:]^y[:s], on the comm_list table); B goes
    // before the look-ahead: its comms_u gate the transcript, and the
    // look-ahead enqueue below costs the host tens of launches
    TPST_HIP(ctx, hipStreamWaitEvent(sB, ev_up(r), 0));
    if (r > 0) TPST_HIP(ctx, compress_fr(sB, Y.u(), len, dcp));  // y_l + c' y_r (mipp.rs:124-136)
    {  // (round 0 as two variable-base K2 MSMs over comm_list, skipping the
       // table build, measured slower: 3.4 vs 1.7 ms at 2^20)
      TPST_HIP(ctx, hipStreamWaitEvent(sB, ev[EV_TABLE], 0));
      FbGroups g;
      g.groups = 2;
      g.glv = true;
      if (loc) {  // partial sums over this rank's rows, gathered and summed
        TPST_HIP(ctx, mipp_scalars(sB, dW, Y.u(), len, s, Cl, ScB.u(), W, rho));
        g.members = C / len * s / W;
        g.L = len / W;
        g.D = s / W;
        const Slot sl = slot(2 * X1);
        TPST_HIP(ctx, fbt_msm<Fq>(arB, sB, tA, ScB.u(), g, (Xyzz<Fq>*)sl.send));
        if (int rc = gather(sB, sl, 2 * X1)) return rc;
        TPST_HIP(ctx, xyzz_sum_groups(sB, (const Xyzz<Fq>*)sl.recv, W, 2, (Xyzz<Fq>*)xb.p));
      } else {
        TPST_HIP(ctx, mipp_scalars(sB, dW, Y.u(), len, s, Ca, ScB.u()));
        g.members = Ca / len * s;
        g.L = len;
        g.D = s;
        TPST_HIP(ctx, fbt_msm<Fq>(arB, sB, tA, ScB.u(), g, (Xyzz<Fq>*)xb.p));
      }
    }
    TPST_HIP(ctx, hipMemcpyAsync(dn_r, xb.p, 2 * X1, hipMemcpyDeviceToHost, sB));
    TPST_HIP(ctx, hipEventRecord(ev_b(r), sB));
    const double hb = open_trace() ? host_us() : 0.0;
    if (!a_first)
      if (int rc = enqueue_a()) return rc;
    const double ha = open_trace() ? host_us() : 0.0;
    auto enqueue_c = [&]() -> int {
      // -- C: h^(r) prepared for the look-ahead of round r+1: at this rank's
      // positions (sharded look-aheads) and / or at all
      const bool c_glob = need_glob[r];
      if (need_loc[r] || c_glob) {
        TPST_HIP(ctx, hipStreamWaitEvent(sC, ev_up(r), 0));
        if (r >= 3) TPST_HIP(ctx, hipStreamWaitEvent(sC, ev_la(r - 2), 0));  // last reader of h^(r-3)'s slot
      }
      if (need_loc[r]) {
        const size_t ln = len / W;
        TPST_HIP(ctx, mipp_scalars(sC, dWi, nullptr, len, 0, Cl, ScC.u(), W, rho));
        FbGroups g;
        g.groups = ln;
        g.members = C / len;
        g.L = ln;
        g.D = 1;
        TPST_HIP(ctx, fbt_msm<Fq2>(arC, sC, tHl, ScC.u(), g, (Xyzz<Fq2>*)xh.p));
        TPST_HIP(ctx, xyzz_to_affine_mont<Fq2>(sC, (Xyzz<Fq2>*)xh.p, Hbl[r % 3].u(), ln));
        TPST_HIP(ctx, g2_prepare_batch(sC, Hbl[r % 3].u(), ln, (LineCoeff*)Lbl[r % 3].p,
                                       st->prep_scratch.u()));
        TPST_HIP(ctx, hipEventRecord(ev_cl(r), sC));
        last_c = r;
      }
      if (c_glob) {
        TPST_HIP(ctx, mipp_scalars(sC, dWi, nullptr, len, 0, C, ScC.u()));
        FbGroups g;
        g.groups = len;
        g.members = C / len;
        g.L = len;
        g.D = 1;
        TPST_HIP(ctx, fbt_msm<Fq2>(arC, sC, tH, ScC.u(), g, (Xyzz<Fq2>*)xh.p));
        TPST_HIP(ctx, xyzz_to_affine_mont<Fq2>(sC, (Xyzz<Fq2>*)xh.p, Hb[r % 3].u(), len));
        TPST_HIP(ctx, g2_prepare_batch(sC, Hb[r % 3].u(), len, (LineCoeff*)Lb[r % 3].p,
                                       st->prep_scratch.u()));
        TPST_HIP(ctx, hipEventRecord(ev_c(r), sC));
        last_c = r;
      }
      return TPST_OK;
    };
    const bool c_first = r == 1;  // look-ahead 1 pairs this round's h
    if (c_first)
      if (int rc = enqueue_c()) return rc;
    // -- D: look-ahead products of this round's vectors for round r+1
    if (len >= 4) {
      hipStream_t sD = sLA[r & 1];
      Arena& arD = *arLA[r & 1];
      if (r > 0) TPST_HIP(ctx, hipStreamWaitEvent(sD, ev_up(r), 0));
      if (ev_t1) TPST_HIP(ctx, hipStreamWaitEvent(sD, ev_t1, 0));
      const size_t ln = loc ? len / W : len;  // positions this rank pairs
      arD.reset();
      TPST_HIP(ctx, arD.reserve(mipp_lookahead_scratch(ln / 4, E) + 4096));
      Slot sl{};
      Fq12* la_out = (Fq12*)LAo[r & 1].p;
      if (loc) {
        sl = slot(8 * sizeof(Fq12));
        la_out = (Fq12*)sl.send;
      }
      if (r == 0) {  // a^(0) = comm_list (affine), h^(0) prepared
        if (loc)
          TPST_HIP(ctx, mipp_lookahead(arD, sD, L0l, Cl, H0l, A.u(), false, ln, 1, la_out, false));
        else
          TPST_HIP(ctx, mipp_lookahead(arD, sD, L0, C, H0, A.u(), false, len, 1, la_out));
      } else {
        // E fold sets f_j a^(r): h^(r)_q = sum_j f_j h^(s)[q + j len]
        TPST_HIP(ctx, hipStreamWaitEvent(sD, ev[EV_TABLE], 0));
        uint32_t* sc = ScD[r & 1].u();
        FbGroups g;
        g.groups = ln;
        g.L = ln;
        g.D = 1;
        g.sets = (size_t)E;
        g.glv = true;
        if (loc) {
          TPST_HIP(ctx, mipp_scalar_sets(sD, dW, dfs, E, len, Cl, sc, W, rho));
          g.members = C / len;
          g.set_stride = Cl;
        } else {
          TPST_HIP(ctx, mipp_scalar_sets(sD, dW, dfs, E, len, Ca, sc));
          g.members = Ca / len;
          g.set_stride = Ca;
        }
        TPST_HIP(ctx, fbt_msm<Fq>(arD, sD, tA, sc, g, (Xyzz<Fq>*)xl[r & 1].p));
        const int src = la_src(r);  // h^(0), or h^(src) prepared by stream C in round src
        const uint32_t* hp = loc ? H0l : H0;
        const LineCoeff* lp = loc ? L0l : L0;
        if (src > 0) {
          TPST_HIP(ctx, hipStreamWaitEvent(sD, loc ? ev_cl(src) : ev_c(src), 0));
          hp = (loc ? Hbl : Hb)[src % 3].u();
          lp = (const LineCoeff*)(loc ? Lbl : Lb)[src % 3].p;
        }
        TPST_HIP(ctx, mipp_lookahead(arD, sD, lp, (size_t)E * ln, hp, xl[r & 1].u(), true, ln, E, la_out, !loc));
      }
      if (loc) {
        if (int rc = gather(sD, sl, 8 * sizeof(Fq12))) return rc;
        TPST_HIP(ctx, gt_prod_final(sD, (const Fq12*)sl.recv, W, 8, (Fq12*)LAo[r & 1].p));
      }
      TPST_HIP(ctx, mipp_sq_tables(sD, (Fq12*)LAo[r & 1].p, (Fq12*)SqT[r & 1].p, (Fq12*)SqG[r & 1].p));
      TPST_HIP(ctx, hipEventRecord(ev_la(r), sD));
    }

    const double hd = open_trace() ? host_us() : 0.0;
    if (r == 0 && lead)
      if (int rc = pst_q()) return rc;

    const double hp = open_trace() ? host_us() : 0.0;
    if (!c_first)
      if (int rc = enqueue_c()) return rc;

    if (r == rb) {  // the rebase (see rb above), consumed from round rb + 1 on
      const hipStream_t sR = ctx->comm;
      TPST_HIP(ctx, hipStreamWaitEvent(sR, ev_up(r), 0));
      TPST_HIP(ctx, hipStreamWaitEvent(sR, ev[EV_TABLE], 0));
      TPST_HIP(ctx, mipp_scalars(sR, dW, nullptr, len, 0, C, ScA.u()));
      FbGroups g;
      g.groups = len;
      g.members = C / len;
      g.L = len;
      g.D = 1;
      g.glv = true;
      TPST_HIP(ctx, fbt_msm<Fq>(ctx->io, sR, tA, ScA.u(), g, (Xyzz<Fq>*)A1x.p));
      TPST_HIP(ctx, xyzz_to_affine_mont<Fq>(sR, (const Xyzz<Fq>*)A1x.p, A1.u(), len));
      TPST_HIP(ctx, fbt_build<Fq>(ctx->io, sR, A1.u(), len, tA1.u(), true));
      ev_t1 = ev[EV_REBASE];
      TPST_HIP(ctx, hipEventRecord(ev_t1, sR));
    }

    // -- host: transcript (mipp.rs:56, 97-101) and the challenge
    if (!have_U) {
      TPST_HIP(ctx, hipEventSynchronize(ev[EV_U]));
      if (U_given)
        memcpy(proof->U, U_given, 96);
      else
        xyzz_to_canonical_host<Fq>(pin + dn_U, 1, proof->U);
      uint8_t b[96];
      g1_bytes(proof->U, b);
      sp.absorb_bytes(b, 96);
      have_U = true;
    }
    // comms_u (stream B) is ready well before comms_t (the final
    // exponentiations): absorb it while stream A finishes (mipp.rs:97-100
    // order: u_l, u_r, t_l, t_r)
    const double h0 = host_us();
    TPST_HIP(ctx, hipEventSynchronize(ev_b(r)));
    const double h1 = host_us();
    xyzz_to_canonical_host<Fq>(dn_r, 2, proof->comms_u[r][0]);
    uint8_t b[96];
    g1_bytes(proof->comms_u[r][0], b);
    sp.absorb_bytes(b, 96);
    g1_bytes(proof->comms_u[r][1], b);
    sp.absorb_bytes(b, 96);
    const double h2 = host_us();
    TPST_HIP(ctx, hipEventSynchronize(ev_a(r)));
    const double h3 = host_us();
    memcpy(proof->comms_t[r][0], dn_r + 2 * X1, 576);
    memcpy(proof->comms_t[r][1], dn_r + 2 * X1 + 576, 576);
    sp.absorb_bytes((const uint8_t*)proof->comms_t[r][0], 576);
    sp.absorb_bytes((const uint8_t*)proof->comms_t[r][1], 576);
    const double h4 = host_us();
    uint64_t ci_c[4];
    sp.challenge(ci_c);  // mipp.rs:101
    const Fr c_inv = fr_canon(ci_c);
    const double h5 = host_us();
    const Fr c = fr_inv(c_inv);  // mipp.rs:106
    if (open_trace())
      fprintf(stderr,
              "open round %d%s: enqueue %.0f (B %.0f A %.0f D %.0f pst %.0f C %.0f) wait_u %.0f absorb_u %.0f wait_t %.0f "
              "absorb_t %.0f challenge %.0f inv %.0f us\n",
              r, loc ? " (sharded)" : "", h0 - hq, hb - hq, ha - hb, hd - ha, hp - hd, h0 - hp, h1 - h0, h2 - h1,
              h3 - h2, h4 - h3, h5 - h4, host_us() - h5);
    xs_inv.push_back(c_inv);
    cprev = c_inv;
    cprev_c = c;
    // base-x digits of (c^-1, c, c^-1, c) for the next round's combination
    {
      uint64_t ci[4], cc[4];
      fr_out(c_inv, ci);
      fr_out(c, cc);
      base_x_digits(ci, la_digits);
      base_x_digits(cc, la_digits + 4);
      memcpy(la_digits + 8, la_digits, 64);
    }
  }
  if (!have_U) {
    TPST_HIP(ctx, hipEventSynchronize(ev[EV_U]));
    if (U_given)
      memcpy(proof->U, U_given, 96);
    else
      xyzz_to_canonical_host<Fq>(pin + dn_U, 1, proof->U);
    uint8_t b[96];
    g1_bytes(proof->U, b);
    sp.absorb_bytes(b, 96);
  }

  // ---- epilogue: final_a (A), final_h (C), pst_proof_h (B); rs need only the
  // transcript state after the last round (mipp.rs:138-141)
  // final weights W_m, Wi_m (device); the p_h evaluations of mipp.rs:159-180,
  // prod over the set bits j of t of c^-1_{m-1-j}, are exactly Wi_m[t]
  {
    uint8_t* stg = pin + up_off[m];
    memcpy(stg, cprev_c.v, 32);
    memcpy(stg + 32, cprev.v, 32);
    for (int i = 0; i < m; i++) {
      uint64_t cc[4];
      sp.challenge(cc);
      const Fr rr = fr_canon(cc);
      memcpy(stg + 32 * (2 + i), rr.v, 32);
    }
  }
  uint32_t* dfin = dup(up_off[m]);
  TPST_HIP(ctx, hipMemcpyAsync(dfin, pin + up_off[m], (2 + m) * 32, hipMemcpyHostToDevice, sA));
  TPST_HIP(ctx, mipp_weights(sA, Wall.u(), Wiall.u(), m, dfin, dfin + 8));
  const uint32_t* dWm = Wall.u() + 8 * (C - 1);
  const uint32_t* dWim = Wiall.u() + 8 * (C - 1);
  TPST_HIP(ctx, hipEventRecord(ev[EV_FINAL_UP], sA));
  TPST_HIP(ctx, hipStreamWaitEvent(sA, ev[EV_TABLE], 0));
  if (ev_t1) TPST_HIP(ctx, hipStreamWaitEvent(sA, ev_t1, 0));
  {  // final_a = a^(m)_0 (one group over the a-side bases: all C, or the gathered a^(r1))
    FbGroups g;
    g.members = Ca;
    TPST_HIP(ctx, mipp_scalars(sA, dWm, nullptr, 1, 0, Ca, ScA.u()));
    g.glv = true;
    TPST_HIP(ctx, fbt_msm<Fq>(arA, sA, tA, ScA.u(), g, (Xyzz<Fq>*)xa.p));
    TPST_HIP(ctx, hipMemcpyAsync(pin + dn_final, xa.p, X1, hipMemcpyDeviceToHost, sA));
  }
  TPST_HIP(ctx, hipStreamWaitEvent(sCe, ev[EV_FINAL_UP], 0));
  if (last_c >= 0) TPST_HIP(ctx, hipStreamWaitEvent(sCe, ev_c(last_c), 0));  // xh / ScC / arC reuse
  if (last_c >= 0 && need_loc[last_c]) TPST_HIP(ctx, hipStreamWaitEvent(sCe, ev_cl(last_c), 0));
  {  // final_h = h^(m)_0
    FbGroups g;
    g.members = C;
    TPST_HIP(ctx, mipp_scalars(sCe, dWim, nullptr, 1, 0, C, ScC.u()));
    TPST_HIP(ctx, fbt_msm<Fq2>(arC, sCe, tH, ScC.u(), g, (Xyzz<Fq2>*)xh.p));
    TPST_HIP(ctx, hipMemcpyAsync(pin + dn_fh, xh.p, X2, hipMemcpyDeviceToHost, sCe));
    TPST_HIP(ctx, hipEventRecord(ev[EV_C_DONE], sCe));
  }
  if (m > 0) {  // pst_proof_h = open_g1(p_h, rs) (mipp.rs:144)
    TPST_HIP(ctx, hipStreamWaitEvent(sB, ev[EV_FINAL_UP], 0));
    TPST_HIP(ctx, pst_open_fbt_s<Fq>(sB, arB, st, st->t_pgp.u(), st->nv - m, dWim, m, dfin + 16,
                                     (Xyzz<Fq>*)xp.p, pstA.u()));
    TPST_HIP(ctx, xyzz_to_affine_canonical<Fq>(sB, (Xyzz<Fq>*)xp.p, canC.u() + 48, m));
    TPST_HIP(ctx, hipMemcpyAsync(pin + dn_ph, canC.u() + 48, (size_t)m * 96, hipMemcpyDeviceToHost, sB));
  }
  TPST_HIP(ctx, hipEventRecord(ev[EV_B_DONE], sB));
  if (pf.on) {  // device spans end when every stream of the opening has drained
    TPST_HIP(ctx, hipEventRecord(ev[EV_D_DONE], sLA[0]));
    TPST_HIP(ctx, hipEventRecord(ev[EV_A_DONE], sLA[1]));
    for (int e : {(int)EV_B_DONE, (int)EV_C_DONE, (int)EV_D_DONE, (int)EV_A_DONE})
      TPST_HIP(ctx, hipStreamWaitEvent(sA, ev[e], 0));
    pf.end(ST_MIPP_PROVE, sA);
    pf.end(ST_SQRT_OPEN, sA);
  }
  for (hipStream_t s2 : {sA, sB, sLA[0], sLA[1], sC}) TPST_HIP(ctx, hipStreamSynchronize(s2));
  if (shd || rb >= 0) TPST_HIP(ctx, hipStreamSynchronize(ctx->comm));
  xyzz_to_canonical_host<Fq>(pin + dn_final, 1, proof->final_a);
  xyzz_to_canonical_host<Fq2>(pin + dn_fh, 1, proof->final_h);
  if (m > 0) memcpy(proof->pst_proof_h, pin + dn_ph, (size_t)m * 96);
  memcpy(proof->pst_proof, pin + dn_pst, (size_t)k * 192);
  sp.store(tr);
  return TPST_OK;
}

extern "C" int tpst_poly_open(tpst_ctx* ctx, tpst_poly* p, tpst_transcript* tr, const uint64_t* comms,
                              const uint64_t* point, const uint64_t* T, tpst_open_proof* proof) {
  (void)T;  // the reference passes T but the prover does not use it (mipp.rs:38)
  if (!ctx || !p || !tr || !comms || !point || !proof) return fail(ctx, TPST_E_ARG, "null argument");
  return poly_open(ctx, p, tr, p->n, comms, point, proof, nullptr);
}

extern "C" int tpst_poly_open_sharded(tpst_ctx* ctx, tpst_poly* p, tpst_transcript* tr, int n, const uint64_t* comms,
                                      const uint64_t* point, const uint64_t* U, const tpst_exchange* x,
                                      tpst_open_proof* proof) {
  if (!ctx || !tr || !comms || !point || !U || !x) return fail(ctx, TPST_E_ARG, "null argument");
  if (x->world < 1 || (x->world & (x->world - 1)) || x->rank < 0 || x->rank >= x->world)
    return fail(ctx, TPST_E_ARG, "world must be a power of two and 0 <= rank < world");
  if (x->rank == 0 && (!p || !proof)) return fail(ctx, TPST_E_ARG, "rank 0 needs the opening handle and the proof");
  if (p && p->n != n) return fail(ctx, TPST_E_ARG, "handle num_vars != n");
  if (!point_valid<Fq>(U)) return fail(ctx, TPST_E_ARG, "c_u is not a valid G1 point");
  for (int i = 0; i < n; i++)
    if (!fr_ok(point + 4 * i)) return fail(ctx, TPST_E_ARG, "point coordinate >= r");
  const int m = n / 2;
  if (shard_rounds(m, x->world) == 0) {  // too few rows to split: rank 0 opens alone
    if (x->rank != 0) return TPST_OK;
    const bool had = p->has_u;
    uint64_t keep[12];
    memcpy(keep, p->U, 96);
    memcpy(p->U, U, 96);
    p->has_u = true;
    const int rc = poly_open(ctx, p, tr, n, comms, point, proof, nullptr);
    memcpy(p->U, keep, 96);
    p->has_u = had;
    return rc;
  }
  Shard sh;
  sh.W = x->world;
  sh.rank = x->rank;
  sh.x = x;
  sh.U = U;
  return poly_open(ctx, p, tr, n, comms, point, proof, &sh);
}

// -------------------------------------------------------------- verify ---
// The verifier is a handful of short serial chains (two-term scalar
// combinations, subgroup checks) plus three pairing products and the GT
// exponentiations: the chains run on host threads (host_curve.h, ~30 ns per
// Fq product against ~1.6 us on a lone GPU lane), the pairing products in ONE
// device launch (groups padded with infinity pairs), the GT powers on a side
// stream (pairing.hip k_gt_pow_wave).
static bool gt_is_one(const uint64_t* gt) {
  if (gt[0] != 1) return false;
  for (int i = 1; i < 72; i++)
    if (gt[i]) return false;
  return true;
}

static void push(std::vector<uint64_t>& v, const uint64_t* p, size_t n) { v.insert(v.end(), p, p + n); }

// pairs of one pairing-product check (canonical affine G1 12 u64, G2 24 u64)
struct PairSet {
  std::vector<uint64_t> g1, g2;
  size_t n() const { return g1.size() / 12; }
};

// prod_{pairs in group g} e(P, Q) for every group, one multi-pairing launch
// (groups padded to a common length with infinity pairs, which contribute 1)
static int pairing_groups(tpst_ctx* ctx, const std::vector<const PairSet*>& sets, std::vector<uint64_t>& gts) {
  const size_t G = sets.size();
  size_t n = 1;
  for (const PairSet* p : sets) n = std::max(n, p->n());
  std::vector<uint64_t> g1(G * n * 12, 0), g2(G * n * 24, 0);
  for (size_t g = 0; g < G; g++) {
    std::copy(sets[g]->g1.begin(), sets[g]->g1.end(), g1.begin() + g * n * 12);
    std::copy(sets[g]->g2.begin(), sets[g]->g2.end(), g2.begin() + g * n * 24);
  }
  hipStream_t s = ctx->stream;
  DevBuf a, b, f, o;
  TPST_HIP(ctx, a.alloc(G * n * 96));
  TPST_HIP(ctx, b.alloc(G * n * 192));
  TPST_HIP(ctx, f.alloc(G * sizeof(Fq12)));
  TPST_HIP(ctx, o.alloc(G * 576));
  TPST_HIP(ctx, hipMemcpyAsync(a.p, g1.data(), G * n * 96, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, hipMemcpyAsync(b.p, g2.data(), G * n * 192, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, points_to_mont<Fq>(s, a.u(), a.u(), G * n));
  TPST_HIP(ctx, points_to_mont<Fq2>(s, b.u(), b.u(), G * n));
  TPST_HIP(ctx, multi_pairing(ctx->arena, s, a.u(), b.u(), G, n, (Fq12*)f.p));
  TPST_HIP(ctx, fq12_from_mont(s, (Fq12*)f.p, o.u(), G));
  gts.assign(G * 72, 0);
  TPST_HIP(ctx, hipMemcpyAsync(gts.data(), o.p, G * 576, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

// MultilinearPC::check (circuit_verifier.rs:245-314): for k points pt (LSB-first,
// canonical Fr) and k G2 proofs,
//   e(C - g^v, h) * prod_i e(g^{pt_i} - g_mask[nv - k + i], pi_i) == 1.
// A polynomial of k < ck.nv variables lives on SRS level ck.nv - k, i.e. on
// the trapdoor coordinates t[ck.nv - k ..], hence the mask offset (the same
// offset check_2 applies to h_mask, circuit_verifier.rs:214); the reference
// only checks full-level polynomials (sqrt_pst.rs:261), where it is 0.
static void mlpc_check_pairs(const SrsState* st, int k, const uint64_t* comm, const uint64_t* pt, const uint64_t* v,
                             const uint64_t* proofs, PairSet& ps) {
  const uint64_t* flat = st->flat.data();
  const uint64_t* g = flat;
  const uint64_t* h = flat + 12;
  const uint64_t* gmask = flat + tpst_srs_flat_len(st->nv) - 36 * st->nv;
  uint64_t negv[4];
  fr_out(sub(Fr::zero(), fr_canon(v)), negv);
  ps.g1.assign((size_t)(k + 1) * 12, 0);
  ps.g2.clear();
  push(ps.g2, h, 24);
  for (int i = 0; i < k; i++) push(ps.g2, proofs + 24 * i, 24);
  host::parallel_for((size_t)k + 1, [&](size_t i) {
    if (i == 0)
      host::mul_add<Fq>(g, negv, comm, 1, &ps.g1[0]);  // C - g^v
    else
      host::mul_add<Fq>(g, pt + 4 * (i - 1), gmask + 12 * (st->nv - k + i - 1), -1, &ps.g1[12 * i]);
  });
}

// check_2 (circuit_verifier.rs:175-243; mipp.rs:307): G2 commitment C_h, k G1
// proofs,  e(g, C_h - h^v) * prod_i e(pi_i, h^{pt_i} - h_mask[nv - k + i]) == 1
static void mlpc_check2_pairs(const SrsState* st, int k, const uint64_t* comm_h, const uint64_t* pt,
                              const uint64_t* v, const uint64_t* proofs, PairSet& ps) {
  const uint64_t* flat = st->flat.data();
  const uint64_t* g = flat;
  const uint64_t* h = flat + 12;
  const uint64_t* hmask = flat + tpst_srs_flat_len(st->nv) - 24 * st->nv;
  uint64_t negv[4];
  fr_out(sub(Fr::zero(), fr_canon(v)), negv);
  ps.g1.clear();
  push(ps.g1, g, 12);
  for (int i = 0; i < k; i++) push(ps.g1, proofs + 12 * i, 12);
  ps.g2.assign((size_t)(k + 1) * 24, 0);
  host::parallel_for((size_t)k + 1, [&](size_t i) {
    if (i == 0)
      host::mul_add<Fq2>(h, negv, comm_h, 1, &ps.g2[0]);  // C_h - h^v
    else
      host::mul_add<Fq2>(h, pt + 4 * (i - 1), hmask + 24 * (st->nv - k + i - 1), -1, &ps.g2[24 * i]);
  });
}

static int mlpc_check_impl(tpst_ctx* ctx, SrsState* st, int k, const uint64_t* comm, const uint64_t* pt,
                           const uint64_t* v, const uint64_t* proofs) {
  PairSet ps;
  mlpc_check_pairs(st, k, comm, pt, v, proofs, ps);
  std::vector<uint64_t> gt;
  if (int rc = pairing_groups(ctx, {&ps}, gt)) return rc;
  return gt_is_one(gt.data()) ? TPST_OK : TPST_E_VERIFY;
}

static int mlpc_check2_impl(tpst_ctx* ctx, SrsState* st, int k, const uint64_t* comm_h, const uint64_t* pt,
                            const uint64_t* v, const uint64_t* proofs) {
  PairSet ps;
  mlpc_check2_pairs(st, k, comm_h, pt, v, proofs, ps);
  std::vector<uint64_t> gt;
  if (int rc = pairing_groups(ctx, {&ps}, gt)) return rc;
  return gt_is_one(gt.data()) ? TPST_OK : TPST_E_VERIFY;
}

// ------------------------------------------------- MultilinearPC calls ---
// Single-call forms of the ark-poly-commit fork's MultilinearPC<E> used by the
// reference: commit (sqrt_pst.rs:124), commit_g2
// (mipp.rs:133), open (sqrt_pst.rs:225), open_g1 (mipp.rs:144), check
// (sqrt_pst.rs:261), check_2 (mipp.rs:307).  A polynomial of nv variables uses
// SRS level ck.nv - nv (the variable-CRS offset); points are LSB-first as
// MultilinearPC takes them; values canonical.
static int mlpc_args(tpst_ctx* ctx, SrsState* st, int nv) {
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  if (nv < 0 || nv > st->nv) return fail(ctx, TPST_E_ARG, "num_vars > SRS num_vars");
  return TPST_OK;
}

template <class F>
static int mlpc_commit_impl(tpst_ctx* ctx, const uint64_t* evals, int nv, uint64_t* out) {
  if (!ctx || !evals || !out) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  int rc = mlpc_args(ctx, st, nv);
  if (rc) return rc;
  const size_t n = (size_t)1 << nv;
  const int lvl = st->nv - nv;
  constexpr size_t PW = 2 * Words<F>::n;
  const uint32_t* bases;
  if (lvl < st->nv) {
    bases = (sizeof(F) == sizeof(Fq) ? st->pg[lvl] : st->ph[lvl])->u();
  } else {  // nv = 0: the level of one base is g (h), the constant polynomial
    bases = (sizeof(F) == sizeof(Fq) ? st->g : st->h).u();
  }
  hipStream_t s = ctx->stream;
  DevBuf sc, r, o;
  TPST_HIP(ctx, sc.alloc(n * 32));
  TPST_HIP(ctx, r.alloc(sizeof(Xyzz<F>)));
  TPST_HIP(ctx, o.alloc(PW * 4));
  TPST_HIP(ctx, hipMemcpyAsync(sc.p, evals, n * 32, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, msm_var<F>(ctx->arena, s, bases, sc.u(), n, (Xyzz<F>*)r.p));
  TPST_HIP(ctx, xyzz_to_affine_canonical<F>(s, (Xyzz<F>*)r.p, o.u(), 1));
  TPST_HIP(ctx, hipMemcpyAsync(out, o.p, PW * 4, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_mlpc_commit(tpst_ctx* ctx, const uint64_t* evals, int nv, uint64_t* g_product) {
  return mlpc_commit_impl<Fq>(ctx, evals, nv, g_product);
}

extern "C" int tpst_mlpc_commit_g2(tpst_ctx* ctx, const uint64_t* evals, int nv, uint64_t* h_product) {
  return mlpc_commit_impl<Fq2>(ctx, evals, nv, h_product);
}

template <class F>
static int mlpc_open_impl(tpst_ctx* ctx, const uint64_t* evals, int nv, const uint64_t* point, uint64_t* proofs) {
  if (!ctx || !evals || !point || !proofs) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  int rc = mlpc_args(ctx, st, nv);
  if (rc) return rc;
  if (nv == 0) return TPST_OK;  // no quotients
  for (int i = 0; i < nv; i++)
    if (!fr_ok(point + 4 * i)) return fail(ctx, TPST_E_ARG, "point coordinate >= r");
  const size_t n = (size_t)1 << nv;
  constexpr size_t PW = 2 * Words<F>::n;
  hipStream_t s = ctx->stream;
  DevBuf ev, pt, r, o;
  TPST_HIP(ctx, ev.alloc(n * 32));
  TPST_HIP(ctx, pt.alloc(nv * 32));
  TPST_HIP(ctx, r.alloc(nv * sizeof(Xyzz<F>)));
  TPST_HIP(ctx, o.alloc(nv * PW * 4));
  TPST_HIP(ctx, hipMemcpyAsync(ev.p, evals, n * 32, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, hipMemcpyAsync(pt.p, point, nv * 32, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, fr_to_mont(s, ev.u(), ev.u(), n));
  TPST_HIP(ctx, fr_to_mont(s, pt.u(), pt.u(), nv));
  const uint32_t* table = sizeof(F) == sizeof(Fq) ? st->t_pgp.u() : st->t_php.u();
  rc = pst_open_fbt<F>(ctx, st, table, st->nv - nv, ev.u(), nv, pt.u(), (Xyzz<F>*)r.p);
  if (rc) return rc;
  TPST_HIP(ctx, xyzz_to_affine_canonical<F>(s, (Xyzz<F>*)r.p, o.u(), nv));
  TPST_HIP(ctx, hipMemcpyAsync(proofs, o.p, nv * PW * 4, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_mlpc_open(tpst_ctx* ctx, const uint64_t* evals, int nv, const uint64_t* point,
                              uint64_t* proofs) {
  return mlpc_open_impl<Fq2>(ctx, evals, nv, point, proofs);
}

extern "C" int tpst_mlpc_open_g1(tpst_ctx* ctx, const uint64_t* evals, int nv, const uint64_t* point,
                                 uint64_t* proofs) {
  return mlpc_open_impl<Fq>(ctx, evals, nv, point, proofs);
}

extern "C" int tpst_mlpc_check(tpst_ctx* ctx, int nv, const uint64_t* comm, const uint64_t* point,
                               const uint64_t* value, const uint64_t* proofs) {
  if (!ctx || !comm || !point || !value || (nv && !proofs)) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  int rc = mlpc_args(ctx, st, nv);
  if (rc) return rc;
  if (!fr_ok(value) || !point_valid<Fq>(comm)) return fail(ctx, TPST_E_VERIFY, "malformed input");
  for (int i = 0; i < nv; i++)
    if (!fr_ok(point + 4 * i) || !point_valid<Fq2>(proofs + 24 * i)) return fail(ctx, TPST_E_VERIFY, "malformed input");
  return mlpc_check_impl(ctx, st, nv, comm, point, value, proofs);
}

extern "C" int tpst_mlpc_check_2(tpst_ctx* ctx, int nv, const uint64_t* comm_h, const uint64_t* point,
                                 const uint64_t* value, const uint64_t* proofs) {
  if (!ctx || !comm_h || !point || !value || (nv && !proofs)) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  int rc = mlpc_args(ctx, st, nv);
  if (rc) return rc;
  if (!fr_ok(value) || !point_valid<Fq2>(comm_h)) return fail(ctx, TPST_E_VERIFY, "malformed input");
  for (int i = 0; i < nv; i++)
    if (!fr_ok(point + 4 * i) || !point_valid<Fq>(proofs + 12 * i)) return fail(ctx, TPST_E_VERIFY, "malformed input");
  return mlpc_check2_impl(ctx, st, nv, comm_h, point, value, proofs);
}

// Every proof element is validated before the transcript absorbs it (a
// non-canonical encoding of a point would otherwise change the Fiat-Shamir
// challenges without changing the point): Fq limbs < p, points on the curve
// and in the r-torsion (host threads), GT coefficients < p (GT membership of
// comms_t is tested on the device with its exponentiation), scalars < r.
static bool proof_valid(const tpst_open_proof* pr, int n, const uint64_t* point, const uint64_t* v,
                        const uint64_t* T) {
  for (int i = 0; i < n; i++)
    if (!fr_ok(point + 4 * i)) return false;
  if (!fr_ok(v) || !gt_ok(T)) return false;
  for (int i = 0; i < pr->m_col; i++)
    if (!gt_ok(pr->comms_t[i][0]) || !gt_ok(pr->comms_t[i][1])) return false;
  std::vector<const uint64_t*> g1 = {pr->U, pr->final_a}, g2 = {pr->final_h};
  for (int i = 0; i < pr->m_col; i++) {
    g1.push_back(pr->comms_u[i][0]);
    g1.push_back(pr->comms_u[i][1]);
    g1.push_back(pr->pst_proof_h[i]);
  }
  for (int i = 0; i < pr->m_row; i++) g2.push_back(pr->pst_proof[i]);
  std::atomic<bool> ok(true);
  host::parallel_for(g1.size() + g2.size(), [&](size_t t) {
    if (!ok.load(std::memory_order_relaxed)) return;
    const bool good = t < g2.size() ? point_valid<Fq2>(g2[t]) : point_valid<Fq>(g1[t - g2.size()]);
    if (!good) ok.store(false);
  });
  return ok.load();
}

// Polynomial::verify (sqrt_pst.rs:232-264) with MippProof::verify (mipp.rs:182-320)
extern "C" int tpst_pst_verify(tpst_ctx* ctx, tpst_transcript* tr, int n, const uint64_t* point, const uint64_t* v,
                               const uint64_t* T, const tpst_open_proof* proof) {
  if (!ctx || !tr || !point || !v || !T || !proof) return fail(ctx, TPST_E_ARG, "null argument");
  int m_col, m_row, odd;
  if (poly_dims(n, m_col, m_row, odd)) return fail(ctx, TPST_E_ARG, "bad num_vars");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  SrsState* st = srs_of(ctx);
  if (!st) return fail(ctx, TPST_E_STATE, "no SRS loaded");
  if (st->nv != m_row || proof->m_col != m_col || proof->m_row != m_row) return fail(ctx, TPST_E_ARG, "size mismatch");
  if (!proof_valid(proof, n, point, v, T)) return fail(ctx, TPST_E_VERIFY, "malformed proof element (non-canonical, off-curve or outside the subgroup)");
  const int m = m_col;
  Sponge sp;
  sp.load(tr);
  uint8_t b[96];
  g1_bytes(proof->U, b);
  sp.absorb_bytes(b, 96);
  std::vector<Fr> xs(m), xs_inv(m);
  Fr final_y = Fr::one();
  for (int i = 0; i < m; i++) {  // mipp.rs:207-227
    g1_bytes(proof->comms_u[i][0], b);
    sp.absorb_bytes(b, 96);
    g1_bytes(proof->comms_u[i][1], b);
    sp.absorb_bytes(b, 96);
    sp.absorb_bytes((const uint8_t*)proof->comms_t[i][0], 576);
    sp.absorb_bytes((const uint8_t*)proof->comms_t[i][1], 576);
    uint64_t cc[4];
    sp.challenge(cc);
    xs_inv[i] = fr_canon(cc);
    xs[i] = fr_inv(xs_inv[i]);
    const Fr bi = fr_canon(point + 4 * (m_row + i));
    final_y = mul(final_y, sub(add(Fr::one(), mul(xs_inv[i], bi)), bi));
  }
  std::vector<Fr> rs(m);
  for (int i = 0; i < m; i++) {
    uint64_t cc[4];
    sp.challenge(cc);
    rs[i] = fr_canon(cc);
  }
  Fr vh = Fr::one();
  for (int i = 0; i < m; i++) vh = mul(vh, sub(add(Fr::one(), mul(rs[i], xs_inv[m - i - 1])), rs[i]));
  auto canon4 = [](const Fr& x) {
    std::vector<uint64_t> c(4);
    fr_out(x, c.data());
    return c;
  };
  // T check, device side first (side stream): t_l^{c_inv}, t_r^{c} for every
  // round after a GT membership test of each (mipp.rs:263-283)
  const size_t k = 2 * (size_t)m;
  if (int rc = open_streams(ctx, 8, k * (sizeof(Fq12) + 4))) return rc;
  hipStream_t s2 = ctx->side[0];
  DevBuf db, de, dout, dok;
  // the powers and flags come back into the context's pinned staging (a true
  // async copy); every return path below drains s2 first (the guard is
  // destroyed before the device buffers the copies read)
  Fq12* pw = reinterpret_cast<Fq12*>(ctx->pinned);
  uint32_t* okv = reinterpret_cast<uint32_t*>(pw + k);
  struct Drain {
    hipStream_t s;
    ~Drain() { (void)hipStreamSynchronize(s); }
  } drain{s2};
  if (k) {
    std::vector<uint32_t> bases;
    std::vector<uint64_t> dg(4 * k);
    for (int i = 0; i < m; i++) {
      for (int j = 0; j < 2; j++) {
        Fq12 f;
        Fq* c = reinterpret_cast<Fq*>(&f);
        for (int q = 0; q < 12; q++) c[q] = fq_canon(proof->comms_t[i][j] + 6 * q);
        const uint32_t* fw = reinterpret_cast<const uint32_t*>(&f);
        bases.insert(bases.end(), fw, fw + sizeof(Fq12) / 4);
        uint64_t e4[4];  // base-x digits of the exponent (e < r < x^4)
        fr_out(j == 0 ? xs_inv[i] : xs[i], e4);
        base_x_digits(e4, &dg[4 * (2 * i + j)]);
      }
    }
    TPST_HIP(ctx, db.alloc(k * sizeof(Fq12)));
    TPST_HIP(ctx, de.alloc(k * 32));
    TPST_HIP(ctx, dout.alloc(k * sizeof(Fq12)));
    TPST_HIP(ctx, dok.alloc(k * 4));
    TPST_HIP(ctx, hipMemcpyAsync(db.p, bases.data(), k * sizeof(Fq12), hipMemcpyHostToDevice, s2));
    TPST_HIP(ctx, hipMemcpyAsync(de.p, dg.data(), k * 32, hipMemcpyHostToDevice, s2));
    TPST_HIP(ctx, gt_pow_wave(s2, (const Fq12*)db.p, (const uint64_t*)de.p, k, (Fq12*)dout.p, dok.u()));
    TPST_HIP(ctx, hipMemcpyAsync(pw, dout.p, k * sizeof(Fq12), hipMemcpyDeviceToHost, s2));
    TPST_HIP(ctx, hipMemcpyAsync(okv, dok.p, k * 4, hipMemcpyDeviceToHost, s2));
  }
  // host threads meanwhile: the U check's terms and the check / check_2 pairs
  // U check: uc = U + sum(c_inv u_l + c u_r) == final_y * final_a (mipp.rs:239-251)
  std::vector<Xyzz<host::HFq>> terms(2 * (size_t)m + 1);
  std::vector<std::vector<uint64_t>> tsc(2 * (size_t)m + 1);
  for (int i = 0; i < m; i++) {
    tsc[2 * i] = canon4(xs_inv[i]);
    tsc[2 * i + 1] = canon4(xs[i]);
  }
  tsc[2 * m] = canon4(sub(Fr::zero(), final_y));
  PairSet chk2, chk;
  {
    std::vector<uint64_t> rsc(4 * (size_t)m);
    for (int i = 0; i < m; i++) fr_out(rs[i], &rsc[4 * i]);
    uint64_t vhc[4];
    fr_out(vh, vhc);
    std::vector<uint64_t> arev(4 * (size_t)m_row);
    for (int i = 0; i < m_row; i++) memcpy(&arev[4 * i], point + 4 * (m_row - 1 - i), 32);
    host::parallel_for(terms.size(), [&](size_t t) {
      const uint64_t* P = t == 2 * (size_t)m ? proof->final_a : proof->comms_u[t / 2][t % 2];
      terms[t] = scalar_mul(host::aff_in<host::HFq>(P), reinterpret_cast<const uint32_t*>(tsc[t].data()), 253);
    });
    mlpc_check2_pairs(st, m, proof->final_h, rsc.data(), vhc, &proof->pst_proof_h[0][0], chk2);  // mipp.rs:307
    mlpc_check_pairs(st, m_row, proof->U, arev.data(), v, &proof->pst_proof[0][0], chk);         // sqrt_pst.rs:261
  }
  Xyzz<host::HFq> uc = to_xyzz(host::aff_in<host::HFq>(proof->U));
  for (auto& t : terms) uc = add(uc, t);
  if (!is_inf(uc)) return TPST_E_VERIFY;
  // the three pairing products in one launch: e(final_a, final_h), check_2, check
  PairSet fin;
  push(fin.g1, proof->final_a, 12);
  push(fin.g2, proof->final_h, 24);
  std::vector<uint64_t> gts;
  if (int rc = pairing_groups(ctx, {&fin, &chk2, &chk}, gts)) return rc;
  TPST_HIP(ctx, hipStreamSynchronize(s2));
  for (size_t i = 0; i < k; i++)
    if (!okv[i]) return fail(ctx, TPST_E_VERIFY, "comms_t element outside GT");
  // T * prod t_l^{c_inv} t_r^{c} == e(final_a, final_h)
  Fq12 acc;
  {
    Fq* c = reinterpret_cast<Fq*>(&acc);
    for (int q = 0; q < 12; q++) c[q] = fq_canon(T + 6 * q);
  }
  for (size_t i = 0; i < k; i++) acc = mul(acc, pw[i]);
  {
    const Fq* c = reinterpret_cast<const Fq*>(&acc);
    for (int q = 0; q < 12; q++) {
      uint64_t lim[6];
      fq_out(c[q], lim);
      if (memcmp(lim, gts.data() + 6 * q, 48) != 0) return TPST_E_VERIFY;
    }
  }
  if (!gt_is_one(gts.data() + 72) || !gt_is_one(gts.data() + 144)) return TPST_E_VERIFY;
  sp.store(tr);
  return TPST_OK;
}
