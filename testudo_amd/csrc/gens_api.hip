// Pedersen / Hyrax row commitments over caller-supplied generators
// (include/tpst.h, "shared-base batch MSM").
//
// Reference: MultiCommitGens {n, G, h} (commitments.rs:9-15),
// PedersenCommit::commit_slice = msm_unchecked(G, scalars) + h * blind
// (commitments.rs:79-86), driven row by row from rayon by
// DensePolynomial::commit_inner (dense_mlpoly.rs:314-329).  Here a generator
// set is uploaded once (tpst_gens_load: Montgomery bases plus the K1 window
// tables T[w][j] = 2^(c w) G_j), and every batch of rows is ONE launch of the
// K1 pipeline (msm.h msm_batch) over a strided view of the caller's scalars --
// the same kernels as the sqrt-PST row commit (sqrt_pst.rs:121-125), so a
// Hyrax commit of 2^n evaluations costs one device pass, not 2^(n/2) MSMs.
#include <cstring>
#include "../../include/tpst.h"
#include "ctx.h"
#include "device_util.h"
#include "pst_kernels.h"

using namespace tpst;

struct tpst_gens {
  tpst_ctx* ctx = nullptr;
  size_t n = 0;
  bool has_h = false;
  uint32_t* d_G = nullptr;   // n affine G1, Montgomery
  uint32_t* d_h = nullptr;   // 1 affine G1, Montgomery
  BatchTables tables;        // K1 window tables over G
  ~tpst_gens() {
    if (d_G) (void)hipFree(d_G);
    if (d_h) (void)hipFree(d_h);
    batch_tables_free(tables);
  }
};

namespace {

__global__ void k_add_affine_rows(Xyzz<Fq>* __restrict__ rows, const uint32_t* __restrict__ pts, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_xyzz(rows, i, add_affine(load_xyzz(rows, i), load_affine<Fq>(pts, i)));
}

// canonical limbs < p for every coordinate of n affine points
bool points_canonical(const uint64_t* pts, size_t n_fq) {
  for (size_t k = 0; k < n_fq; k++) {
    const uint64_t* a = pts + 6 * k;
    for (int i = 5; i >= 0; i--) {
      const uint64_t pi = (uint64_t)params::FQ_P[2 * i] | ((uint64_t)params::FQ_P[2 * i + 1] << 32);
      if (a[i] != pi) {
        if (a[i] > pi) return false;
        break;
      }
      if (i == 0) return false;  // == p
    }
  }
  return true;
}

// the span (in scalars) a strided rows x cols view touches; 0 on overflow
size_t strided_span(size_t rows, size_t cols, size_t rs, size_t cs) {
  if (!rows || !cols) return 0;
  const size_t lim = (size_t)1 << 40;
  if (rows > lim || cols > lim || rs > lim || cs > lim) return 0;
  return (rows - 1) * rs + (cols - 1) * cs + 1;
}

// K1 over the generator tables, plus optional per-row blind * h; writes rows
// canonical affine G1 to the host
int batch_commit(tpst_ctx* ctx, const tpst_gens* g, const uint32_t* d_sc, size_t rows, size_t rs, size_t cs,
                 const uint64_t* blinds, uint64_t* out_host, uint32_t* out_dev) {
  hipStream_t s = ctx->stream;
  ctx->arena2.reset();
  TPST_HIP(ctx, ctx->arena2.reserve(Arena::need(rows, sizeof(Xyzz<Fq>)) + Arena::need(rows * 24, 4) * 2 +
                                    Arena::need(rows * 8, 4) + 1024));
  Xyzz<Fq>* acc = ctx->arena2.take<Xyzz<Fq>>(rows);
  uint32_t* aff = ctx->arena2.take<uint32_t>(rows * 24);
  uint32_t* bh = ctx->arena2.take<uint32_t>(rows * 24);
  uint32_t* d_bl = ctx->arena2.take<uint32_t>(rows * 8);
  if (g->n == 0) {  // empty MSM: every row is the identity (plus its blind)
    std::vector<Xyzz<Fq>> inf(rows, Xyzz<Fq>::inf());
    TPST_HIP(ctx, hipMemcpyAsync(acc, inf.data(), rows * sizeof(Xyzz<Fq>), hipMemcpyHostToDevice, s));
  } else {
    TPST_HIP(ctx, msm_batch(ctx->arena, s, g->tables, d_sc, rows, rs, cs, acc));
  }
  if (blinds) {
    TPST_HIP(ctx, hipMemcpyAsync(d_bl, blinds, rows * 32, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, fixed_base_mul<Fq>(s, g->d_h, d_bl, rows, bh));
    k_add_affine_rows<<<(unsigned)((rows + 63) / 64), 64, 0, s>>>(acc, bh, rows);
    TPST_HIP(ctx, hipGetLastError());
  }
  uint32_t* dst = out_dev ? out_dev : aff;
  TPST_HIP(ctx, xyzz_to_affine_canonical<Fq>(s, acc, dst, rows));
  if (out_host) {
    TPST_HIP(ctx, hipMemcpyAsync(out_host, dst, rows * 96, hipMemcpyDeviceToHost, s));
    TPST_HIP(ctx, hipStreamSynchronize(s));
  }
  return TPST_OK;
}

// upload the scalar span of a strided view and run batch_commit
int host_batch(tpst_ctx* ctx, const tpst_gens* g, const uint64_t* scalars, size_t rows, size_t cols, size_t rs,
               size_t cs, const uint64_t* blinds, uint64_t* out) {
  if (cols != g->n) return fail(ctx, TPST_E_ARG, "cols != number of generators (commitments.rs:84 assert)");
  if (!rows) return TPST_OK;
  const size_t span = g->n ? strided_span(rows, cols, rs, cs) : 0;
  if (g->n && !span) return fail(ctx, TPST_E_ARG, "bad strides");
  if (span && !scalars) return fail(ctx, TPST_E_ARG, "null scalars");
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(span ? span * 8 : 1, 4) + 256));
  uint32_t* d_sc = ctx->io.take<uint32_t>(span ? span * 8 : 1);
  if (span) TPST_HIP(ctx, hipMemcpyAsync(d_sc, scalars, span * 32, hipMemcpyHostToDevice, ctx->stream));
  return batch_commit(ctx, g, d_sc, rows, rs, cs, blinds, out, nullptr);
}

}  // namespace

extern "C" int tpst_gens_load(tpst_ctx* ctx, const uint64_t* G, size_t n, const uint64_t* h, tpst_gens** out) {
  if (!ctx || !out || (n && !G)) return fail(ctx, TPST_E_ARG, "null argument");
  if (n >= ((size_t)1 << 26)) return fail(ctx, TPST_E_ARG, "too many generators");
  if (!points_canonical(G, 2 * n) || (h && !points_canonical(h, 2)))
    return fail(ctx, TPST_E_ARG, "generator coordinate >= p");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  auto g = new tpst_gens();
  g->ctx = ctx;
  g->n = n;
  int rc = TPST_OK;
  auto bail = [&](hipError_t e, const char* where) {
    delete g;
    return hip_fail(ctx, e, where);
  };
  uint32_t* up = nullptr;
  hipError_t e = hipMalloc(&up, (n + 1) * 96);
  if (e != hipSuccess) return bail(e, "hipMalloc");
  if ((e = hipMalloc(&g->d_G, (n ? n : 1) * 96)) != hipSuccess || (e = hipMalloc(&g->d_h, 96)) != hipSuccess) {
    (void)hipFree(up);
    return bail(e, "hipMalloc");
  }
  if (n) e = hipMemcpyAsync(up, G, n * 96, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && h) e = hipMemcpyAsync(up + 24 * n, h, 96, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && n) e = points_to_mont<Fq>(s, up, g->d_G, n);
  if (e == hipSuccess && h) e = points_to_mont<Fq>(s, up + 24 * n, g->d_h, 1);
  if (e == hipSuccess && n) e = batch_tables_build(s, g->d_G, n, batch_window_bits(n), g->tables);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(up);
  if (e != hipSuccess) return bail(e, "tpst_gens_load");
  g->has_h = h != nullptr;
  *out = g;
  return rc;
}

extern "C" void tpst_gens_free(tpst_gens* g) { delete g; }

extern "C" int tpst_g1_msm_batch(tpst_ctx* ctx, const tpst_gens* g, const uint64_t* scalars, size_t rows,
                                 size_t cols, size_t row_stride, size_t col_stride, uint64_t* out) {
  if (!ctx || !g || (rows && !out)) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  return host_batch(ctx, g, scalars, rows, cols, row_stride, col_stride, nullptr, out);
}

extern "C" int tpst_g1_msm_batch_dev(tpst_ctx* ctx, const tpst_gens* g, const void* d_scalars, size_t rows,
                                     size_t cols, size_t row_stride, size_t col_stride, void* d_out) {
  if (!ctx || !g || (rows && (!d_out || (g->n && !d_scalars)))) return fail(ctx, TPST_E_ARG, "null argument");
  if (cols != g->n) return fail(ctx, TPST_E_ARG, "cols != number of generators");
  if (g->n && rows && !strided_span(rows, cols, row_stride, col_stride)) return fail(ctx, TPST_E_ARG, "bad strides");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  if (!rows) return TPST_OK;
  return batch_commit(ctx, g, (const uint32_t*)d_scalars, rows, row_stride, col_stride, nullptr, nullptr,
                      (uint32_t*)d_out);
}

extern "C" int tpst_pedersen_commit_slice(tpst_ctx* ctx, const tpst_gens* g, const uint64_t* scalars, size_t n,
                                          const uint64_t* blind, uint64_t* out) {
  if (!ctx || !g || !blind || !out) return fail(ctx, TPST_E_ARG, "null argument");
  if (!g->has_h) return fail(ctx, TPST_E_STATE, "generator set has no blinding base h");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  return host_batch(ctx, g, scalars, 1, n, n, 1, blind, out);
}

extern "C" int tpst_pedersen_commit_rows(tpst_ctx* ctx, const tpst_gens* g, const uint64_t* Z, size_t n_z,
                                         const uint64_t* blinds, size_t n_rows, uint64_t* out) {
  if (!ctx || !g || !out || (n_rows && !blinds)) return fail(ctx, TPST_E_ARG, "null argument");
  if (!g->has_h) return fail(ctx, TPST_E_STATE, "generator set has no blinding base h");
  if (!n_rows || n_z % n_rows) return fail(ctx, TPST_E_ARG, "L_size * R_size != |Z| (dense_mlpoly.rs:320)");
  const size_t R = n_z / n_rows;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  return host_batch(ctx, g, Z, n_rows, R, R, 1, blinds, out);
}
