// Field / curve microbenchmarks (tpst_microbench): the measured compute peak
// used in bench.py's roofline, and A/B variants of the Fq multiply.
#include <vector>
#include "../../include/tpst.h"
#include "ctx.h"
#include "device_util.h"

using namespace tpst;

static inline unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

// ------------------------------------------------------ microbenchmark ----
__global__ void k_mb_fqmul(int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = Fq::one(), b = Fq::one();
  a.v[0] ^= t;
  b.v[1] ^= t * 7u + 1;
  for (int i = 0; i < iters; i++) a = mul(a, b);
  store_f<Fq>(out + 12 * (size_t)t, a);
}

__global__ void k_mb_madd(int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  G1A g = {Fq::from_limbs(params::G1_GEN_X), Fq::from_limbs(params::G1_GEN_Y)};
  Xyzz<Fq> acc = dbl_affine(g);
  acc.X.v[0] ^= (t & 1);  // keep threads independent of each other's values
  for (int i = 0; i < iters; i++) acc = add_affine(acc, g);
  store_f<Fq>(out + 12 * (size_t)t, acc.X);
}

extern "C" int tpst_microbench(tpst_ctx* ctx, int kind, size_t threads, int iters, double* ms) {
  if (!ctx || !ms || threads == 0 || iters <= 0) return fail(ctx, TPST_E_ARG, "bad argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  const unsigned bs = threads < 256 ? (unsigned)threads : 256u;
  const unsigned grid = grid_for(threads, bs);
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need((size_t)grid * bs * 12, 4)));
  uint32_t* d = ctx->io.take<uint32_t>((size_t)grid * bs * 12);
  hipEvent_t e0, e1;
  TPST_HIP(ctx, hipEventCreate(&e0));
  TPST_HIP(ctx, hipEventCreate(&e1));
  TPST_HIP(ctx, hipEventRecord(e0, ctx->stream));
  if (kind == 0)
    k_mb_fqmul<<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 1)
    k_mb_madd<<<grid, bs, 0, ctx->stream>>>(iters, d);
  else
    return fail(ctx, TPST_E_ARG, "unknown microbench kind");
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, hipEventRecord(e1, ctx->stream));
  TPST_HIP(ctx, hipEventSynchronize(e1));
  float f = 0;
  TPST_HIP(ctx, hipEventElapsedTime(&f, e0, e1));
  *ms = f;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return TPST_OK;
}

