// C-ABI entry points (include/tpst.h): context management, device
// primitives (MSM, multi-pairing, generator multiples) and the field
// microbenchmark.  The sqrt-PST protocol entry points live in pst_api.hip.
#include <cstring>
#include "../../include/tpst.h"
#include "ctx.h"
#include "device_util.h"
#include "fbt.h"

using namespace tpst;

namespace tpst {

int fail(tpst_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int hip_fail(tpst_ctx* ctx, hipError_t e, const char* where) {
  return fail(ctx, TPST_E_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

}  // namespace tpst

static inline unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

extern "C" int tpst_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" int tpst_create(int device, tpst_ctx** out) {
  if (!out) return TPST_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return TPST_E_NODEV;
  if (device < 0 || device >= n) return TPST_E_ARG;
  if (hipSetDevice(device) != hipSuccess) return TPST_E_HIP;
  tpst_ctx* c = new tpst_ctx();
  c->device = device;
  c->arena.prof = &c->prof;
  for (int i = 0; i < tpst_ctx::MSM_SLOTS; i++) {
    c->arena_msm[i].prof = &c->prof;
    if (i) c->arena_msm[i].aux_from = &c->arena_msm[0];  // one pair of aux streams
  }
  c->mu.stream = &c->stream;
  // the library stream carries every critical path (the opening's transcript
  // chain in particular); the opening's side streams (pst_api.hip) are
  // created at the lowest priority so the dispatcher favours this one
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
  if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest) != hipSuccess) {
    delete c;
    return TPST_E_HIP;
  }
  *out = c;
  return TPST_OK;
}

extern "C" void tpst_destroy(tpst_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  ctx->arena.release();
  ctx->io.release();
  ctx->arena2.release();
  for (int i = 0; i < 3; i++) {
    if (ctx->side[i]) {
      (void)hipStreamSynchronize(ctx->side[i]);
      (void)hipStreamDestroy(ctx->side[i]);
    }
    ctx->arena_side[i].release();
  }
  for (hipStream_t st : {ctx->comm, ctx->side_c}) {
    if (!st) continue;
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
  }
  if (ctx->msm_tail) {
    (void)hipStreamSynchronize(ctx->msm_tail);
    (void)hipStreamDestroy(ctx->msm_tail);
  }
  // slots 1.. borrow slot 0's aux streams (aux_from): release them first, so
  // no arena synchronizes a stream slot 0 has already destroyed
  for (int i = tpst_ctx::MSM_SLOTS - 1; i >= 0; i--) {
    if (ctx->msm_in[i]) (void)hipEventDestroy(ctx->msm_in[i]);
    if (ctx->msm_done[i]) (void)hipEventDestroy(ctx->msm_done[i]);
    if (ctx->msm_out[i]) (void)hipFree(ctx->msm_out[i]);
    ctx->arena_msm[i].release();
  }
  for (hipEvent_t e : ctx->events) (void)hipEventDestroy(e);
  if (ctx->ev_wait) (void)hipEventDestroy(ctx->ev_wait);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  tpst_release_pst_state(ctx);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

extern "C" const char* tpst_last_error(const tpst_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

extern "C" void* tpst_stream(tpst_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

extern "C" int tpst_synchronize(tpst_ctx* ctx) {
  if (!ctx) return TPST_E_ARG;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);  // the stream waits for pending pipelined MSMs
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return TPST_OK;
}

// one event per direction, re-recorded per call (a stream wait captures the
// event's state at the time of the wait call, so re-use is safe)
static int order_streams(tpst_ctx* ctx, hipStream_t before, hipStream_t after, hipEvent_t& ev) {
  if (!ev) TPST_HIP(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  TPST_HIP(ctx, hipEventRecord(ev, before));
  TPST_HIP(ctx, hipStreamWaitEvent(after, ev, 0));
  return TPST_OK;
}

extern "C" int tpst_wait_stream(tpst_ctx* ctx, void* stream) {
  if (!ctx) return TPST_E_ARG;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  return order_streams(ctx, (hipStream_t)stream, ctx->stream, ctx->ev_wait);
}

extern "C" int tpst_join_stream(tpst_ctx* ctx, void* stream) {
  if (!ctx) return TPST_E_ARG;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  return order_streams(ctx, ctx->stream, (hipStream_t)stream, ctx->ev_join);
}

// ---------------------------------------------------------------- MSM ----
template <class F>
static int msm_host(tpst_ctx* ctx, const uint64_t* bases, size_t nb, const uint64_t* scalars, size_t ns,
                    uint64_t* out) {
  if (!ctx || !out || (nb && !bases) || (ns && !scalars)) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  const size_t n = nb < ns ? nb : ns;  // msm_unchecked truncates
  if (n > MSM_MAX_POINTS) return fail(ctx, TPST_E_ARG, "MSM longer than 2^27 points: split it");
  constexpr size_t PW = 2 * Words<F>::n;  // u32 per affine point
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(n * PW, 4) * 2 + Arena::need(n * 8, 4) + 4096 +
                                Arena::need(1, sizeof(Xyzz<F>)) + Arena::need(PW, 4)));
  uint32_t* d_b = ctx->io.take<uint32_t>(n * PW);
  uint32_t* d_bm = ctx->io.take<uint32_t>(n * PW);
  uint32_t* d_s = ctx->io.take<uint32_t>(n * 8);
  Xyzz<F>* d_r = ctx->io.take<Xyzz<F>>(1);
  uint32_t* d_o = ctx->io.take<uint32_t>(PW);
  hipStream_t s = ctx->stream;
  if (n) {
    TPST_HIP(ctx, hipMemcpyAsync(d_b, bases, n * PW * 4, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, hipMemcpyAsync(d_s, scalars, n * 32, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, points_to_mont<F>(s, d_b, d_bm, n));
  }
  TPST_HIP(ctx, msm_var<F>(ctx->arena, s, d_bm, d_s, n, d_r));
  TPST_HIP(ctx, xyzz_to_affine_canonical<F>(s, d_r, d_o, 1));
  TPST_HIP(ctx, hipMemcpyAsync(out, d_o, PW * 4, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_g1_msm(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                           size_t n_scalars, uint64_t* out) {
  return msm_host<Fq>(ctx, bases, n_bases, scalars, n_scalars, out);
}

// multiexponentiation (mipp.rs:385-394): lengths must agree
extern "C" int tpst_g1_multiexp(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                                size_t n_scalars, uint64_t* out) {
  if (n_bases != n_scalars) return fail(ctx, TPST_E_ARG, "InvalidIPVectorLength");
  return msm_host<Fq>(ctx, bases, n_bases, scalars, n_scalars, out);
}

extern "C" int tpst_g2_multiexp(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                                size_t n_scalars, uint64_t* out) {
  if (n_bases != n_scalars) return fail(ctx, TPST_E_ARG, "InvalidIPVectorLength");
  return msm_host<Fq2>(ctx, bases, n_bases, scalars, n_scalars, out);
}

extern "C" int tpst_g2_msm(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                           size_t n_scalars, uint64_t* out) {
  return msm_host<Fq2>(ctx, bases, n_bases, scalars, n_scalars, out);
}

// fixed-base table path (fbt.h): builds the table of the n bases, then the
// grouped MSM out[g] = sum_{k in g} s_k B_k with strided groups (L, D)
template <class F>
static int msm_fixed_host(tpst_ctx* ctx, const uint64_t* bases, size_t n, const uint64_t* scalars, size_t L,
                          size_t D, uint64_t* out) {
  if (!ctx || !out || (n && (!bases || !scalars))) return fail(ctx, TPST_E_ARG, "null argument");
  if (!n || !L || !D || n % L || L % D) return fail(ctx, TPST_E_ARG, "bad group shape");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  constexpr size_t PW = 2 * Words<F>::n;
  const size_t G = L / D;
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(n * PW, 4) * 2 + Arena::need(n * 8, 4) + Arena::need(G, sizeof(Xyzz<F>)) +
                                Arena::need(G * PW, 4) + Arena::need(fbt_words<F>(n), 4) + 4096));
  uint32_t* d_b = ctx->io.take<uint32_t>(n * PW);
  uint32_t* d_bm = ctx->io.take<uint32_t>(n * PW);
  uint32_t* d_s = ctx->io.take<uint32_t>(n * 8);
  Xyzz<F>* d_r = ctx->io.take<Xyzz<F>>(G);
  uint32_t* d_o = ctx->io.take<uint32_t>(G * PW);
  uint32_t* d_t = ctx->io.take<uint32_t>(fbt_words<F>(n));
  hipStream_t s = ctx->stream;
  TPST_HIP(ctx, hipMemcpyAsync(d_b, bases, n * PW * 4, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, hipMemcpyAsync(d_s, scalars, n * 32, hipMemcpyHostToDevice, s));
  TPST_HIP(ctx, points_to_mont<F>(s, d_b, d_bm, n));
  TPST_HIP(ctx, fbt_build<F>(ctx->arena, s, d_bm, n, d_t));
  FbGroups g;
  g.groups = G;
  g.members = (n / L) * D;
  g.L = L;
  g.D = D;
  TPST_HIP(ctx, fbt_msm<F>(ctx->arena, s, d_t, d_s, g, d_r));
  TPST_HIP(ctx, xyzz_to_affine_canonical<F>(s, d_r, d_o, G));
  TPST_HIP(ctx, hipMemcpyAsync(out, d_o, G * PW * 4, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_g1_msm_fixed(tpst_ctx* ctx, const uint64_t* bases, size_t n, const uint64_t* scalars, size_t L,
                                 size_t D, uint64_t* out) {
  return msm_fixed_host<Fq>(ctx, bases, n, scalars, L, D, out);
}

extern "C" int tpst_g2_msm_fixed(tpst_ctx* ctx, const uint64_t* bases, size_t n, const uint64_t* scalars, size_t L,
                                 size_t D, uint64_t* out) {
  return msm_fixed_host<Fq2>(ctx, bases, n, scalars, L, D, out);
}

// Pipelined (tpst_g1_msm_dev_async): consecutive calls overlap.  Call i decomposes and sorts its
// scalars on ctx->side[0], accumulates on ctx->side[1] and runs its
// latency-bound tail (the last window group's fixup, bucket reduction and
// window chain, and the affine output; ~0.7 ms of a few waves at 2^20) on
// ctx->msm_tail, with one of three arenas: call i+1's sort runs under call
// i's accumulation, its accumulation under call i's tail (with two arenas the
// sort of call i+1 waited for call i-1's tail, itself stretched by call i's
// accumulation: 0.85 ms idle between accumulations, profiles/r05/f).  Stream order is kept
// for the caller: each call starts after the work already on ctx->stream (its
// inputs), the next entry point of any other kind (and tpst_synchronize /
// tpst_join_stream) first waits for the pending tails (CtxMutex::lock), and a
// call reusing an arena waits for the tail that last used it.
// tpst_g1_msm_dev (stream-safe): the same work, then ctx->stream waits for its
// end, so work the caller queues on tpst_stream() afterwards (reading d_out,
// overwriting the inputs, freeing them) is ordered after the MSM; consecutive
// calls then run one after another on the device (the host still returns at
// once).
static int msm_dev_impl(tpst_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n, void* d_out,
                        bool async) {
  if (!ctx || !d_out || (n && (!d_bases || !d_scalars))) return fail(ctx, TPST_E_ARG, "null argument");
  if (n > MSM_MAX_POINTS) return fail(ctx, TPST_E_ARG, "MSM longer than 2^27 points: split it");
  tpst::CtxKeep lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  if (!ctx->msm_tail) {
    int least = 0, greatest = 0;
    TPST_HIP(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
    for (int i = 0; i < 2; i++)  // as pst_api.hip open_streams creates them
      if (!ctx->side[i]) TPST_HIP(ctx, hipStreamCreateWithPriority(&ctx->side[i], hipStreamNonBlocking, least));
    TPST_HIP(ctx, hipStreamCreateWithPriority(&ctx->msm_tail, hipStreamNonBlocking, greatest));
    for (int i = 0; i < tpst_ctx::MSM_SLOTS; i++) {
      TPST_HIP(ctx, hipEventCreateWithFlags(&ctx->msm_in[i], hipEventDisableTiming));
      TPST_HIP(ctx, hipEventCreateWithFlags(&ctx->msm_done[i], hipEventDisableTiming));
      TPST_HIP(ctx, hipMalloc(&ctx->msm_out[i], sizeof(Xyzz<Fq>)));
    }
  }
  const int k = ctx->msm_slot;
  ctx->msm_slot = (k + 1) % tpst_ctx::MSM_SLOTS;
  Arena& ar = ctx->arena_msm[k];
  // the caller's inputs, and the tail that last used this arena (its
  // buckets, bounds, output slot)
  TPST_HIP(ctx, hipEventRecord(ctx->msm_in[k], ctx->stream));
  const hipStream_t front = ctx->side[0], bulk = ctx->side[1];
  TPST_HIP(ctx, hipStreamWaitEvent(front, ctx->msm_in[k], 0));
  if (ctx->msm_done_set[k]) TPST_HIP(ctx, hipStreamWaitEvent(front, ctx->msm_done[k], 0));
  bool on_tail = false;
  Xyzz<Fq>* d_r = (Xyzz<Fq>*)ctx->msm_out[k];
  TPST_HIP(ctx, hipStreamWaitEvent(bulk, ctx->msm_in[k], 0));  // n = 0: no front work
  // n = 0 writes msm_out[k] on bulk without front work: order it after the
  // tail of the call that last used slot k (it may still read msm_out[k])
  if (ctx->msm_done_set[k]) TPST_HIP(ctx, hipStreamWaitEvent(bulk, ctx->msm_done[k], 0));
  TPST_HIP(ctx, msm_var<Fq>(ar, bulk, (const uint32_t*)d_bases, (const uint32_t*)d_scalars, n, d_r, ctx->msm_tail,
                            &on_tail, front));
  hipStream_t t = on_tail ? ctx->msm_tail : bulk;
  TPST_HIP(ctx, xyzz_to_affine_canonical<Fq>(t, d_r, (uint32_t*)d_out, 1));
  TPST_HIP(ctx, hipEventRecord(ctx->msm_done[k], t));
  ctx->msm_done_set[k] = true;
  if (!async) {
    TPST_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->msm_done[k], 0));
    return TPST_OK;
  }
  bool listed = false;
  for (hipEvent_t e : ctx->mu.pending) listed |= e == ctx->msm_done[k];
  if (!listed) ctx->mu.pending.push_back(ctx->msm_done[k]);
  return TPST_OK;
}

extern "C" int tpst_g1_msm_dev(tpst_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n, void* d_out) {
  return msm_dev_impl(ctx, d_bases, d_scalars, n, d_out, false);
}

extern "C" int tpst_g1_msm_dev_async(tpst_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n,
                                     void* d_out) {
  return msm_dev_impl(ctx, d_bases, d_scalars, n, d_out, true);
}

// strong-scaled MSM pieces: one rank's share as the raw XYZZ sum (no affine
// inversion per rank), and the combine of the gathered shares on one device
extern "C" int tpst_g1_msm_xyzz_dev(tpst_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n,
                                    void* d_out_xyzz) {
  if (!ctx || !d_out_xyzz || (n && (!d_bases || !d_scalars))) return fail(ctx, TPST_E_ARG, "null argument");
  if (n > MSM_MAX_POINTS) return fail(ctx, TPST_E_ARG, "MSM longer than 2^27 points: split it");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  TPST_HIP(ctx, msm_var<Fq>(ctx->arena, ctx->stream, (const uint32_t*)d_bases, (const uint32_t*)d_scalars, n,
                            (Xyzz<Fq>*)d_out_xyzz));
  return TPST_OK;
}

static __global__ void __launch_bounds__(64) k_xyzz_sum(const uint8_t* __restrict__ parts, size_t k, size_t stride,
                                                        Xyzz<Fq>* __restrict__ out) {
  if (threadIdx.x != 0) return;
  Xyzz<Fq> acc = Xyzz<Fq>::inf();
  for (size_t i = 0; i < k; i++) acc = add(acc, load_xyzz(reinterpret_cast<const Xyzz<Fq>*>(parts + i * stride), 0));
  store_xyzz(out, 0, acc);
}

extern "C" int tpst_g1_xyzz_sum_dev(tpst_ctx* ctx, const void* d_parts, size_t k, size_t stride_bytes, void* d_out) {
  if (!ctx || !d_out || (k && !d_parts)) return fail(ctx, TPST_E_ARG, "null argument");
  // k_xyzz_sum reads each share with 16-byte vector loads
  if (k && (stride_bytes < sizeof(Xyzz<Fq>) || stride_bytes % 16 || ((uintptr_t)d_parts & 15)))
    return fail(ctx, TPST_E_ARG, "shares must be 16-byte aligned with a 16-byte-multiple stride");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(1, sizeof(Xyzz<Fq>)) + 256));
  Xyzz<Fq>* d_r = ctx->io.take<Xyzz<Fq>>(1);
  k_xyzz_sum<<<1, 64, 0, ctx->stream>>>((const uint8_t*)d_parts, k, stride_bytes, d_r);
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, xyzz_to_affine_canonical<Fq>(ctx->stream, d_r, (uint32_t*)d_out, 1));
  return TPST_OK;
}

// ------------------------------------------------------------ pairing ----
extern "C" int tpst_multi_pairing(tpst_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n,
                                  uint64_t* out_gt) {
  if (!ctx || !out_gt || (n && (!g1 || !g2))) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(n * 24, 4) * 2 + Arena::need(n * 48, 4) * 2 +
                                Arena::need(1, sizeof(Fq12)) + Arena::need(144, 4) + 4096));
  uint32_t* d1 = ctx->io.take<uint32_t>(n * 24);
  uint32_t* d1m = ctx->io.take<uint32_t>(n * 24);
  uint32_t* d2 = ctx->io.take<uint32_t>(n * 48);
  uint32_t* d2m = ctx->io.take<uint32_t>(n * 48);
  Fq12* d_f = ctx->io.take<Fq12>(1);
  uint32_t* d_o = ctx->io.take<uint32_t>(144);
  if (n) {
    TPST_HIP(ctx, hipMemcpyAsync(d1, g1, n * 96, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, hipMemcpyAsync(d2, g2, n * 192, hipMemcpyHostToDevice, s));
    TPST_HIP(ctx, points_to_mont<Fq>(s, d1, d1m, n));
    TPST_HIP(ctx, points_to_mont<Fq2>(s, d2, d2m, n));
  }
  TPST_HIP(ctx, multi_pairing(ctx->arena, s, d1m, d2m, 1, n, d_f));
  TPST_HIP(ctx, fq12_from_mont(s, d_f, d_o, 1));
  TPST_HIP(ctx, hipMemcpyAsync(out_gt, d_o, 576, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

// ------------------------------------------------- generator multiples ----
template <class F>
__global__ void __launch_bounds__(64, 1) k_mul_gen(const uint32_t* __restrict__ scalars, size_t n, uint32_t* __restrict__ out, int canonical) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<F> g;
  if constexpr (sizeof(F) == sizeof(Fq)) {
    g = {Fq::from_limbs(params::G1_GEN_X), Fq::from_limbs(params::G1_GEN_Y)};
  } else {
    g = {fq2_const(params::G2_GEN_X), fq2_const(params::G2_GEN_Y)};
  }
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; j++) k[j] = scalars[8 * i + j];
  Affine<F> a = to_affine(scalar_mul(g, k, 253));
  if (canonical) {
    Fq* c = reinterpret_cast<Fq*>(&a);
#pragma unroll
    for (int j = 0; j < (int)(sizeof(Affine<F>) / sizeof(Fq)); j++) c[j] = from_mont(c[j]);
  }
  store_affine(out, i, a);
}

template <class F>
static int mul_gen_host(tpst_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out) {
  if (!ctx || (n && (!scalars || !out))) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  if (!n) return TPST_OK;
  constexpr size_t PW = 2 * Words<F>::n;
  hipStream_t s = ctx->stream;
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(Arena::need(n * 8, 4) + Arena::need(n * PW, 4) + 512));
  uint32_t* d_s = ctx->io.take<uint32_t>(n * 8);
  uint32_t* d_o = ctx->io.take<uint32_t>(n * PW);
  TPST_HIP(ctx, hipMemcpyAsync(d_s, scalars, n * 32, hipMemcpyHostToDevice, s));
  k_mul_gen<F><<<grid_for(n, 64), 64, 0, s>>>(d_s, n, d_o, 1);
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, hipMemcpyAsync(out, d_o, n * PW * 4, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

extern "C" int tpst_g1_mul_generator(tpst_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out) {
  return mul_gen_host<Fq>(ctx, scalars, n, out);
}

extern "C" int tpst_g2_mul_generator(tpst_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out) {
  return mul_gen_host<Fq2>(ctx, scalars, n, out);
}

extern "C" int tpst_g1_mul_generator_dev(tpst_ctx* ctx, const void* d_scalars, size_t n, void* d_out_mont) {
  if (!ctx || (n && (!d_scalars || !d_out_mont))) return fail(ctx, TPST_E_ARG, "null argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  if (!n) return TPST_OK;
  k_mul_gen<Fq><<<grid_for(n, 64), 64, 0, ctx->stream>>>((const uint32_t*)d_scalars, n, (uint32_t*)d_out_mont, 0);
  TPST_HIP(ctx, hipGetLastError());
  return TPST_OK;
}

// ------------------------------------------------------ stage profiling ----
extern "C" int tpst_profile_enable(tpst_ctx* ctx, int on) {
  if (!ctx) return TPST_E_ARG;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  ctx->prof.on = on != 0;
  return TPST_OK;
}

extern "C" int tpst_profile_reset(tpst_ctx* ctx) {
  if (!ctx) return TPST_E_ARG;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->prof.collect();
  ctx->prof.reset();
  return TPST_OK;
}

extern "C" int tpst_profile_read(tpst_ctx* ctx, int stage, double* total_ms, uint64_t* launches) {
  if (!ctx || !total_ms || !launches || stage < 0 || stage >= N_STAGES) return fail(ctx, TPST_E_ARG, "bad stage");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->prof.collect();
  *total_ms = ctx->prof.total_ms[stage];
  *launches = ctx->prof.count[stage];
  return TPST_OK;
}
