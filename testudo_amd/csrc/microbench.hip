// Field / curve microbenchmarks (tpst_microbench): the measured compute peak
// used in bench.py's roofline, and A/B variants of the Fq multiply.
#include <vector>
#include "../../include/tpst.h"
#include "ctx.h"
#include "device_util.h"
#include "wave_tower.h"
#include "rns_engine.h"
#include "field29.h"
#include "inv_wave.h"

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

// ---- single-instruction issue rates: 8 independent chains per lane -------
// kind 6: v_mad_u64_u32, 7: v_mad_u32_u24, 8: v_mul_lo_u32, 9: v_add_u32,
// 10: v_fma_f64, 11: v_mul_hi_u32 (iters x 4 x 8 instructions per lane);
// kinds 112..115 (tpst_microbench): 12 v_lshl_add_u64, 13 v_lshrrev_b64,
// 14 v_alignbit_b32, 15 v_add3_u32
template <int K>
__global__ void k_mb_insn(int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a64[8];
  uint32_t a32[8];
  double f[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    a64[j] = t * 13u + j;
    a32[j] = t * 7u + j;
    f[j] = (double)(t + j);
  }
  const uint32_t x = t | 1u, y = t * 3u + 5u;
  const double fx = 1.0000001, fy = 1e-9;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if constexpr (K == 6) {
          uint64_t c;
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a64[j]), "=&s"(c) : "v"(x), "v"(y));
        } else if constexpr (K == 7) {
          asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(a32[j]) : "v"(x), "v"(y));
        } else if constexpr (K == 8) {
          asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a32[j]) : "v"(x));
        } else if constexpr (K == 9) {
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(a32[j]) : "v"(x));
        } else if constexpr (K == 10) {
          asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(f[j]) : "v"(fx), "v"(fy));
        } else if constexpr (K == 12) {  // the column carry add of the radix-2^29 product
          asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a64[j]) : "v"(a64[(j + 1) & 7]));
        } else if constexpr (K == 13) {  // the column shift acc >>= 29
          asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(a64[j]));
        } else if constexpr (K == 14) {
          asm volatile("v_alignbit_b32 %0, %0, %1, 29" : "+v"(a32[j]) : "v"(x));
        } else if constexpr (K == 15) {
          asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a32[j]) : "v"(x), "v"(y));
        } else {
          asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a32[j]) : "v"(x));
        }
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= (uint32_t)a64[j] ^ a32[j] ^ (uint32_t)f[j];
  out[t] = r;
}

// ---- A/B variants of the device Montgomery product (latency experiments) --
// ILP2: product scanning with the terms of every column split over two
// independent (acc, hi) chains, merged when the column completes.
__device__ __forceinline__ Fq mul_ilp2(const Fq& a, const Fq& b) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return mul(a, b);
#else
  constexpr int N = 12;
  uint32_t m[N], t[N];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t a1 = 0;
    uint32_t h1 = 0;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j >= 0 && j < N) {
        if (cnt++ & 1) mac_vv(a1, h1, a.v[i], b.v[j]);
        else mac_vv(acc, hi, a.v[i], b.v[j]);
      }
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N) {
        if (cnt++ & 1) mac_vs(a1, h1, m[i], FqCfg::p(j));
        else mac_vs(acc, hi, m[i], FqCfg::p(j));
      }
    }
    {  // merge the chains: (hi:acc) += (h1:a1)
      const uint64_t s = acc + a1;
      hi += h1 + (s < acc ? 1u : 0u);
      acc = s;
    }
    if (k < N) {
      const uint32_t lo = (uint32_t)acc;
      m[k] = 0u - lo;
      acc = ((acc >> 32) | ((uint64_t)hi << 32)) + (lo != 0u ? 1u : 0u);
      hi = 0;
      continue;
    } else {
      t[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[N - 1] = (uint32_t)acc;
  Fq r;
#pragma unroll
  for (int j = 0; j < N; j++) r.v[j] = t[j];
  reduce_once(r);
  return r;
#endif
}

// COLS: the 23 columns of a*b accumulate independently (no chain between
// columns), then a word-serial Montgomery reduction over the column sums.
__device__ __forceinline__ Fq mul_cols(const Fq& a, const Fq& b) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return mul(a, b);
#else
  constexpr int N = 12;
  uint64_t c[2 * N];
  uint32_t h[2 * N];
#pragma unroll
  for (int k = 0; k < 2 * N; k++) {
    c[k] = 0;
    h[k] = 0;
  }
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int j = 0; j < N; j++) mac_vv(c[i + j], h[i + j], a.v[i], b.v[j]);
  // REDC: word k exact once column k - 1's carry is in
#pragma unroll
  for (int k = 0; k < N; k++) {
    const uint32_t lo = (uint32_t)c[k];
    const uint32_t mk = 0u - lo;  // p0 = 1
#pragma unroll
    for (int j = 1; j < N; j++) mac_vs(c[k + j], h[k + j], mk, FqCfg::p(j));
    // column k + mk*p0 = (c[k] - lo) + 2^32*(lo != 0): carry up
    const uint64_t up = (c[k] >> 32) | ((uint64_t)h[k] << 32);
    const uint64_t add = up + (lo != 0u ? 1u : 0u);
    const uint64_t s = c[k + 1] + add;
    h[k + 1] += (s < c[k + 1] ? 1u : 0u);
    c[k + 1] = s;
  }
  Fq r;
#pragma unroll
  for (int j = 0; j < N; j++) {
    const int k = N + j;
    r.v[j] = (uint32_t)c[k];
    const uint64_t up = (c[k] >> 32) | ((uint64_t)h[k] << 32);
    if (k + 1 < 2 * N) {
      const uint64_t s = c[k + 1] + up;
      h[k + 1] += (s < c[k + 1] ? 1u : 0u);
      c[k + 1] = s;
    }
  }
  reduce_once(r);
  return r;
#endif
}

__global__ void k_mb_fqmul_v(int variant, int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = Fq::one(), b = Fq::one();
  a.v[0] ^= t;
  b.v[1] ^= t * 7u + 1;
  if (variant == 1)
    for (int i = 0; i < iters; i++) a = mul_ilp2(a, b);
  else
    for (int i = 0; i < iters; i++) a = mul_cols(a, b);
  store_f<Fq>(out + 12 * (size_t)t, a);
}

// radix-2^29 field (field29.h): product / square chains and the XYZZ mixed
// add over it, same shapes as kinds 0 and 1 (kinds 12, 14, 13)
__global__ void k_mb_fq29(int sq, int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Fq29 a = Fq29::one(), b = Fq29::one();
  a.v[0] ^= t & 0xffffu;
  b.v[1] ^= (t * 7u + 1) & 0xffffu;
  if (sq)
    for (int i = 0; i < iters; i++) a = sqr(a);
  else
    for (int i = 0; i < iters; i++) a = mul(a, b);
#pragma unroll
  for (int i = 0; i < 12; i++) out[12 * (size_t)t + i] = a.v[i] ^ (i == 0 ? a.v[12] : 0u);
}

__global__ void k_mb_madd29(int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const Affine<Fq29> g = {from_std(Fq::from_limbs(params::G1_GEN_X)), from_std(Fq::from_limbs(params::G1_GEN_Y))};
  Xyzz<Fq29> acc = dbl_affine(g);
  acc.X.v[0] ^= (t & 1);
  for (int i = 0; i < iters; i++) acc = add_affine(acc, g);
  const Fq x = to_std(acc.X);
  store_f<Fq>(out + 12 * (size_t)t, x);
}

__global__ void k_mb_dbl(int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  G1A g = {Fq::from_limbs(params::G1_GEN_X), Fq::from_limbs(params::G1_GEN_Y)};
  Xyzz<Fq> acc = dbl_affine(g);
  acc.X.v[0] ^= (t & 1);
  for (int i = 0; i < iters; i++) acc = dbl(acc);
  store_f<Fq>(out + 12 * (size_t)t, acc.X);
}

__global__ void k_mb_madd(int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  G1A g = {Fq::from_limbs(params::G1_GEN_X), Fq::from_limbs(params::G1_GEN_Y)};
  Xyzz<Fq> acc = dbl_affine(g);
  acc.X.v[0] ^= (t & 1);  // keep threads independent of each other's values
  for (int i = 0; i < iters; i++) acc = add_affine(acc, g);
  store_f<Fq>(out + 12 * (size_t)t, acc.X);
}

__global__ void k_mb_inv(int iters, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = Fq::one();
  a.v[0] ^= t * 0x9E3779B9u;
  a.v[3] ^= t;
  for (int i = 0; i < iters; i++) {
    a = inv(a);
    a.v[1] ^= 1u;
  }
  store_f<Fq>(out + 12 * (size_t)t, a);
}

// one wave per 64 threads, `iters` dependent wave-cooperative inverses
__global__ void __launch_bounds__(64) k_mb_inv_wave(int iters, uint32_t* out) {
  const uint32_t w = blockIdx.x;
  Fq a = Fq::one();
  a.v[0] ^= w * 0x9E3779B9u;
  a.v[3] ^= w;
  for (int i = 0; i < iters; i++) {
    a = inv_w(a);
    a.v[1] ^= 1u;
  }
  if (threadIdx.x == 0) store_f<Fq>(out + 12 * (size_t)w, a);
}

// inverses of n Montgomery-form Fq values by both inverse routines
__global__ void __launch_bounds__(64) k_selftest_inv(const uint32_t* __restrict__ in, uint32_t* __restrict__ o_lane,
                                                     uint32_t* __restrict__ o_wave, size_t n) {
  const size_t i = blockIdx.x;
  if (i >= n) return;
  const Fq a = load_f<Fq>(in + 12 * i);
  const Fq rw = inv_w(a);
  if (threadIdx.x == 0) {
    store_f<Fq>(o_wave + 12 * i, rw);
    store_f<Fq>(o_lane + 12 * i, inv(a));
  }
}

extern "C" int tpst_selftest_inv(tpst_ctx* ctx, size_t n, const uint64_t* in, uint64_t* out_lane, uint64_t* out_wave) {
  if (!ctx || (n && (!in || !out_lane || !out_wave))) return fail(ctx, TPST_E_ARG, "bad argument");
  if (!n) return TPST_OK;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(3 * Arena::need(n * 12, 4)));
  uint32_t* d_in = ctx->io.take<uint32_t>(n * 12);
  uint32_t* d_l = ctx->io.take<uint32_t>(n * 12);
  uint32_t* d_w = ctx->io.take<uint32_t>(n * 12);
  TPST_HIP(ctx, hipMemcpyAsync(d_in, in, n * 48, hipMemcpyHostToDevice, ctx->stream));
  k_selftest_inv<<<(unsigned)n, 64, 0, ctx->stream>>>(d_in, d_l, d_w, n);
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, hipMemcpyAsync(out_lane, d_l, n * 48, hipMemcpyDeviceToHost, ctx->stream));
  TPST_HIP(ctx, hipMemcpyAsync(out_wave, d_w, n * 48, hipMemcpyDeviceToHost, ctx->stream));
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return TPST_OK;
}

// one wave running `iters` stages of wave-engine op `op` (wave_tower.h)
__global__ void __launch_bounds__(64) k_mb_wave(int op, int iters, uint32_t* out) {
  extern __shared__ uint4 smem4[];
  wave::lds_t* prog = (wave::lds_t*)(smem4);
  const uint32_t len = wave::OP_LEN[op];
  for (uint32_t i = threadIdx.x; i < len; i += 64) prog[i] = wave::BLOB[wave::OP_OFF[op] + i];
  wave::lds_t* vals = prog + ((len + 3) & ~3u);
  wave::load_consts(vals, 0);
  const int base = wave::N_CONSTS;
  for (int i = threadIdx.x; i < 64 + 4 * 48; i += 64) {
    Fq v = Fq::one();
    v.v[0] ^= i;
    wave::put_slot(vals, base + i, v);
  }
  __syncthreads();
  const wave::Eng e{vals, base, 0};
  const int A = base + 64, B = A + 48, Cr = B + 48, D = Cr + 48;
  for (int it = 0; it < iters; it++) wave::run(e, prog, A, B, Cr, D);
  if (threadIdx.x < 12) out[threadIdx.x] = vals[Cr * wave::SLOT + threadIdx.x];
}

// the same stage with s_memtime stamps between its parts (lane 0 totals):
// [0] X/Y forms, [1] Montgomery product, [2] product store + sync,
// [3] output forms, [4] output reduce + store + sync
__global__ void __launch_bounds__(64) k_mb_wave_prof(int op, int iters, unsigned long long* out) {
  extern __shared__ uint4 smem4[];
  wave::lds_t* prog = (wave::lds_t*)(smem4);
  const uint32_t len = wave::OP_LEN[op];
  for (uint32_t i = threadIdx.x; i < len; i += 64) prog[i] = wave::BLOB[wave::OP_OFF[op] + i];
  wave::lds_t* vals = prog + ((len + 3) & ~3u);
  wave::load_consts(vals, 0);
  const int base = wave::N_CONSTS;
  for (int i = threadIdx.x; i < 64 + 4 * 48; i += 64) {
    Fq v = Fq::one();
    v.v[0] ^= i;
    wave::put_slot(vals, base + i, v);
  }
  __syncthreads();
  const wave::Eng e{vals, base, 0};
  const int A = base + 64, B = A + 48, Cr = B + 48;
  unsigned long long acc[5] = {0, 0, 0, 0, 0};
  const int lane = threadIdx.x;
  const wave::lds_t* blk = prog;
  for (int it = 0; it < iters; it++) {
    const uint32_t hdr = __builtin_amdgcn_readfirstlane(blk[0]);
    const uint32_t hdr1 = __builtin_amdgcn_readfirstlane(blk[1]);
    const int np = hdr & 0xff, no = (hdr >> 8) & 0xff, nc = hdr >> 24;
    const int tx = hdr1 & 0xff, ty = (hdr1 >> 8) & 0xff, tc = (hdr1 >> 16) & 0xff;
    const bool sq = (hdr >> 17) & 1;
    const uint64_t bases = wave::pack_bases(e, A, B);
    const wave::lds_t* X = blk + 2;
    const wave::lds_t* Y = X + tx * np;
    const wave::lds_t* CH = Y + ty * np;
    const wave::lds_t* DST = CH + tc * nc + no;
    unsigned long long t0 = clock64();
    uint32_t xw[13], yw[13];
    Fq x, y, pr;
    if (lane < np) {
      wave::form(e, X + lane, np, tx, bases, xw);
      if (!sq) wave::form(e, Y + lane, np, ty, bases, yw);
#pragma unroll
      for (int i = 0; i < 12; i++) {
        x.v[i] = xw[i];
        y.v[i] = yw[i];
      }
    }
    unsigned long long t1 = clock64();
    if (lane < np) pr = sq ? wave::stage_sqr(x) : wave::stage_mul(x, y);
    unsigned long long t2 = clock64();
    if (lane < np) wave::put_slot(vals, base + lane, pr);
    wave::wave_sync();
    unsigned long long t3 = clock64();
    uint32_t w[13];
    if (lane < nc) wave::form(e, CH + lane, nc, tc, bases, w);
    unsigned long long t4 = clock64();
    if (lane < no) wave::put_slot(vals, Cr + (DST[lane] & 0xff), wave::reduce_wide(w));
    wave::wave_sync();
    unsigned long long t5 = clock64();
    acc[0] += t1 - t0;
    acc[1] += t2 - t1;
    acc[2] += t3 - t2;
    acc[3] += t4 - t3;
    acc[4] += t5 - t4;
  }
  if (lane == 0)
    for (int i = 0; i < 5; i++) out[i] = acc[i];
}

// RNS engine stages (rns_engine.h): each 12-wave workgroup (two chains) runs
// `iters` dependent stages of OP; grid = threads / 768 workgroups, so one
// workgroup measures the stage latency and a full grid the throughput
template <int OP, class LT>
__device__ __forceinline__ void mb_rns_body(const LT& L, uint32_t* s_slots, uint32_t* s_xch, int iters,
                                            uint32_t* __restrict__ sink);

template <int OP>
__global__ void __launch_bounds__(768) k_mb_rns(int iters, uint32_t* __restrict__ sink) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 36) * rns::SLOT];
  __shared__ uint32_t s_xch[12 * rns::XCH];
  rns::load_consts((rns::lds_t*)s_slots);
  mb_rns_body<OP>(rns::load_lane(), s_slots, s_xch, iters, sink);
}

// the same with the extension rows in LDS (rns::LaneL), two workgroups per CU
template <int OP>
__global__ void __launch_bounds__(768, 2) k_mb_rns_l(int iters, uint32_t* __restrict__ sink) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 36) * rns::SLOT];
  __shared__ uint32_t s_xch[12 * rns::XCH];
  __shared__ uint32_t s_rows[2 * rns::NB * 32];
  rns::load_consts((rns::lds_t*)s_slots);
  mb_rns_body<OP>(rns::load_lane_lds((rns::lds_t*)s_rows), s_slots, s_xch, iters, sink);
}

template <int OP, class LT>
__device__ __forceinline__ void mb_rns_body(const LT& L, uint32_t* s_slots, uint32_t* s_xch, int iters,
                                            uint32_t* __restrict__ sink) {
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  for (int i = threadIdx.x; i < 24 * rns::SLOT; i += blockDim.x)
    s_slots[rns::N_CONSTS * rns::SLOT + i] = s_slots[((i / rns::SLOT) % rns::N_CONSTS) * rns::SLOT + (i % rns::SLOT)];
  __syncthreads();
  int acc = rns::N_CONSTS, in_r = acc + 12, tmp = acc + 24;
  for (int it = 0; it < iters; it++) {
    rns::stage<OP>(e, L, acc, in_r, tmp);
    const int t = acc;
    acc = tmp;
    tmp = t;
  }
  rns::store_res(e, acc, sink + (size_t)blockIdx.x * 2 * rns::RES_WORDS, sink + ((size_t)blockIdx.x * 2 + 1) * rns::RES_WORDS, 12);
}

extern "C" int tpst_microbench_wave_phases(tpst_ctx* ctx, int op, int iters, uint64_t* cycles5) {
  if (!ctx || !cycles5 || op < 0 || op >= wave::N_OPS || iters <= 0) return fail(ctx, TPST_E_ARG, "bad argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  ctx->io.reset();
  TPST_HIP(ctx, ctx->io.reserve(256));
  unsigned long long* d = ctx->io.take<unsigned long long>(8);
  const size_t lds = (((wave::OP_LEN[op] + 3) & ~3u) + (size_t)(wave::N_CONSTS + 64 + 4 * 48) * wave::SLOT) * 4;
  k_mb_wave_prof<<<1, 64, lds, ctx->stream>>>(op, iters, d);
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, hipMemcpyAsync(cycles5, d, 40, hipMemcpyDeviceToHost, ctx->stream));
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return TPST_OK;
}

extern "C" int tpst_microbench(tpst_ctx* ctx, int kind, size_t threads, int iters, double* ms) {
  if (!ctx || !ms || threads == 0 || iters <= 0) return fail(ctx, TPST_E_ARG, "bad argument");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  const bool rnsk = kind >= 64 && kind < 96;
  const unsigned bs = rnsk ? 768u : (threads < 256 ? (unsigned)threads : 256u);
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
  else if (kind == 2)
    k_mb_inv<<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 3 || kind == 4)
    k_mb_fqmul_v<<<grid, bs, 0, ctx->stream>>>(kind - 2, iters, d);
  else if (kind == 5)
    k_mb_dbl<<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 6)
    k_mb_insn<6><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 7)
    k_mb_insn<7><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 8)
    k_mb_insn<8><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 9)
    k_mb_insn<9><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 10)
    k_mb_insn<10><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 11)
    k_mb_insn<11><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 12 || kind == 14)
    k_mb_fq29<<<grid, bs, 0, ctx->stream>>>(kind == 14, iters, d);
  else if (kind == 15)
    k_mb_inv_wave<<<grid_for(threads, 64), 64, 0, ctx->stream>>>(iters, d);
  else if (kind == 13)
    k_mb_madd29<<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 112)
    k_mb_insn<12><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 113)
    k_mb_insn<13><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 114)
    k_mb_insn<14><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind == 115)
    k_mb_insn<15><<<grid, bs, 0, ctx->stream>>>(iters, d);
  else if (kind >= 16 && kind < 16 + wave::N_OPS) {
    const int op = kind - 16;
    const size_t lds = (((wave::OP_LEN[op] + 3) & ~3u) + (size_t)(wave::N_CONSTS + 64 + 4 * 48) * wave::SLOT) * 4;
    k_mb_wave<<<1, 64, lds, ctx->stream>>>(op, iters, d);
  } else if (kind == 64 + rns::OP_F12_MUL) {
    k_mb_rns<rns::OP_F12_MUL><<<grid, bs, 0, ctx->stream>>>(iters, d);
  } else if (kind == 64 + rns::OP_F12_SQR) {
    k_mb_rns<rns::OP_F12_SQR><<<grid, bs, 0, ctx->stream>>>(iters, d);
  } else if (kind == 64 + rns::OP_CYC_SQR) {
    k_mb_rns<rns::OP_CYC_SQR><<<grid, bs, 0, ctx->stream>>>(iters, d);
  } else if (kind == 80 + rns::OP_F12_MUL) {
    k_mb_rns_l<rns::OP_F12_MUL><<<grid, bs, 0, ctx->stream>>>(iters, d);
  } else if (kind == 80 + rns::OP_CYC_SQR) {
    k_mb_rns_l<rns::OP_CYC_SQR><<<grid, bs, 0, ctx->stream>>>(iters, d);
  } else
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

