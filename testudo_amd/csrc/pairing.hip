// K4: optimal-ate multi-pairing on gfx950.
//
// Layout: prepared line coefficients are coefficient-major (all pairs' step
// idx coefficients contiguous) so the Miller kernel's per-step loads are
// coalesced across threads.  A thread owns `k` pairs of one group and keeps
// one running f (Fq12), so f^2 is paid once per step for k pairs
// (arkworks does the same with chunks of 4, bls12/mod.rs multi_miller_loop).
#include "device_util.h"
#include "pairing_kernels.h"

namespace tpst {

#define TPST_TRY(x)                  \
  do {                               \
    hipError_t _e = (x);             \
    if (_e != hipSuccess) return _e; \
  } while (0)

static inline unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

__global__ void k_g2_prepare(const uint32_t* __restrict__ g2, size_t n, LineCoeff* __restrict__ coeffs) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G2A q = load_affine<Fq2>(g2, i);
  if (is_inf(q)) return;
  g2_prepare(q, coeffs + i, (long)n);
}

hipError_t g2_prepare_batch(hipStream_t s, const uint32_t* d_g2, size_t n, LineCoeff* d_coeffs) {
  if (!n) return hipSuccess;
  k_g2_prepare<<<grid_for(n, 64), 64, 0, s>>>(d_g2, n, d_coeffs);
  return hipGetLastError();
}

// thread (g, t) handles pairs t, t+T, ... of group g; writes its partial f
__global__ void k_miller(const uint32_t* __restrict__ g1, const uint32_t* __restrict__ g2,
                         const LineCoeff* __restrict__ coeffs, size_t groups, size_t n, size_t T,
                         Fq12* __restrict__ partial) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= groups * T) return;
  const size_t g = tid / T, t = tid % T;
  const size_t stride = groups * n;
  Fq12 f = Fq12::one();
  int idx = 0;
  for (int b = X_BITS - 2; b >= 0; b--) {
    f = sqr(f);
    const bool add_step = (params::BLS_X >> b) & 1;
    for (size_t i = t; i < n; i += T) {
      const size_t pi = g * n + i;
      const G1A p = load_affine<Fq>(g1, pi);
      const G2A q = load_affine<Fq2>(g2, pi);
      if (is_inf(p) || is_inf(q)) continue;
      f = ell(f, coeffs[(size_t)idx * stride + pi], p);
      if (add_step) f = ell(f, coeffs[(size_t)(idx + 1) * stride + pi], p);
    }
    idx += add_step ? 2 : 1;
  }
  partial[tid] = f;
}

// one workgroup per group: product of T partials, then final exponentiation
template <int BS>
__global__ void __launch_bounds__(BS) k_gt_reduce_final(const Fq12* __restrict__ partial, size_t T,
                                                       Fq12* __restrict__ out) {
  __shared__ Fq12 sh[BS];
  const size_t g = blockIdx.x;
  Fq12 acc = Fq12::one();
  for (size_t k = threadIdx.x; k < T; k += BS) acc = mul(acc, partial[g * T + k]);
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int h = BS / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) sh[threadIdx.x] = mul(sh[threadIdx.x], sh[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[g] = final_exponentiation(sh[0]);
}

hipError_t multi_pairing_prepared(Arena& ar, hipStream_t s, const uint32_t* d_g1, const uint32_t* d_g2,
                                  const LineCoeff* d_coeffs, size_t groups, size_t n, Fq12* d_out) {
  if (!groups) return hipSuccess;
  // one pair per thread: latency-bound chains favour width
  size_t T = n ? n : 1;
  Fq12* partial = ar.take<Fq12>(groups * T);
  k_miller<<<grid_for(groups * T, 64), 64, 0, s>>>(d_g1, d_g2, d_coeffs, groups, n, T, partial);
  TPST_TRY(hipGetLastError());
  k_gt_reduce_final<32><<<(unsigned)groups, 32, 0, s>>>(partial, T, d_out);
  return hipGetLastError();
}

hipError_t multi_pairing(Arena& ar, hipStream_t s, const uint32_t* d_g1, const uint32_t* d_g2, size_t groups,
                         size_t n, Fq12* d_out) {
  const size_t np = groups * n;
  size_t need = Arena::need(np * N_LINE_COEFFS, sizeof(LineCoeff)) + Arena::need(np ? np : groups, sizeof(Fq12)) + 4096;
  ar.reset();
  TPST_TRY(ar.reserve(need));
  LineCoeff* coeffs = ar.take<LineCoeff>(np * N_LINE_COEFFS);
  TPST_TRY(g2_prepare_batch(s, d_g2, np, coeffs));
  return multi_pairing_prepared(ar, s, d_g1, d_g2, coeffs, groups, n, d_out);
}

__global__ void k_fq12_from_mont(const Fq12* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 12) return;
  const Fq* c = reinterpret_cast<const Fq*>(in);
  store_f<Fq>(out + 12 * i, from_mont(c[i]));
}

hipError_t fq12_from_mont(hipStream_t s, const Fq12* d_in, uint32_t* d_out, size_t n) {
  if (!n) return hipSuccess;
  k_fq12_from_mont<<<grid_for(n * 12, 64), 64, 0, s>>>(d_in, d_out, n);
  return hipGetLastError();
}

}  // namespace tpst
