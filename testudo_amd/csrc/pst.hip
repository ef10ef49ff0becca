// sqrt-PST protocol kernels for gfx950 (see pst_kernels.h).
#include "device_util.h"
#include "inv_wave.h"
#include "pst_kernels.h"
#include <cstdlib>

namespace tpst {

static inline unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

__global__ void k_fr_conv(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n, int to_mont_flag) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr a = load_f<Fr>(in + 8 * i);
  store_f<Fr>(out + 8 * i, to_mont_flag ? to_mont(a) : from_mont(a));
}

hipError_t fr_to_mont(hipStream_t s, const uint32_t* in, uint32_t* out, size_t n) {
  if (!n) return hipSuccess;
  k_fr_conv<<<grid_for(n, 256), 256, 0, s>>>(in, out, n, 1);
  return hipGetLastError();
}

hipError_t fr_from_mont(hipStream_t s, const uint32_t* in, uint32_t* out, size_t n) {
  if (!n) return hipSuccess;
  k_fr_conv<<<grid_for(n, 256), 256, 0, s>>>(in, out, n, 0);
  return hipGetLastError();
}

__global__ void k_chi(const uint32_t* __restrict__ b, int m, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ((size_t)1 << m)) return;
  Fr prod = Fr::one();
  for (int j = 0; j < m; j++) {
    const Fr bj = load_f<Fr>(b + 8 * j);
    prod = mul(prod, ((i >> (m - j - 1)) & 1) ? bj : sub(Fr::one(), bj));
  }
  store_f<Fr>(out + 8 * i, prod);
}

hipError_t chi_table(hipStream_t s, const uint32_t* d_b, int m, uint32_t* d_out) {
  const size_t n = (size_t)1 << m;
  k_chi<<<grid_for(n, 256), 256, 0, s>>>(d_b, m, d_out);
  return hipGetLastError();
}

// one workgroup per output j: q[j] = sum_{i < nr} Z[j cs + i] chis[i], the run
// Z[j cs .. j cs + nr) contiguous and read coalesced (the whole polynomial:
// cs = nr = 2^m_col; a row shard: the shard's block, nr of its rows)
template <int BS>
__global__ void __launch_bounds__(BS) k_get_q(const uint32_t* __restrict__ Z, size_t cs, size_t nr,
                                              const uint32_t* __restrict__ chis, uint32_t* __restrict__ q,
                                              int canonical_out) {
  __shared__ Fr sh[BS];
  const size_t j = blockIdx.x;
  Fr acc = Fr::zero();
  for (size_t i = threadIdx.x; i < nr; i += BS) {
    const Fr z = to_mont(load_f<Fr>(Z + 8 * (j * cs + i)));
    acc = add(acc, mul(z, load_f<Fr>(chis + 8 * i)));
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int h = BS / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) sh[threadIdx.x] = add(sh[threadIdx.x], sh[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) store_f<Fr>(q + 8 * j, canonical_out ? from_mont(sh[0]) : sh[0]);
}

hipError_t get_q(hipStream_t s, const uint32_t* d_Z, int m_col, int m_row, const uint32_t* d_chis, uint32_t* d_q) {
  const size_t C = (size_t)1 << m_col;
  k_get_q<256><<<(unsigned)((size_t)1 << m_row), 256, 0, s>>>(d_Z, C, C, d_chis, d_q, 0);
  return hipGetLastError();
}

hipError_t get_q_rows(hipStream_t s, const uint32_t* d_Z, size_t cs, size_t nr, int m_row, const uint32_t* d_chis,
                      uint32_t* d_q_canonical) {
  k_get_q<256><<<(unsigned)((size_t)1 << m_row), 256, 0, s>>>(d_Z, cs, nr, d_chis, d_q_canonical, 1);
  return hipGetLastError();
}

// out[j] = sum_t parts[t n + j] (mod r), canonical in and out
__global__ void k_fr_sum_parts(const uint32_t* __restrict__ parts, size_t k, size_t n, uint32_t* __restrict__ out) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  Fr acc = Fr::zero();
  for (size_t t = 0; t < k; t++) acc = add(acc, load_f<Fr>(parts + 8 * (t * n + j)));
  store_f<Fr>(out + 8 * j, acc);
}

hipError_t fr_sum_parts(hipStream_t s, const uint32_t* d_parts, size_t k, size_t n, uint32_t* d_out) {
  if (!n) return hipSuccess;
  k_fr_sum_parts<<<grid_for(n, 256), 256, 0, s>>>(d_parts, k, n, d_out);
  return hipGetLastError();
}

template <int BS>
__global__ void __launch_bounds__(BS) k_fr_dot(const uint32_t* __restrict__ x, const uint32_t* __restrict__ y, size_t n,
                                               uint32_t* __restrict__ v) {
  __shared__ Fr sh[BS];
  Fr acc = Fr::zero();
  for (size_t i = threadIdx.x; i < n; i += BS) acc = add(acc, mul(load_f<Fr>(x + 8 * i), load_f<Fr>(y + 8 * i)));
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int h = BS / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) sh[threadIdx.x] = add(sh[threadIdx.x], sh[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) store_f<Fr>(v, sh[0]);
}

hipError_t fr_dot(hipStream_t s, const uint32_t* d_x, const uint32_t* d_y, size_t n, uint32_t* d_v) {
  k_fr_dot<256><<<1, 256, 0, s>>>(d_x, d_y, n, d_v);
  return hipGetLastError();
}

__global__ void k_pst_step(const uint32_t* __restrict__ r, size_t half, const uint32_t* __restrict__ pt,
                           uint32_t* __restrict__ qcan, uint32_t* __restrict__ rnext) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= half) return;
  const Fr p = load_f<Fr>(pt);
  const Fr r0 = load_f<Fr>(r + 16 * b), r1 = load_f<Fr>(r + 16 * b + 8);
  const Fr d = sub(r1, r0);
  store_f<Fr>(qcan + 8 * b, from_mont(d));
  store_f<Fr>(rnext + 8 * b, add(r0, mul(d, p)));  // r0(1-p) + r1 p
}

hipError_t pst_step(hipStream_t s, const uint32_t* d_r, size_t half, const uint32_t* d_pt, uint32_t* d_qcan,
                    uint32_t* d_rnext) {
  if (!half) return hipSuccess;
  k_pst_step<<<grid_for(half, 256), 256, 0, s>>>(d_r, half, d_pt, d_qcan, d_rnext);
  return hipGetLastError();
}

template <class F>
__global__ void __launch_bounds__(64, 1) k_compress(uint32_t* __restrict__ v, size_t split, const uint32_t* __restrict__ k) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= split) return;
  uint32_t sc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) sc[j] = k[j];
  const Affine<F> l = load_affine<F>(v, i), r = load_affine<F>(v, i + split);
  Xyzz<F> acc = scalar_mul(r, sc, 253);
  acc = add_affine(acc, l);
  store_affine(v, i, to_affine(acc));
}

template <class F>
hipError_t compress_points(hipStream_t s, uint32_t* d_v, size_t split, const uint32_t* d_k) {
  if (!split) return hipSuccess;
  k_compress<F><<<grid_for(split, 64), 64, 0, s>>>(d_v, split, d_k);
  return hipGetLastError();
}

__global__ void k_compress_fr(uint32_t* __restrict__ y, size_t split, const uint32_t* __restrict__ k) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= split) return;
  const Fr c = load_f<Fr>(k);
  store_f<Fr>(y + 8 * i, add(load_f<Fr>(y + 8 * i), mul(load_f<Fr>(y + 8 * (i + split)), c)));
}

hipError_t compress_fr(hipStream_t s, uint32_t* d_y, size_t split, const uint32_t* d_kmont) {
  if (!split) return hipSuccess;
  k_compress_fr<<<grid_for(split, 256), 256, 0, s>>>(d_y, split, d_kmont);
  return hipGetLastError();
}

template <class F>
__global__ void __launch_bounds__(64, 1) k_fixed_base(const uint32_t* __restrict__ p, const uint32_t* __restrict__ scalars, size_t n,
                             uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Affine<F> P = load_affine<F>(p, 0);
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; j++) k[j] = scalars[8 * i + j];
  store_affine(out, i, to_affine(scalar_mul(P, k, 253)));
}

template <class F>
hipError_t fixed_base_mul(hipStream_t s, const uint32_t* d_p, const uint32_t* d_scalars, size_t n, uint32_t* d_out) {
  if (!n) return hipSuccess;
  k_fixed_base<F><<<grid_for(n, 64), 64, 0, s>>>(d_p, d_scalars, n, d_out);
  return hipGetLastError();
}

template <class F>
__global__ void __launch_bounds__(64, 1) k_pair_sum(const uint32_t* __restrict__ in, size_t half, uint32_t* __restrict__ out) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= half) return;
  Xyzz<F> a = to_xyzz(load_affine<F>(in, 2 * b));
  a = add_affine(a, load_affine<F>(in, 2 * b + 1));
  store_affine(out, b, to_affine(a));
}

template <class F>
hipError_t pair_sum(hipStream_t s, const uint32_t* d_in, size_t half, uint32_t* d_out) {
  if (!half) return hipSuccess;
  k_pair_sum<F><<<grid_for(half, 64), 64, 0, s>>>(d_in, half, d_out);
  return hipGetLastError();
}

template <class F>
__global__ void __launch_bounds__(64, 1) k_xyzz_to_affine_mont(const Xyzz<F>* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_affine(out, i, to_affine(load_xyzz(in, i)));
}

// (one inverse per wave by Montgomery's batch trick across the lanes was
// measured within noise for the h vector of the opening: not kept)

// one wave per point, the wave-cooperative inverse (inv_wave.h): the
// latency-bound conversions of the opening (the h vector each round before
// its G2 preparation, <= C / 2 points; the gathered a^(r1))
template <class F>
__global__ void __launch_bounds__(64) k_xyzz_to_affine_mont_wave(const Xyzz<F>* __restrict__ in,
                                                                 uint32_t* __restrict__ out, size_t n) {
  const size_t i = blockIdx.x;
  if (i >= n) return;
  const Affine<F> a = to_affine_w(load_xyzz(in, i));
  if (threadIdx.x == 0) store_affine(out, i, a);
}

constexpr size_t MONT_WAVE_MAX = 4096;

template <class F>
hipError_t xyzz_to_affine_mont(hipStream_t s, const Xyzz<F>* d_in, uint32_t* d_out, size_t n) {
  if (!n) return hipSuccess;
  if (n <= MONT_WAVE_MAX)
    k_xyzz_to_affine_mont_wave<F><<<(unsigned)n, 64, 0, s>>>(d_in, d_out, n);
  else
    k_xyzz_to_affine_mont<F><<<grid_for(n, 64), 64, 0, s>>>(d_in, d_out, n);
  return hipGetLastError();
}

__global__ void k_affine_rot(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n, size_t words) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * words) return;
  const size_t j = t / words, w = t % words;
  out[t] = in[((j + n / 2) % n) * words + w];
}

hipError_t affine_rot(hipStream_t s, const uint32_t* d_in, uint32_t* d_out, size_t n, size_t words) {
  if (!n) return hipSuccess;
  k_affine_rot<<<grid_for(n * words, 256), 256, 0, s>>>(d_in, d_out, n, words);
  return hipGetLastError();
}

// MIPP fold scalars over the original bases (fbt.h strided groups):
// fold:  out[k] = W[k / len]                      (a^(r)_i = sum_t W_t a_{i + t len})
// cross: out[k] = W[k / len] * y[(k % len + s) % len]   (u_l / u_r, mipp.rs:66-75)
// out[kl] for the base k = sub kl + off (sub = 1, off = 0: every base; a
// rank of a row-sharded opening takes its rows k = off mod sub)
__global__ void k_mipp_scalars(const uint32_t* __restrict__ W, const uint32_t* __restrict__ y, size_t len, size_t s,
                               size_t n, size_t sub, size_t off, uint32_t* __restrict__ out) {
  const size_t kl = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (kl >= n) return;
  const size_t k = sub * kl + off;
  Fr v = load_f<Fr>(W + 8 * (k / len));
  if (y) v = mul(v, load_f<Fr>(y + 8 * ((k % len + s) % len)));
  store_f<Fr>(out + 8 * kl, from_mont(v));
}

hipError_t mipp_scalars(hipStream_t s, const uint32_t* d_W, const uint32_t* d_y, size_t len, size_t split, size_t n,
                        uint32_t* d_out, size_t sub, size_t off) {
  if (!n) return hipSuccess;
  k_mipp_scalars<<<grid_for(n, 256), 256, 0, s>>>(d_W, d_y, len, split, n, sub, off, d_out);
  return hipGetLastError();
}

// E fold sets at once: out[j n + kl] = canonical(W[k / len] * f[j]), k = sub kl + off
__global__ void k_mipp_scalar_sets(const uint32_t* __restrict__ W, const uint32_t* __restrict__ f, int E, size_t len,
                                   size_t n, size_t sub, size_t off, uint32_t* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)E * n) return;
  const size_t j = t / n, k = sub * (t % n) + off;
  store_f<Fr>(out + 8 * t, from_mont(mul(load_f<Fr>(W + 8 * (k / len)), load_f<Fr>(f + 8 * j))));
}

hipError_t mipp_scalar_sets(hipStream_t s, const uint32_t* d_W, const uint32_t* d_f, int E, size_t len, size_t n,
                            uint32_t* d_out, size_t sub, size_t off) {
  if (!n || E <= 0) return hipSuccess;
  k_mipp_scalar_sets<<<grid_for((size_t)E * n, 256), 256, 0, s>>>(d_W, d_f, E, len, n, sub, off, d_out);
  return hipGetLastError();
}

// out[g] = sum_{w < W} parts[w G + g] (XYZZ): the combine of gathered per-rank
// partial sums, one lane per group
__global__ void __launch_bounds__(64, 1) k_xyzz_sum_groups(const Xyzz<Fq>* __restrict__ parts, size_t W, size_t G,
                                                          Xyzz<Fq>* __restrict__ out) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  Xyzz<Fq> acc = load_xyzz(parts, g);
  for (size_t w = 1; w < W; w++) acc = add(acc, load_xyzz(parts, w * G + g));
  store_xyzz(out, g, acc);
}

hipError_t xyzz_sum_groups(hipStream_t s, const Xyzz<Fq>* d_parts, size_t W, size_t G, Xyzz<Fq>* d_out) {
  if (!G || !W) return hipSuccess;
  k_xyzz_sum_groups<<<grid_for(G, 64), 64, 0, s>>>(d_parts, W, G, d_out);
  return hipGetLastError();
}

// MIPP fold weights of round r from round r-1's (mipp.rs:58-120 unrolled):
// W_r[2t] = W_{r-1}[t], W_r[2t+1] = W_{r-1}[t] c, and Wi likewise with c^-1;
// round r's 2^r weights live at offset 2^r - 1 of W / Wi (r = 0: W_0 = Wi_0 = 1)
__global__ void k_mipp_weights(uint32_t* __restrict__ W, uint32_t* __restrict__ Wi, int r,
                               const uint32_t* __restrict__ c, const uint32_t* __restrict__ cinv) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nw = (size_t)1 << r;
  if (t >= nw) return;
  const size_t o = nw - 1 + t;
  if (r == 0) {
    store_f<Fr>(W + 8 * o, Fr::one());
    store_f<Fr>(Wi + 8 * o, Fr::one());
    return;
  }
  const size_t src = (nw / 2 - 1) + (t >> 1);
  Fr w = load_f<Fr>(W + 8 * src), wi = load_f<Fr>(Wi + 8 * src);
  if (t & 1) {
    w = mul(w, load_f<Fr>(c));
    wi = mul(wi, load_f<Fr>(cinv));
  }
  store_f<Fr>(W + 8 * o, w);
  store_f<Fr>(Wi + 8 * o, wi);
}

hipError_t mipp_weights(hipStream_t s, uint32_t* d_W, uint32_t* d_Wi, int r, const uint32_t* d_c,
                        const uint32_t* d_cinv) {
  const size_t nw = (size_t)1 << r;
  k_mipp_weights<<<grid_for(nw, 256), 256, 0, s>>>(d_W, d_Wi, r, d_c, d_cinv);
  return hipGetLastError();
}

template hipError_t compress_points<Fq>(hipStream_t, uint32_t*, size_t, const uint32_t*);
template hipError_t compress_points<Fq2>(hipStream_t, uint32_t*, size_t, const uint32_t*);
template hipError_t fixed_base_mul<Fq>(hipStream_t, const uint32_t*, const uint32_t*, size_t, uint32_t*);
template hipError_t fixed_base_mul<Fq2>(hipStream_t, const uint32_t*, const uint32_t*, size_t, uint32_t*);
template hipError_t pair_sum<Fq>(hipStream_t, const uint32_t*, size_t, uint32_t*);
template hipError_t pair_sum<Fq2>(hipStream_t, const uint32_t*, size_t, uint32_t*);
template hipError_t xyzz_to_affine_mont<Fq>(hipStream_t, const Xyzz<Fq>*, uint32_t*, size_t);
template hipError_t xyzz_to_affine_mont<Fq2>(hipStream_t, const Xyzz<Fq2>*, uint32_t*, size_t);

}  // namespace tpst
