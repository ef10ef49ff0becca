// Fixed-base lookup tables + grouped fixed-base MSM (see fbt.h).
#include "fbt.h"

namespace tpst {

#define TPST_TRY(x)                  \
  do {                               \
    hipError_t _e = (x);             \
    if (_e != hipSuccess) return _e; \
  } while (0)

static inline unsigned fbt_grid(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

// 2^(4w) B_k for w < 64 (XYZZ): one thread per base, 252 doublings
template <class F>
__global__ void __launch_bounds__(64) k_fbt_pow(const uint32_t* __restrict__ bases, size_t n,
                                                Xyzz<F>* __restrict__ tmp) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  Xyzz<F> p = to_xyzz(load_affine<F>(bases, k));
  for (int w = 0; w < FBT_W; w++) {
    store_xyzz(tmp, k * FBT_W + w, p);
    if (w + 1 < FBT_W) {
      p = dbl(p);
      p = dbl(p);
      p = dbl(p);
      p = dbl(p);
    }
  }
}

// entry (k, w, m) = (m+1) * tmp[k, w], normalised to affine
template <class F>
__global__ void __launch_bounds__(64) k_fbt_mult(const Xyzz<F>* __restrict__ tmp, size_t n,
                                                 uint32_t* __restrict__ table) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= fbt_entries<F>(n)) return;
  const int m = (int)(i % FBT_M) + 1;
  const Xyzz<F> p = load_xyzz(tmp, i / FBT_M);
  Xyzz<F> q = p;
  for (int b = 30 - __clz(m); b >= 0; b--) {
    q = dbl(q);
    if ((m >> b) & 1) q = add(q, p);
  }
  store_affine<F>(table, i, to_affine(q));
}

template <class F>
hipError_t fbt_build(Arena& ar, hipStream_t s, const uint32_t* d_bases, size_t n, uint32_t* d_table) {
  if (!n) return hipSuccess;
  ar.reset();
  TPST_TRY(ar.reserve(Arena::need(n * FBT_W, sizeof(Xyzz<F>))));
  Xyzz<F>* tmp = ar.take<Xyzz<F>>(n * FBT_W);
  k_fbt_pow<F><<<fbt_grid(n, 64), 64, 0, s>>>(d_bases, n, tmp);
  TPST_TRY(hipGetLastError());
  k_fbt_mult<F><<<fbt_grid(fbt_entries<F>(n), 64), 64, 0, s>>>(tmp, n, d_table);
  return hipGetLastError();
}

// signed 4-bit digit of window w given the incoming carry
__device__ __forceinline__ int fbt_digit(const uint32_t* s, int w, int& carry) {
  int d = (int)((s[w >> 3] >> ((w & 7) * 4)) & 15u) + carry;
  carry = d > 8;
  return carry ? d - 16 : d;
}

// thread (g, m, chunk): sum of the 8 lookups of windows [8 chunk, 8 chunk + 8)
template <class F>
__global__ void __launch_bounds__(64) k_fbt_partial(const uint32_t* __restrict__ table,
                                                    const uint32_t* __restrict__ scal, FbGroups gr,
                                                    Xyzz<F>* __restrict__ partial) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= gr.sets * gr.groups * gr.members * 8) return;
  const int ch = (int)(i & 7);
  const size_t per_set = gr.groups * gr.members;
  const size_t qgm = i >> 3, q = qgm / per_set, gm = qgm % per_set;
  const size_t g = gm / gr.members, m = gm % gr.members;
  size_t k;
  bool valid = true;
  if (gr.d_seg) {
    const size_t lo = gr.d_seg[g], hi = gr.d_seg[g + 1];
    valid = m < hi - lo;
    k = lo + m;
  } else {
    k = (m / gr.D) * gr.L + g * gr.D + m % gr.D;
  }
  Xyzz<F> acc = Xyzz<F>::inf();
  if (valid) {
    uint32_t s[8];
    const uint4* sp = reinterpret_cast<const uint4*>(scal + 8 * (k + q * gr.set_stride));
    const uint4 a = sp[0], b = sp[1];
    s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
    s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
    int carry = 0;
    for (int w = 0; w < 8 * ch; w++) fbt_digit(s, w, carry);
    for (int j = 0; j < 8; j++) {
      const int w = 8 * ch + j;
      const int d = fbt_digit(s, w, carry);
      if (d) {
        Affine<F> t = load_affine<F>(table, (k * FBT_W + w) * FBT_M + (d < 0 ? -d : d) - 1);
        if (d < 0) t = neg(t);
        acc = add_affine(acc, t);
      }
    }
  }
  store_xyzz(partial, i, acc);
}

// out[seg * out_len + part] = sum of in[seg * seg_len + part * per .. + per)
template <class F, int BS>
__global__ void __launch_bounds__(BS) k_seg_sum(const Xyzz<F>* __restrict__ in, size_t seg_len, size_t per,
                                                size_t parts, Xyzz<F>* __restrict__ out) {
  __shared__ Xyzz<F> sh[BS];
  const size_t seg = blockIdx.x / parts, part = blockIdx.x % parts;
  const size_t lo = part * per, hi = lo + per < seg_len ? lo + per : seg_len;
  Xyzz<F> acc = Xyzz<F>::inf();
  for (size_t j = lo + threadIdx.x; j < hi; j += BS) acc = add(acc, load_xyzz(in, seg * seg_len + j));
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int h = BS / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) sh[threadIdx.x] = add(sh[threadIdx.x], sh[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) store_xyzz(out, blockIdx.x, sh[0]);
}

template <class F>
hipError_t fbt_msm(Arena& ar, hipStream_t s, const uint32_t* d_table, const uint32_t* d_scalars, const FbGroups& g,
                   Xyzz<F>* d_out) {
  if (!g.groups || !g.sets) return hipSuccess;
  constexpr int BS = sizeof(F) > 48 ? 64 : 128;
  constexpr size_t R = 4;
  const size_t G = g.groups * g.sets;
  size_t len = g.members * 8;
  const size_t np = G * (len ? len : 1);
  ar.reset();
  TPST_TRY(ar.reserve(2 * Arena::need(np, sizeof(Xyzz<F>))));
  Xyzz<F>* a = ar.take<Xyzz<F>>(np);
  Xyzz<F>* b = ar.take<Xyzz<F>>(np);
  if (!len) {
    len = 1;
    TPST_TRY(hipMemsetAsync(a, 0, G * sizeof(Xyzz<F>), s));
  } else {
    k_fbt_partial<F><<<fbt_grid(G * len, 64), 64, 0, s>>>(d_table, d_scalars, g, a);
    TPST_TRY(hipGetLastError());
  }
  while (len > 1) {
    const size_t per = BS * R;
    const size_t parts = (len + per - 1) / per;
    Xyzz<F>* dst = parts == 1 ? d_out : b;
    k_seg_sum<F, BS><<<(unsigned)(G * parts), BS, 0, s>>>(a, len, per, parts, dst);
    TPST_TRY(hipGetLastError());
    if (parts == 1) return hipSuccess;
    len = parts;
    Xyzz<F>* t = a;
    a = b;
    b = t;
  }
  return hipMemcpyAsync(d_out, a, G * sizeof(Xyzz<F>), hipMemcpyDeviceToDevice, s);
}

template hipError_t fbt_build<Fq>(Arena&, hipStream_t, const uint32_t*, size_t, uint32_t*);
template hipError_t fbt_build<Fq2>(Arena&, hipStream_t, const uint32_t*, size_t, uint32_t*);
template hipError_t fbt_msm<Fq>(Arena&, hipStream_t, const uint32_t*, const uint32_t*, const FbGroups&, Xyzz<Fq>*);
template hipError_t fbt_msm<Fq2>(Arena&, hipStream_t, const uint32_t*, const uint32_t*, const FbGroups&, Xyzz<Fq2>*);

}  // namespace tpst
