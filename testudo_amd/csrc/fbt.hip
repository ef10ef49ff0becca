// Fixed-base lookup tables + grouped fixed-base MSM (see fbt.h).
#include "acc_field.h"
#include "coop.h"
#include "fbt.h"
#include "glv.h"
#include <cstdlib>

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

// the same chain on a quad of lanes per base (coop.h): 3 product latencies
// per doubling instead of 9
template <class F>
__global__ void __launch_bounds__(64) k_fbt_pow_quad(const uint32_t* __restrict__ bases, size_t n, int nw,
                                                     Xyzz<F>* __restrict__ tmp) {
  using A = AccField<F>;
  const size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const int qi = threadIdx.x & 3;
  if (k >= n) return;  // quad-uniform
  Xyzz<typename A::T> p = to_xyzz(A::in(load_affine<F>(bases, k)));
  for (int w = 0; w < nw; w++) {
    if (qi == 0) store_acc(tmp, k * nw + w, p);
    if (w + 1 < nw) {
      p = dbl_quad(p, qi);
      p = dbl_quad(p, qi);
      p = dbl_quad(p, qi);
      p = dbl_quad(p, qi);
    }
  }
}

// entries (k, w, 0..7) = (1..8) * tmp[k, w] from one thread: the multiples by
// repeated addition, normalised to affine with ONE inversion (Montgomery's
// batch trick over d_m = ZZ_m ZZZ_m; the multiples are recomputed for the
// output pass instead of being held in registers).  Arithmetic in the
// accumulation field (field29.h for G1: ~1.4x field.h's product rate).
template <class F>
__global__ void __launch_bounds__(64) k_fbt_mult8(const Xyzz<F>* __restrict__ tmp, size_t n, int nw,
                                                  uint32_t* __restrict__ table) {
  using C = typename AccField<F>::T;
  // d_m and the prefix products live in LDS (a lane's column), not in
  // dynamically indexed registers
  __shared__ C sd[FBT_M][64], spre[FBT_M][64];
  const int l = threadIdx.x;
  const size_t i = (size_t)blockIdx.x * blockDim.x + l;
  if (i >= n * (size_t)nw) return;
  const Xyzz<C> P = load_acc(tmp, i);
  Xyzz<C> q = P;
  C pre = C::one();
  for (int j = 0; j < FBT_M; j++) {
    const C d = is_zero(q.ZZ) ? C::one() : mul(q.ZZ, q.ZZZ);
    pre = j ? mul(pre, d) : d;
    sd[j][l] = d;
    spre[j][l] = pre;
    if (j + 1 < FBT_M) q = add(q, P);
  }
  C acc = inv(pre);  // 1 / (d_0 ... d_7)
  for (int j = FBT_M - 1; j >= 0; j--) {
    const C t = j ? mul(acc, spre[j - 1][l]) : acc;  // 1 / d_j
    if (j) acc = mul(acc, sd[j][l]);
    spre[j][l] = t;
  }
  q = P;
  for (int j = 0; j < FBT_M; j++) {
    Affine<F> a = Affine<F>::inf();
    if (!is_zero(q.ZZ)) {
      const C t = spre[j][l];
      const C izz = mul(t, q.ZZZ), izzz = mul(t, q.ZZ);
      a = {to_std(mul(q.X, izz)), to_std(mul(q.Y, izzz))};
    }
    store_affine<F>(table, i * FBT_M + j, a);
    if (j + 1 < FBT_M) q = add(q, P);
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
hipError_t fbt_build(Arena& ar, hipStream_t s, const uint32_t* d_bases, size_t n, uint32_t* d_table, bool glv) {
  if (!n) return hipSuccess;
  ar.reset();
  TPST_TRY(ar.reserve(Arena::need(n * FBT_W, sizeof(Xyzz<F>))));
  Xyzz<F>* tmp = ar.take<Xyzz<F>>(n * FBT_W);
  if constexpr (sizeof(F) == sizeof(Fq)) {  // G1 (timed: the opening's comm_list table)
    const int nw = glv ? FBT_WG : FBT_W;
    k_fbt_pow_quad<F><<<fbt_grid(4 * n, 64), 64, 0, s>>>(d_bases, n, nw, tmp);
    TPST_TRY(hipGetLastError());
    k_fbt_mult8<F><<<fbt_grid(n * nw, 64), 64, 0, s>>>(tmp, n, nw, d_table);
  } else {  // G2 tables are built once per SRS
    if (glv) return hipErrorInvalidValue;
    k_fbt_pow<F><<<fbt_grid(n, 64), 64, 0, s>>>(d_bases, n, tmp);
    TPST_TRY(hipGetLastError());
    k_fbt_mult<F><<<fbt_grid(fbt_entries<F>(n), 64), 64, 0, s>>>(tmp, n, d_table);
  }
  return hipGetLastError();
}

// signed 4-bit digit of window w given the incoming carry
__device__ __forceinline__ int fbt_digit(const uint32_t* s, int w, int& carry) {
  int d = (int)((s[w >> 3] >> ((w & 7) * 4)) & 15u) + carry;
  carry = d > 8;
  return carry ? d - 16 : d;
}

// quad of lanes (coop.h): sum of the lookups of windows [8 ch + j0, 8 ch +
// j0 + nj) of member m of group g in scalar set q
template <class F>
__device__ __forceinline__ Xyzz<typename AccField<F>::T> fbt_lookups(const uint32_t* __restrict__ table,
                                                                      const uint32_t* __restrict__ scal,
                                                                      const FbGroups& gr, size_t q, size_t g, size_t m,
                                                                      int ch, int j0, int nj, int qi) {
  using A = AccField<F>;
  using C = typename A::T;
  size_t k;
  if (gr.d_seg) {
    const size_t lo = gr.d_seg[g], hi = gr.d_seg[g + 1];
    if (m >= hi - lo) return Xyzz<C>::inf();
    k = lo + m;
  } else {
    k = (m / gr.D) * gr.L + g * gr.D + m % gr.D;
  }
  Xyzz<C> acc = Xyzz<C>::inf();
  uint32_t s[8];
  const uint4* sp = reinterpret_cast<const uint4*>(scal + 8 * (k + q * gr.set_stride));
  const uint4 a = sp[0], b = sp[1];
  s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
  s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
  // GLV table: chunks 0-3 take k1's windows from T, chunks 4-7 k2's from
  // phi(T) = (beta x, y)
  int wb = 8 * ch, nw = FBT_W;
  bool phi = false;
  if constexpr (sizeof(F) == sizeof(Fq)) {
    if (gr.glv) {
      uint32_t k1[4], k2[4];
      glv_split(s, k1, k2);
      phi = ch >= 4;
#pragma unroll
      for (int t = 0; t < 4; t++) {
        s[t] = phi ? k2[t] : k1[t];
        s[4 + t] = 0;
      }
      wb = 8 * (ch & 3);
      nw = FBT_WG;
    }
  }
  wb += j0;
  int carry = 0;
  for (int w = 0; w < wb; w++) fbt_digit(s, w, carry);
  // the next lookup is in flight during the current addition; the phi
  // chunks sum the lookups of T and map the sum once (phi(sum T_j) =
  // sum phi(T_j), phi(X, Y, ZZ, ZZZ) = (beta X, Y, ZZ, ZZZ))
  auto look = [&](int w, int d) { return load_affine<F>(table, (k * nw + w) * FBT_M + (d < 0 ? -d : d) - 1); };
  int dn = fbt_digit(s, wb, carry);
  Affine<F> nx;
  if (dn) nx = look(wb, dn);
  for (int j = 0; j < nj; j++) {
    const Affine<F> cur = nx;
    const int d = dn;
    if (j + 1 < nj) {
      dn = fbt_digit(s, wb + j + 1, carry);
      if (dn) nx = look(wb + j + 1, dn);
    }
    if (d) {
      Affine<C> t = A::in(cur);
      if (d < 0) t = neg(t);
      acc = add_affine_quad(acc, t, qi);
    }
  }
  if constexpr (sizeof(F) == sizeof(Fq)) {
    if (phi) acc.X = mul(acc.X, A::in(Affine<F>{Fq::from_limbs(params::G1_BETA), Fq::zero()}).x);
  }
  return acc;
}

// quad of lanes per (group, member, chunk): sum of the 8 lookups of windows
// [8 chunk, 8 chunk + 8)
template <class F>
__global__ void __launch_bounds__(64) k_fbt_partial_quad(const uint32_t* __restrict__ table,
                                                         const uint32_t* __restrict__ scal, FbGroups gr,
                                                         Xyzz<F>* __restrict__ partial) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const int qi = threadIdx.x & 3;
  if (i >= gr.sets * gr.groups * gr.members * 8) return;  // quad-uniform
  const int ch = (int)(i & 7);
  const size_t per_set = gr.groups * gr.members;
  const size_t qgm = i >> 3, q = qgm / per_set, gm = qgm % per_set;
  const size_t g = gm / gr.members, m = gm % gr.members;
  const auto acc = fbt_lookups<F>(table, scal, gr, q, g, m, ch, 0, 8, qi);
  if (qi == 0) store_acc(partial, i, acc);
}

// pairwise tree over the quads [0, n) of a block, n <= the block's quads:
// sh[0] ends with the sum (n > 0)
template <class C>
__device__ __forceinline__ void quad_tree(Xyzz<C>* sh, int n, int quad, int qi) {
  int h = 1;
  while (h < n) h <<= 1;
  for (h >>= 1; h > 0; h >>= 1) {
    if (quad < h && quad + h < n) {
      const Xyzz<C> v = add_quad(sh[quad], sh[quad + h], qi);
      if (qi == 0) sh[quad] = v;
    }
    __syncthreads();
  }
}

// workgroup size: four waves, one per SIMD (two waves per SIMD doubled every
// addition's latency: 2^24 open 24.0 -> 26.8 ms)
template <class F>
constexpr int fbt_block() { return 256; }

// one workgroup per (set, group) of few members: quad u sums the lpq lookups
// of unit u = (member, chunk, sub-chunk), then a tree in LDS -- lpq + log2
// (units) serial additions in one launch instead of 8 + the two-launch
// segmented tree
template <class F>
__global__ void __launch_bounds__(fbt_block<F>()) k_fbt_small_quad(const uint32_t* __restrict__ table,
                                                                   const uint32_t* __restrict__ scal, FbGroups gr,
                                                                   int lpq, Xyzz<F>* __restrict__ out) {
  using C = typename AccField<F>::T;
  __shared__ Xyzz<C> sh[fbt_block<F>() / 4];
  const int quad = threadIdx.x >> 2, qi = threadIdx.x & 3;
  const size_t q = blockIdx.x / gr.groups, g = blockIdx.x % gr.groups;
  const int spc = 8 / lpq;  // units per chunk
  const int units = (int)gr.members * 8 * spc;
  Xyzz<C> acc = Xyzz<C>::inf();
  if (quad < units) {
    const int m = quad / (8 * spc), ch = (quad / spc) & 7, sub = quad % spc;
    acc = fbt_lookups<F>(table, scal, gr, q, g, m, ch, sub * lpq, lpq, qi);
  }
  if (qi == 0) sh[quad] = acc;
  __syncthreads();
  quad_tree(sh, units, quad, qi);
  if (threadIdx.x == 0) store_acc(out, blockIdx.x, sh[0]);
}

// out[seg * parts + part] = sum of in[seg * seg_len + part * per .. + per):
// each quad sums its strided elements, then a tree over the quads in use
template <class F>
__global__ void __launch_bounds__(fbt_block<F>()) k_seg_sum_quad(const Xyzz<F>* __restrict__ in, size_t seg_len,
                                                                 size_t per, size_t parts, Xyzz<F>* __restrict__ out) {
  using C = typename AccField<F>::T;
  constexpr int Q = fbt_block<F>() / 4;
  __shared__ Xyzz<C> sh[Q];
  const int quad = threadIdx.x >> 2, qi = threadIdx.x & 3;
  const size_t seg = blockIdx.x / parts, part = blockIdx.x % parts;
  const size_t lo = part * per, hi = lo + per < seg_len ? lo + per : seg_len;
  Xyzz<C> acc = Xyzz<C>::inf();
  size_t j = lo + quad;
  if (j < hi) {
    acc = load_acc(in, seg * seg_len + j);
    for (j += Q; j < hi; j += Q) acc = add_quad(acc, load_acc(in, seg * seg_len + j), qi);
  }
  if (qi == 0) sh[quad] = acc;
  __syncthreads();
  quad_tree(sh, (int)(hi - lo < (size_t)Q ? hi - lo : (size_t)Q), quad, qi);
  if (threadIdx.x == 0) store_acc(out, blockIdx.x, sh[0]);
}

template <class F>
hipError_t fbt_msm(Arena& ar, hipStream_t s, const uint32_t* d_table, const uint32_t* d_scalars, const FbGroups& g,
                   Xyzz<F>* d_out) {
  if (!g.groups || !g.sets) return hipSuccess;
  constexpr int BS = fbt_block<F>();
  constexpr size_t Q = BS / 4;  // quads per block
  const size_t G = g.groups * g.sets;
  // few members in few groups: one launch (latency-bound shapes; with many
  // groups the tree levels' idle quads cost throughput: 2^24's first h fold,
  // 2048 groups of 2 members, 3.2 ms in one launch; 2^24 open 22.85 -> 22.45
  // ms with the cap, profiles/r06/ab/ab_fbt_small.txt)
  if (!g.d_seg && g.members && g.members * 8 <= Q && G <= 256) {
    int lpq = 1;
    while (g.members * 8 * (8 / lpq) > Q) lpq <<= 1;
    k_fbt_small_quad<F><<<(unsigned)G, BS, 0, s>>>(d_table, d_scalars, g, lpq, d_out);
    return hipGetLastError();
  }
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
    k_fbt_partial_quad<F><<<fbt_grid(4 * G * len, 64), 64, 0, s>>>(d_table, d_scalars, g, a);
    TPST_TRY(hipGetLastError());
  }
  while (len > 1) {
    // four serial additions per quad before the tree, one when a block holds
    // the whole segment
    const size_t per = len <= Q ? Q : 4 * Q;
    const size_t parts = (len + per - 1) / per;
    Xyzz<F>* dst = parts == 1 ? d_out : b;
    k_seg_sum_quad<F><<<(unsigned)(G * parts), BS, 0, s>>>(a, len, per, parts, dst);
    TPST_TRY(hipGetLastError());
    if (parts == 1) return hipSuccess;
    len = parts;
    Xyzz<F>* t = a;
    a = b;
    b = t;
  }
  return hipMemcpyAsync(d_out, a, G * sizeof(Xyzz<F>), hipMemcpyDeviceToDevice, s);
}

template hipError_t fbt_build<Fq>(Arena&, hipStream_t, const uint32_t*, size_t, uint32_t*, bool);
template hipError_t fbt_build<Fq2>(Arena&, hipStream_t, const uint32_t*, size_t, uint32_t*, bool);
template hipError_t fbt_msm<Fq>(Arena&, hipStream_t, const uint32_t*, const uint32_t*, const FbGroups&, Xyzz<Fq>*);
template hipError_t fbt_msm<Fq2>(Arena&, hipStream_t, const uint32_t*, const uint32_t*, const FbGroups&, Xyzz<Fq2>*);

}  // namespace tpst
