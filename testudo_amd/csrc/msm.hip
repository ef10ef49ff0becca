// Pippenger MSM kernels for gfx950 (see msm.h for the pipeline).
#include <cstdlib>
#include <string>
#include "device_util.h"
#include "coop.h"
#include "msm.h"
#include "pair_fq2.h"
#include "glv.h"
#include "acc_field.h"
#include "inv_wave.h"
#include <type_traits>

namespace tpst {

#define TPST_TRY(x)                          \
  do {                                       \
    hipError_t _e = (x);                     \
    if (_e != hipSuccess) return _e;         \
  } while (0)

static inline unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

static inline int bit_length(uint64_t v) {
  int b = 0;
  while (v) {
    b++;
    v >>= 1;
  }
  return b;
}

// signed-digit windows covering `bits` bits: ceil(bits / c) keeps the top
// digit <= 2^(c-1) (bits = 254 for full scalars, 128 for GLV halves)
static inline int num_windows_bits(int c, int bits) { return (bits + c - 1) / c; }
static inline int num_windows(int c) { return num_windows_bits(c, 254); }

// entries per thread in the balanced bucket accumulation: 2^lg with lg the
// largest in [5, 8] that still leaves >= TPST_ACC_WAVES (default 8) waves per
// SIMD.  Long chunks matter for the batch commit, whose buckets (~44 entries
// at 2^24) would otherwise nearly all straddle chunk boundaries.
// SIMDs of the current device (4 per CU on CDNA)
static size_t device_simds() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;  // MI355X
  return (size_t)cus * 4;
}

static int acc_chunk_lg(size_t m) {
  static const size_t threads = (size_t)8 * 64 * device_simds();  // 8 waves of chunks per SIMD
  int lg = 5;
  while (lg < 8 && (m >> (lg + 1)) >= threads) lg++;
  return lg;
}
constexpr int ACC_BLOCK_LG = 6;  // chunks (threads) per accumulation workgroup: one wave
constexpr int ACC_BLOCK = 1 << ACC_BLOCK_LG;

// c-bit window of an nw-word canonical scalar starting at bit `off`
__device__ __forceinline__ uint32_t window_bits(const uint32_t* s, int nw, int off, int c) {
  const int w = off >> 5, b = off & 31;
  const uint64_t lo = (w < nw) ? s[w] : 0u;
  const uint64_t hi = (w + 1 < nw) ? s[w + 1] : 0u;
  return (uint32_t)(((lo | (hi << 32)) >> b) & ((1ull << c) - 1));
}

// signed digit of window w given the running carry (arkworks make_digits,
// except the top window keeps its carry instead of recentering)
__device__ __forceinline__ int signed_digit(const uint32_t* s, int nw, int w, int c, int W, uint32_t& carry) {
  const uint32_t coef = window_bits(s, nw, w * c, c) + carry;
  if (w == W - 1) {
    carry = 0;
    return (int)coef;
  }
  carry = (coef + (1u << (c - 1))) >> c;
  return (int)coef - (int)(carry << c);
}

__device__ __forceinline__ void load_scalar(const uint32_t* p, uint32_t* s) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
  s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
}

// wave issue priority on its SIMD (s_setprio): the latency-bound reduction and
// chain kernels of the window-grouped MSM share SIMDs with accumulation waves
__device__ __forceinline__ void set_wave_prio(int prio) {
  if (prio == 1)
    __builtin_amdgcn_s_setprio(1);
  else if (prio == 2)
    __builtin_amdgcn_s_setprio(2);
  else if (prio >= 3)
    __builtin_amdgcn_s_setprio(3);
}

// ------------------------------------------------------- K2 bucket sort ---
// The decomposed entries (key = window*nb + |digit|-1, val = point index |
// sign<<31; with GLV, index i < n is P_i and n + i is phi(P_i); zero digits
// get the sentinel key nb*W) are grouped by key in two passes, no library sort:
//  * k_decompose_hist writes a tile of scalars' entries window-major and
//    counts them per bin (key >> lo) in LDS -> tab[tile][bin];
//  * k_sort_colscan / k_sort_binscan turn the counts into every tile's slot
//    range inside every bin and the bin starts;
//  * k_sort_scatter moves each tile's entries to its slots of their bins;
//  * k_sort_bin sorts one bin by the low lo key bits in LDS and writes the
//    entries in key order, the bucket bounds [bstart, bend), zeroes (=
//    infinity) the buckets without entries and the window starts range[w].
// Entries of one bucket land in an unspecified order: the bucket sum is a
// group element, so the MSM result does not depend on it.
// Workgroups of at most 256 threads (one wave per SIMD of a CU): a pipelined
// caller's next MSM decomposes and sorts while this one accumulates, and the
// accumulation's 2 waves per SIMD at ~200 VGPRs leave room for one more wave
// of <= 104 VGPRs per SIMD -- a wider workgroup waits for a whole CU to drain.
constexpr int SORT_THREADS = 256;                    // decomposition / scatter workgroup
constexpr uint32_t SORT_MAX_BINS = 16384;            // LDS histogram of a tile
constexpr int SORTB_THREADS = 256;                   // bin-sort workgroup
constexpr int SORTB_IT = 24;                         // entries per thread kept in registers
constexpr int SORTB_CAP = SORTB_THREADS * SORTB_IT;  // largest bin sorted in LDS
constexpr int SORTB_LO_MAX = 10;  // bin-sort LDS: 2^(lo+3) + 4 SORTB_CAP bytes <= 64 KB

struct SortPlan {
  int lo = 0;          // key bits sorted inside a bin
  uint32_t nbins = 0;  // (sent >> lo) + 1: the last bin holds the sentinel
  size_t tile = 0;     // scalars per decomposition tile
  uint32_t ntile = 0;
};

static bool sort_plan(uint32_t sent, size_t n, size_t m, SortPlan& p) {
  p.lo = 1;
  while ((sent >> p.lo) + 1 > SORT_MAX_BINS) p.lo++;
  // fewer, larger bins while a mean bin stays <= CAP/2 (headroom for skewed digits)
  while (p.lo < SORTB_LO_MAX && m / ((size_t)(sent >> (p.lo + 1)) + 1) <= (size_t)SORTB_CAP / 2) p.lo++;
  if (p.lo > SORTB_LO_MAX) return false;
  p.nbins = (sent >> p.lo) + 1;
  p.tile = 2048;
  while ((n + p.tile - 1) / p.tile > 1024) p.tile *= 2;
  p.ntile = (uint32_t)((n + p.tile - 1) / p.tile);
  return true;
}

// phi(P) = (beta x, y), the GLV endomorphism (phi(P) = [x^2 - 1] P on G1).
// On G2 (E'(Fq2), also j = 0) the same beta has eigenvalue lambda^2, so G2
// uses beta^2: (beta^2 x, y) = [x^2 - 1] Q, and one scalar decomposition
// serves both groups.
__constant__ uint32_t G2_GLV_BETA[12] = {0x5a7b8727u, 0x2c766f92u, 0x253d58b5u, 0x03d7f6b0u,
                                         0xec122131u, 0x838ec0deu, 0xf658bb10u, 0xbd5eb3e9u,
                                         0x6ed3e52eu, 0x6942bd12u, 0xdd04ed6au, 0x01673786u};  // Montgomery
template <class F>
__device__ __forceinline__ void glv_phi_point(const uint32_t* __restrict__ bases, size_t i, uint32_t* __restrict__ out) {
  Affine<F> p = load_affine<F>(bases, i);
  if (!is_inf(p)) {
    if constexpr (sizeof(F) == sizeof(Fq)) {
      p.x = mul(p.x, Fq::from_limbs(params::G1_BETA));
    } else {
      const Fq b2 = Fq::from_limbs(G2_GLV_BETA);
      p.x.c0 = mul(p.x.c0, b2);
      p.x.c1 = mul(p.x.c1, b2);
    }
  }
  store_affine(out, i, p);
}

// K2 (G1, GLV) gather records: P_i at index i and phi(P_i) at n + i in the
// accumulation field, fetch_rec29's 128-byte layout (written by the
// decomposition; TPST_K2_REC29=0 builds keep field.h points + phi(P) only)
#ifndef TPST_K2_REC29
#define TPST_K2_REC29 1
#endif
constexpr int REC29_WORDS = 32;
__device__ __forceinline__ void store_rec29(uint32_t* table, size_t idx, const Fq29& x, const Fq29& y) {
  uint32_t rec[REC29_WORDS];
#pragma unroll
  for (int i = 0; i < REC29_WORDS; i++) rec[i] = i < r29::N ? x.v[i] : i < 2 * r29::N ? y.v[i - r29::N] : 0u;
  uint4* dst = reinterpret_cast<uint4*>(table + idx * REC29_WORDS);
#pragma unroll
  for (int i = 0; i < REC29_WORDS / 4; i++) dst[i] = make_uint4(rec[4 * i], rec[4 * i + 1], rec[4 * i + 2], rec[4 * i + 3]);
}
__device__ __forceinline__ void store_rec29(uint32_t* table, size_t idx, const Affine<Fq>& p) {
  store_rec29(table, idx, from_std(p.x), from_std(p.y));
}

// one tile of scalars: signed digits (arkworks make_digits over the GLV
// halves), entries at slot (h W + w) n + i, bin counts, and phi of the bases
// (or, rec != nullptr, the gather records of P and phi(P))
template <class F>
static __global__ void __launch_bounds__(SORT_THREADS)
    k_decompose_hist(const uint32_t* __restrict__ scalars, size_t n, int c, int W, int glv, uint32_t sent, int lo,
                     uint32_t nbins, size_t tile, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                     uint32_t* __restrict__ tab, const uint32_t* __restrict__ bases, uint32_t* __restrict__ phib,
                     uint32_t* __restrict__ rec) {
  extern __shared__ uint32_t hist[];
  for (uint32_t b = threadIdx.x; b < nbins; b += SORT_THREADS) hist[b] = 0;
  __syncthreads();
  const uint32_t nb = 1u << (c - 1);
  const size_t i0 = (size_t)blockIdx.x * tile;
  const size_t i1 = (i0 + tile < n) ? i0 + tile : n;
  for (size_t i = i0 + threadIdx.x; i < i1; i += SORT_THREADS) {
    uint32_t s[8];
    load_scalar(scalars + 8 * i, s);
    const int halves = glv ? 2 : 1;
    uint32_t parts[2][4];
    if (glv) glv_split(s, parts[0], parts[1]);
    for (int h = 0; h < halves; h++) {
      const uint32_t* sc = glv ? parts[h] : s;
      const int nw = glv ? 4 : 8;
      const uint32_t idx = (uint32_t)(h * n + i);
      uint32_t carry = 0;
      for (int w = 0; w < W; w++) {
        const int d = signed_digit(sc, nw, w, c, W, carry);
        uint32_t key = sent, val = 0;
        if (d != 0) {
          key = (uint32_t)w * nb + (uint32_t)(abs(d) - 1);
          val = idx | (d < 0 ? 0x80000000u : 0u);
        }
        const size_t slot = ((size_t)h * W + w) * n + i;
        keys[slot] = key;
        vals[slot] = val;
        atomicAdd(&hist[key >> lo], 1u);
      }
    }
    if constexpr (sizeof(F) == sizeof(Fq)) {
      if (rec) {  // P and phi(P) = (beta x, y) in the accumulation field (infinity: x = y = 0 both)
        const Affine<Fq> p = load_affine<Fq>(bases, i);
        const Fq29 x = from_std(p.x), y = from_std(p.y);
        store_rec29(rec, i, x, y);
        store_rec29(rec, n + i, mul(x, from_std(Fq::from_limbs(params::G1_BETA))), y);
        continue;
      }
    }
    if (glv) glv_phi_point<F>(bases, i, phib);
  }
  __syncthreads();
  uint32_t* row = tab + (size_t)blockIdx.x * nbins;
  for (uint32_t b = threadIdx.x; b < nbins; b += SORT_THREADS) row[b] = hist[b];
}

// per bin: exclusive scan of the tiles' counts (in place: tab[t][bin] becomes
// tile t's first slot inside the bin) and the bin total.  64 bins x
// COLSCAN_CH tile chunks per workgroup.
constexpr int COLSCAN_CH = 4;
static __global__ void __launch_bounds__(64 * COLSCAN_CH) k_sort_colscan(uint32_t* __restrict__ tab, uint32_t ntile,
                                                                         uint32_t nbins, uint32_t* __restrict__ tot) {
  __shared__ uint32_t part[COLSCAN_CH][64];
  const uint32_t lane = threadIdx.x & 63, ch = threadIdx.x >> 6;
  const uint32_t bin = blockIdx.x * 64 + lane;
  const uint32_t per = (ntile + COLSCAN_CH - 1) / COLSCAN_CH;
  const uint32_t t0 = (ch * per < ntile) ? ch * per : ntile;
  const uint32_t t1 = (t0 + per < ntile) ? t0 + per : ntile;
  uint32_t sum = 0;
  if (bin < nbins)
    for (uint32_t t = t0; t < t1; t++) sum += tab[(size_t)t * nbins + bin];
  part[ch][lane] = sum;
  __syncthreads();
  if (ch == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < COLSCAN_CH; k++) {
      const uint32_t v = part[k][lane];
      part[k][lane] = acc;
      acc += v;
    }
    if (bin < nbins) tot[bin] = acc;
  }
  __syncthreads();
  if (bin < nbins) {
    uint32_t acc = part[ch][lane];
    for (uint32_t t = t0; t < t1; t++) {
      const size_t o = (size_t)t * nbins + bin;
      const uint32_t v = tab[o];
      tab[o] = acc;
      acc += v;
    }
  }
}

// start[b] = sum of the totals of bins < b, start[nbins] = entry count (one workgroup)
constexpr int BINSCAN_THREADS = 256;
static __global__ void __launch_bounds__(BINSCAN_THREADS) k_sort_binscan(const uint32_t* __restrict__ tot,
                                                                         uint32_t nbins, uint32_t* __restrict__ start) {
  __shared__ uint32_t ws[BINSCAN_THREADS];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nbins + BINSCAN_THREADS - 1) / BINSCAN_THREADS;
  const uint32_t b0 = t * per;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; k++)
    if (b0 + k < nbins) sum += tot[b0 + k];
  ws[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < BINSCAN_THREADS; off <<= 1) {
    const uint32_t v = t >= off ? ws[t - off] : 0u;
    __syncthreads();
    ws[t] += v;
    __syncthreads();
  }
  uint32_t acc = ws[t] - sum;
  for (uint32_t k = 0; k < per; k++)
    if (b0 + k < nbins) {
      start[b0 + k] = acc;
      acc += tot[b0 + k];
    }
  if (t == BINSCAN_THREADS - 1) start[nbins] = ws[BINSCAN_THREADS - 1];
}

// tile -> bins: each entry takes the next slot of its bin from the tile's
// cursors in LDS (reads coalesced; writes in runs of the tile's entries per bin)
static __global__ void __launch_bounds__(SORT_THREADS)
    k_sort_scatter(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, size_t n, uint32_t segs,
                   int lo, uint32_t nbins, size_t tile, const uint32_t* __restrict__ tab,
                   const uint32_t* __restrict__ start, uint32_t* __restrict__ keys2, uint32_t* __restrict__ vals2) {
  extern __shared__ uint32_t cur[];
  const uint32_t* row = tab + (size_t)blockIdx.x * nbins;
  for (uint32_t b = threadIdx.x; b < nbins; b += SORT_THREADS) cur[b] = start[b] + row[b];
  __syncthreads();
  const size_t i0 = (size_t)blockIdx.x * tile;
  const uint32_t cnt = (uint32_t)((i0 + tile < n) ? tile : n - i0);
  const uint32_t total = segs * cnt;
  constexpr int U = 4;
  for (uint32_t q0 = 0; q0 < total; q0 += U * SORT_THREADS) {
    uint32_t k[U], v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t q = q0 + u * SORT_THREADS + threadIdx.x;
      if (q < total) {
        const uint32_t sg = q / cnt;
        const size_t slot = (size_t)sg * n + i0 + (q - sg * cnt);
        k[u] = keys[slot];
        v[u] = vals[slot];
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t q = q0 + u * SORT_THREADS + threadIdx.x;
      if (q < total) {
        const uint32_t pos = atomicAdd(&cur[k[u] >> lo], 1u);
        keys2[pos] = k[u];
        vals2[pos] = v[u];
      }
    }
  }
}

// exclusive prefix sums of a[0, len) into o (may alias a) by NT threads:
// per-thread runs, wave scan, wave totals; returns the total
template <int NT>
__device__ uint32_t block_scan_excl(const uint32_t* a, uint32_t* o, uint32_t len, uint32_t* wsum) {
  const uint32_t t = threadIdx.x;
  const uint32_t per = (len + NT - 1) / NT, d0 = t * per;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; k++)
    if (d0 + k < len) sum += a[d0 + k];
  uint32_t incl = sum;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const uint32_t v = __shfl_up(incl, s, 64);
    if ((t & 63) >= (uint32_t)s) incl += v;
  }
  if ((t & 63) == 63) wsum[t >> 6] = incl;
  __syncthreads();
  uint32_t acc = incl - sum, total = 0;
  for (uint32_t w = 0; w < NT / 64; w++) {
    if (w < (t >> 6)) acc += wsum[w];
    total += wsum[w];
  }
  for (uint32_t k = 0; k < per; k++)
    if (d0 + k < len) {
      const uint32_t v = a[d0 + k];
      o[d0 + k] = acc;
      acc += v;
    }
  __syncthreads();
  return total;
}

// k_sort_scatter with the tile staged per window through LDS (bins aligned to
// windows: lo <= c - 1): the tile's entries of window w (both GLV halves)
// are ordered by bin in LDS, then written out in per-bin runs, so a wave's
// store covers a few runs instead of 64 scattered words
template <int E>
static __global__ void __launch_bounds__(SORT_THREADS)
    k_sort_scatter_win(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, size_t n, int halves,
                       int W, uint32_t sent, int lo, uint32_t nbins, uint32_t bpw, size_t tile,
                       const uint32_t* __restrict__ tab, const uint32_t* __restrict__ start,
                       uint32_t* __restrict__ keys2, uint32_t* __restrict__ vals2) {
  extern __shared__ uint32_t sm[];
  __shared__ uint32_t wsum[SORT_THREADS / 64];
  uint32_t* cur = sm;              // global cursor of every bin
  uint32_t* lc = cur + nbins;      // the window's bins + the sentinel bin: counts
  uint32_t* lo_ = lc + bpw + 1;    //   and their first staged slot
  uint32_t* sk = lo_ + bpw + 1;    // staged keys / values
  uint32_t* sv = sk + (size_t)E * SORT_THREADS;
  const uint32_t t = threadIdx.x;
  const uint32_t* row = tab + (size_t)blockIdx.x * nbins;
  for (uint32_t b = t; b < nbins; b += SORT_THREADS) cur[b] = start[b] + row[b];
  const size_t sub = (size_t)E * SORT_THREADS / halves;
  const size_t t0 = (size_t)blockIdx.x * tile, t1 = (t0 + tile < n) ? t0 + tile : n;
  for (size_t i0 = t0; i0 < t1; i0 += sub)  // sub-tiles append at the tile's cursors
  for (int w = 0; w < W; w++) {
    const uint32_t cnt = (uint32_t)((i0 + sub < t1) ? sub : t1 - i0);
    const uint32_t tot = (uint32_t)halves * cnt;
    const uint32_t wb = (uint32_t)w * bpw;
    for (uint32_t j = t; j <= bpw; j += SORT_THREADS) lc[j] = 0;
    __syncthreads();
    uint32_t k[E], v[E], r[E];
#pragma unroll
    for (int u = 0; u < E; u++) {
      const uint32_t q = u * SORT_THREADS + t;
      if (q < tot) {
        const uint32_t h = q >= cnt ? 1u : 0u;
        const size_t slot = ((size_t)h * W + w) * n + i0 + (q - h * cnt);
        k[u] = keys[slot];
        v[u] = vals[slot];
      }
    }
#pragma unroll
    for (int u = 0; u < E; u++)
      if (u * SORT_THREADS + t < tot) r[u] = atomicAdd(&lc[k[u] >= sent ? bpw : (k[u] >> lo) - wb], 1u);
    __syncthreads();
    block_scan_excl<SORT_THREADS>(lc, lo_, bpw + 1, wsum);
#pragma unroll
    for (int u = 0; u < E; u++)
      if (u * SORT_THREADS + t < tot) {
        const uint32_t p = lo_[k[u] >= sent ? bpw : (k[u] >> lo) - wb] + r[u];
        sk[p] = k[u];
        sv[p] = v[u];
      }
    __syncthreads();
    for (uint32_t p = t; p < tot; p += SORT_THREADS) {
      const uint32_t key = sk[p];
      const bool z = key >= sent;
      const uint32_t lb = z ? bpw : (key >> lo) - wb;
      const uint32_t pos = cur[z ? nbins - 1 : key >> lo] + (p - lo_[lb]);
      keys2[pos] = key;
      vals2[pos] = sv[p];
    }
    __syncthreads();
    for (uint32_t j = t; j <= bpw; j += SORT_THREADS) cur[j == bpw ? nbins - 1 : wb + j] += lc[j];
    __syncthreads();
  }
}

// one bin: counting sort by the low lo key bits.  A bin of <= SORTB_CAP
// entries is staged in registers + LDS and written out contiguously; a larger
// one (skewed digits) scatters straight to its slots.
static __global__ void __launch_bounds__(SORTB_THREADS)
    k_sort_bin(const uint32_t* __restrict__ keys2, const uint32_t* __restrict__ vals2,
               const uint32_t* __restrict__ start, int lo, uint32_t sent, uint32_t nb, int W,
               uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t* __restrict__ bstart,
               uint32_t* __restrict__ bend, uint4* __restrict__ buckets, uint32_t bucket_u4,
               uint32_t* __restrict__ range) {
  extern __shared__ uint32_t sm[];
  __shared__ uint32_t wsum[SORTB_THREADS / 64];
  const uint32_t D = 1u << lo, mask = D - 1;
  uint32_t* off = sm;           // bucket offsets inside the bin (counts first)
  uint32_t* cur = sm + D;       // placement cursors
  uint32_t* sval = sm + 2 * D;  // staged values
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  const uint32_t s = start[b], len = start[b + 1] - s;
  if ((b << lo) >= sent) {
    // the sentinel bin (zero digits; sent = W nb is a multiple of 2^lo when
    // lo <= c - 1): nothing reads entries past range[W] -- the short chunks
    // stop at range[whi], the long-chunk pass at range[W] -- so a bin that can
    // hold most of m entries (small or boolean scalars) costs nothing here
    if (t == 0 && (b << lo) == sent) range[W] = s;
    return;
  }
  for (uint32_t d = t; d < D; d += SORTB_THREADS) off[d] = 0;
  __syncthreads();
  const bool fits = len <= (uint32_t)SORTB_CAP;
  uint32_t kk[SORTB_IT], vv[SORTB_IT];
  // sentinel entries of a mixed last bin (lo > c - 1: small MSMs) are not
  // counted: they fill the bin's tail [nz, len) after the sorted entries
  if (fits) {
#pragma unroll
    for (int k = 0; k < SORTB_IT; k++) {
      const uint32_t p = k * SORTB_THREADS + t;
      if (p < len) {
        kk[k] = keys2[s + p];
        vv[k] = vals2[s + p];
      }
    }
#pragma unroll
    for (int k = 0; k < SORTB_IT; k++)
      if (k * SORTB_THREADS + t < len && kk[k] < sent) atomicAdd(&off[kk[k] & mask], 1u);
  } else {
    for (uint32_t p = t; p < len; p += SORTB_THREADS) {
      const uint32_t key = keys2[s + p];
      if (key < sent) atomicAdd(&off[key & mask], 1u);
    }
  }
  __syncthreads();
  // exclusive scan of the counts: per-thread runs, wave scan, wave totals
  const uint32_t per = (D + SORTB_THREADS - 1) / SORTB_THREADS;
  const uint32_t d0 = t * per;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; k++)
    if (d0 + k < D) sum += off[d0 + k];
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if ((t & 63) >= (uint32_t)o) incl += v;
  }
  if ((t & 63) == 63) wsum[t >> 6] = incl;
  __syncthreads();
  uint32_t acc = incl - sum, nz = 0;
  for (uint32_t w = 0; w < SORTB_THREADS / 64; w++) {
    if (w < (t >> 6)) acc += wsum[w];
    nz += wsum[w];  // entries with a bucket key
  }
  for (uint32_t k = 0; k < per; k++) {
    const uint32_t d = d0 + k;
    if (d >= D) break;
    const uint32_t cn = off[d];
    cur[d] = acc;
    const uint32_t key = (b << lo) | d;
    if (key < sent) {
      bstart[key] = s + acc;
      bend[key] = s + acc + cn;
      if (cn == 0 && buckets)
        for (uint32_t u = 0; u < bucket_u4; u++) buckets[(size_t)key * bucket_u4 + u] = make_uint4(0, 0, 0, 0);
    }
    acc += cn;
  }
  __syncthreads();
  for (uint32_t d = t; d < D; d += SORTB_THREADS) off[d] = cur[d];
  if (t <= (uint32_t)W) {
    const uint32_t target = t * nb;  // first key of window t (t = W: the sentinel)
    if ((target >> lo) == b) range[t] = s + cur[target & mask];
  }
  __syncthreads();
  if (fits) {
#pragma unroll
    for (int k = 0; k < SORTB_IT; k++)
      if (k * SORTB_THREADS + t < len && kk[k] < sent) sval[atomicAdd(&cur[kk[k] & mask], 1u)] = vv[k];
    __syncthreads();
    for (uint32_t p = t; p < nz; p += SORTB_THREADS) {
      uint32_t a = 0, z = D;  // first bucket offset > p
      while (a < z) {
        const uint32_t mid = (a + z) >> 1;
        if (off[mid] <= p)
          a = mid + 1;
        else
          z = mid;
      }
      keys[s + p] = (b << lo) | (a - 1);
      vals[s + p] = sval[p];
    }
  } else {
    for (uint32_t p = t; p < len; p += SORTB_THREADS) {
      const uint32_t key = keys2[s + p];
      if (key >= sent) continue;
      const uint32_t pos = s + atomicAdd(&cur[key & mask], 1u);
      keys[pos] = key;
      vals[pos] = vals2[s + p];
    }
  }
  for (uint32_t p = nz + t; p < len; p += SORTB_THREADS) keys[s + p] = sent;
}

// K1 window-table record (msm_batch): one affine point already in the
// accumulation field (field29.h radix 2^29, canonical), x (13 words) | y
// (13 words) | 6 pad words = 128 bytes, so a gather is ONE aligned 128-byte
// line (a 96-byte field.h point straddles two lines 3 times in 4) and needs
// no conversion in the accumulation loop
__device__ __forceinline__ Affine<Fq29> fetch_rec29(const uint32_t* table, uint32_t v) {
  const uint4* r = reinterpret_cast<const uint4*>(table + (size_t)(v & 0x7fffffffu) * REC29_WORDS);
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 7; i++) {
    const uint4 q = r[i];
    w[4 * i] = q.x;
    w[4 * i + 1] = q.y;
    w[4 * i + 2] = q.z;
    w[4 * i + 3] = q.w;
  }
  Affine<Fq29> p;
#pragma unroll
  for (int i = 0; i < r29::N; i++) {
    p.x.v[i] = w[i];
    p.y.v[i] = w[r29::N + i];
  }
  p.y = cneg(p.y, (v >> 31) != 0);
  return p;
}

template <class F>
__device__ __forceinline__ Affine<F> fetch_point(const uint32_t* bases, const uint32_t* phib, uint32_t nbase,
                                                uint32_t v) {
  const uint32_t idx = v & 0x7fffffffu;
  Affine<F> p = (idx < nbase) ? load_affine<F>(bases, idx) : load_affine<F>(phib, idx - nbase);
  if (v >> 31) p.y = neg(p.y);
  return p;
}

// Balanced bucket accumulation over the key-sorted entries: thread t owns the
// chunk of entries [t 2^lg, (t+1) 2^lg).  A bucket lying wholly inside the
// chunk is stored directly.  A bucket crossing chunk boundaries is finished by
// its owner (the chunk holding its first entry): the owner keeps its tail
// piece in registers while every later chunk parks its leading piece in
// part[t]; after the workgroup barrier the owner adds the pieces of the
// following chunks of its workgroup (still in L2) and stores the bucket.  Only
// the bucket crossing the workgroup's last chunk is left to k_bucket_fixup
// (its owner's partial goes to bpart[workgroup]), so the fixup runs one thread
// per workgroup instead of one per bucket.  The next point is loaded before
// the current mixed add runs (software prefetch).
// REC29: `bases` is a K1 window table of fetch_rec29 records (Fq only)
template <class F, int MINW = (sizeof(F) > 48 ? 1 : 2), bool REC29 = false>
__global__ void __launch_bounds__(ACC_BLOCK, MINW)
    k_bucket_acc_chunk(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, size_t m_all,
                       const uint32_t* __restrict__ mend, uint32_t sent, const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bend,
                       const uint32_t* __restrict__ bases, const uint32_t* __restrict__ phib, uint32_t nbase,
                       int lg, Xyzz<F>* __restrict__ buckets, Xyzz<F>* __restrict__ part,
                       Xyzz<F>* __restrict__ bpart) {
  const size_t t = (size_t)blockIdx.x * ACC_BLOCK + threadIdx.x;
  const size_t c0 = t << lg;
  // entries with a bucket key: range[W] for msm_var (its sentinel tail is never sorted)
  const size_t m = mend ? (size_t)*mend : m_all;
  using A = AccField<F>;
  using C = typename A::T;
  // the chunk's last segment, when its bucket continues past the chunk, is
  // left in acc at the loop's end (no second accumulator live in the loop)
  uint32_t tail_key = sent;
  Xyzz<C> acc = Xyzz<C>::inf();
  if (c0 < m) {
    const size_t c1 = (c0 + ((size_t)1 << lg) < m) ? c0 + ((size_t)1 << lg) : m;
    auto fetch = [&](uint32_t v) -> Affine<C> {
      if constexpr (REC29)
        return fetch_rec29(bases, v);
      else
        return A::in(fetch_point<F>(bases, phib, nbase, v));
    };
    uint32_t key = keys[c0];
    Affine<C> pt;
    if (key < sent) pt = fetch(vals[c0]);
    for (size_t e = c0; e < c1; e++) {
      uint32_t key_n = sent;
      Affine<C> pt_n;
      if (e + 1 < c1) {
        key_n = keys[e + 1];
        if (key_n < sent) pt_n = fetch(vals[e + 1]);
      }
      if (key < sent) {
        acc = add_affine(acc, pt);
        if (key_n != key) {
          if (bend[key] <= c1) {  // the bucket ends in this chunk
            // began here: complete; began earlier: the chunk's first segment
            if (bstart[key] >= c0)
              store_pk(buckets, key, acc);
            else
              store_pk(part, t, acc);
            acc = Xyzz<C>::inf();
          } else {  // continues: the chunk's last segment (e + 1 == c1)
            tail_key = key;
          }
        }
      }
      key = key_n;
      pt = pt_n;
    }
    if (tail_key < sent && bstart[tail_key] < c0) {  // spans the whole chunk
      store_pk(part, t, acc);
      tail_key = sent;
    }
  }
  __threadfence_block();
  __syncthreads();
  if (tail_key >= sent) return;
  const size_t t1 = ((size_t)bend[tail_key] - 1) >> lg;  // chunk of the bucket's last entry
  const size_t tb = (size_t)blockIdx.x * ACC_BLOCK + (ACC_BLOCK - 1);
  const size_t stop = t1 < tb ? t1 : tb;
  for (size_t u = t + 1; u <= stop; u++) acc = add(acc, load_pk(part, u));
  if (t1 <= tb)
    store_pk(buckets, tail_key, acc);
  else
    store_pk(bpart, blockIdx.x, acc);
}

// k_bucket_acc_chunk over K1's record table (REC29) with the next record
// staged through LDS, as k_bucket_acc_short_lds: seven global_load_lds_dwordx4
// per step land lane i's 16-byte pieces at stage[buf][j][i] while the current
// mixed add runs; the loop runs to the wave's longest chunk (every lane
// issues every staging load), then the same tail / owner walk
#ifndef TPST_K1_NBUF
#define TPST_K1_NBUF 2
#endif
#ifndef TPST_K1_MINW
#define TPST_K1_MINW 2
#endif
template <int MINW>
__global__ void __launch_bounds__(ACC_BLOCK, MINW)
    k_bucket_acc_chunk_lds(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, size_t m_all,
                           const uint32_t* __restrict__ mend, uint32_t sent, const uint32_t* __restrict__ bstart,
                           const uint32_t* __restrict__ bend, const uint32_t* __restrict__ table, int lg,
                           Xyzz<Fq>* __restrict__ buckets, Xyzz<Fq>* __restrict__ part,
                           Xyzz<Fq>* __restrict__ bpart) {
  constexpr int NP = 7;  // the first 112 bytes of a 128-byte record
  constexpr int NBUF = TPST_K1_NBUF;  // 1: refilled once the current record's ds_reads returned
  __shared__ uint4 stage[NBUF][NP][ACC_BLOCK];
  using A = AccField<Fq>;
  using C = typename A::T;
  const int lane = threadIdx.x;
  const size_t t = (size_t)blockIdx.x * ACC_BLOCK + lane;
  const size_t c0 = t << lg;
  const size_t m = mend ? (size_t)*mend : m_all;
  if ((((size_t)blockIdx.x * ACC_BLOCK) << lg) >= m) return;  // the whole workgroup (one wave) idle
  const bool active = c0 < m;
  const size_t c1 = active ? ((c0 + ((size_t)1 << lg) < m) ? c0 + ((size_t)1 << lg) : m) : c0;
  auto stage_load = [&](int buf, uint32_t v, bool want) {
    const uint32_t* src = want ? table + (size_t)REC29_WORDS * (v & 0x7fffffffu) : table;
#pragma unroll
    for (int j = 0; j < NP; j++)
      __builtin_amdgcn_global_load_lds((const void*)(src + 4 * j),
                                       (__attribute__((address_space(3))) void*)&stage[buf][j][0], 16, 0, 0);
  };
  auto stage_read = [&](int buf, uint32_t v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t w[4 * NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
      const uint4 q = stage[buf][j][lane];
      w[4 * j] = q.x;
      w[4 * j + 1] = q.y;
      w[4 * j + 2] = q.z;
      w[4 * j + 3] = q.w;
    }
    Affine<C> p;
#pragma unroll
    for (int i = 0; i < r29::N; i++) {
      p.x.v[i] = w[i];
      p.y.v[i] = w[r29::N + i];
    }
    p.y = cneg(p.y, (v >> 31) != 0);
    return p;
  };
  uint32_t tail_key = sent;
  Xyzz<C> acc = Xyzz<C>::inf();
  uint32_t key = active ? keys[c0] : sent;
  uint32_t val = active && key < sent ? vals[c0] : 0u;
  stage_load(0, val, key < sent);
  const size_t steps = c1 - c0;
  const size_t maxsteps = (size_t)1 << lg;
  for (size_t s = 0; s < maxsteps; s++) {
    const size_t e = c0 + s;
    const bool live = s < steps;
    uint32_t key_n = sent, val_n = 0;
    if (s + 1 < steps) {
      key_n = keys[e + 1];
      if (key_n < sent) val_n = vals[e + 1];
    }
    const Affine<C> pt = stage_read(NBUF == 1 ? 0 : (int)(s & 1), val);
    if constexpr (NBUF == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // pt read out of the buffer
    stage_load(NBUF == 1 ? 0 : (int)((s + 1) & 1), val_n, key_n < sent);
    if (live && key < sent) {
      acc = add_affine(acc, pt);
      if (key_n != key) {
        if (bend[key] <= c1) {  // the bucket ends in this chunk
          if (bstart[key] >= c0)
            store_pk(buckets, key, acc);
          else
            store_pk(part, t, acc);
          acc = Xyzz<C>::inf();
        } else {  // continues: the chunk's last segment
          tail_key = key;
        }
      }
    }
    key = key_n;
    val = val_n;
    if (__all(s + 1 >= steps ? 1 : 0)) break;  // wave-uniform exit
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no staging load outstanding
  if (tail_key < sent && bstart[tail_key] < c0) {  // spans the whole chunk
    store_pk(part, t, acc);
    tail_key = sent;
  }
  __threadfence_block();
  __syncthreads();
  if (tail_key >= sent) return;
  const size_t t1 = ((size_t)bend[tail_key] - 1) >> lg;  // chunk of the bucket's last entry
  const size_t tb = (size_t)blockIdx.x * ACC_BLOCK + (ACC_BLOCK - 1);
  const size_t stop = t1 < tb ? t1 : tb;
  for (size_t u = t + 1; u <= stop; u++) acc = add(acc, load_pk(part, u));
  if (t1 <= tb)
    store_pk(buckets, tail_key, acc);
  else
    store_pk(bpart, blockIdx.x, acc);
}

// buckets crossing a workgroup boundary: thread B finishes the bucket holding
// workgroup B's last entry when that bucket began in B -- its owner's partial
// plus the leading pieces of the chunks after B up to the bucket's last one
template <class F>
__global__ void __launch_bounds__(64, (sizeof(F) > 48 ? 1 : 2))
    k_bucket_fixup(const uint32_t* __restrict__ keys, size_t m_all, const uint32_t* __restrict__ mend, uint32_t sent,
                   const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bend, int lg, size_t nblk,
                   const Xyzz<F>* __restrict__ part, const Xyzz<F>* __restrict__ bpart,
                   Xyzz<F>* __restrict__ buckets) {
  using C = typename AccField<F>::T;
  const size_t B = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (B + 1 >= nblk) return;
  const int lb = lg + ACC_BLOCK_LG;
  const size_t e = (B + 1) << lb;  // first entry of workgroup B + 1
  if (e >= (mend ? (size_t)*mend : m_all)) return;
  const uint32_t key = keys[e];
  if (key >= sent || keys[e - 1] != key || ((size_t)bstart[key] >> lb) != B) return;
  const size_t t1 = ((size_t)bend[key] - 1) >> lg;
  Xyzz<C> acc = load_pk(bpart, B);
  for (size_t u = (B + 1) << ACC_BLOCK_LG; u <= t1; u++) acc = add(acc, load_pk(part, u));
  store_pk(buckets, key, acc);
}

// Short-chunk accumulation for the variable-base MSM (32-entry chunks over
// ~64-entry buckets): no in-workgroup owner walk (it costs registers and a
// barrier that the short chunks do not amortise); every piece of a bucket
// that crosses a chunk boundary is parked -- the chunk's trailing piece in
// part[2t + 1], its leading piece in part[2t] -- and k_bucket_fixup_short
// sums them per bucket.  One launch covers the entries of windows [wlo, whi)
// (range[w] = first sorted entry of window w, device-side): chunk indices stay
// global (t = entry >> lg) so a chunk straddling two window groups is split
// between their launches without sharing a part[] slot.
template <class F, int MINW = (sizeof(F) > 48 ? 1 : 2), bool REC29 = false>
__global__ void __launch_bounds__(64, MINW)
    k_bucket_acc_short(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                       const uint32_t* __restrict__ range, int wlo, int whi, uint32_t sent,
                       const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bend,
                       const uint32_t* __restrict__ bases, const uint32_t* __restrict__ phib, uint32_t nbase,
                       int lg, Xyzz<F>* __restrict__ buckets, Xyzz<F>* __restrict__ part) {
  const size_t e_lo = range[wlo], e_hi = range[whi];
  const size_t t = (e_lo >> lg) + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t c0 = t << lg;
  if (c0 >= e_hi) return;
  const size_t c1 = (c0 + ((size_t)1 << lg) < e_hi) ? c0 + ((size_t)1 << lg) : e_hi;
  if (c0 < e_lo) c0 = e_lo;
  using A = AccField<F>;
  using C = typename A::T;
  auto fetch = [&](uint32_t v) -> Affine<C> {
    if constexpr (REC29)
      return fetch_rec29(bases, v);
    else
      return A::in(fetch_point<F>(bases, phib, nbase, v));
  };
  uint32_t key = keys[c0];
  Affine<C> pt;
  if (key < sent) pt = fetch(vals[c0]);
  Xyzz<C> acc = Xyzz<C>::inf();
  for (size_t e = c0; e < c1; e++) {
    uint32_t key_n = sent;
    Affine<C> pt_n;
    if (e + 1 < c1) {
      key_n = keys[e + 1];
      if (key_n < sent) pt_n = fetch(vals[e + 1]);
    }
    if (key < sent) {
      acc = add_affine(acc, pt);
      if (key_n != key) {
        const bool starts = bstart[key] >= c0;
        const bool ends = bend[key] <= c1;
        if (starts && ends)
          store_pk(buckets, key, acc);
        else
          store_pk(part, 2 * t + (starts ? 1 : 0), acc);
        acc = Xyzz<C>::inf();
      }
    }
    key = key_n;
    pt = pt_n;
  }
}

// k_bucket_acc_short<Fq> with the next point staged through LDS instead of
// registers: the wave issues six global_load_lds_dwordx4 for the 64 lanes'
// next points (lane i's 16-byte piece j lands at stage[buf][j][i]; no VGPR
// destination), runs the current mixed add meanwhile, and reads the staged
// point back with six ds_read_b128.  Frees the prefetched point's VGPRs
// (occupancy) and moves the gathers off the register file.  The default for
// G1 (TPST_ACC_LDS=0: k_bucket_acc_short's register prefetch).
#ifndef TPST_K2_NBUF
#define TPST_K2_NBUF 2
#endif
#ifndef TPST_K2_MINW
#define TPST_K2_MINW 2  // waves per SIMD the register allocation targets (G1 records)
#endif
template <int MINW, bool REC29>
__global__ void __launch_bounds__(64, MINW)
    k_bucket_acc_short_lds(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                           const uint32_t* __restrict__ range, int wlo, int whi, uint32_t sent,
                           const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bend,
                           const uint32_t* __restrict__ bases, const uint32_t* __restrict__ phib, uint32_t nbase,
                           int lg, Xyzz<Fq>* __restrict__ buckets, Xyzz<Fq>* __restrict__ part) {
  // double-buffered points, piece-major: 96-byte field.h points or the
  // first 112 bytes of a 128-byte record (REC29)
  constexpr int NP = REC29 ? 7 : 6;
  // NBUF = 1: one staging buffer, refilled once the current point's ds_reads
  // have returned (half the LDS per wave)
  constexpr int NBUF = TPST_K2_NBUF;
  __shared__ uint4 stage[NBUF][NP][64];
  using A = AccField<Fq>;
  using C = typename A::T;
  const int lane = threadIdx.x;
  const size_t e_lo = range[wlo], e_hi = range[whi];
  const size_t t = (e_lo >> lg) + (size_t)blockIdx.x * blockDim.x + lane;
  size_t c0 = t << lg;
  if ((e_lo >> lg) + (size_t)blockIdx.x * blockDim.x >= e_hi) return;  // wave-uniform: no lane has work
  const bool active = c0 < e_hi;
  const size_t c1 = active ? ((c0 + ((size_t)1 << lg) < e_hi) ? c0 + ((size_t)1 << lg) : e_hi) : c0;
  if (c0 < e_lo) c0 = e_lo;
  // every lane issues every staging load (the instruction is wave-wide);
  // lanes without a point load bases[0]
  auto stage_load = [&](int buf, uint32_t v, bool want) {
    const uint32_t idx = v & 0x7fffffffu;
    const uint32_t* src = !want ? bases
                          : REC29 ? bases + (size_t)REC29_WORDS * idx
                                  : ((idx < nbase) ? bases + 24 * (size_t)idx : phib + 24 * (size_t)(idx - nbase));
#pragma unroll
    for (int j = 0; j < NP; j++)
      __builtin_amdgcn_global_load_lds((const void*)(src + 4 * j),
                                       (__attribute__((address_space(3))) void*)&stage[buf][j][0], 16, 0, 0);
  };
  auto stage_read = [&](int buf, uint32_t v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t w[4 * NP];
#pragma unroll
    for (int j = 0; j < NP; j++) {
      const uint4 q = stage[buf][j][lane];
      w[4 * j] = q.x;
      w[4 * j + 1] = q.y;
      w[4 * j + 2] = q.z;
      w[4 * j + 3] = q.w;
    }
    if constexpr (REC29) {
      Affine<C> p;
#pragma unroll
      for (int i = 0; i < r29::N; i++) {
        p.x.v[i] = w[i];
        p.y.v[i] = w[r29::N + i];
      }
      p.y = cneg(p.y, (v >> 31) != 0);
      return p;
    } else {
      Affine<Fq> p = {Fq::from_limbs(w), Fq::from_limbs(w + 12)};
      if (v >> 31) p.y = neg(p.y);
      return A::in(p);
    }
  };
  uint32_t key = active ? keys[c0] : sent;
  uint32_t val = active && key < sent ? vals[c0] : 0u;
  stage_load(0, val, key < sent);
  Xyzz<C> acc = Xyzz<C>::inf();
  const size_t steps = c1 - c0;  // per lane; the loop runs to the wave's longest chunk
  const size_t maxsteps = (size_t)1 << lg;
  for (size_t s = 0; s < maxsteps; s++) {
    const size_t e = c0 + s;
    const bool live = s < steps;
    uint32_t key_n = sent, val_n = 0;
    if (s + 1 < steps) {
      key_n = keys[e + 1];
      if (key_n < sent) val_n = vals[e + 1];
    }
    const Affine<C> pt = stage_read(NBUF == 1 ? 0 : (int)(s & 1), val);
    if constexpr (NBUF == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // pt read out of the buffer
    stage_load(NBUF == 1 ? 0 : (int)((s + 1) & 1), val_n, key_n < sent);
    if (live && key < sent) {
      acc = add_affine(acc, pt);
      if (key_n != key) {
        const bool starts = bstart[key] >= c0;
        const bool ends = bend[key] <= c1;
        if (starts && ends)
          store_pk(buckets, key, acc);
        else
          store_pk(part, 2 * t + (starts ? 1 : 0), acc);
        acc = Xyzz<C>::inf();
      }
    }
    key = key_n;
    val = val_n;
    if (__all(s + 1 >= steps ? 1 : 0)) break;  // wave-uniform exit
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no staging load outstanding at exit
}

// k_bucket_acc_short over G2 with pair-distributed Fq2 (pair_fq2.h): lanes
// 2t and 2t+1 run chunk t's bucket chain together, each holding one Fq
// coordinate of every Fq2 value; same chunking, parking and bucket stores.
static __device__ __forceinline__ Affine<Fq2P> fetch_point_pair(const uint32_t* bases, const uint32_t* phib, uint32_t nbase,
                                                        uint32_t v) {
  const uint32_t idx = v & 0x7fffffffu;
  Affine<Fq2P> p = (idx < nbase) ? load_affine_pair(bases, idx) : load_affine_pair(phib, idx - nbase);
  if (v >> 31) p.y = neg(p.y);
  return p;
}

static __global__ void __launch_bounds__(64, 2)
    k_bucket_acc_short_pair(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                            const uint32_t* __restrict__ range, int wlo, int whi, uint32_t sent,
                            const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bend,
                            const uint32_t* __restrict__ bases, const uint32_t* __restrict__ phib, uint32_t nbase,
                            int lg, Xyzz<Fq2>* __restrict__ buckets, Xyzz<Fq2>* __restrict__ part) {
  const size_t e_lo = range[wlo], e_hi = range[whi];
  const size_t t = (e_lo >> lg) + (((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 1);
  size_t c0 = t << lg;
  if (c0 >= e_hi) return;  // pair-uniform
  const size_t c1 = (c0 + ((size_t)1 << lg) < e_hi) ? c0 + ((size_t)1 << lg) : e_hi;
  if (c0 < e_lo) c0 = e_lo;
  uint32_t key = keys[c0];
  Affine<Fq2P> pt;
  if (key < sent) pt = fetch_point_pair(bases, phib, nbase, vals[c0]);
  Xyzz<Fq2P> acc = Xyzz<Fq2P>::inf();
  for (size_t e = c0; e < c1; e++) {
    uint32_t key_n = sent;
    Affine<Fq2P> pt_n;
    if (e + 1 < c1) {
      key_n = keys[e + 1];
      if (key_n < sent) pt_n = fetch_point_pair(bases, phib, nbase, vals[e + 1]);
    }
    if (key < sent) {
      acc = add_affine(acc, pt);
      if (key_n != key) {
        const bool starts = bstart[key] >= c0;
        const bool ends = bend[key] <= c1;
        if (starts && ends)
          store_xyzz_pair(buckets, key, acc);
        else
          store_xyzz_pair(part, 2 * t + (starts ? 1 : 0), acc);
        acc = Xyzz<Fq2P>::inf();
      }
    }
    key = key_n;
    pt = pt_n;
  }
}

// bucket-array input of a reduction kernel: the accumulation's packed format
// (PK) or a reduction's own output
template <bool PK, class F>
__device__ __forceinline__ Xyzz<typename AccField<F>::T> load_in(const Xyzz<F>* p, size_t i) {
  if constexpr (PK)
    return load_pk(p, i);
  else
    return load_acc(p, i);
}

// Buckets spanning more than LONG_PARTS chunks (many equal digits: small or
// boolean scalars put most entries of a window into one bucket) are not
// walked by one lane of the fixups below -- 2^20 entries of one bucket would
// be a 32 768-add serial chain -- but appended to a per-group list and summed
// by k_bucket_fixup_long, one workgroup per bucket (strided partial sums, then
// a tree in LDS).  cap bounds the list: every listed bucket covers more than
// LONG_PARTS whole chunks of its group's entries.
constexpr uint32_t LONG_PARTS = 64;
constexpr int LONG_THREADS = 256;
constexpr unsigned LONG_GRID = 32;
struct LongList {
  uint32_t* cnt;
  uint32_t* list;
  uint32_t cap;
  __device__ __forceinline__ void push(uint32_t b) const {
    const uint32_t i = atomicAdd(cnt, 1u);
    if (i < cap) list[i] = b;
  }
};

template <class F>
__global__ void __launch_bounds__(LONG_THREADS) k_bucket_fixup_long(const uint32_t* __restrict__ bstart,
                                                                    const uint32_t* __restrict__ bend, int lg,
                                                                    const Xyzz<F>* __restrict__ part,
                                                                    Xyzz<F>* __restrict__ buckets, LongList ll) {
  using C = typename AccField<F>::T;
  __shared__ Xyzz<C> sh[LONG_THREADS];
  const uint32_t n = *ll.cnt < ll.cap ? *ll.cnt : ll.cap;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t b = ll.list[i];
    const size_t t0 = (size_t)bstart[b] >> lg, t1 = (size_t)(bend[b] - 1) >> lg;
    Xyzz<C> acc = tid == 0 ? load_pk(part, 2 * t0 + 1) : Xyzz<C>::inf();
    for (size_t t = t0 + 1 + tid; t <= t1; t += LONG_THREADS) acc = add(acc, load_pk(part, 2 * t));
    sh[tid] = acc;
    __syncthreads();
    for (uint32_t h = LONG_THREADS / 2; h > 0; h >>= 1) {
      if (tid < h) sh[tid] = add(sh[tid], sh[tid + h]);
      __syncthreads();
    }
    if (tid == 0) store_pk(buckets, b, sh[0]);
    __syncthreads();
  }
}

// k_bucket_fixup_short over G2 with pair-distributed Fq2: lanes 2b, 2b+1
// finish bucket b0 + b together
static __global__ void __launch_bounds__(64, 2)
    k_bucket_fixup_short_pair(const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bend, size_t b0,
                              size_t b1, int lg, const Xyzz<Fq2>* __restrict__ part, Xyzz<Fq2>* __restrict__ buckets,
                              int prio, LongList ll) {
  set_wave_prio(prio);
  const size_t b = b0 + (((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 1);
  if (b >= b1) return;
  const uint32_t s = bstart[b], e = bend[b];
  if (e <= s) return;
  const size_t t0 = (size_t)s >> lg, t1 = (size_t)(e - 1) >> lg;
  if (t0 == t1) return;
  if (t1 - t0 > LONG_PARTS) {
    if (!(threadIdx.x & 1)) ll.push((uint32_t)b);
    return;
  }
  Xyzz<Fq2P> acc = load_xyzz_pair(part, 2 * t0 + 1);
  for (size_t t = t0 + 1; t <= t1; t++) acc = add(acc, load_xyzz_pair(part, 2 * t));
  store_xyzz_pair(buckets, b, acc);
}

// buckets crossing chunk boundaries: trailing piece of the first chunk plus
// the leading pieces of the following ones
template <class F>
__global__ void __launch_bounds__(64, (sizeof(F) > 48 ? 1 : 2))
    k_bucket_fixup_short(const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ bend, size_t b0,
                         size_t b1, int lg, const Xyzz<F>* __restrict__ part, Xyzz<F>* __restrict__ buckets,
                         int prio, LongList ll) {
  using C = typename AccField<F>::T;
  set_wave_prio(prio);
  const size_t b = b0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= b1) return;
  const uint32_t s = bstart[b], e = bend[b];
  if (e <= s) return;
  const size_t t0 = (size_t)s >> lg, t1 = (size_t)(e - 1) >> lg;
  if (t0 == t1) return;
  if (t1 - t0 > LONG_PARTS) {
    ll.push((uint32_t)b);
    return;
  }
  Xyzz<C> acc = load_pk(part, 2 * t0 + 1);
  for (size_t t = t0 + 1; t <= t1; t++) acc = add(acc, load_pk(part, 2 * t));
  store_pk(buckets, b, acc);
}

// the same fixup, one quad of lanes per bucket (coop.h: 4 product latencies
// per addition instead of ~14): for the last window group, whose fixup sits on
// the MSM's tail with one lone lane per bucket at ~2 waves per CU
template <class F>
__global__ void __launch_bounds__(64) k_bucket_fixup_quad(const uint32_t* __restrict__ bstart,
                                                          const uint32_t* __restrict__ bend, size_t b0, size_t b1,
                                                          int lg, const Xyzz<F>* __restrict__ part,
                                                          Xyzz<F>* __restrict__ buckets, LongList ll) {
  using C = typename AccField<F>::T;
  const size_t b = b0 + (((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2);
  const int qi = threadIdx.x & 3;
  if (b >= b1) return;  // quad-uniform
  const uint32_t s = bstart[b], e = bend[b];
  if (e <= s) return;
  const size_t t0 = (size_t)s >> lg, t1 = (size_t)(e - 1) >> lg;
  if (t0 == t1) return;
  if (t1 - t0 > LONG_PARTS) {
    if (qi == 0) ll.push((uint32_t)b);
    return;
  }
  Xyzz<C> acc = load_pk(part, 2 * t0 + 1);
  for (size_t t = t0 + 1; t <= t1; t++) acc = add_quad(acc, load_pk(part, 2 * t), qi);
  if (qi == 0) store_pk(buckets, b, acc);
}

// segment t of group g: sum_{b in seg} (b+1) * S_b with b the bucket index
// inside the group (bucket b holds digit value b+1): running sums over the L
// buckets plus (segment offset) * (segment sum).  One quad of lanes per
// segment (coop.h): 4 / 3 product latencies per addition / doubling.
template <class F, bool PK>
__global__ void __launch_bounds__(64) k_seg_reduce_quad(const Xyzz<F>* __restrict__ buckets, uint32_t nb, uint32_t L,
                                                        size_t nseg, Xyzz<F>* __restrict__ seg_out, int prio = 0) {
  using C = typename AccField<F>::T;
  set_wave_prio(prio);
  const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const int qi = threadIdx.x & 3;
  if (t >= nseg) return;  // quad-uniform
  const uint32_t S = nb / L;
  const size_t g = t / S;
  const uint32_t k = (uint32_t)(t % S);
  const size_t base = g * nb + (size_t)k * L;
  Xyzz<C> acc = Xyzz<C>::inf(), sum = Xyzz<C>::inf();
  for (int b = (int)L - 1; b >= 0; b--) {
    acc = add_quad(acc, load_in<PK>(buckets, base + b), qi);
    sum = add_quad(sum, acc, qi);
  }
  const uint32_t s0 = k * L;
  if (s0 != 0 && !is_inf(acc)) sum = add_quad(sum, scalar_mul_quad(acc, s0, 32 - __builtin_clz(s0), qi), qi);
  if (qi == 0) store_acc(seg_out, t, sum);
}

// the same segment sums, one lane per segment: for reductions with enough
// segments to fill the chip (the 4096-row commit at 2^24: 262 144 segments)
// the quad-cooperative form only adds exchange overhead to a throughput-bound
// pass
template <class F, bool PK>
__global__ void __launch_bounds__(64) k_seg_reduce_lane(const Xyzz<F>* __restrict__ buckets, uint32_t nb, uint32_t L,
                                                        size_t nseg, Xyzz<F>* __restrict__ seg_out) {
  using C = typename AccField<F>::T;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nseg) return;
  const uint32_t S = nb / L;
  const size_t g = t / S;
  const uint32_t k = (uint32_t)(t % S);
  const size_t base = g * nb + (size_t)k * L;
  Xyzz<C> acc = Xyzz<C>::inf(), sum = Xyzz<C>::inf();
  for (int b = (int)L - 1; b >= 0; b--) {
    acc = add(acc, load_in<PK>(buckets, base + b));
    sum = add(sum, acc);
  }
  const uint32_t s0 = k * L;
  if (s0 != 0 && !is_inf(acc)) sum = add(sum, scalar_mul_xyzz(acc, &s0, 32 - __builtin_clz(s0)));
  store_acc(seg_out, t, sum);
}

// one workgroup of BS / 4 quads per group: sum its S partial points
template <class F, int BS>
__global__ void __launch_bounds__(BS) k_group_reduce_quad(const Xyzz<F>* __restrict__ seg, uint32_t S,
                                                          Xyzz<F>* __restrict__ out, int prio = 0) {
  using C = typename AccField<F>::T;
  set_wave_prio(prio);
  constexpr int Q = BS / 4;
  __shared__ Xyzz<C> sh[Q];
  const size_t g = blockIdx.x;
  const int quad = threadIdx.x >> 2, qi = threadIdx.x & 3;
  Xyzz<C> acc = Xyzz<C>::inf();
  for (uint32_t k = quad; k < S; k += Q) acc = add_quad(acc, load_acc(seg, g * S + k), qi);
  if (qi == 0) sh[quad] = acc;
  __syncthreads();
  for (int h = Q / 2; h > 0; h >>= 1) {
    if (quad < h) {  // a quad reads its two operands before its lane 0 writes (one wave, in order)
      const Xyzz<C> v = add_quad(sh[quad], sh[quad + h], qi);
      if (qi == 0) sh[quad] = v;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) store_acc(out, g, sh[0]);
}

// Contribution of the window group [wlo, whi) on one wave:
// 2^(c wlo) sum_{wlo <= w < whi} 2^(c (w - wlo)) G_w (Horner, then c wlo more
// doublings), plus the `nextra` finished contributions of the other groups.
// Every quad runs the same chain, its doublings and additions
// quad-cooperative (coop.h: 3 / 4 product latencies).
template <class F>
static __global__ void __launch_bounds__(64, 1) k_window_chain(const Xyzz<F>* __restrict__ win, int wlo, int whi,
                                                              int c, const Xyzz<F>* __restrict__ extra, int nextra,
                                                              Xyzz<F>* __restrict__ out) {
  using C = typename AccField<F>::T;
  if (blockIdx.x != 0) return;
  __builtin_amdgcn_s_setprio(3);  // a lone latency chain beside accumulation waves
  const int qi = threadIdx.x & 3;
  Xyzz<C> acc = load_acc(win, whi - 1);
  for (int w = whi - 2; w >= wlo; w--) {
    for (int i = 0; i < c; i++) acc = dbl_quad(acc, qi);
    acc = add_quad(acc, load_acc(win, w), qi);
  }
  for (int i = 0; i < c * wlo; i++) acc = dbl_quad(acc, qi);
  for (int k = 0; k < nextra; k++) acc = add_quad(acc, load_acc(extra, k), qi);
  if (threadIdx.x == 0) store_acc(out, 0, acc);
}

template <class F>
__global__ void k_points_to_mont(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<F> a = load_affine<F>(in, i);
  Fq* c = reinterpret_cast<Fq*>(&a);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(Affine<F>) / sizeof(Fq)); k++) c[k] = to_mont(c[k]);
  store_affine(out, i, a);
}

template <class F>
__global__ void k_affine_from_mont(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<F> a = load_affine<F>(in, i);
  Fq* c = reinterpret_cast<Fq*>(&a);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(Affine<F>) / sizeof(Fq)); k++) c[k] = from_mont(c[k]);
  store_affine(out, i, a);
}

template <class F>
__global__ void __launch_bounds__(64, 1) k_xyzz_to_affine_canonical(const Xyzz<F>* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<F> a = to_affine(load_xyzz(in, i));
  Fq* c = reinterpret_cast<Fq*>(&a);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(Affine<F>) / sizeof(Fq)); k++) c[k] = from_mont(c[k]);
  store_affine(out, i, a);
}

// the same with one wave per point and the wave-cooperative inverse
// (inv_wave.h): for the few-point conversions on a latency path
template <class F>
__global__ void __launch_bounds__(64) k_xyzz_to_affine_wave(const Xyzz<F>* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  const size_t i = blockIdx.x;
  if (i >= n) return;
  Affine<F> a = to_affine_w(load_xyzz(in, i));
  Fq* c = reinterpret_cast<Fq*>(&a);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(Affine<F>) / sizeof(Fq)); k++) c[k] = from_mont(c[k]);
  if (threadIdx.x == 0) store_affine(out, i, a);
}

// up to this many points one wave-cooperative inverse per point
// (k_xyzz_to_affine_wave); above it one lone-lane inverse per point
constexpr size_t INV_WAVE_MAX = 4096;

#ifndef TPST_MSM_LAB  // tools/lab: the kernels above only, instantiated there
template <class F>
hipError_t points_to_mont(hipStream_t s, const uint32_t* d_in, uint32_t* d_out, size_t n) {
  if (!n) return hipSuccess;
  k_points_to_mont<F><<<grid_for(n, 256), 256, 0, s>>>(d_in, d_out, n);
  return hipGetLastError();
}

template <class F>
hipError_t affine_from_mont(hipStream_t s, const uint32_t* d_in, uint32_t* d_out, size_t n) {
  if (!n) return hipSuccess;
  k_affine_from_mont<F><<<grid_for(n, 256), 256, 0, s>>>(d_in, d_out, n);
  return hipGetLastError();
}

template <class F>
hipError_t xyzz_to_affine_canonical(hipStream_t s, const Xyzz<F>* d_in, uint32_t* d_out, size_t n) {
  if (!n) return hipSuccess;
  if (n <= INV_WAVE_MAX)
    k_xyzz_to_affine_wave<F><<<(unsigned)n, 64, 0, s>>>(d_in, d_out, n);
  else
    k_xyzz_to_affine_canonical<F><<<grid_for(n, 64), 64, 0, s>>>(d_in, d_out, n);
  return hipGetLastError();
}

// reduce `groups` bucket sets of nb buckets each into one point per group:
// short weighted segments (L = 4) then two tree passes
// segment length of the weighted bucket reduction: short segments (L = 4)
// when the groups are few (latency-bound: many short chains); longer ones when
// there are enough segments to fill the chip anyway (throughput-bound: every
// segment pays one scalar multiplication by its offset, so fewer, longer
// segments do less work) -- the 4096-row commit at 2^24 runs L = 32
static uint32_t reduce_seg_len(size_t groups, uint32_t nb) {
  uint32_t L = 4;
  while (L < 32 && 2 * L <= nb && groups * (nb / (2 * L)) >= ((size_t)1 << 18)) L *= 2;
  return nb >= L ? L : nb;
}

template <class F>
static size_t reduce_scratch(size_t groups, uint32_t nb) {
  const uint32_t L = reduce_seg_len(groups, nb);
  const size_t nseg = groups * (nb / L);
  return Arena::need(nseg, sizeof(Xyzz<F>)) + Arena::need(nseg / 64 + groups + 1, sizeof(Xyzz<F>));
}

template <class F>
static hipError_t reduce_buckets(Arena& ar, hipStream_t s, const Xyzz<F>* d_buckets, size_t groups, uint32_t nb,
                                 Xyzz<F>* d_group_out, int prio = 0, bool pk = true) {
  const uint32_t L = reduce_seg_len(groups, nb);
  const uint32_t S = nb / L;
  const size_t nseg = groups * S;
  Xyzz<F>* seg = ar.take<Xyzz<F>>(nseg);
  // d_buckets: the accumulation's bucket format (pk) or a reduction's output
  if (std::is_same<F, Fq>::value && nseg >= ((size_t)1 << 18)) {
    if (pk)
      k_seg_reduce_lane<F, true><<<grid_for(nseg, 64), 64, 0, s>>>(d_buckets, nb, L, nseg, seg);
    else
      k_seg_reduce_lane<F, false><<<grid_for(nseg, 64), 64, 0, s>>>(d_buckets, nb, L, nseg, seg);
  } else if (pk) {
    k_seg_reduce_quad<F, true><<<grid_for(4 * nseg, 64), 64, 0, s>>>(d_buckets, nb, L, nseg, seg, prio);
  } else {
    k_seg_reduce_quad<F, false><<<grid_for(4 * nseg, 64), 64, 0, s>>>(d_buckets, nb, L, nseg, seg, prio);
  }
  TPST_TRY(hipGetLastError());
  if (S >= 256 && S % 64 == 0) {  // two-pass tree: 64 -> 1, then per group
    Xyzz<F>* mid = ar.take<Xyzz<F>>(nseg / 64);
    k_group_reduce_quad<F, 256><<<(unsigned)(nseg / 64), 256, 0, s>>>(seg, 64, mid, prio);
    TPST_TRY(hipGetLastError());
    k_group_reduce_quad<F, 256><<<(unsigned)groups, 256, 0, s>>>(mid, S / 64, d_group_out, prio);
  } else {
    k_group_reduce_quad<F, 256><<<(unsigned)groups, 256, 0, s>>>(seg, S, d_group_out, prio);
  }
  return hipGetLastError();
}

// Two-level weighted reduction without per-segment scalar multiplications
// (work ~1/3 of reduce_buckets at the K2 shape, for the window groups whose
// reduction runs under other groups' accumulation -- throughput, not latency).
// Level 1: segments of L1 buckets -> S_k = sum_{b in seg} (b - k L1 + 1) X_b and
// T_k = sum_{b in seg} X_b; then sum_b (b+1) X_b = sum_k S_k + L1 sum_k k T_k,
// the second sum being the same weighted reduction over Tn_{k-1} = T_k.
template <class F, bool PK = true>
__global__ void __launch_bounds__(64) k_seg_run_quad(const Xyzz<F>* __restrict__ buckets, uint32_t nb, uint32_t L,
                                                     size_t nseg, Xyzz<F>* __restrict__ S_out,
                                                     Xyzz<F>* __restrict__ Tn, int prio = 0) {
  using C = typename AccField<F>::T;
  set_wave_prio(prio);
  const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const int qi = threadIdx.x & 3;
  if (t >= nseg) return;  // quad-uniform
  const uint32_t S = nb / L;
  const size_t g = t / S;
  const uint32_t k = (uint32_t)(t % S);
  const size_t base = g * nb + (size_t)k * L;
  Xyzz<C> acc = Xyzz<C>::inf(), sum = Xyzz<C>::inf();
  for (int b = (int)L - 1; b >= 0; b--) {
    acc = add_quad(acc, load_in<PK>(buckets, base + b), qi);
    sum = add_quad(sum, acc, qi);
  }
  if (qi == 0) {
    store_acc(S_out, t, sum);
    store_acc(Tn, g * S + (k ? k - 1 : S - 1), k ? acc : Xyzz<C>::inf());
  }
}

// k_seg_run_quad with one lane per segment (throughput shape: >= 2^18
// segments, e.g. the 2^24 commit's 4096 rows x 128 segments)
template <class F, bool PK = true>
__global__ void __launch_bounds__(64) k_seg_run_lane(const Xyzz<F>* __restrict__ buckets, uint32_t nb, uint32_t L,
                                                     size_t nseg, Xyzz<F>* __restrict__ S_out,
                                                     Xyzz<F>* __restrict__ Tn) {
  using C = typename AccField<F>::T;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nseg) return;
  const uint32_t S = nb / L;
  const size_t g = t / S;
  const uint32_t k = (uint32_t)(t % S);
  const size_t base = g * nb + (size_t)k * L;
  Xyzz<C> acc = Xyzz<C>::inf(), sum = Xyzz<C>::inf();
  for (int b = (int)L - 1; b >= 0; b--) {
    acc = add(acc, load_in<PK>(buckets, base + b));
    sum = add(sum, acc);
  }
  store_acc(S_out, t, sum);
  store_acc(Tn, g * S + (k ? k - 1 : S - 1), k ? acc : Xyzz<C>::inf());
}

// out[g] = a[g] + 2^lg b[g], one quad per group
template <class F>
__global__ void __launch_bounds__(64) k_lift_add_quad(const Xyzz<F>* __restrict__ a, const Xyzz<F>* __restrict__ b,
                                                      int lg, size_t groups, Xyzz<F>* __restrict__ out,
                                                      int prio = 0) {
  using C = typename AccField<F>::T;
  set_wave_prio(prio);
  const size_t g = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const int qi = threadIdx.x & 3;
  if (g >= groups) return;
  Xyzz<C> r = load_acc(b, g);
  for (int i = 0; i < lg; i++) r = dbl_quad(r, qi);
  r = add_quad(r, load_acc(a, g), qi);
  if (qi == 0) store_acc(out, g, r);
}

// sum of S points per group (tree passes of k_group_reduce_quad)
template <class F>
static hipError_t sum_groups(Arena& ar, hipStream_t s, const Xyzz<F>* in, size_t groups, uint32_t S, Xyzz<F>* out,
                             int prio) {
  if (S >= 256 && S % 64 == 0) {
    Xyzz<F>* mid = ar.take<Xyzz<F>>(groups * S / 64);
    k_group_reduce_quad<F, 256><<<(unsigned)(groups * S / 64), 256, 0, s>>>(in, 64, mid, prio);
    TPST_TRY(hipGetLastError());
    k_group_reduce_quad<F, 256><<<(unsigned)groups, 256, 0, s>>>(mid, S / 64, out, prio);
  } else {
    k_group_reduce_quad<F, 256><<<(unsigned)groups, 256, 0, s>>>(in, S, out, prio);
  }
  return hipGetLastError();
}

constexpr int RED2_LG = 4;  // level-1 segment length 16

static bool red2_ok(uint32_t nb) { return nb >= (16u << RED2_LG); }

template <class F>
static size_t reduce2_scratch(size_t groups, uint32_t nb) {
  const uint32_t S1 = nb >> RED2_LG;
  return 2 * Arena::need(groups * S1, sizeof(Xyzz<F>)) + reduce_scratch<F>(groups, S1) +
         Arena::need(groups * S1 / 64 + 1, sizeof(Xyzz<F>)) + 2 * Arena::need(groups, sizeof(Xyzz<F>));
}

#ifndef TPST_RED2_LANE
#define TPST_RED2_LANE 1
#endif
// lane_ok: a throughput reduction (under other accumulation work) -- one lane
// per segment costs fewer VALU issue slots per addition than a quad
template <class F>
static hipError_t reduce_buckets2(Arena& ar, hipStream_t s, const Xyzz<F>* d_buckets, size_t groups, uint32_t nb,
                                  Xyzz<F>* d_group_out, int prio, bool lane_ok = false) {
  const uint32_t L1 = 1u << RED2_LG, S1 = nb / L1;
  const size_t nseg = groups * S1;
  Xyzz<F>* Sk = ar.take<Xyzz<F>>(nseg);
  Xyzz<F>* Tn = ar.take<Xyzz<F>>(nseg);
  Xyzz<F>* R = ar.take<Xyzz<F>>(groups);
  Xyzz<F>* SS = ar.take<Xyzz<F>>(groups);
  if (std::is_same<F, Fq>::value && (nseg >= ((size_t)1 << 18) || (TPST_RED2_LANE && lane_ok)))
    k_seg_run_lane<F><<<grid_for(nseg, 64), 64, 0, s>>>(d_buckets, nb, L1, nseg, Sk, Tn);
  else
    k_seg_run_quad<F><<<grid_for(4 * nseg, 64), 64, 0, s>>>(d_buckets, nb, L1, nseg, Sk, Tn, prio);
  TPST_TRY(hipGetLastError());
  TPST_TRY(reduce_buckets<F>(ar, s, Tn, groups, S1, R, prio, false));  // Tn: a reduction's output
  TPST_TRY(sum_groups<F>(ar, s, Sk, groups, S1, SS, prio));
  k_lift_add_quad<F><<<grid_for(4 * groups, 64), 64, 0, s>>>(SS, R, RED2_LG, groups, d_group_out, prio);
  return hipGetLastError();
}

// the last window group's fixup (on the MSM's tail) runs one quad of lanes
// per bucket; the aux-stream groups one lane per bucket at s_setprio 2
constexpr int RED_PRIO = 2;

// window groups of the variable-base MSM (3; sweep of 1-5 in
// profiles/r02/sw2): with more than one, the groups' bucket accumulations run
// top group first on the main stream; each finished group's reduction (the
// two-level one) and doubling chain run on an aux stream under the next
// group's accumulation, so only the last group's reduction and its
// c-doubling Horner remain after the accumulation
static int msm_groups(size_t n, int W) {
  if (n < ((size_t)1 << 17) || W < 4) return 1;
  int g = 3;
  if (g > (Arena::N_AUX_EV - 1) / 2) g = (Arena::N_AUX_EV - 1) / 2;
  return g > W ? W : g;
}

// window boundaries wb[0..NG] of the groups: a short bottom group (~W/8
// windows: its reduction and chain are the tail left after the accumulation)
// and an even split of the rest -- 1,3,4 for the 2^20 G1 MSM, 1.3 % faster
// than 2,3,3 in an interleaved A/B (profiles/r02/sw2)
static void msm_group_bounds(int W, int NG, int* wb) {
  if (NG == 1) {
    wb[0] = 0;
    wb[1] = W;
  } else {
    const int lo = W / 8 > 1 ? W / 8 : 1;
    wb[0] = 0;
    for (int g = 1; g <= NG; g++) wb[g] = lo + (g - 1) * (W - lo) / (NG - 1);
  }
}

template <class F>
hipError_t msm_var(Arena& ar, hipStream_t s, const uint32_t* d_bases, const uint32_t* d_scalars, size_t n,
                   Xyzz<F>* d_out, hipStream_t tail, bool* on_tail, hipStream_t front) {
  if (on_tail) *on_tail = false;
  if (n == 0) {
    Xyzz<F> inf = Xyzz<F>::inf();
    return hipMemcpyAsync(d_out, &inf, sizeof(inf), hipMemcpyHostToDevice, s);
  }
  if (n > MSM_MAX_POINTS) return hipErrorInvalidValue;
  const bool glv = n >= 64;  // phi(x, y) = (beta x, y) on G1, (beta^2 x, y) on G2
  // G1 with GLV: gather records of P and phi(P) (fetch_rec29) instead of phi(P) alone
  constexpr bool g1 = std::is_same<F, Fq>::value;
  const bool rec29 = TPST_K2_REC29 && glv && g1;
  constexpr size_t PW = 2 * Words<F>::n;
  const int c = msm_window_bits(glv ? 2 * n : n);
  const int W = glv ? num_windows_bits(c, 128) : num_windows(c);
  const uint32_t nb = 1u << (c - 1);
  const size_t per_win = (size_t)(glv ? 2 : 1) * n;  // entries of one window (zero digits included)
  const size_t m = per_win * W;
  if (m >= ((size_t)1 << 31)) return hipErrorInvalidValue;
  const size_t nbk = (size_t)W * nb;
  const uint32_t sent = (uint32_t)nbk;  // zero digits; sorts after every bucket key
  SortPlan sp;
  if (!sort_plan(sent, n, m, sp)) return hipErrorInvalidValue;
  const int NG = msm_groups(n, W);
  int wb[Arena::N_AUX_EV / 2 + 1];
  msm_group_bounds(W, NG, wb);
  if (NG > 1) TPST_TRY(ar.aux_init());
  int lg;
  if (NG > 1) {  // per-group launches: keep >= 4 waves per SIMD in each
    static const size_t simds = device_simds();
    lg = 4;  // 16-entry chunks: 8 / 32 / 64 measured 4 / 7 / 18 % slower (profiles/r05/g)
    while (lg < 8 && ((m / NG) >> (lg + 1)) >= (size_t)4 * 64 * simds) lg++;
  } else {
    lg = acc_chunk_lg(m);
  }
  const bool short_chunks = NG > 1 || lg == 5;  // K2 at every size up to ~2^24 points
  const size_t nchunk = (m + ((size_t)1 << lg) - 1) >> lg;
  const size_t nblk = (nchunk + ACC_BLOCK - 1) / ACC_BLOCK;
  size_t red_need = 0;
  for (int g = 0; g < NG; g++) {
    const size_t gw = (size_t)(wb[g + 1] - wb[g]);
    red_need += reduce_scratch<F>(gw, nb) + (red2_ok(nb) ? reduce2_scratch<F>(gw, nb) : 0);
  }
  size_t need = Arena::need(m, 4) * 4 + Arena::need(nbk, 4) * 2 + Arena::need(nbk, sizeof(Xyzz<F>)) +
                Arena::need(2 * nchunk, sizeof(Xyzz<F>)) + Arena::need(nblk, sizeof(Xyzz<F>)) + red_need +
                Arena::need(W, sizeof(Xyzz<F>)) + Arena::need(NG, sizeof(Xyzz<F>)) + Arena::need(W + 1, 4) +
                Arena::need(glv && !rec29 ? n * PW : 1, 4) + Arena::need(rec29 ? 2 * n * REC29_WORDS : 1, 4) +
                Arena::need((size_t)sp.ntile * sp.nbins, 4) +
                Arena::need(sp.nbins, 4) + Arena::need(sp.nbins + 1, 4) + Arena::need(NG, 4) +
                Arena::need((size_t)NG * (m / ((size_t)LONG_PARTS << lg) + 1), 4) + 8192;
  ar.reset();
  TPST_TRY(ar.reserve(need));
  uint32_t* keys = ar.take<uint32_t>(m);
  uint32_t* vals = ar.take<uint32_t>(m);
  uint32_t* keys2 = ar.take<uint32_t>(m);
  uint32_t* vals2 = ar.take<uint32_t>(m);
  uint32_t* bstart = ar.take<uint32_t>(nbk);
  uint32_t* bend = ar.take<uint32_t>(nbk);
  Xyzz<F>* buckets = ar.take<Xyzz<F>>(nbk);
  Xyzz<F>* part = ar.take<Xyzz<F>>(2 * nchunk);
  Xyzz<F>* bpart = ar.take<Xyzz<F>>(nblk);
  Xyzz<F>* win = ar.take<Xyzz<F>>(W);
  Xyzz<F>* contrib = ar.take<Xyzz<F>>(NG);
  uint32_t* range = ar.take<uint32_t>(W + 1);
  uint32_t* phib = ar.take<uint32_t>(glv && !rec29 ? n * PW : 1);
  uint32_t* rec = rec29 ? ar.take<uint32_t>(2 * n * REC29_WORDS) : nullptr;
  const uint32_t* gb = rec29 ? rec : d_bases;  // what the accumulation gathers
  const uint32_t gnb = rec29 ? 0x7fffffffu : (uint32_t)n;
  uint32_t* tab = ar.take<uint32_t>((size_t)sp.ntile * sp.nbins);
  uint32_t* btot = ar.take<uint32_t>(sp.nbins);
  uint32_t* bin0 = ar.take<uint32_t>(sp.nbins + 1);
  // a listed bucket spans more than LONG_PARTS chunks, so more than
  // LONG_PARTS << lg entries, and buckets are disjoint: at most m / (LONG_PARTS
  // << lg) of them in any group (the list can never overflow)
  const uint32_t lcap = (uint32_t)(m / ((size_t)LONG_PARTS << lg)) + 1;
  uint32_t* lcnt = ar.take<uint32_t>(NG);
  uint32_t* llist = ar.take<uint32_t>((size_t)NG * lcap);

  Profiler* pf = ar.prof;
  Profiler dummy;
  if (!pf) pf = &dummy;
  const hipStream_t fs = front ? front : s;
  pf->begin(ST_DECOMPOSE, fs);
  if (short_chunks) TPST_TRY(hipMemsetAsync(lcnt, 0, NG * sizeof(uint32_t), fs));
  k_decompose_hist<F><<<sp.ntile, SORT_THREADS, sp.nbins * 4, fs>>>(d_scalars, n, c, W, glv ? 1 : 0, sent, sp.lo,
                                                                  sp.nbins, sp.tile, keys, vals, tab, d_bases, phib,
                                                                  rec);
  TPST_TRY(hipGetLastError());
  pf->end(ST_DECOMPOSE, fs);
  pf->begin(ST_SORT, fs);
  k_sort_colscan<<<grid_for(sp.nbins, 64), 64 * COLSCAN_CH, 0, fs>>>(tab, sp.ntile, sp.nbins, btot);
  TPST_TRY(hipGetLastError());
  k_sort_binscan<<<1, BINSCAN_THREADS, 0, fs>>>(btot, sp.nbins, bin0);
  TPST_TRY(hipGetLastError());
  const int halves = glv ? 2 : 1;
  const uint32_t bpw = nb >> sp.lo;
  // stage of E entries per thread (E = 4, or 2 when the bin cursors are many)
  const auto scat_lds = [&](int E) { return ((size_t)sp.nbins + 2 * (bpw + 1) + 2 * (size_t)E * SORT_THREADS) * 4; };
  const int E = scat_lds(4) <= 60 * 1024 ? 4 : (scat_lds(2) <= 60 * 1024 ? 2 : 0);
  if (sp.lo <= c - 1 && E) {  // bins aligned to windows, stage fits
    if (E == 4)
      k_sort_scatter_win<4><<<sp.ntile, SORT_THREADS, scat_lds(4), fs>>>(keys, vals, n, halves, W, sent, sp.lo,
                                                                       sp.nbins, bpw, sp.tile, tab, bin0, keys2, vals2);
    else
      k_sort_scatter_win<2><<<sp.ntile, SORT_THREADS, scat_lds(2), fs>>>(keys, vals, n, halves, W, sent, sp.lo,
                                                                       sp.nbins, bpw, sp.tile, tab, bin0, keys2, vals2);
  } else {
    k_sort_scatter<<<sp.ntile, SORT_THREADS, sp.nbins * 4, fs>>>(keys, vals, n, (uint32_t)(halves * W), sp.lo,
                                                                sp.nbins, sp.tile, tab, bin0, keys2, vals2);
  }
  TPST_TRY(hipGetLastError());
  // sorted entries back into keys / vals; bucket bounds, empty buckets, range
  k_sort_bin<<<sp.nbins, SORTB_THREADS, (2u << sp.lo) * 4 + SORTB_CAP * 4, fs>>>(
      keys2, vals2, bin0, sp.lo, sent, nb, W, keys, vals, bstart, bend, reinterpret_cast<uint4*>(buckets),
      (uint32_t)(sizeof(Xyzz<F>) / 16), range);
  TPST_TRY(hipGetLastError());
  pf->end(ST_SORT, fs);
  if (fs != s) {  // the accumulation waits for the sort
    TPST_TRY(ar.aux_init());
    TPST_TRY(hipEventRecord(ar.aux_ev[Arena::N_AUX_EV - 1], fs));
    TPST_TRY(hipStreamWaitEvent(s, ar.aux_ev[Arena::N_AUX_EV - 1], 0));
  }
  if (!short_chunks) {  // one launch, long chunks (more than ~2^21 points)
    pf->begin(ST_BUCKET_ACC, s);
    bool done = false;
    if constexpr (g1) {
      if (rec29) {
        k_bucket_acc_chunk<Fq, 2, true><<<(unsigned)nblk, ACC_BLOCK, 0, s>>>(keys, vals, m, range + W, sent, bstart,
                                                                              bend, gb, nullptr, gnb, lg, buckets,
                                                                              part, bpart);
        done = true;
      }
    }
    if (!done)
      k_bucket_acc_chunk<F><<<(unsigned)nblk, ACC_BLOCK, 0, s>>>(keys, vals, m, range + W, sent, bstart, bend,
                                                                  d_bases, phib, (uint32_t)n, lg, buckets, part, bpart);
    TPST_TRY(hipGetLastError());
    k_bucket_fixup<F><<<grid_for(nblk, 64), 64, 0, s>>>(keys, m, range + W, sent, bstart, bend, lg, nblk, part, bpart,
                                                        buckets);
    TPST_TRY(hipGetLastError());
    pf->end(ST_BUCKET_ACC, s);
    pf->begin(ST_REDUCE, s);
    TPST_TRY(reduce_buckets<F>(ar, s, buckets, W, nb, win));
    pf->end(ST_REDUCE, s);
    pf->begin(ST_COMBINE, s);
    k_window_chain<F><<<1, 64, 0, s>>>(win, 0, W, c, nullptr, 0, d_out);
    TPST_TRY(hipGetLastError());
    pf->end(ST_COMBINE, s);
    return hipSuccess;
  }
  // groups accumulate on the context stream; the fixup / reduction / chain of
  // group g > 0 run on an aux stream (a separate low-priority accumulation
  // stream measured slower: 4+ streams share the hardware queues)
  hipStream_t bulk = s;
  // the last group's tail: on `tail` when the caller pipelines calls
  const hipStream_t t0 = (tail && NG > 1) ? tail : s;
  if (on_tail) *on_tail = t0 != s;
  pf->begin(ST_BUCKET_ACC, bulk);
  for (int g = NG - 1; g >= 0; g--) {  // top windows first: their chains are the longest
    const int wlo = wb[g], whi = wb[g + 1];
    const size_t gchunks = ((per_win * (size_t)(whi - wlo)) >> lg) + 2;
    if constexpr (std::is_same<F, Fq2>::value) {
      k_bucket_acc_short_pair<<<grid_for(2 * gchunks, 64), 64, 0, bulk>>>(keys, vals, range, wlo, whi, sent,
                                                                          bstart, bend, d_bases, phib, (uint32_t)n,
                                                                          lg, buckets, part);
    } else {
      // the next point staged through LDS (default: 277-279 vs 273 Mscalar/s
      // with the register prefetch, profiles/r05/l); TPST_ACC_LDS=0 selects
      // the register prefetch
      static const bool lds = [] {
        const char* e = getenv("TPST_ACC_LDS");
        return !e || atoi(e) != 0;
      }();
      const unsigned grid = grid_for(gchunks, 64);
      if (lds && rec29)
        k_bucket_acc_short_lds<TPST_K2_MINW, true><<<grid, 64, 0, bulk>>>(keys, vals, range, wlo, whi, sent, bstart, bend, gb,
                                                                nullptr, gnb, lg, buckets, part);
      else if (lds)
        k_bucket_acc_short_lds<2, false><<<grid, 64, 0, bulk>>>(keys, vals, range, wlo, whi, sent, bstart, bend,
                                                                 d_bases, phib, (uint32_t)n, lg, buckets, part);
      else if (rec29)
        k_bucket_acc_short<F, 2, true><<<grid, 64, 0, bulk>>>(keys, vals, range, wlo, whi, sent, bstart, bend, gb,
                                                               nullptr, gnb, lg, buckets, part);
      else
        k_bucket_acc_short<F><<<grid, 64, 0, bulk>>>(keys, vals, range, wlo, whi, sent, bstart, bend, d_bases, phib,
                                                      (uint32_t)n, lg, buckets, part);
    }
    TPST_TRY(hipGetLastError());
    if (g == 0) pf->end(ST_BUCKET_ACC, bulk);
    const size_t b0 = (size_t)wlo * nb, b1 = (size_t)whi * nb;
    hipStream_t a = g ? ar.aux[g % Arena::N_AUX] : t0;
    if (NG > 1) {
      TPST_TRY(hipEventRecord(ar.aux_ev[2 * g], bulk));
      TPST_TRY(hipStreamWaitEvent(a, ar.aux_ev[2 * g], 0));
    }
    const LongList ll{lcnt + g, llist + (size_t)g * lcap, lcap};
    if constexpr (std::is_same<F, Fq2>::value)
      k_bucket_fixup_short_pair<<<grid_for(2 * (b1 - b0), 64), 64, 0, a>>>(bstart, bend, b0, b1, lg, part, buckets,
                                                                          g ? RED_PRIO : 0, ll);
    else if (g == 0)
      k_bucket_fixup_quad<F><<<grid_for(4 * (b1 - b0), 64), 64, 0, a>>>(bstart, bend, b0, b1, lg, part, buckets, ll);
    else
      k_bucket_fixup_short<F><<<grid_for(b1 - b0, 64), 64, 0, a>>>(bstart, bend, b0, b1, lg, part, buckets,
                                                                    RED_PRIO, ll);
    TPST_TRY(hipGetLastError());
    k_bucket_fixup_long<F><<<LONG_GRID, LONG_THREADS, 0, a>>>(bstart, bend, lg, part, buckets, ll);
    TPST_TRY(hipGetLastError());
    if (g == 0) break;
    if (red2_ok(nb))
      // lane form (fewer issue slots) for the groups with slack; the group
      // before the last keeps the quads: its tail ends right after the last
      // group's in a lone call
      TPST_TRY(reduce_buckets2<F>(ar, a, buckets + b0, (size_t)(whi - wlo), nb, win + wlo, RED_PRIO, g >= 2));
    else
      TPST_TRY(reduce_buckets<F>(ar, a, buckets + b0, (size_t)(whi - wlo), nb, win + wlo, RED_PRIO));
    k_window_chain<F><<<1, 64, 0, a>>>(win, wlo, whi, c, nullptr, 0, contrib + g);
    TPST_TRY(hipGetLastError());
    TPST_TRY(hipEventRecord(ar.aux_ev[2 * g + 1], a));
  }
  const int w1 = wb[1];  // group 0 = windows [0, w1)
  pf->begin(ST_REDUCE, t0);
#ifndef TPST_G0_RED2
#define TPST_G0_RED2 0  // 1: the two-level form for the last group (slower: 285-290 vs 295 Mscalar/s, a lone call 5.5 vs 5.1 ms, profiles/r06/ab_g0_red2.jsonl)
#endif
  // the last group's reduction is the call's tail: the two-level form (no
  // per-segment scalar multiplications; quads) or the short-segment one
  if (TPST_G0_RED2 && red2_ok(nb))
    TPST_TRY(reduce_buckets2<F>(ar, t0, buckets, (size_t)w1, nb, win, 0, false));
  else
    TPST_TRY(reduce_buckets<F>(ar, t0, buckets, (size_t)w1, nb, win));
  pf->end(ST_REDUCE, t0);
  pf->begin(ST_COMBINE, t0);
  for (int g = 1; g < NG; g++) TPST_TRY(hipStreamWaitEvent(t0, ar.aux_ev[2 * g + 1], 0));
  k_window_chain<F><<<1, 64, 0, t0>>>(win, 0, w1, c, contrib + 1, NG - 1, d_out);
  TPST_TRY(hipGetLastError());
  pf->end(ST_COMBINE, t0);
  return hipSuccess;
}

#ifndef TPST_MSM_G2_ONLY
hipError_t Arena::reserve(size_t bytes) {
  if (bytes <= cap) return hipSuccess;
  if (base) {
    hipError_t e = hipFree(base);
    if (e != hipSuccess) return e;
    base = nullptr;
    cap = 0;
  }
  size_t want = bytes + (bytes >> 3);
  hipError_t e = hipMalloc(&base, want);
  if (e != hipSuccess) return e;
  cap = want;
  return hipSuccess;
}

void Profiler::begin(int st, hipStream_t s) {
  if (!on) return;
  if (used[st] + 2 > ev[st].size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    ev[st].push_back(a);
    ev[st].push_back(b);
  }
  (void)hipEventRecord(ev[st][used[st]], s);
}

void Profiler::end(int st, hipStream_t s) {
  if (!on || used[st] + 2 > ev[st].size()) return;
  (void)hipEventRecord(ev[st][used[st] + 1], s);
  used[st] += 2;
}

void Profiler::collect() {
  for (int st = 0; st < N_STAGES; st++) {
    for (size_t i = 0; i + 1 < used[st]; i += 2) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ev[st][i], ev[st][i + 1]) == hipSuccess) {
        total_ms[st] += ms;
        count[st] += 1;
      }
    }
    used[st] = 0;
  }
}

void Profiler::reset() {
  for (int st = 0; st < N_STAGES; st++) {
    used[st] = 0;
    total_ms[st] = 0;
    count[st] = 0;
  }
}

Profiler::~Profiler() {
  for (auto& v : ev)
    for (auto e : v) (void)hipEventDestroy(e);
}

void Arena::release() {
  if (base) (void)hipFree(base);
  base = nullptr;
  cap = off = 0;
  if (aux_ready) {
    for (auto& st : aux) {
      (void)hipStreamSynchronize(st);
      if (!aux_from) (void)hipStreamDestroy(st);
      st = nullptr;
    }
    for (auto& e : aux_ev) {
      (void)hipEventDestroy(e);
      e = nullptr;
    }
    aux_ready = false;
  }
}

hipError_t Arena::aux_init() {
  if (aux_ready) return hipSuccess;
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
  if (aux_from) {
    TPST_TRY(aux_from->aux_init());
    for (int i = 0; i < N_AUX; i++) aux[i] = aux_from->aux[i];
  } else {
    for (auto& st : aux) TPST_TRY(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, greatest));
  }
  for (auto& e : aux_ev) TPST_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  aux_ready = true;
  return hipSuccess;
}

int msm_window_bits(size_t n) {
  // 16-bit signed windows are the sweet spot for ~2^18..2^22 points; smaller
  // inputs use smaller windows so buckets stay populated.
  int lg = bit_length(n ? n - 1 : 0);
  if (lg >= 20) return 16;
  if (lg >= 16) return 13;
  if (lg >= 12) return 10;
  if (lg >= 8) return 7;
  return 4;
}

int batch_window_bits(size_t N) {
  // rows of 1024 / 2048 scalars: 11-bit windows (2^20 commit 7.35 -> 7.05 ms
  // against 10; 12 -> 13 at 4096 was slower, 65.2 -> 65.8 ms:
  // profiles/r06/ab/ab_k1_window.txt)
  int lg = bit_length(N ? N - 1 : 0);
  if (lg >= 12) return 12;
  if (lg >= 10) return 11;
  if (lg >= 6) return 7;
  return 4;
}

// ------------------------------------------------------------------ K1 ---
// T[w][j] = 2^(c w) B_j, one thread per base
__global__ void __launch_bounds__(64, 1) k_build_tables(const uint32_t* __restrict__ bases, size_t N, int c, int W, uint32_t* __restrict__ table) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  G1A p = load_affine<Fq>(bases, j);
  for (int w = 0; w < W; w++) {
    store_rec29(table, (size_t)w * N + j, p);  // an infinity base stays all-zero: x = y = 0
    if (w + 1 < W) {
      Xyzz<Fq> x = to_xyzz(p);
      for (int i = 0; i < c; i++) x = dbl(x);
      p = to_affine(x);
    }
  }
}

hipError_t batch_tables_build(hipStream_t s, const uint32_t* d_bases, size_t N, int c, BatchTables& t) {
  batch_tables_free(t);
  t.N = N;
  t.c = c;
  t.W = num_windows(c);
  TPST_TRY(hipMalloc(&t.d_table, (size_t)t.W * N * REC29_WORDS * sizeof(uint32_t)));
  k_build_tables<<<grid_for(N, 64), 64, 0, s>>>(d_bases, N, c, t.W, t.d_table);
  return hipGetLastError();
}

void batch_tables_free(BatchTables& t) {
  if (t.d_table) (void)hipFree(t.d_table);
  t.d_table = nullptr;
  t.N = 0;
}

// an empty bucket of the row MSMs = infinity (ZZ = 0): written by the sort,
// which knows the empty ones (no memset of all buckets)
__device__ __forceinline__ void zero_bucket(uint4* zb, size_t key) {
  constexpr int Q = sizeof(Xyzz<Fq>) / 16;
#pragma unroll
  for (int i = 0; i < Q; i++) zb[key * Q + i] = make_uint4(0, 0, 0, 0);
}

// one workgroup per row: LDS counting sort of the row's N*W signed digits
// by bucket; writes the row's entries and bucket bounds.
__global__ void __launch_bounds__(256) k_batch_sort(const uint32_t* __restrict__ scalars, size_t rows, size_t N,
                                                    size_t row_stride, size_t col_stride, int c, int W,
                                                    uint32_t* __restrict__ keys, uint32_t* __restrict__ entries,
                                                    uint32_t* __restrict__ bstart, uint32_t* __restrict__ bend,
                                                    uint4* __restrict__ zb) {
  extern __shared__ uint32_t cnt[];  // nb counters
  // XCD-aware: consecutive rows on the same XCD (blocks b, b+8, ... share one)
  const size_t nblk = gridDim.x;
  size_t r = blockIdx.x;
  if (nblk % 8 == 0) r = (blockIdx.x % 8) * (nblk / 8) + blockIdx.x / 8;
  if (r >= rows) return;
  const uint32_t nb = 1u << (c - 1);
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  for (size_t j = threadIdx.x; j < N; j += blockDim.x) {
    uint32_t s[8];
    load_scalar(scalars + 8 * (r * row_stride + j * col_stride), s);
    uint32_t carry = 0;
    for (int w = 0; w < W; w++) {
      const int d = signed_digit(s, 8, w, c, W, carry);
      if (d) atomicAdd(&cnt[abs(d) - 1], 1u);
    }
  }
  __syncthreads();
  // exclusive scan of nb counters: thread t owns a contiguous slice
  __shared__ uint32_t part[256];
  __shared__ uint32_t total_sh;
  const uint32_t per = (nb + blockDim.x - 1) / blockDim.x;
  const uint32_t b0 = threadIdx.x * per;
  uint32_t local = 0;
  for (uint32_t b = b0; b < b0 + per && b < nb; b++) local += cnt[b];
  part[threadIdx.x] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (unsigned t = 0; t < blockDim.x; t++) {
      const uint32_t v = part[t];
      part[t] = run;
      run += v;
    }
    total_sh = run;
  }
  __syncthreads();
  const size_t rowbase = r * N * (size_t)W;
  uint32_t run = part[threadIdx.x];
  for (uint32_t b = b0; b < b0 + per && b < nb; b++) {
    const uint32_t v = cnt[b];
    if (!v) zero_bucket(zb, r * nb + b);
    bstart[r * nb + b] = (uint32_t)(rowbase + run);
    bend[r * nb + b] = (uint32_t)(rowbase + run + v);
    cnt[b] = run;
    run += v;
  }
  __syncthreads();
  for (size_t j = threadIdx.x; j < N; j += blockDim.x) {
    uint32_t s[8];
    load_scalar(scalars + 8 * (r * row_stride + j * col_stride), s);
    uint32_t carry = 0;
    for (int w = 0; w < W; w++) {
      const int d = signed_digit(s, 8, w, c, W, carry);
      if (d) {
        const uint32_t b = (uint32_t)abs(d) - 1;
        const uint32_t pos = atomicAdd(&cnt[b], 1u);
        keys[rowbase + pos] = (uint32_t)(r * nb + b);
        entries[rowbase + pos] = (uint32_t)(w * N + j) | (d < 0 ? 0x80000000u : 0u);
      }
    }
  }
  // zero digits leave the row's region short: pad it with the sentinel
  const uint32_t total = total_sh;
  const uint32_t sent = (uint32_t)(rows * nb);
  for (size_t e = total + threadIdx.x; e < N * (size_t)W; e += blockDim.x) keys[rowbase + e] = sent;
}

// Staged variant (N <= SB_THREADS * SB_SPT, nb <= SB_NB): one 1024-thread
// workgroup per row.  After the LDS counting pass and the scan, the row's
// output is produced in position ranges of at most SB_STAGE entries: a pass
// takes the buckets [b_lo, b_hi) whose entries fit the range, recomputes the
// row's signed digits (the scalars are L2-resident after the counting pass),
// scatters the pass's digits into LDS and flushes the range to global memory
// with consecutive (coalesced) stores.  The direct scatter of k_batch_sort
// writes every 4-byte key and entry to a random position of a ~720 KB row
// region while dozens of rows per XCD are in flight (far over the L2), so
// nearly every store was a partial-line write; here the row's keys and
// entries are written once, contiguously.  A bucket larger than the stage
// (degenerate scalars) is scattered directly in a pass of its own.
constexpr int SB_THREADS = 1024;
constexpr int SB_SPT = 4;                 // scalars per thread: N <= 4096
constexpr uint32_t SB_NB = 2048;          // buckets per row (c <= 12)
constexpr uint32_t SB_STAGE = 15 * 1024;  // staged entries per pass (120 KB)

// WC > 0 (c = CC, W = WC: the commit's row MSMs, 12 / 22 at 2^24 and 11 /
// 24 at 2^20): the window loop is unrolled, so every digit is a funnel shift
// at a constant bit offset; with a runtime W the offset is runtime and the
// word select a chain of conditional moves over the scalar's 8 words (x 7
// passes over every digit of the row; 2^20 sort 172 -> 95 us)
template <int WC, int CC = 12>
__global__ void __launch_bounds__(SB_THREADS) k_batch_sort_staged(const uint32_t* __restrict__ scalars, size_t rows,
                                                                 size_t N, size_t row_stride, size_t col_stride, int c,
                                                                 int W, uint32_t* __restrict__ keys,
                                                                 uint32_t* __restrict__ entries,
                                                                 uint32_t* __restrict__ bstart,
                                                                 uint32_t* __restrict__ bend,
                                                                 uint4* __restrict__ zb) {
  __shared__ uint32_t start[SB_NB + 1];
  __shared__ uint32_t cur[SB_NB];
  __shared__ uint2 stage[SB_STAGE];
  __shared__ uint32_t part[SB_THREADS / 64];
  __shared__ uint32_t pass_lo, pass_hi;
  const size_t nblk = gridDim.x;
  size_t r = blockIdx.x;
  if (nblk % 8 == 0) r = (blockIdx.x % 8) * (nblk / 8) + blockIdx.x / 8;  // XCD-aware, as k_batch_sort
  if (r >= rows) return;
  const uint32_t nb = 1u << (c - 1);
  const int tid = threadIdx.x;
  for (uint32_t b = tid; b < nb; b += SB_THREADS) cur[b] = 0;
  __syncthreads();
  for (int k = 0; k < SB_SPT; k++) {
    const size_t j = (size_t)tid + (size_t)k * SB_THREADS;
    if (j >= N) break;
    uint32_t sc[8];
    load_scalar(scalars + 8 * (r * row_stride + j * col_stride), sc);
    uint32_t carry = 0;
    if constexpr (WC > 0) {
#pragma unroll
      for (int w = 0; w < WC; w++) {
        const int d = signed_digit(sc, 8, w, CC, WC, carry);
        if (d) atomicAdd(&cur[abs(d) - 1], 1u);
      }
    } else {
      for (int w = 0; w < W; w++) {
        const int d = signed_digit(sc, 8, w, c, W, carry);
        if (d) atomicAdd(&cur[abs(d) - 1], 1u);
      }
    }
  }
  __syncthreads();
  // exclusive scan of the counts -> start[] (row-relative)
  {
    const uint32_t per = (nb + SB_THREADS - 1) / SB_THREADS;
    const uint32_t b0 = tid * per;
    uint32_t local = 0;
    for (uint32_t b = b0; b < b0 + per && b < nb; b++) local += cur[b];
    const int lane = tid & 63, wv = tid >> 6;
    uint32_t incl = local;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) part[wv] = incl;
    __syncthreads();
    if (tid == 0) {
      uint32_t run = 0;
      for (int i = 0; i < SB_THREADS / 64; i++) {
        const uint32_t v = part[i];
        part[i] = run;
        run += v;
      }
      start[nb] = run;
    }
    __syncthreads();
    uint32_t run = part[wv] + incl - local;
    for (uint32_t b = b0; b < b0 + per && b < nb; b++) {
      const uint32_t v = cur[b];
      start[b] = run;
      run += v;
    }
  }
  __syncthreads();
  const size_t rowbase = r * N * (size_t)W;
  for (uint32_t b = tid; b < nb; b += SB_THREADS) {
    if (start[b + 1] == start[b]) zero_bucket(zb, r * nb + b);
    bstart[r * nb + b] = (uint32_t)(rowbase + start[b]);
    bend[r * nb + b] = (uint32_t)(rowbase + start[b + 1]);
    cur[b] = start[b];
  }
  const uint32_t total = start[nb];
  if (tid == 0) pass_hi = 0;
  __syncthreads();
  for (;;) {
    // next pass: buckets [lo, hi) from the end of the previous one, as many
    // as fit the stage (at least one)
    if (tid == 0) {
      const uint32_t lo = pass_hi;
      uint32_t hi = lo;
      if (lo < nb) {
        const uint32_t lim = start[lo] + SB_STAGE;
        uint32_t a = lo + 1, z = nb;  // largest hi in (lo, nb] with start[hi] <= lim
        while (a < z) {
          const uint32_t m = (a + z + 1) >> 1;
          if (start[m] <= lim) a = m; else z = m - 1;
        }
        hi = a;
      }
      pass_lo = lo;
      pass_hi = hi;
    }
    __syncthreads();
    const uint32_t lo = pass_lo, hi = pass_hi;
    if (lo >= nb) break;
    const uint32_t p0 = start[lo], cnt = start[hi] - p0;
    const bool direct = cnt > SB_STAGE;  // one oversized bucket
    auto place = [&](int d, int w, size_t j) {
      if (!d) return;
      const uint32_t b = (uint32_t)abs(d) - 1;
      if (b < lo || b >= hi) return;
      const uint32_t pos = atomicAdd(&cur[b], 1u);
      const uint2 e = make_uint2((uint32_t)(r * nb + b), (uint32_t)(w * N + j) | (d < 0 ? 0x80000000u : 0u));
      if (direct) {
        keys[rowbase + pos] = e.x;
        entries[rowbase + pos] = e.y;
      } else {
        stage[pos - p0] = e;
      }
    };
    for (int k = 0; k < SB_SPT; k++) {
      const size_t j = (size_t)tid + (size_t)k * SB_THREADS;
      if (j >= N) break;
      uint32_t sc[8];
      load_scalar(scalars + 8 * (r * row_stride + j * col_stride), sc);
      uint32_t carry = 0;
      if constexpr (WC > 0) {
#pragma unroll
        for (int w = 0; w < WC; w++) place(signed_digit(sc, 8, w, CC, WC, carry), w, j);
      } else {
        for (int w = 0; w < W; w++) place(signed_digit(sc, 8, w, c, W, carry), w, j);
      }
    }
    __syncthreads();
    if (!direct) {
      for (uint32_t i = tid; i < cnt; i += SB_THREADS) {
        const uint2 e = stage[i];
        keys[rowbase + p0 + i] = e.x;
        entries[rowbase + p0 + i] = e.y;
      }
    }
    __syncthreads();
  }
  // zero digits leave the row's region short: pad it with the sentinel
  const uint32_t sent = (uint32_t)(rows * nb);
  for (size_t e = total + tid; e < N * (size_t)W; e += SB_THREADS) keys[rowbase + e] = sent;
}

hipError_t msm_batch(Arena& ar, hipStream_t s, const BatchTables& t, const uint32_t* d_scalars, size_t rows,
                     size_t row_stride, size_t col_stride, Xyzz<Fq>* d_out) {
  if (rows == 0) return hipSuccess;
    const int c = t.c, W = t.W;
  const size_t N = t.N;
  const uint32_t nb = 1u << (c - 1);
  const size_t m = rows * N * (size_t)W;
  if (m >= (1ull << 32)) return hipErrorInvalidValue;  // entry offsets are u32
  const size_t nbk = rows * nb;
  // chunk length: at least 4 waves of chunks per SIMD (TPST_K1_WAVES; the
  // 2^20 commit's 26.6 M entries take 64-entry chunks, measured 8.7 -> 8.4 ms
  // against the 32-entry chunks 8 waves per SIMD would give)
  static const size_t k1_threads = (size_t)4 * 64 * device_simds();
  int lg = 5;
  while (lg < 8 && (m >> (lg + 1)) >= k1_threads) lg++;
  const size_t nchunk = (m + ((size_t)1 << lg) - 1) >> lg;
  const size_t nblk = (nchunk + ACC_BLOCK - 1) / ACC_BLOCK;
  size_t need = 2 * Arena::need(m, 4) + 2 * Arena::need(nbk, 4) + Arena::need(nbk, sizeof(Xyzz<Fq>)) +
                Arena::need(nchunk, sizeof(Xyzz<Fq>)) + Arena::need(nblk, sizeof(Xyzz<Fq>)) +
                reduce_scratch<Fq>(rows, nb) + (red2_ok(nb) ? reduce2_scratch<Fq>(rows, nb) : 0) + 4096;
  ar.reset();
  TPST_TRY(ar.reserve(need));
  uint32_t* keys = ar.take<uint32_t>(m);
  uint32_t* entries = ar.take<uint32_t>(m);
  Xyzz<Fq>* part = ar.take<Xyzz<Fq>>(nchunk);
  Xyzz<Fq>* bpart = ar.take<Xyzz<Fq>>(nblk);
  uint32_t* bstart = ar.take<uint32_t>(nbk);
  uint32_t* bend = ar.take<uint32_t>(nbk);
  Xyzz<Fq>* buckets = ar.take<Xyzz<Fq>>(nbk);
  const unsigned nrow_blk = (unsigned)rows;
  Profiler* pf = ar.prof;
  Profiler dummy;
  if (!pf) pf = &dummy;
  pf->begin(ST_BATCH_SORT, s);
  if (N <= (size_t)SB_THREADS * SB_SPT && c == 12 && W == 22)
    k_batch_sort_staged<22, 12><<<nrow_blk, SB_THREADS, 0, s>>>(d_scalars, rows, N, row_stride, col_stride, c, W, keys,
                                                                 entries, bstart, bend, reinterpret_cast<uint4*>(buckets));
  else if (N <= (size_t)SB_THREADS * SB_SPT && c == 11 && W == 24)
    k_batch_sort_staged<24, 11><<<nrow_blk, SB_THREADS, 0, s>>>(d_scalars, rows, N, row_stride, col_stride, c, W, keys,
                                                                 entries, bstart, bend, reinterpret_cast<uint4*>(buckets));
  else if (N <= (size_t)SB_THREADS * SB_SPT && nb <= SB_NB)
    k_batch_sort_staged<0><<<nrow_blk, SB_THREADS, 0, s>>>(d_scalars, rows, N, row_stride, col_stride, c, W, keys,
                                                            entries, bstart, bend, reinterpret_cast<uint4*>(buckets));
  else
    k_batch_sort<<<nrow_blk, 256, nb * sizeof(uint32_t), s>>>(d_scalars, rows, N, row_stride, col_stride, c, W, keys,
                                                          entries, bstart, bend, reinterpret_cast<uint4*>(buckets));
  TPST_TRY(hipGetLastError());
  pf->end(ST_BATCH_SORT, s);
  pf->begin(ST_BUCKET_ACC, s);
  // the LDS-staged gathers (2^24 commit 68.7-69.3 -> 68.6-68.8 ms against
  // k_bucket_acc_chunk<Fq, 2, true>'s register prefetch, profiles/r05/l)
  k_bucket_acc_chunk_lds<TPST_K1_MINW><<<(unsigned)nblk, ACC_BLOCK, 0, s>>>(keys, entries, m, nullptr, (uint32_t)nbk, bstart, bend,
                                                                  t.d_table, lg, buckets, part, bpart);
  TPST_TRY(hipGetLastError());
  k_bucket_fixup<Fq><<<grid_for(nblk, 64), 64, 0, s>>>(keys, m, nullptr, (uint32_t)nbk, bstart, bend, lg, nblk,
                                                       part, bpart, buckets);
  TPST_TRY(hipGetLastError());
  pf->end(ST_BUCKET_ACC, s);
  pf->begin(ST_REDUCE, s);
  // the two-level reduction (no per-segment scalar multiplications; 2^20
  // commit 8.7 -> 8.2 ms, 2^24 unchanged)
  if (red2_ok(nb))
    TPST_TRY(reduce_buckets2<Fq>(ar, s, buckets, rows, nb, d_out, 0));
  else
    TPST_TRY(reduce_buckets<Fq>(ar, s, buckets, rows, nb, d_out));
  pf->end(ST_REDUCE, s);
  return hipSuccess;
}

// explicit instantiations (G1)
template hipError_t msm_var<Fq>(Arena&, hipStream_t, const uint32_t*, const uint32_t*, size_t, Xyzz<Fq>*, hipStream_t,
                                bool*, hipStream_t);
template hipError_t points_to_mont<Fq>(hipStream_t, const uint32_t*, uint32_t*, size_t);
template hipError_t affine_from_mont<Fq>(hipStream_t, const uint32_t*, uint32_t*, size_t);
template hipError_t xyzz_to_affine_canonical<Fq>(hipStream_t, const Xyzz<Fq>*, uint32_t*, size_t);
#else
// explicit instantiations (G2)
template hipError_t msm_var<Fq2>(Arena&, hipStream_t, const uint32_t*, const uint32_t*, size_t, Xyzz<Fq2>*,
                                 hipStream_t, bool*, hipStream_t);
template hipError_t points_to_mont<Fq2>(hipStream_t, const uint32_t*, uint32_t*, size_t);
template hipError_t affine_from_mont<Fq2>(hipStream_t, const uint32_t*, uint32_t*, size_t);
template hipError_t xyzz_to_affine_canonical<Fq2>(hipStream_t, const Xyzz<Fq2>*, uint32_t*, size_t);
#endif
#endif  // TPST_MSM_LAB

}  // namespace tpst
