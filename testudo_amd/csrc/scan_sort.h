// Hand-written device scan and stable key-value sort for the R1CS instance
// paths (r1cs.hip: CSR / CSC construction, SPARK memory-checking timestamps),
// replacing the library primitives those paths used.
//
//   scan_excl_u32      exclusive prefix sums of n u32 (n < 2^26): per-block
//                      totals, one block scanning the totals, per-block apply
//   stable_sort_pairs  LSD radix sort of (key, value) u32 pairs by the low
//                      key_bits bits, 8-bit digits, each pass a stable
//                      counting sort: tile histograms (digit-major, so one
//                      flat exclusive scan gives every (digit, tile) its first
//                      slot) and a scatter that ranks equal digits in input
//                      order -- inside a wave by an 8-ballot match, across the
//                      tile's waves and its 8 slices through LDS counters
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tpst {
namespace scan_sort {

constexpr int SCAN_THREADS = 256, SCAN_ITEMS = 16, SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;
constexpr int SORT_THREADS = 256, SORT_SLICES = 8, SORT_TILE = SORT_THREADS * SORT_SLICES;
constexpr int DIGIT_BITS = 8, DIGITS = 1 << DIGIT_BITS;

// exclusive scan of v over the block; returns the block total
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* sh, uint32_t& excl) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
    if (k < w) before += sh[k];
    total += sh[k];
  }
  __syncthreads();
  excl = before + incl - v;
  return total;
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_totals(const uint32_t* __restrict__ in, size_t n,
                                                             uint32_t* __restrict__ tot) {
  __shared__ uint32_t sh[SCAN_THREADS / 64];
  const size_t b0 = (size_t)blockIdx.x * SCAN_TILE;
  uint32_t s = 0;
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const size_t i = b0 + (size_t)k * SCAN_THREADS + threadIdx.x;
    if (i < n) s += in[i];
  }
  uint32_t ex;
  const uint32_t total = block_excl(s, sh, ex);
  if (threadIdx.x == 0) tot[blockIdx.x] = total;
}

// one block: exclusive scan of the nb <= 1024 * 16 block totals in place
__global__ void __launch_bounds__(1024) k_scan_block_totals(uint32_t* __restrict__ tot, uint32_t nb) {
  __shared__ uint32_t sh[1024 / 64];
  const uint32_t per = (nb + 1023) / 1024, b0 = threadIdx.x * per;
  uint32_t s = 0;
  for (uint32_t k = 0; k < per; k++)
    if (b0 + k < nb) s += tot[b0 + k];
  uint32_t ex;
  block_excl(s, sh, ex);
  for (uint32_t k = 0; k < per; k++)
    if (b0 + k < nb) {
      const uint32_t v = tot[b0 + k];
      tot[b0 + k] = ex;
      ex += v;
    }
}

// each thread scans SCAN_ITEMS consecutive elements of its block's tile
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_apply(const uint32_t* __restrict__ in, size_t n,
                                                            const uint32_t* __restrict__ tot,
                                                            uint32_t* __restrict__ out) {
  __shared__ uint32_t sh[SCAN_THREADS / 64];
  const size_t i0 = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS], s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    v[k] = i0 + k < n ? in[i0 + k] : 0u;
    s += v[k];
  }
  uint32_t ex;
  block_excl(s, sh, ex);
  ex += tot[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++)
    if (i0 + k < n) {
      out[i0 + k] = ex;
      ex += v[k];
    }
}

// scratch: (n + SCAN_TILE - 1) / SCAN_TILE u32; in == out allowed
inline size_t scan_scratch(size_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }

inline hipError_t scan_excl_u32(hipStream_t s, const uint32_t* in, uint32_t* out, size_t n, uint32_t* scratch) {
  if (!n) return hipSuccess;
  const size_t nb = scan_scratch(n);
  if (nb > 1024 * 16) return hipErrorInvalidValue;
  k_scan_totals<<<(unsigned)nb, SCAN_THREADS, 0, s>>>(in, n, scratch);
  k_scan_block_totals<<<1, 1024, 0, s>>>(scratch, (uint32_t)nb);
  k_scan_apply<<<(unsigned)nb, SCAN_THREADS, 0, s>>>(in, n, scratch, out);
  return hipGetLastError();
}

// ------------------------------------------------------- stable LSD sort --
// item (k, t) of a tile = element tile_base + k * SORT_THREADS + t: the input
// order is slice-major, thread-minor, which is the order ranks are assigned in
__global__ void __launch_bounds__(SORT_THREADS) k_radix_hist(const uint32_t* __restrict__ keys, size_t n, int sh,
                                                            uint32_t ntile, uint32_t* __restrict__ hist) {
  __shared__ uint32_t cnt[DIGITS];
  cnt[threadIdx.x] = 0;  // SORT_THREADS == DIGITS
  __syncthreads();
  const size_t b0 = (size_t)blockIdx.x * SORT_TILE;
  for (int k = 0; k < SORT_SLICES; k++) {
    const size_t i = b0 + (size_t)k * SORT_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(keys[i] >> sh) & (DIGITS - 1)], 1u);
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * ntile + blockIdx.x] = cnt[threadIdx.x];  // digit-major
}

__global__ void __launch_bounds__(SORT_THREADS) k_radix_scatter(const uint32_t* __restrict__ keys,
                                                               const uint32_t* __restrict__ vals, size_t n, int sh,
                                                               uint32_t ntile, const uint32_t* __restrict__ off,
                                                               uint32_t* __restrict__ keys_out,
                                                               uint32_t* __restrict__ vals_out) {
  constexpr int NW = SORT_THREADS / 64;
  __shared__ uint32_t base[DIGITS];       // this tile's next slot per digit
  __shared__ uint32_t wcnt[NW][DIGITS];   // the slice's count per wave and digit
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  base[t] = off[(size_t)t * ntile + blockIdx.x];
#pragma unroll
  for (int k = 0; k < NW; k++) wcnt[k][t] = 0;
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const size_t b0 = (size_t)blockIdx.x * SORT_TILE;
  for (int k = 0; k < SORT_SLICES; k++) {
    const size_t i = b0 + (size_t)k * SORT_THREADS + t;
    const bool valid = i < n;
    const uint32_t key = valid ? keys[i] : 0u;
    const uint32_t val = valid ? vals[i] : 0u;
    // 9-bit tag: invalid items never match a digit
    const uint32_t tag = valid ? ((key >> sh) & (DIGITS - 1)) : (uint32_t)DIGITS;
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b <= DIGIT_BITS; b++) {
      const uint64_t bal = __ballot((tag >> b) & 1u);
      peers &= ((tag >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t rank_w = (uint32_t)__popcll(peers & lt);
    const bool leader = rank_w == 0;
    if (valid && leader) wcnt[w][tag] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t before = base[tag];
      for (int q = 0; q < w; q++) before += wcnt[q][tag];
      const size_t dst = before + rank_w;
      keys_out[dst] = key;
      vals_out[dst] = val;
    }
    __syncthreads();
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < NW; q++) {
      sum += wcnt[q][t];
      wcnt[q][t] = 0;
    }
    base[t] += sum;
    __syncthreads();
  }
}

// scratch u32 words for stable_sort_pairs of n items
inline size_t sort_scratch(size_t n) {
  const size_t ntile = (n + SORT_TILE - 1) / SORT_TILE;
  return 2 * n + DIGITS * ntile + scan_scratch(DIGITS * ntile) + 64;
}

// stable sort of (keys, vals) by the low key_bits bits into (keys_out, vals_out)
inline hipError_t stable_sort_pairs(hipStream_t s, const uint32_t* keys, const uint32_t* vals, uint32_t* keys_out,
                                    uint32_t* vals_out, size_t n, int key_bits, uint32_t* scratch) {
  if (!n) return hipSuccess;
  const uint32_t ntile = (uint32_t)((n + SORT_TILE - 1) / SORT_TILE);
  uint32_t* tk = scratch;
  uint32_t* tv = tk + n;
  uint32_t* hist = tv + n;
  uint32_t* sc = hist + (size_t)DIGITS * ntile;
  const int passes = key_bits <= 0 ? 1 : (key_bits + DIGIT_BITS - 1) / DIGIT_BITS;
  // ping-pong so the last pass lands in (keys_out, vals_out)
  const uint32_t* ik = keys;
  const uint32_t* iv = vals;
  for (int p = 0; p < passes; p++) {
    const bool last = p + 1 == passes;
    uint32_t* ok = ((passes - 1 - p) & 1) ? tk : keys_out;
    uint32_t* ov = ((passes - 1 - p) & 1) ? tv : vals_out;
    if (last) {
      ok = keys_out;
      ov = vals_out;
    }
    k_radix_hist<<<ntile, SORT_THREADS, 0, s>>>(ik, n, p * DIGIT_BITS, ntile, hist);
    hipError_t e = scan_excl_u32(s, hist, hist, (size_t)DIGITS * ntile, sc);
    if (e != hipSuccess) return e;
    k_radix_scatter<<<ntile, SORT_THREADS, 0, s>>>(ik, iv, n, p * DIGIT_BITS, ntile, hist, ok, ov);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    ik = ok;
    iv = ov;
  }
  return hipSuccess;
}

}  // namespace scan_sort
}  // namespace tpst
