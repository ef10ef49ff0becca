// Fixed-base lookup tables and grouped fixed-base MSMs (host API of fbt.hip).
//
// For a base vector that stays fixed across many MSMs (SRS levels, the row
// commitments of one opening, powers_of_h) the doublings of Pippenger's
// window combination are paid once: entry (k, w, m) of the table is
// (m+1) * 2^(4w) * B_k (affine, Montgomery), w < 64, m < 8.  An MSM is then a
// sum of one signed lookup per (base, window) -- 64 mixed additions per
// scalar, no doublings and no bucket sort -- reduced by a segmented tree.
// This turns the latency-bound small MSMs of the opening (MIPP folding, the
// PST level proofs) from ~250 serial doublings into ~20 serial additions.
#pragma once
#include "device_util.h"
#include "msm.h"

namespace tpst {

constexpr int FBT_C = 4;   // window bits (signed digits in [-8, 8])
constexpr int FBT_W = 64;  // windows: 64 * 4 >= 253 + carry
constexpr int FBT_M = 8;   // multiples per window
constexpr int FBT_WG = 32;  // GLV tables (G1): windows of the two 127-bit halves

template <class F>
constexpr size_t fbt_entries(size_t n) { return n * FBT_W * FBT_M; }
template <class F>
constexpr size_t fbt_words(size_t n) { return fbt_entries<F>(n) * 2 * Words<F>::n; }

// Build the table of n affine Montgomery bases into d_table (fbt_words(n) u32).
// glv (G1 only): windows w < 32 only -- a scalar is split k = k1 + lambda k2
// (both < 2^127) and k2's digits look up phi(T) = (beta x, y) = lambda T, so
// the same 64 lookups per scalar need half the table and half the doublings.
template <class F>
hipError_t fbt_build(Arena& ar, hipStream_t s, const uint32_t* d_bases, size_t n, uint32_t* d_table,
                     bool glv = false);

// Grouped fixed-base MSM: out[g] = sum_{k in group g} S_k * B_k, S canonical
// Fr indexed by base.  Membership:
//   strided  (d_seg == nullptr): k(g, m) = (m / D) L + g D + m % D,
//            g < L / D, m < (n / L) D   -- MIPP folds (D = 1) and cross
//            products (D = L / 2), a plain MSM is L = D = n;
//   segments (d_seg != nullptr): k = seg[g] + m, m < seg[g+1] - seg[g].
// sets > 1: the same groups again for each of `sets` scalar vectors (set q
// reads S at d_scalars + 8 q set_stride), out[q groups + g].
struct FbGroups {
  size_t groups = 1;
  size_t members = 0;  // per group (max over groups for segments)
  size_t L = 1, D = 1;
  const uint32_t* d_seg = nullptr;
  size_t sets = 1, set_stride = 0;
  bool glv = false;  // the table was built with glv = true
};

template <class F>
hipError_t fbt_msm(Arena& ar, hipStream_t s, const uint32_t* d_table, const uint32_t* d_scalars, const FbGroups& g,
                   Xyzz<F>* d_out);

}  // namespace tpst
