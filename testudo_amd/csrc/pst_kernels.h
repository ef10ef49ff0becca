// Device kernels for the sqrt-PST protocol layer (pst.hip): Fr vector
// kernels (chi tables, get_q mat-vec, PST quotient recurrence, MIPP y fold),
// MIPP compress (fixed-scalar point folds) and SRS generation.
#pragma once
#include <hip/hip_runtime.h>
#include "msm.h"
#include "pairing_kernels.h"

namespace tpst {

// canonical <-> Montgomery Fr vectors (8 u32 each)
hipError_t fr_to_mont(hipStream_t s, const uint32_t* in, uint32_t* out, size_t n);
hipError_t fr_from_mont(hipStream_t s, const uint32_t* in, uint32_t* out, size_t n);

// out[i] = chi_i(b) = prod_j (bit (m-1-j) of i ? b_j : 1-b_j), b Montgomery (sqrt_pst.rs:152-166)
hipError_t chi_table(hipStream_t s, const uint32_t* d_b, int m, uint32_t* d_out);

// q[j] = sum_i Z[(j << m_col) | i] * chis[i]  (sqrt_pst.rs:93-96); Z canonical, chis/q Montgomery
hipError_t get_q(hipStream_t s, const uint32_t* d_Z, int m_col, int m_row, const uint32_t* d_chis, uint32_t* d_q);
// a row shard's share of q: out[j] = sum_{i < nr} Z[j cs + i] chis[i] (canonical out)
hipError_t get_q_rows(hipStream_t s, const uint32_t* d_Z, size_t cs, size_t nr, int m_row, const uint32_t* d_chis,
                      uint32_t* d_q_canonical);
// the combine of the shares: out = sum of k canonical Fr vectors of length n, mod r
hipError_t fr_sum_parts(hipStream_t s, const uint32_t* d_parts, size_t k, size_t n, uint32_t* d_out);

// v = sum_j x[j] * y[j] (Montgomery), one value
hipError_t fr_dot(hipStream_t s, const uint32_t* d_x, const uint32_t* d_y, size_t n, uint32_t* d_v);

// PST open step: from r (2h, Montgomery) and pt (Montgomery
// scalar at d_pt): q_can[b] = canonical(r[2b+1]-r[2b]), r_next[b] = r[2b](1-pt)+r[2b+1]pt
hipError_t pst_step(hipStream_t s, const uint32_t* d_r, size_t half, const uint32_t* d_pt, uint32_t* d_qcan,
                    uint32_t* d_rnext);

// MIPP compress (mipp.rs:354-383): v[i] = v[i] + k * v[i+split] for i < split;
// k is a canonical Fr at d_k.  In place; points stay affine Montgomery.
template <class F>
hipError_t compress_points(hipStream_t s, uint32_t* d_v, size_t split, const uint32_t* d_k);
hipError_t compress_fr(hipStream_t s, uint32_t* d_y, size_t split, const uint32_t* d_kmont);

// MIPP scalars over the original bases (Montgomery W, y; canonical out):
// y == nullptr: out[k] = W[k / len]; else out[k] = W[k / len] * y[(k % len + split) % len].
// sub / off: n scalars of the bases k = sub kl + off only (out[kl]; a rank's
// rows of the row-sharded opening)
hipError_t mipp_scalars(hipStream_t s, const uint32_t* d_W, const uint32_t* d_y, size_t len, size_t split, size_t n,
                        uint32_t* d_out, size_t sub = 1, size_t off = 0);
// E fold sets: out[j n + kl] = canonical(W[k / len] * f[j]), k = sub kl + off (Montgomery W, f)
hipError_t mipp_scalar_sets(hipStream_t s, const uint32_t* d_W, const uint32_t* d_f, int E, size_t len, size_t n,
                            uint32_t* d_out, size_t sub = 1, size_t off = 0);
// out[g] = sum_{w < W} parts[w G + g]: gathered per-rank XYZZ partials -> sums
hipError_t xyzz_sum_groups(hipStream_t s, const Xyzz<Fq>* d_parts, size_t W, size_t G, Xyzz<Fq>* d_out);
// round r's fold weights W_r / Wi_r (2^r Montgomery Fr at offset 2^r - 1) from
// round r-1's and its challenge c (and c^-1), both Montgomery Fr on the device
hipError_t mipp_weights(hipStream_t s, uint32_t* d_W, uint32_t* d_Wi, int r, const uint32_t* d_c,
                        const uint32_t* d_cinv);

// out[i] = k_i * P for a fixed affine (Montgomery) point P at d_p; scalars canonical
template <class F>
hipError_t fixed_base_mul(hipStream_t s, const uint32_t* d_p, const uint32_t* d_scalars, size_t n, uint32_t* d_out);

// pair sums for the halved PST-open MSM: out[b] = in[2b] + in[2b+1] (affine)
template <class F>
hipError_t pair_sum(hipStream_t s, const uint32_t* d_in, size_t half, uint32_t* d_out);

// batch XYZZ -> affine (Montgomery)
template <class F>
hipError_t xyzz_to_affine_mont(hipStream_t s, const Xyzz<F>* d_in, uint32_t* d_out, size_t n);

// affine rotation by half: out[j] = in[(j + n/2) % n], `words` u32 per point
hipError_t affine_rot(hipStream_t s, const uint32_t* d_in, uint32_t* d_out, size_t n, size_t words);

}  // namespace tpst
