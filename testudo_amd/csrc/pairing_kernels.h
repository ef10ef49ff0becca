// Host-side API of pairing.hip (K4): batched multi-Miller loop, Fq12 tree
// product and final exponentiation on the device.
#pragma once
#include <hip/hip_runtime.h>
#include "msm.h"
#include "pairing.h"

namespace tpst {

// G2Prepared for n points: coeffs laid out coefficient-major,
// d_coeffs[idx * n + i] (idx < 69).  Infinity points get no use (the Miller
// kernel skips pairs whose G1 or G2 point is infinity).
// scratch: g2_prepare_scratch(n) bytes for the RNS engine's residue lines
// (nullptr: the radix engine)
size_t g2_prepare_scratch(size_t n);
hipError_t g2_prepare_batch(hipStream_t s, const uint32_t* d_g2, size_t n, LineCoeff* d_coeffs,
                            uint32_t* scratch = nullptr);

// groups x n pairs -> groups GT elements (after final exponentiation).
// d_g1: groups*n affine G1 (Montgomery); d_coeffs: prepared G2 of the same
// pairs, coefficient-major with row length groups*n; d_g2 only for the
// infinity test.  Output Montgomery Fq12 per group.
// final_exp = false: the Miller-loop product of each group only (unreduced GT
// partial of a row-sharded IPP, finished by gt_product_final).  Scratch from
// `ar`: multi_pairing_scratch(groups, n) bytes.
// map_s != 0 (MIPP cross pairings, groups = 2, n = H map_s with H in {1, 2}):
// pair k of group g uses column j = (k / map_s) 2 map_s + (g ? 0 : map_s) +
// k % map_s of d_g1 / d_g2 / d_coeffs (row length groups * n), i.e. group 0
// pairs the upper half of every 2 map_s block of prepared G2 points, group 1
// the lower half -- t_l / t_r of mipp.rs:87-94 against an unswapped h.
// rot_L != 0: d_g1 is XYZZ (Montgomery) and column j's G1 point is
// d_g1[(j / rot_L) rot_L + ((j % rot_L) + rot_L / 2) % rot_L] (the MIPP
// rotation); the pairing is computed without normalising it (its lines are
// scaled by an Fq factor that the final exponentiation removes, so with
// final_exp = false the partial differs from the affine one by such a factor).
hipError_t multi_pairing_prepared(Arena& ar, hipStream_t s, const uint32_t* d_g1, const uint32_t* d_g2,
                                  const LineCoeff* d_coeffs, size_t groups, size_t n, Fq12* d_out,
                                  bool final_exp = true, size_t map_s = 0, size_t rot_L = 0);
size_t multi_pairing_scratch(size_t groups, size_t n);

// groups x n Montgomery Fq12 partials -> groups final-exponentiated products
// (uses `ar` for the tree levels, <= multi_pairing_scratch(groups, n))
hipError_t gt_product_final(Arena& ar, hipStream_t s, const Fq12* d_partials, size_t groups, size_t n, Fq12* d_out);

// convenience: prepare + pair
hipError_t multi_pairing(Arena& ar, hipStream_t s, const uint32_t* d_g1, const uint32_t* d_g2, size_t groups,
                         size_t n, Fq12* d_out);

// GT exponentiations (verifier): out[i] = base[i]^e_i with e_i given by its
// base-x digits (4 x u64, e = sum_j digits[4 i + j] x^j) after a GT membership
// test of base[i]; ok[i] = 1 iff base[i] is in GT.  Montgomery Fq12.
hipError_t gt_pow_wave(hipStream_t s, const Fq12* d_base, const uint64_t* d_digits, size_t n, Fq12* d_out,
                       uint32_t* d_ok);

// MIPP look-ahead (tpst_poly_open): the 8 pairing products of round-r vectors
// (pairing.hip, groups A0 A3 A1 A2 B0 B3 B1 B2) into d_out8 (Montgomery);
// d_g1 affine (xyzz = false, E = 1) or the fold's E XYZZ sets f_j a (xyzz =
// true), paired against an earlier round's prepared h of row length
// ncol = E len (E = 1, 2, 4, 8).  Scratch: mipp_lookahead_scratch(len / 4, E).
size_t mipp_lookahead_scratch(size_t sp, int E);
// final_exp = false: the 8 unreduced Miller products (a rank's partials of
// the row-sharded opening, combined by gt_prod_final)
hipError_t mipp_lookahead(Arena& ar, hipStream_t s, const LineCoeff* d_coeffs, size_t ncol, const uint32_t* d_g2,
                          const uint32_t* d_g1, bool xyzz, size_t len, int E, Fq12* d_out8, bool final_exp = true);
// out[g] = FE(prod_{w < W} parts[w G + g]) for gathered Montgomery Miller
// partials (W ranks x G groups), RNS engine
hipError_t gt_prod_final(hipStream_t s, const Fq12* d_parts, size_t W, size_t G, Fq12* d_out);
// round r+1's cross terms from the look-ahead products and c = c_r:
// t_l = A0 A3 A1^(c^-1) A2^c, t_r = B0 B3 B1^(c^-1) B2^c.  d_digits: base-x
// digits of (c^-1, c, c^-1, c) (4 x 4 u64); d_la8 is overwritten.
hipError_t mipp_combine(hipStream_t s, Fq12* d_la8, const uint64_t* d_digits, Fq12* d_out2);
// the same combination from squaring tables built off the critical path:
// mipp_sq_tables right after the look-ahead (d_tab: 4 x 64 Fq12, d_G: 2 x 10
// Fq12 product lists, A0 A3 / B0 B3 copied in), then once c is known
// mipp_combine_tab (d_mid: 2 x 3 Fq12 scratch) -> d_out2 = (t_l, t_r)
hipError_t mipp_sq_tables(hipStream_t s, const Fq12* d_la8, Fq12* d_tab, Fq12* d_G);
// bytes per table / partial entry of either engine (d_tab: 4 x 64, d_G: 2 x 10,
// d_mid: 128 entries of this size; the RNS engine keeps them in residue form)
constexpr size_t MIPP_TAB_F12_BYTES = 12 * 32 * 4;
hipError_t mipp_combine_tab(hipStream_t s, const Fq12* d_tab, const uint64_t* d_digits, Fq12* d_G, Fq12* d_mid,
                            Fq12* d_out2);

hipError_t fq12_from_mont(hipStream_t s, const Fq12* d_in, uint32_t* d_out, size_t n);

}  // namespace tpst
