// K4: optimal-ate multi-pairing on gfx950.
//
// Layout: prepared line coefficients are coefficient-major (all pairs' step
// idx coefficients contiguous) so the line evaluation's loads are coalesced
// across threads.  The Miller loop itself is restructured as a product of
// per-bit line products (see "multi-pairing by line products" below).
#include "device_util.h"
#include "pairing_kernels.h"
#include "wave_tower.h"
#include "rns_engine.h"
#include "inv_wave.h"
#include <cstdlib>

namespace tpst {

#define TPST_TRY(x)                  \
  do {                               \
    hipError_t _e = (x);             \
    if (_e != hipSuccess) return _e; \
  } while (0)

static inline unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

// ---- G2Prepared on the RNS engine ------------------------------------------
// The doubling / addition chain of pairing.h per G2 point (one 44-slot region
// per point, the two halves of a 12-wave workgroup holding two points):
// G2_DBL1-4 / G2_ADD1-4 (tools/gen_rns_ops.py) as RNS stages,
// each step's line (region slots 6..11) dumped in residue form, then
// k_rns_to_fq converts every coefficient to field.h form in bulk -- ~280
// stages of ~1 us against the radix engine's ~6 us stages.
__global__ void __launch_bounds__(768, 2) k_g2_prepare_rns(const uint32_t* __restrict__ g2, size_t n,
                                                           uint32_t* __restrict__ lres) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 44) * rns::SLOT];
  __shared__ uint32_t s_xch[12 * rns::XCH];
  __shared__ uint32_t s_rows[2 * rns::NB * 32];
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::LaneL L = rns::load_lane_lds((rns::lds_t*)s_rows);
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  const int w = rns::wave_id(), lane = threadIdx.x & 63;
  const size_t p0 = 2 * (size_t)blockIdx.x, p1 = p0 + 1 < n ? p0 + 1 : p0;
  const int R = rns::N_CONSTS;
  __syncthreads();
  // x, y (and the copy of Q at 26..29); z = 1
  const Fq* q0 = reinterpret_cast<const Fq*>(g2 + p0 * 48);
  const Fq* q1 = reinterpret_cast<const Fq*>(g2 + p1 * 48);
  rns::load(e, L, q0, q1, R, 4);
  if (w < 4) e.slots[(R + 26 + w) * rns::SLOT + lane] = e.slots[(R + w) * rns::SLOT + lane];
  if (w == 4) e.slots[(R + 4) * rns::SLOT + lane] = e.slots[e.kon * rns::SLOT + lane];
  if (w == 5) e.slots[(R + 5) * rns::SLOT + lane] = 0;
  __syncthreads();
  const size_t p = (lane & 32) ? p1 : p0;
  size_t idx = 0;
  auto dump = [&]() {  // line (c0, c1, c2) of step idx
    if (w < 6) lres[((idx * n + p) * 6 + w) * 32 + (lane & 31)] = e.slots[(R + 6 + w) * rns::SLOT + lane];
    __syncthreads();
    idx++;
  };
  for (int b = X_BITS - 2; b >= 0; b--) {
    rns::stage<rns::OP_G2_DBL1, rns::OP_RW[rns::OP_G2_DBL1] != 0>(e, L, R, R, R);
    rns::stage<rns::OP_G2_DBL2, rns::OP_RW[rns::OP_G2_DBL2] != 0>(e, L, R, R, R);
    rns::stage<rns::OP_G2_DBL3, rns::OP_RW[rns::OP_G2_DBL3] != 0>(e, L, R, R, R);
    rns::stage<rns::OP_G2_DBL4, rns::OP_RW[rns::OP_G2_DBL4] != 0>(e, L, R, R, R);
    dump();
    if ((params::BLS_X >> b) & 1) {
      rns::stage<rns::OP_G2_ADD1, rns::OP_RW[rns::OP_G2_ADD1] != 0>(e, L, R, R, R);
      rns::stage<rns::OP_G2_ADD2, rns::OP_RW[rns::OP_G2_ADD2] != 0>(e, L, R, R, R);
      rns::stage<rns::OP_G2_ADD3, rns::OP_RW[rns::OP_G2_ADD3] != 0>(e, L, R, R, R);
      rns::stage<rns::OP_G2_ADD4, rns::OP_RW[rns::OP_G2_ADD4] != 0>(e, L, R, R, R);
      dump();
    }
  }
}

// count M-domain residue vectors (32 u32 each) -> field.h Montgomery Fq,
// two per wave and pass
__global__ void __launch_bounds__(256) k_rns_to_fq(const uint32_t* __restrict__ res, size_t count,
                                                   Fq* __restrict__ out) {
  __shared__ uint32_t s_slots[rns::N_CONSTS * rns::SLOT];
  __shared__ uint32_t s_xch[4 * rns::XCH];
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + (threadIdx.x >> 6) * rns::XCH, 0};
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const size_t pairs = (count + 1) / 2;
  for (size_t pw = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); pw < pairs; pw += (size_t)gridDim.x * 4) {
    const size_t v0 = 2 * pw, v1 = v0 + 1 < count ? v0 + 1 : v0;
    const uint32_t x = res[((lane & 32) ? v1 : v0) * 32 + (lane & 31)];
    rns::to_fq_wave(e, L, x, out + v0, out + v1);
  }
}

size_t g2_prepare_scratch(size_t n) { return n * N_LINE_COEFFS * 6 * 32 * sizeof(uint32_t); }

// scratch: g2_prepare_scratch(n) bytes (the residue lines)
hipError_t g2_prepare_batch(hipStream_t s, const uint32_t* d_g2, size_t n, LineCoeff* d_coeffs, uint32_t* scratch) {
  if (!n) return hipSuccess;
  if (!scratch) return hipErrorInvalidValue;
  k_g2_prepare_rns<<<(unsigned)((n + 1) / 2), 768, 0, s>>>(d_g2, n, scratch);
  TPST_TRY(hipGetLastError());
  const size_t count = n * N_LINE_COEFFS * 6;
  const size_t waves = (count + 1) / 2;
  const unsigned grid = (unsigned)(waves / 4 < 2048 ? (waves + 3) / 4 : 2048);
  k_rns_to_fq<<<grid, 256, 0, s>>>(scratch, count, reinterpret_cast<Fq*>(d_coeffs));
  return hipGetLastError();
}

// ---- product of a group's partials + final exponentiation ----------------
constexpr int FW = 2;  // waves per workgroup
constexpr int FW_SLOTS = 64 + 36;          // PROD, ACC, IN, TMP per wave
constexpr int FE_SLOTS = 10 * 12 + 24;     // wave 0: 10 registers + inversion temporaries
constexpr int FE_OPS[] = {wave::OP_F12_MUL, wave::OP_CYC_SQR, wave::OP_FROB1, wave::OP_FROB2, wave::OP_CONJ,
                          wave::OP_INV1,    wave::OP_INV2,    wave::OP_INV3,  wave::OP_INV4,  wave::OP_INV5,
                          wave::OP_INV6,    wave::OP_INV7,    wave::OP_F12_SQR};
constexpr int N_FE_OPS = sizeof(FE_OPS) / sizeof(FE_OPS[0]);
constexpr wave::OpSet<N_FE_OPS> FE_SET(FE_OPS);
constexpr int FW_PROG = FE_SET.words;
constexpr size_t FW_LDS = (size_t)(FW_PROG + (wave::N_CONSTS + FW * FW_SLOTS + FE_SLOTS) * wave::SLOT) * 4;
static_assert(FW_LDS <= 65536, "final-exponentiation kernel LDS");

enum { FE_MUL, FE_CYC, FE_FROB1, FE_FROB2, FE_CONJ, FE_INV1, FE_SQR12 = 12 };

__device__ int fe_exp_by_x(const wave::Eng& e, const wave::lds_t* prog, int src, int r1, int r2) {
  int cur = src;
  for (int b = X_BITS - 2; b >= 0; b--) {
    int nxt = cur == r1 ? r2 : r1;
    wave::run(e, prog + FE_SET.off[FE_CYC], cur, 0, nxt);
    cur = nxt;
    if ((params::BLS_X >> b) & 1) {
      nxt = cur == r1 ? r2 : r1;
      wave::run(e, prog + FE_SET.off[FE_MUL], cur, src, nxt);
      cur = nxt;
    }
  }
  return cur;
}

// f (register F) -> f^(3(p^12-1)/r); returns the result register.  Same chain
// as final_exponentiation() in pairing.h (eprint 2020/875).
// ninv: the inverse of f's Fq-norm N(f) computed elsewhere in the workgroup
// (k_chain_final's second wave), or nullptr to invert N(f) here on lane 0;
// with ninv the function contains one __syncthreads (the hand-over).
__device__ int fe_final_exp(const wave::Eng& e, const wave::lds_t* prog, int F, int regs, int I,
                            const Fq* ninv = nullptr) {
  const int lane = threadIdx.x & 63;
#define R(i) (regs + 12 * (i))
  // f^-1 through the tower norms and one Fq inversion
  wave::run(e, prog + FE_SET.off[FE_INV1 + 0], F, 0, I + 0);        // t = c0^2 - v c1^2
  wave::run(e, prog + FE_SET.off[FE_INV1 + 1], I + 0, 0, I + 6);    // Fq6 adjugate c'
  wave::run(e, prog + FE_SET.off[FE_INV1 + 2], I + 6, I + 0, I + 12);  // Fq6 norm t'
  wave::run(e, prog + FE_SET.off[FE_INV1 + 3], I + 12, 0, I + 14);  // Fq2 norm n
  if (ninv) {
    __syncthreads();
    if (lane == 0) wave::put_slot(e.lds, I + 15, *ninv);
  } else if (lane == 0) {
    wave::put_slot(e.lds, I + 15, inv(wave::get_slot(e.lds, I + 14)));
  }
  wave::wave_sync();
  wave::run(e, prog + FE_SET.off[FE_INV1 + 4], I + 12, I + 15, I + 16);  // t'^-1
  wave::run(e, prog + FE_SET.off[FE_INV1 + 5], I + 6, I + 16, I + 18);   // t^-1
  wave::run(e, prog + FE_SET.off[FE_INV1 + 6], F, I + 18, R(0));         // f^-1
  // easy part
  wave::run(e, prog + FE_SET.off[FE_CONJ], F, 0, R(1));
  wave::run(e, prog + FE_SET.off[FE_MUL], R(1), R(0), R(2));  // r = conj(f) f^-1
  wave::run(e, prog + FE_SET.off[FE_FROB2], R(2), 0, R(1));
  wave::run(e, prog + FE_SET.off[FE_MUL], R(1), R(2), R(3));  // r = r^(p^2) r
  // hard part
  wave::run(e, prog + FE_SET.off[FE_CYC], R(3), 0, R(4));  // y0
  int t = fe_exp_by_x(e, prog, R(3), R(5), R(6));
  wave::run(e, prog + FE_SET.off[FE_CONJ], R(3), 0, R(7));  // y2 = conj(r)
  wave::run(e, prog + FE_SET.off[FE_MUL], t, R(7), R(8));   // y1 = y1 y2
  t = fe_exp_by_x(e, prog, R(8), R(5), R(6));  // y2
  wave::run(e, prog + FE_SET.off[FE_CONJ], R(8), 0, R(7));
  wave::run(e, prog + FE_SET.off[FE_MUL], R(7), t, R(9));   // y1 = conj(y1) y2
  t = fe_exp_by_x(e, prog, R(9), R(5), R(6));  // y2
  wave::run(e, prog + FE_SET.off[FE_FROB1], R(9), 0, R(7));
  wave::run(e, prog + FE_SET.off[FE_MUL], R(7), t, R(8));   // y1 = frob(y1) y2
  wave::run(e, prog + FE_SET.off[FE_MUL], R(3), R(4), R(0));  // r = r y0
  const int y0 = fe_exp_by_x(e, prog, R(8), R(5), R(6));
  const int y2 = fe_exp_by_x(e, prog, y0, y0 == R(5) ? R(6) : R(5), R(1));
  wave::run(e, prog + FE_SET.off[FE_FROB2], R(8), 0, R(2));  // y0 = frob2(y1)
  wave::run(e, prog + FE_SET.off[FE_CONJ], R(8), 0, R(3));
  wave::run(e, prog + FE_SET.off[FE_MUL], R(3), y2, R(4));   // y1 = conj(y1) y2
  wave::run(e, prog + FE_SET.off[FE_MUL], R(4), R(2), R(7));  // y1 = y1 y0
  wave::run(e, prog + FE_SET.off[FE_MUL], R(0), R(7), R(9));  // r = r y1
  return R(9);
#undef R
}

__global__ void __launch_bounds__(64 * FW) k_final_wave(const Fq12* __restrict__ partial, size_t T,
                                                        Fq12* __restrict__ out, int do_final) {
  extern __shared__ uint4 smem4[];
  __shared__ int acc_slot[FW];
  wave::lds_t* prog = (wave::lds_t*)(smem4);
  wave::lds_t* vals = prog + FW_PROG;
  wave::load_set(prog, FE_SET);
  wave::load_consts(vals, 0);
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const size_t g = blockIdx.x;
  const int base = wave::N_CONSTS + w * FW_SLOTS;
  const wave::Eng e{vals, base, 0};
  int acc = base + 64, in = base + 76, tmp = base + 88;
  size_t cnt = 0;
  for (size_t k = w; k < T; k += FW, cnt++) {
    if (cnt == 0) {
      wave::load_f12(vals, acc, partial + g * T + k);
    } else {
      wave::load_f12(vals, in, partial + g * T + k);
      wave::run(e, prog + FE_SET.off[FE_MUL], acc, in, tmp);
      const int t = acc;
      acc = tmp;
      tmp = t;
    }
  }
  if (cnt == 0) wave::set_one(vals, acc);
  if ((threadIdx.x & 63) == 0) acc_slot[w] = acc;
  __syncthreads();
  if (w != 0) return;
  for (int v = 1; v < FW; v++) {
    wave::run(e, prog + FE_SET.off[FE_MUL], acc, acc_slot[v], tmp);
    const int t = acc;
    acc = tmp;
    tmp = t;
  }
  if (!do_final) {  // Miller-loop product only (row-sharded IPP partial)
    wave::store_f12(vals, acc, out + g);
    return;
  }
  const int fe = wave::N_CONSTS + FW * FW_SLOTS;
  const int r = fe_final_exp(e, prog, acc, fe, fe + 120);
  wave::store_f12(vals, r, out + g);
}

// ---- parallel tree product of Miller partials -----------------------------
// One wave per output: out[g][j] = prod of partials [g][j*CH .. j*CH+CH) (the
// tail chunk shorter).  Keeps k_final_wave's serial product short: without it
// a 4096-pair IPP would be 1024 dependent Fq12 products per wave.
constexpr int RW = 4;
constexpr int RW_SLOTS = 64 + 36;
constexpr int RW_OPS[] = {wave::OP_F12_MUL};
constexpr wave::OpSet<1> RW_SET(RW_OPS);
constexpr int RW_PROG = RW_SET.words;
constexpr size_t RW_LDS = (size_t)(RW_PROG + (wave::N_CONSTS + RW * RW_SLOTS) * wave::SLOT) * 4;
constexpr size_t RW_CHUNK = 8;
static_assert(RW_LDS <= 65536, "tree-product kernel LDS");

__global__ void __launch_bounds__(64 * RW) k_f12_chunk_prod(const Fq12* __restrict__ in, size_t groups, size_t n,
                                                            size_t nout, Fq12* __restrict__ out, size_t chunk) {
  extern __shared__ uint4 smem4[];
  wave::lds_t* prog = (wave::lds_t*)(smem4);
  wave::lds_t* vals = prog + RW_PROG;
  wave::load_set(prog, RW_SET);
  wave::load_consts(vals, 0);
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const size_t o = (size_t)blockIdx.x * RW + w;
  if (o >= groups * nout) return;
  const size_t g = o / nout, j = o % nout;
  const size_t k0 = j * chunk, k1 = (k0 + chunk < n) ? k0 + chunk : n;
  const int base = wave::N_CONSTS + w * RW_SLOTS;
  const wave::Eng e{vals, base, 0};
  int acc = base + 64, in_r = base + 76, tmp = base + 88;
  // the next factor's global load is issued before the current product runs
  // (12 lanes hold it in VGPRs), so its latency hides under the stage
  const int lane = threadIdx.x & 63;
  const Fq* src = reinterpret_cast<const Fq*>(in + g * n);
  wave::load_f12(vals, acc, in + g * n + k0);
  Fq nxt = lane < 12 && k0 + 1 < k1 ? src[12 * (k0 + 1) + lane] : Fq::zero();
  for (size_t k = k0 + 1; k < k1; k++) {
    if (lane < 12) wave::put_slot(vals, in_r + lane, nxt);
    wave::wave_sync();
    if (lane < 12 && k + 1 < k1) nxt = src[12 * (k + 1) + lane];
    wave::run(e, prog + RW_SET.off[0], acc, in_r, tmp);
    const int t = acc;
    acc = tmp;
    tmp = t;
  }
  wave::store_f12(vals, acc, out + o);
}

// groups x n Miller partials -> groups x n' (n' <= 4 FW-wave shares) by
// chunked tree products; returns the buffer holding them and sets n
static hipError_t tree_partials(Arena& ar, hipStream_t s, Fq12*& partial, size_t groups, size_t& n) {
  while (n > 2 * FW) {
    const size_t nout = (n + RW_CHUNK - 1) / RW_CHUNK;
    Fq12* nxt = ar.take<Fq12>(groups * nout);
    k_f12_chunk_prod<<<grid_for(groups * nout, RW), 64 * RW, RW_LDS, s>>>(partial, groups, n, nout, nxt, RW_CHUNK);
    TPST_TRY(hipGetLastError());
    partial = nxt;
    n = nout;
  }
  return hipSuccess;
}

// ---- multi-pairing by line products ---------------------------------------
// With m_{p,b} the line value(s) of pair p at bit b (b = 62..0), the Miller
// product of a group is
//     prod_p f_p = prod_b M_b^(2^b),   M_b = prod_p m_{p,b}.
// The M_b do not depend on f, so they are a parallel tree over the pairs
// (k_line_pair, then k_f12_chunk_prod levels); the only serial chain left is
// Horner over the bits: per block of LB bits a block multiplier
// MB_j = prod_{b in block} M_b^(2^(b - lo_j)) (k_miller_blocks, all blocks in
// parallel), then F = MB_top, F = F^(2^LB) MB_j for the lower blocks, and the
// final exponentiation in the same wave (k_chain_final): 56 squarings + 7
// products instead of 63 x (square + line product) per pair.
// G1 operands may be XYZZ: the line of column j is scaled by
// lambda = ZZ ZZZ in Fq (c0 Y ZZ, c1 X ZZZ, c2 ZZ ZZZ), a factor the final
// exponentiation removes, so no inversion is needed before pairing.
constexpr int LB = 8;                                     // bits per block
constexpr int N_BITS = X_BITS - 1;                        // 63 Miller bits
constexpr int NBLK = (N_BITS + LB - 1) / LB;              // 8 blocks
constexpr int TREE_CHUNK = 4;

__device__ __forceinline__ size_t pair_column(size_t g, size_t k, size_t n, size_t map_s) {
  return map_s ? (k / map_s) * 2 * map_s + (g == 0 ? map_s : 0) + k % map_s : g * n + k;
}

__global__ void k_set_one(Fq12* __restrict__ v, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = Fq12::one();
}

// Sparse line value c0' + c3' w + c4' v w of one pair at its G1 point
// (ark ell(): c0 py, c1 px, c2), or the G1 point's lambda = ZZ ZZZ scaling of
// all three when P is XYZZ (a factor the final exponentiation removes).
// Returns false when the pair contributes 1 (either point at infinity).
// Products kept in program order: sched_barrier stops the scheduler from
// interleaving independent Montgomery products, which multiplies the live
// limbs past the register file (hundreds of spilled VGPRs otherwise).
__device__ __forceinline__ Fq smul(const Fq& a, const Fq& b) {
  const Fq r = mul(a, b);
  __builtin_amdgcn_sched_barrier(0);
  return r;
}
__device__ __forceinline__ Fq2 smul(const Fq2& a, const Fq2& b) {
  const Fq v0 = smul(a.c0, b.c0);
  const Fq v1 = smul(a.c1, b.c1);
  const Fq t = smul(add(a.c0, a.c1), add(b.c0, b.c1));
  return {sub(v0, mul5(v1)), sub(sub(t, v0), v1)};
}
__device__ __forceinline__ Fq2 smul_fq(const Fq2& a, const Fq& b) { return {smul(a.c0, b), smul(a.c1, b)}; }

__device__ __forceinline__ bool line_at(const LineCoeff* __restrict__ coeffs, size_t col, const uint32_t* g1, size_t p,
                                        bool xyzz, Fq2& c0, Fq2& c3, Fq2& c4) {
  Fq px, py, lam;
  if (xyzz) {
    const Xyzz<Fq> P = load_xyzz(reinterpret_cast<const Xyzz<Fq>*>(g1), p);
    if (is_inf(P)) return false;
    px = smul(P.X, P.ZZZ);
    py = smul(P.Y, P.ZZ);
    lam = smul(P.ZZ, P.ZZZ);
  } else {
    const G1A P = load_affine<Fq>(g1, p);
    if (is_inf(P)) return false;
    px = P.x;
    py = P.y;
  }
  const LineCoeff c = coeffs[col];
  c0 = smul_fq(c.c0, py);
  c3 = smul_fq(c.c1, px);
  c4 = xyzz ? smul_fq(c.c2, lam) : c.c2;
  return true;
}

// Pair maps: pair (g, k) of a multi-pairing -> (G1 index, G2 column).
// Standard: column pair_column(g, k), G1 = the same index (affine), or the
// half-rotated XYZZ index within blocks of rot_L (MIPP's t_l / t_r pairs).
struct PairMapStd {
  size_t n, map_s, rot_L;
  __device__ void at(size_t g, size_t k, size_t& p, size_t& q) const {
    q = pair_column(g, k, n, map_s);
    p = rot_L ? (q / rot_L) * rot_L + ((q % rot_L) + rot_L / 2) % rot_L : q;
  }
};

// Pair products of the lines: out[(g 69 + idx) nout + c] = line idx of pair
// (g, 2c) times that of pair (g, 2c + 1) (the lone line when n is odd), one
// lane per product.  Two sparse line values A = a0 + (a3 + a4 v) w and B
// multiply to
//   (a0 b0 + u a4 b4, a3 b3, a3 b4 + a4 b3) + (a0 b3 + a3 b0, a0 b4 + a4 b0, 0) w
// -- six Fq2 products with Karatsuba cross terms -- stored as a dense Fq12:
// half as many values for the wave-cooperative tree that follows, and none of
// its dense x dense products at the widest level (its lone waves are
// latency-bound at their LDS-limited occupancy; this is throughput work).
template <class Map>
__global__ void __launch_bounds__(64, 1) k_line_pair(const LineCoeff* __restrict__ coeffs, size_t ncol,
                                                     const uint32_t* __restrict__ g1, int xyzz,
                                                     const uint32_t* __restrict__ g2, size_t groups, size_t n,
                                                     Map map, size_t nout, Fq12* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= groups * N_LINE_COEFFS * nout) return;
  const size_t c = t % nout, gi = t / nout, idx = gi % N_LINE_COEFFS, g = gi / N_LINE_COEFFS;
  Fq2 a0, a3, a4, b0, b3, b4;
  bool ha = false, hb = false;
  size_t p, q;
  map.at(g, 2 * c, p, q);
  if (!is_inf(load_affine<Fq2>(g2, q))) ha = line_at(coeffs, idx * ncol + q, g1, p, xyzz != 0, a0, a3, a4);
  if (2 * c + 1 < n) {
    map.at(g, 2 * c + 1, p, q);
    if (!is_inf(load_affine<Fq2>(g2, q))) hb = line_at(coeffs, idx * ncol + q, g1, p, xyzz != 0, b0, b3, b4);
  }
  Fq12* o = out + t;
  if (ha && hb) {
    const Fq2 m33 = smul(a3, b3);
    o->c0.c1 = m33;
    const Fq2 m00 = smul(a0, b0);
    o->c1.c0 = sub(sub(smul(add(a0, a3), add(b0, b3)), m00), m33);
    const Fq2 m44 = smul(a4, b4);
    o->c0.c2 = sub(sub(smul(add(a3, a4), add(b3, b4)), m33), m44);
    o->c0.c0 = add(m00, mul_by_u(m44));
    o->c1.c1 = sub(sub(smul(add(a0, a4), add(b0, b4)), m00), m44);
    o->c1.c2 = Fq2::zero();
  } else if (ha || hb) {
    *o = ha ? Fq12{{a0, Fq2::zero(), Fq2::zero()}, {a3, a4, Fq2::zero()}}
            : Fq12{{b0, Fq2::zero(), Fq2::zero()}, {b3, b4, Fq2::zero()}};
  } else {
    *o = Fq12::one();
  }
}

// line index of the doubling at bit b (62..0); its addition line follows it
__device__ __forceinline__ int dbl_idx(int b) {
  int idx = 0;
  for (int c = X_BITS - 2; c > b; c--) idx += 1 + (int)((params::BLS_X >> c) & 1);
  return idx;
}

// one wave per (group, block): MB = prod_{b in block} M_b^(2^(b - lo))
constexpr int BW = 4;
constexpr int BW_SLOTS = 64 + 36;
constexpr int BW_OPS[] = {wave::OP_F12_MUL, wave::OP_F12_SQR, wave::OP_INV1, wave::OP_INV2, wave::OP_INV3,
                          wave::OP_INV4};
constexpr wave::OpSet<6> BW_SET(BW_OPS);
constexpr int BW_PROG = BW_SET.words;
constexpr size_t BW_LDS = (size_t)(BW_PROG + (wave::N_CONSTS + BW * BW_SLOTS) * wave::SLOT) * 4;
static_assert(BW_LDS <= 65536, "block-multiplier kernel LDS");

// ---- the same chain on the RNS engine (rns_engine.h) ------------------------
// Two groups per workgroup (the two halves of every wave), twelve waves: one
// per Fq12 output coefficient, so a stage is a dozen parallel RNS Montgomery
// reductions instead of a wave's lone-lane product chain.  The Fq inversion of
// the final exponentiation runs on lanes 0 / 32 of wave 0 between two stages.
constexpr int RC_WAVES = 12;
constexpr int RC_SLOTS = rns::N_CONSTS + 36 + 10 * 12 + 24;
static_assert((size_t)(RC_SLOTS * rns::SLOT + RC_WAVES * rns::XCH) * 4 <= 65536, "RNS chain LDS");

__device__ __forceinline__ int rc_exp_by_x(const rns::Eng& e, const rns::Lane& L, int src, int r1, int r2) {
  int cur = src;
  for (int b = X_BITS - 2; b >= 0; b--) {
    int nxt = cur == r1 ? r2 : r1;
    rns::stage<rns::OP_CYC_SQR>(e, L, cur, 0, nxt);
    cur = nxt;
    if ((params::BLS_X >> b) & 1) {
      nxt = cur == r1 ? r2 : r1;
      rns::stage<rns::OP_F12_MUL>(e, L, cur, src, nxt);
      cur = nxt;
    }
  }
  return cur;
}

// fe_final_exp on the RNS engine (same chain, eprint 2020/875)
__device__ __forceinline__ int rc_final_exp(const rns::Eng& e, const rns::Lane& L, int F, int regs, int I, Fq* sh_n) {
  using namespace rns;
#define R(i) (regs + 12 * (i))
  stage<OP_INV1>(e, L, F, 0, I + 0);         // t = c0^2 - v c1^2
  stage<OP_INV2>(e, L, I + 0, 0, I + 6);     // Fq6 adjugate c'
  stage<OP_INV3>(e, L, I + 6, I + 0, I + 12);  // Fq6 norm t'
  stage<OP_INV4>(e, L, I + 12, 0, I + 14);   // Fq2 norm n
  store(e, L, I + 14, sh_n, sh_n + 1, 1);
  const int lane = threadIdx.x & 63;
  if (wave_id() < 2) {  // one chain's norm per wave, wave-cooperative inverse
    const Fq ni = inv_w(sh_n[wave_id()]);
    if (lane == 0) sh_n[wave_id()] = ni;
  }
  __syncthreads();
  load(e, L, sh_n, sh_n + 1, I + 15, 1);
  stage<OP_INV5>(e, L, I + 12, I + 15, I + 16);  // t'^-1
  stage<OP_INV6>(e, L, I + 6, I + 16, I + 18);   // t^-1
  stage<OP_INV7>(e, L, F, I + 18, R(0));         // f^-1
  // easy part
  stage<OP_CONJ>(e, L, F, 0, R(1));
  stage<OP_F12_MUL>(e, L, R(1), R(0), R(2));  // r = conj(f) f^-1
  stage<OP_FROB2>(e, L, R(2), 0, R(1));
  stage<OP_F12_MUL>(e, L, R(1), R(2), R(3));  // r = r^(p^2) r
  // hard part
  stage<OP_CYC_SQR>(e, L, R(3), 0, R(4));  // y0
  int t = rc_exp_by_x(e, L, R(3), R(5), R(6));
  stage<OP_CONJ>(e, L, R(3), 0, R(7));      // y2 = conj(r)
  stage<OP_F12_MUL>(e, L, t, R(7), R(8));   // y1 = y1 y2
  t = rc_exp_by_x(e, L, R(8), R(5), R(6));  // y2
  stage<OP_CONJ>(e, L, R(8), 0, R(7));
  stage<OP_F12_MUL>(e, L, R(7), t, R(9));   // y1 = conj(y1) y2
  t = rc_exp_by_x(e, L, R(9), R(5), R(6));  // y2
  stage<OP_FROB1>(e, L, R(9), 0, R(7));
  stage<OP_F12_MUL>(e, L, R(7), t, R(8));   // y1 = frob(y1) y2
  stage<OP_F12_MUL>(e, L, R(3), R(4), R(0));  // r = r y0
  const int y0 = rc_exp_by_x(e, L, R(8), R(5), R(6));
  const int y2 = rc_exp_by_x(e, L, y0, y0 == R(5) ? R(6) : R(5), R(1));
  stage<OP_FROB2>(e, L, R(8), 0, R(2));  // y0 = frob2(y1)
  stage<OP_CONJ>(e, L, R(8), 0, R(3));
  stage<OP_F12_MUL>(e, L, R(3), y2, R(4));   // y1 = conj(y1) y2
  stage<OP_F12_MUL>(e, L, R(4), R(2), R(7));  // y1 = y1 y0
  stage<OP_F12_MUL>(e, L, R(0), R(7), R(9));  // r = r y1
  return R(9);
#undef R
}

// tree products on the RNS engine: out[g][j] = prod in[g][j*CH .. j*CH+CH),
// two outputs per workgroup, the result in RNS form.  From field.h Fq12
// (RES_IN false) the first factor is loaded with K_LOAD[CH] and the others
// raw (no reduction), so a chunk costs CH - 1 stages; a short tail chunk is
// padded with ones so both halves run the same stage sequence.
template <bool RES_IN, int CH>
__global__ void __launch_bounds__(64 * RC_WAVES, 2) k_chunk_prod_rns(const void* __restrict__ in, size_t groups,
                                                                  size_t n, size_t nout, uint32_t* __restrict__ out) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 12 * (CH + 1)) * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  __shared__ uint32_t s_rows[2 * rns::NB * 32];
  const size_t items = groups * nout, pairs = (items + 1) / 2;
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::LaneL L = rns::load_lane_lds((rns::lds_t*)s_rows);
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  const int w = rns::wave_id(), lane = threadIdx.x & 63;
  const int X = rns::N_CONSTS;  // factor i in slots X + 12 i; the product ping-pongs with X + 12 CH
  __syncthreads();
  // persistent: a workgroup walks the output pairs (its setup amortized)
  for (size_t pr = blockIdx.x; pr < pairs; pr += gridDim.x) {
    const size_t o = (lane & 32) ? (2 * pr + 1 < items ? 2 * pr + 1 : 2 * pr) : 2 * pr;
    const size_t k0 = (o % nout) * CH, base = (o / nout) * n;
    // wave w fetches coefficient w of all CH factors at once (one memory
    // latency per chunk, not one per factor)
    uint32_t v[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const bool valid = k0 + i < n;
      if (RES_IN) {
        const uint32_t* r = static_cast<const uint32_t*>(in);
        v[i] = valid ? r[(base + k0 + i) * rns::RES_WORDS + w * 32 + (lane & 31)]
                     : (w == 0 ? e.slots[e.kon * rns::SLOT + lane] : 0u);
      } else {
        const Fq* f = static_cast<const Fq*>(in) + 12 * (base + k0 + i);
        if (valid) {
          v[i] = rns::residue(L, f[w].v);
        } else {
          uint32_t one[12];
#pragma unroll
          for (int k = 0; k < 12; k++) one[k] = w == 0 ? params::FQ_ONE[k] : 0u;
          v[i] = rns::residue(L, one);
        }
      }
    }
    if (!RES_IN) {  // the first of CH raw factors carries the (M/R)^(CH-1) M correction
      const uint32_t kin = e.slots[(e.kon + rns::K_LOAD[CH]) * rns::SLOT + lane];
      v[0] = rns::mont(e, L, rns::red64((uint64_t)v[0] * kin, L));
    }
#pragma unroll
    for (int i = 0; i < CH; i++) e.slots[(X + 12 * i + w) * rns::SLOT + lane] = v[i];
    __syncthreads();
    int acc = X, tmp = X + 12 * CH;
#pragma unroll
    for (int i = 1; i < CH; i++) {
      rns::stage<rns::OP_F12_MUL>(e, L, acc, X + 12 * i, tmp);
      const int t = acc;
      acc = tmp;
      tmp = t;
    }
    rns::store_res(e, acc, out + 2 * pr * rns::RES_WORDS,
                   out + (2 * pr + 1 < items ? 2 * pr + 1 : 2 * pr) * rns::RES_WORDS, 12);
    __syncthreads();  // the next chunk's factors overwrite these slots
  }
}

// workgroups for a persistent RNS kernel over `pairs` work items
static unsigned rns_grid(size_t pairs) {
  const size_t cap = (size_t)256 * 2;  // two workgroups per CU
  return (unsigned)(pairs < cap ? pairs : cap);
}

// block multipliers on the RNS engine: one workgroup per (block, pair of
// groups) -- both halves of a wave must run the same stage sequence, so the
// pair shares the block (and so its bit pattern).  Input: the per-bit line
// products M (field.h Fq12, or RNS form from k_chunk_prod_rns); MB is left
// in RNS form.
constexpr int MB_MAXV = 12;  // line products one block reads (LB doublings + its additions)

template <bool RES_IN>
__global__ void __launch_bounds__(64 * RC_WAVES) k_miller_blocks_rns(const void* __restrict__ M, size_t groups,
                                                                     uint32_t* __restrict__ MBr) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 24 + 12 * MB_MAXV) * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  const size_t pairs = (groups + 1) / 2;
  const int blk = (int)(blockIdx.x / pairs);
  const size_t g0 = 2 * (blockIdx.x % pairs), g1 = g0 + 1 < groups ? g0 + 1 : g0;
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  const int w = rns::wave_id(), lane = threadIdx.x & 63;
  const size_t g = (lane & 32) ? g1 : g0;
  const int lo = blk * LB, hi = (lo + LB < N_BITS ? lo + LB : N_BITS) - 1;
  const int V = rns::N_CONSTS + 24;  // the block's line products, in reading order
  // every line product of the block fetched at once: line index idx(hi) .. ,
  // in the order the Horner below consumes them
  const int idx_hi = dbl_idx(hi);
  const int nv = dbl_idx(lo) + 1 + (int)((params::BLS_X >> lo) & 1) - idx_hi;
  for (int v = 0; v < nv; v++) {
    const size_t li = g * N_LINE_COEFFS + idx_hi + v;
    uint32_t x;
    if (RES_IN) {
      x = static_cast<const uint32_t*>(M)[li * rns::RES_WORDS + w * 32 + (lane & 31)];
    } else {
      const uint32_t r = rns::residue(L, static_cast<const Fq*>(M)[12 * li + w].v);
      x = rns::mont(e, L, rns::red64((uint64_t)r * e.slots[(e.kon + rns::K_IN) * rns::SLOT + lane], L));
    }
    e.slots[(V + 12 * v + w) * rns::SLOT + lane] = x;
  }
  __syncthreads();
  // two work registers; other(x) is the one not holding x
  const int W0 = rns::N_CONSTS, W1 = rns::N_CONSTS + 12;
  auto other = [&](int x) { return x == W0 ? W1 : W0; };
  int acc = V, v = 1;
  for (int b = hi; b >= lo; b--) {
    if (b != hi) {
      const int t = other(acc);
      rns::stage<rns::OP_F12_SQR>(e, L, acc, 0, t);
      acc = other(t);
      rns::stage<rns::OP_F12_MUL>(e, L, t, V + 12 * v++, acc);
    }
    if ((params::BLS_X >> b) & 1) {
      const int t = other(acc);
      rns::stage<rns::OP_F12_MUL>(e, L, acc, V + 12 * v++, t);
      acc = t;
    }
  }
  rns::store_res(e, acc, MBr + (g0 * NBLK + blk) * rns::RES_WORDS, MBr + (g1 * NBLK + blk) * rns::RES_WORDS, 12);
}

__global__ void __launch_bounds__(64 * RC_WAVES) k_chain_final_rns(const uint32_t* __restrict__ MBr, size_t groups,
                                                                   Fq12* __restrict__ out, int do_final) {
  __shared__ uint32_t s_slots[RC_SLOTS * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  __shared__ Fq sh_n[2];
  const size_t g0 = 2 * (size_t)blockIdx.x, g1 = g0 + 1 < groups ? g0 + 1 : g0;
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  __syncthreads();
  int acc = rns::N_CONSTS, in_r = acc + 12, tmp = acc + 24;
  const uint32_t* m0 = MBr + g0 * NBLK * rns::RES_WORDS;
  const uint32_t* m1 = MBr + g1 * NBLK * rns::RES_WORDS;
  rns::load_res(e, m0 + (NBLK - 1) * rns::RES_WORDS, m1 + (NBLK - 1) * rns::RES_WORDS, acc, 12);
  for (int blk = NBLK - 2; blk >= 0; blk--) {
    for (int i = 0; i < LB; i++) {
      rns::stage<rns::OP_F12_SQR>(e, L, acc, 0, tmp);
      const int t = acc;
      acc = tmp;
      tmp = t;
    }
    rns::load_res(e, m0 + blk * rns::RES_WORDS, m1 + blk * rns::RES_WORDS, in_r, 12);
    rns::stage<rns::OP_F12_MUL>(e, L, acc, in_r, tmp);
    const int t = acc;
    acc = tmp;
    tmp = t;
  }
  int r = acc;
  if (do_final) r = rc_final_exp(e, L, acc, rns::N_CONSTS + 36, rns::N_CONSTS + 36 + 120, sh_n);
  rns::store(e, L, r, reinterpret_cast<Fq*>(out + g0), reinterpret_cast<Fq*>(out + g1), 12);
}

static size_t line_tree_len(size_t n) {  // tree levels over n pairs, chunk TREE_CHUNK
  size_t tot = 0;
  while (n > 1) {
    n = (n + TREE_CHUNK - 1) / TREE_CHUNK;
    tot += n;
  }
  return tot;
}

size_t multi_pairing_scratch(size_t groups, size_t n) {
  const size_t G = groups * N_LINE_COEFFS;
  return Arena::need(G * (n ? n : 1), sizeof(Fq12)) + Arena::need(G * (line_tree_len(n) + 1), sizeof(Fq12)) +
         Arena::need(groups * NBLK, sizeof(Fq12)) + Arena::need(groups * NBLK, sizeof(Fq)) +
         Arena::need(groups * NBLK * rns::RES_WORDS, sizeof(uint32_t)) +
         Arena::need(G * line_tree_len(n) * rns::RES_WORDS, sizeof(uint32_t)) + 4096 + 256 * 16;
}

// tree products of the lines, block multipliers, Horner chain (+ final exp)
static hipError_t pairing_from_lines(Arena& ar, hipStream_t s, Fq12* lines, size_t groups, size_t n, Fq12* d_out,
                                     bool final_exp) {
  const size_t G = groups * N_LINE_COEFFS;
  {
    // tree levels in RNS form (the first from the field.h line products)
    const void* cur = lines;
    bool res = false;
    while (n > 1) {
      const size_t nout = (n + TREE_CHUNK - 1) / TREE_CHUNK;
      uint32_t* nxt = ar.take<uint32_t>(G * nout * rns::RES_WORDS);
      const unsigned wg = rns_grid((G * nout + 1) / 2);
      if (res)
        k_chunk_prod_rns<true, TREE_CHUNK><<<wg, 64 * RC_WAVES, 0, s>>>(cur, G, n, nout, nxt);
      else
        k_chunk_prod_rns<false, TREE_CHUNK><<<wg, 64 * RC_WAVES, 0, s>>>(cur, G, n, nout, nxt);
      TPST_TRY(hipGetLastError());
      cur = nxt;
      res = true;
      n = nout;
    }
    uint32_t* MBr = ar.take<uint32_t>(groups * NBLK * rns::RES_WORDS);
    const unsigned pairs = (unsigned)((groups + 1) / 2);
    if (res)
      k_miller_blocks_rns<true><<<pairs * NBLK, 64 * RC_WAVES, 0, s>>>(cur, groups, MBr);
    else
      k_miller_blocks_rns<false><<<pairs * NBLK, 64 * RC_WAVES, 0, s>>>(cur, groups, MBr);
    TPST_TRY(hipGetLastError());
    // (one instantiation: a second one -- e.g. an s_setprio variant -- made
    // rc_final_exp an out-of-line call with its lane tables behind a
    // reference, 0.5 -> 2.2 ms per chain)
    k_chain_final_rns<<<pairs, 64 * RC_WAVES, 0, s>>>(MBr, groups, d_out, final_exp ? 1 : 0);
    return hipGetLastError();
  }
}

hipError_t multi_pairing_prepared(Arena& ar, hipStream_t s, const uint32_t* d_g1, const uint32_t* d_g2,
                                  const LineCoeff* d_coeffs, size_t groups, size_t n, Fq12* d_out, bool final_exp,
                                  size_t map_s, size_t rot_L) {
  if (!groups) return hipSuccess;
  const size_t G = groups * N_LINE_COEFFS;
  Fq12* lines = ar.take<Fq12>(G * (n ? n : 1));
  if (n) {
    const size_t nout = (n + 1) / 2;
    k_line_pair<PairMapStd><<<grid_for(G * nout, 64), 64, 0, s>>>(d_coeffs, groups * n, d_g1, rot_L ? 1 : 0, d_g2,
                                                                 groups, n, PairMapStd{n, map_s, rot_L}, nout, lines);
    TPST_TRY(hipGetLastError());
    n = nout;
  } else {
    k_set_one<<<grid_for(G, 64), 64, 0, s>>>(lines, G);
    TPST_TRY(hipGetLastError());
    n = 1;
  }
  return pairing_from_lines(ar, s, lines, groups, n, d_out, final_exp);
}

// ---- MIPP look-ahead (pst_api.hip tpst_poly_open) --------------------------
// The 8 pairing products of round-r vectors (a, h; len, s = len/2, s' = s/2)
// whose combination with round r's challenge gives round r+1's cross terms:
//   group  0 A0 (i, i+s')   1 A3 (i+s, i+s+s')   2 A1 (i, i+s+s')   3 A2 (i+s, i+s')
//          4 B0 (i+s', i)   5 B3 (i+s+s', i+s)   6 B1 (i+s', i+s)   7 B2 (i+s+s', i)
// (G1 index, G2 index) for i < s'.  E > 1: h is not prepared but an earlier
// round's h_prev is (row length E len), h_q = sum_j f_j h_prev[q + j len];
// each pair (p, q) becomes the E pairs (X[p + j len], h_prev[q + j len]) with
// X = the E fold sets f_j a (XYZZ).
__constant__ uint32_t LA_P[8] = {0, 2, 0, 2, 1, 3, 1, 3};  // G1 offset in units of s'
__constant__ uint32_t LA_Q[8] = {1, 3, 3, 1, 0, 2, 2, 0};  // G2 offset in units of s'

struct PairMapLA {
  size_t sp, len;
  __device__ void at(size_t g, size_t k, size_t& p, size_t& q) const {
    const size_t i = k % sp, j = k / sp;
    p = LA_P[g] * sp + i + j * len;
    q = LA_Q[g] * sp + i + j * len;
  }
};

size_t mipp_lookahead_scratch(size_t sp, int E) {
  const size_t n = sp * (size_t)E;
  return Arena::need(8 * N_LINE_COEFFS * n, sizeof(Fq12)) + multi_pairing_scratch(8, n);
}

hipError_t mipp_lookahead(Arena& ar, hipStream_t s, const LineCoeff* d_coeffs, size_t ncol, const uint32_t* d_g2,
                          const uint32_t* d_g1, bool xyzz, size_t len, int E, Fq12* d_out8, bool final_exp) {
  const size_t sp = len / 4;
  if (!sp || E < 1 || E > 8 || (E & (E - 1)) || ncol < (size_t)E * len) return hipErrorInvalidValue;
  const size_t n = sp * (size_t)E;
  Fq12* lines = ar.take<Fq12>(8 * N_LINE_COEFFS * n);
  const size_t G = 8 * N_LINE_COEFFS, nout = (n + 1) / 2;
  k_line_pair<PairMapLA><<<grid_for(G * nout, 64), 64, 0, s>>>(d_coeffs, ncol, d_g1, xyzz ? 1 : 0, d_g2, 8, n,
                                                              PairMapLA{sp, len}, nout, lines);
  TPST_TRY(hipGetLastError());
  return pairing_from_lines(ar, s, lines, 8, nout, d_out8, final_exp);
}

// ---- gathered Miller partials -> final exponentiation (row-sharded opening)
// out[g] = FE(prod_{w < W} parts[w G + g]): the ranks' unreduced Miller
// products of group g (look-ahead products, round 0's t_l / t_r) multiplied
// and final-exponentiated on the RNS engine, two groups per workgroup (the
// halves of every wave) -- W - 1 products + the chain of k_chain_final_rns
__global__ void __launch_bounds__(64 * RC_WAVES) k_prod_final_rns(const Fq12* __restrict__ parts, size_t W,
                                                                  size_t G, Fq12* __restrict__ out) {
  __shared__ uint32_t s_slots[RC_SLOTS * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  __shared__ Fq sh_n[2];
  const size_t g0 = 2 * (size_t)blockIdx.x, g1 = g0 + 1 < G ? g0 + 1 : g0;
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  __syncthreads();
  int acc = rns::N_CONSTS, in_r = acc + 12, tmp = acc + 24;
  rns::load(e, L, reinterpret_cast<const Fq*>(parts + g0), reinterpret_cast<const Fq*>(parts + g1), acc, 12);
  for (size_t w = 1; w < W; w++) {
    rns::load(e, L, reinterpret_cast<const Fq*>(parts + w * G + g0), reinterpret_cast<const Fq*>(parts + w * G + g1),
              in_r, 12);
    rns::stage<rns::OP_F12_MUL>(e, L, acc, in_r, tmp);
    const int t = acc;
    acc = tmp;
    tmp = t;
  }
  const int r = rc_final_exp(e, L, acc, rns::N_CONSTS + 36, rns::N_CONSTS + 36 + 120, sh_n);
  rns::store(e, L, r, reinterpret_cast<Fq*>(out + g0), reinterpret_cast<Fq*>(out + g1), 12);
}

hipError_t gt_prod_final(hipStream_t s, const Fq12* d_parts, size_t W, size_t G, Fq12* d_out) {
  if (!G) return hipSuccess;
  if (!W) return hipErrorInvalidValue;
  k_prod_final_rns<<<(unsigned)((G + 1) / 2), 64 * RC_WAVES, 0, s>>>(d_parts, W, G, d_out);
  return hipGetLastError();
}

hipError_t gt_product_final(Arena& ar, hipStream_t s, const Fq12* d_partials, size_t groups, size_t n, Fq12* d_out) {
  if (!groups) return hipSuccess;
  Fq12* partial = const_cast<Fq12*>(d_partials);
  if (n) TPST_TRY(tree_partials(ar, s, partial, groups, n));
  k_final_wave<<<(unsigned)groups, 64 * FW, FW_LDS, s>>>(partial, n, d_out, 1);
  return hipGetLastError();
}

hipError_t multi_pairing(Arena& ar, hipStream_t s, const uint32_t* d_g1, const uint32_t* d_g2, size_t groups,
                         size_t n, Fq12* d_out) {
  const size_t np = groups * n;
  size_t need = Arena::need(np * N_LINE_COEFFS, sizeof(LineCoeff)) + multi_pairing_scratch(groups, n) +
                Arena::need(g2_prepare_scratch(np), 1) + 4096;
  ar.reset();
  TPST_TRY(ar.reserve(need));
  LineCoeff* coeffs = ar.take<LineCoeff>(np * N_LINE_COEFFS);
  uint32_t* prep = ar.take<uint32_t>(g2_prepare_scratch(np) / sizeof(uint32_t));
  TPST_TRY(g2_prepare_batch(s, d_g2, np, coeffs, prep));
  return multi_pairing_prepared(ar, s, d_g1, d_g2, coeffs, groups, n, d_out);
}

// ---- GT exponentiation on the wave engine (MippProof::verify, mipp.rs:263-283)
// For f in GT (order r), f^p = f^x since p = x (mod r).  With e = sum_i e_i x^i
// (base-x digits; e < r < x^4, so the digits are exact, each < 2^64),
//     f^e = prod_i frob^i(f)^(e_i),
// a 4-way simultaneous exponentiation with 64-bit digits: 63 cyclotomic
// squarings and <= 64 products from the 16-entry subset table of
// (f, f^p, f^p^2, f^p^3), where the plain square-and-multiply needs 253
// squarings.  Membership first -- what arkworks' Validate::Yes
// deserialisation of a PairingOutput checks: f^(p^4) f == f^(p^2) puts f in
// the cyclotomic subgroup (order Phi12(p), so cyclotomic squaring applies),
// and then f^p == f^x puts it in GT, because gcd(p - x, Phi12(p)) = r for
// BLS12-377 (tests/test_kat_ref.py checks it).  ok[i] = 1 iff f_i is in GT
// (out[i] is only meaningful then); f = 0 is rejected first.
constexpr int GP_REGS = 20;  // R0 scratch, T1..T15 subset table, ACC, TMP, X1, X2
constexpr size_t GP_LDS = (size_t)(FW_PROG + (wave::N_CONSTS + 64 + 12 * GP_REGS) * wave::SLOT) * 4;
static_assert(GP_LDS <= 65536, "GT pow kernel LDS");

__device__ bool regs_equal(const wave::lds_t* lds, int a, int b) {
  const int lane = threadIdx.x & 63;
  const bool same = lane >= 12 || eq(wave::get_slot(lds, a + lane), wave::get_slot(lds, b + lane));
  return __all(same ? 1 : 0) != 0;
}

// mipp: the opening's look-ahead combination (pst_api.hip): wave i raises
// base[MIPP_POW_SEL[i]] in place (out == base), no membership test (the bases
// are final-exponentiation outputs)
__constant__ uint32_t MIPP_POW_SEL[4] = {2, 3, 6, 7};

__global__ void __launch_bounds__(64) k_gt_pow_wave(const Fq12* __restrict__ base, const uint64_t* __restrict__ digits,
                                                    size_t n, Fq12* __restrict__ out, uint32_t* __restrict__ ok,
                                                    int mipp) {
  extern __shared__ uint4 smem4[];
  wave::lds_t* prog = (wave::lds_t*)(smem4);
  wave::lds_t* vals = prog + FW_PROG;
  wave::load_set(prog, FE_SET);
  wave::load_consts(vals, 0);
  __syncthreads();
  if (blockIdx.x >= n) return;
  const size_t i = mipp ? MIPP_POW_SEL[blockIdx.x] : blockIdx.x;
  const uint64_t* d = digits + 4 * blockIdx.x;
  const wave::Eng e{vals, wave::N_CONSTS, 0};
#define R(k) (wave::N_CONSTS + 64 + 12 * (k))
  const int ACC = R(16), TMP = R(17), X1 = R(18), X2 = R(19);
  const wave::lds_t* P = prog;
  wave::load_f12(vals, R(1), base + i);
  const bool check = ok != nullptr;
  bool good = true;
  if (check) {
    // f = 0 passes both equations below but is not in GT (Validate::Yes rejects it)
    const int ln = threadIdx.x & 63;
    good = __any((ln < 12 && !is_zero(wave::get_slot(vals, R(1) + ln))) ? 1 : 0) != 0;
  }
  if (check && good) {  // cyclotomic subgroup: f^(p^4) f == f^(p^2)
    wave::run(e, P + FE_SET.off[FE_FROB2], R(1), 0, X1);
    wave::run(e, P + FE_SET.off[FE_FROB2], X1, 0, X2);
    wave::run(e, P + FE_SET.off[FE_MUL], X2, R(1), R(0));
    good = regs_equal(vals, R(0), X1);
  }
  // GT: f^p == f^x
  wave::run(e, P + FE_SET.off[FE_FROB1], R(1), 0, R(2));
  if (check && good) {
    const int fx = fe_exp_by_x(e, P, R(1), X1, X2);
    good = regs_equal(vals, fx, R(2));
  }
  const int lane = threadIdx.x & 63;
  if (check && lane == 0) ok[i] = good ? 1u : 0u;
  if (!good) return;
  // subset table T[m] = prod_{bit j of m} f^(p^j)
  wave::run(e, P + FE_SET.off[FE_FROB2], R(1), 0, R(4));
  wave::run(e, P + FE_SET.off[FE_FROB1], R(4), 0, R(8));
  for (int m = 3; m < 16; m++) {
    if ((m & (m - 1)) == 0) continue;  // powers of two are the bases themselves
    const int hi = 1 << (31 - __builtin_clz(m));
    wave::run(e, P + FE_SET.off[FE_MUL], R(m - hi), R(hi), R(m));
  }
  int acc = -1;
  for (int b = 63; b >= 0; b--) {
    if (acc >= 0) {
      const int nxt = acc == ACC ? TMP : ACC;
      wave::run(e, P + FE_SET.off[FE_CYC], acc, 0, nxt);
      acc = nxt;
    }
    const int mask = (int)((d[0] >> b) & 1) | (int)(((d[1] >> b) & 1) << 1) | (int)(((d[2] >> b) & 1) << 2) |
                     (int)(((d[3] >> b) & 1) << 3);
    if (!mask) continue;
    if (acc < 0) {
      acc = R(mask);
    } else {
      const int nxt = acc == ACC ? TMP : ACC;
      wave::run(e, P + FE_SET.off[FE_MUL], acc, R(mask), nxt);
      acc = nxt;
    }
  }
  if (acc < 0) {
    wave::set_one(vals, ACC);
    acc = ACC;
  }
  wave::store_f12(vals, acc, out + i);
#undef R
}

hipError_t gt_pow_wave(hipStream_t s, const Fq12* d_base, const uint64_t* d_digits, size_t n, Fq12* d_out,
                       uint32_t* d_ok) {
  if (!n) return hipSuccess;
  k_gt_pow_wave<<<(unsigned)n, 64, GP_LDS, s>>>(d_base, d_digits, n, d_out, d_ok, 0);
  return hipGetLastError();
}

hipError_t mipp_combine(hipStream_t s, Fq12* d_la8, const uint64_t* d_digits, Fq12* d_out2) {
  k_gt_pow_wave<<<4, 64, GP_LDS, s>>>(d_la8, d_digits, 4, d_la8, nullptr, 1);
  TPST_TRY(hipGetLastError());
  k_f12_chunk_prod<<<1, 64 * RW, RW_LDS, s>>>(d_la8, 2, 4, 1, d_out2, 4);
  return hipGetLastError();
}

// ---- look-ahead combination by squaring tables ------------------------------
// The combination t = A0 A3 A1^(c^-1) A2^c needs the four exponentiated
// look-ahead values to 253-bit exponents, known only once c is.  Their
// squarings do not depend on c: right after the look-ahead (off the critical
// path) the table S_b[k] = X_b^(2^k), k < 64, is stored for the four bases
// X_b = la8[MIPP_POW_SEL[b]] (63 cyclotomic squarings each).
// With the base-x digits e = sum_i e_i x^i of the exponent (f^p = f^x in GT),
//     X^e = prod_i frob^i( prod_{bit k of e_i} S[k] ),
// a product of <= 256 table entries per (base, digit), then frob^i, and two
// short tree levels finish t_l = A0 A3 X_A1 X_A2 and t_r = B0 B3 X_B1 X_B2
// (kernels below, on the RNS engine).
// tables of the bases src[sel[b]], b < n (one wave each); blocks n.. copy
// src[cp.src[j]] (or 1 when cp.src[j] < 0) to dst[cp.dst[j]]
struct SqPlan {
  int n;
  int sel[12];
};
struct CopyPlan {
  int n;
  int src[12], dst[12];
};

// block (b, i): G[tp.out[b] + i] = frob^i( prod_{bit k of e_{b,i}} S_b[k] ),
// e_{b,i} = digits[4 tp.dig[b] + i] (base-x digits, 4 x u64 per exponent).
// Wave w multiplies the entries of bit positions [16 w, 16 w + 16) in its
// three registers, then a 2-level tree across the waves (operands read from
// the other wave's slots).
struct TpPlan {
  int n;
  int dig[12], out[12];
};

// ---- the same combination on the RNS engine ---------------------------------
// Tables and partial products stay in RNS form (rns::RES_WORDS u32 per Fq12):
//   k_gt_sq_table_rns   blocks 0, 1: two bases each (the two halves), 63
//                       cyclotomic squarings, every power stored; block 2
//                       converts the plain copies (A0 A3 B0 B3) into G
//   k_gt_tab_prod1_rns  (base, digit, byte j): product of the 8 selected
//                       powers 8j .. 8j+7 (ones where the digit bit is 0)
//   k_gt_tab_prod2_rns  (base, digit): product of its 8 partials, then
//                       frob^digit -- both halves share the digit index, so
//                       they share the Frobenius stages
//   k_gt_final_rns      t_l, t_r = product of the 10 factors of each group,
//                       back to field.h Montgomery form
// about 25 stages on the critical path after the challenge, against the
// radix engine's ~17 slower stages and its table conversions.
__global__ void __launch_bounds__(64 * RC_WAVES) k_gt_sq_table_rns(const Fq12* __restrict__ src, SqPlan sp,
                                                                   uint32_t* __restrict__ tab, CopyPlan cp,
                                                                   uint32_t* __restrict__ G) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 24) * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  __syncthreads();
  int cur = rns::N_CONSTS, nxt = cur + 12;
  if (blockIdx.x < 2) {
    const int b0 = 2 * blockIdx.x, b1 = b0 + 1;
    rns::load(e, L, reinterpret_cast<const Fq*>(src + sp.sel[b0]), reinterpret_cast<const Fq*>(src + sp.sel[b1]),
              cur, 12);
    for (int k = 0; k < 64; k++) {
      rns::store_res(e, cur, tab + (size_t)(b0 * 64 + k) * rns::RES_WORDS,
                     tab + (size_t)(b1 * 64 + k) * rns::RES_WORDS, 12);
      if (k == 63) break;
      rns::stage<rns::OP_CYC_SQR>(e, L, cur, 0, nxt);
      const int t = cur;
      cur = nxt;
      nxt = t;
    }
    return;
  }
  for (int j = 0; j < cp.n; j += 2) {
    const int j1 = j + 1 < cp.n ? j + 1 : j;
    rns::load(e, L, reinterpret_cast<const Fq*>(src + cp.src[j]), reinterpret_cast<const Fq*>(src + cp.src[j1]),
              cur, 12);
    rns::store_res(e, cur, G + (size_t)cp.dst[j] * rns::RES_WORDS, G + (size_t)cp.dst[j1] * rns::RES_WORDS, 12);
    __syncthreads();
  }
}

// product of CH factors already fetched into slots X + 12 i; returns the slot
template <int CH>
__device__ int rns_product(const rns::Eng& e, const rns::Lane& L, int X, int W) {
  int acc = X, tmp = W;
#pragma unroll
  for (int i = 1; i < CH; i++) {
    rns::stage<rns::OP_F12_MUL>(e, L, acc, X + 12 * i, tmp);
    acc = tmp;
    tmp = tmp == W ? W + 12 : W;
  }
  return acc;
}

__global__ void __launch_bounds__(64 * RC_WAVES) k_gt_tab_prod1_rns(const uint32_t* __restrict__ tab,
                                                                    const uint64_t* __restrict__ digits, TpPlan tp,
                                                                    uint32_t* __restrict__ L1) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 12 * 10) * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  const int w = rns::wave_id(), lane = threadIdx.x & 63;
  const int q = 2 * blockIdx.x + (lane >> 5);  // (base, digit, byte) = (q / 32, q / 8 % 4, q % 8)
  const int b = q >> 5, i = (q >> 3) & 3, j = q & 7;
  const uint64_t ei = digits[4 * tp.dig[b] + i];
  const uint32_t one = w == 0 ? e.slots[e.kon * rns::SLOT + lane] : 0u;
  uint32_t v[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int bit = 8 * j + k;
    v[k] = ((ei >> bit) & 1) ? tab[(size_t)(b * 64 + bit) * rns::RES_WORDS + w * 32 + (lane & 31)] : one;
  }
  const int X = rns::N_CONSTS;
#pragma unroll
  for (int k = 0; k < 8; k++) e.slots[(X + 12 * k + w) * rns::SLOT + lane] = v[k];
  __syncthreads();
  const int r = rns_product<8>(e, L, X, X + 96);
  rns::store_res(e, r, L1 + (size_t)(2 * blockIdx.x) * rns::RES_WORDS, L1 + (size_t)(2 * blockIdx.x + 1) * rns::RES_WORDS,
                 12);
}

__global__ void __launch_bounds__(64 * RC_WAVES) k_gt_tab_prod2_rns(const uint32_t* __restrict__ L1, TpPlan tp,
                                                                    uint32_t* __restrict__ G) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 12 * 10) * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  const int w = rns::wave_id(), lane = threadIdx.x & 63;
  const int i = blockIdx.x >> 1, b = 2 * (blockIdx.x & 1) + (lane >> 5);  // both halves: digit i
  const int X = rns::N_CONSTS;
#pragma unroll
  for (int j = 0; j < 8; j++)
    e.slots[(X + 12 * j + w) * rns::SLOT + lane] = L1[(size_t)((b * 4 + i) * 8 + j) * rns::RES_WORDS + w * 32 + (lane & 31)];
  __syncthreads();
  int r = rns_product<8>(e, L, X, X + 96);
  const int o = r == X + 96 ? X + 108 : X + 96;
  if (i == 1) {
    rns::stage<rns::OP_FROB1>(e, L, r, 0, o);
    r = o;
  } else if (i == 2) {
    rns::stage<rns::OP_FROB2>(e, L, r, 0, o);
    r = o;
  } else if (i == 3) {
    rns::stage<rns::OP_FROB3>(e, L, r, 0, o);
    r = o;
  }
  const int b0 = 2 * (blockIdx.x & 1);
  rns::store_res(e, r, G + (size_t)(tp.out[b0] + i) * rns::RES_WORDS, G + (size_t)(tp.out[b0 + 1] + i) * rns::RES_WORDS,
                 12);
}

__global__ void __launch_bounds__(64 * RC_WAVES) k_gt_final_rns(const uint32_t* __restrict__ G, Fq12* __restrict__ out2) {
  __shared__ uint32_t s_slots[(rns::N_CONSTS + 12 * 12) * rns::SLOT];
  __shared__ uint32_t s_xch[RC_WAVES * rns::XCH];
  rns::load_consts((rns::lds_t*)s_slots);
  const rns::Lane L = rns::load_lane();
  const rns::Eng e{(rns::lds_t*)s_slots, (rns::lds_t*)s_xch + rns::wave_id() * rns::XCH, 0};
  const int w = rns::wave_id(), lane = threadIdx.x & 63, h = lane >> 5;
  const int X = rns::N_CONSTS;
#pragma unroll
  for (int f = 0; f < 10; f++)
    e.slots[(X + 12 * f + w) * rns::SLOT + lane] = G[(size_t)(10 * h + f) * rns::RES_WORDS + w * 32 + (lane & 31)];
  __syncthreads();
  const int r = rns_product<10>(e, L, X, X + 120);
  rns::store(e, L, r, reinterpret_cast<Fq*>(out2), reinterpret_cast<Fq*>(out2 + 1), 12);
}

hipError_t mipp_sq_tables(hipStream_t s, const Fq12* d_la8, Fq12* d_tab, Fq12* d_G) {
  // tables of A1 A2 B1 B2; A0 A3 / B0 B3 into slots 0, 1 of the two product lists
  const SqPlan sp{4, {2, 3, 6, 7}};
  const CopyPlan cp{4, {0, 1, 4, 5}, {0, 1, 10, 11}};
  k_gt_sq_table_rns<<<3, 64 * RC_WAVES, 0, s>>>(d_la8, sp, reinterpret_cast<uint32_t*>(d_tab), cp,
                                                reinterpret_cast<uint32_t*>(d_G));
  return hipGetLastError();
}

hipError_t mipp_combine_tab(hipStream_t s, const Fq12* d_tab, const uint64_t* d_digits, Fq12* d_G, Fq12* d_mid,
                            Fq12* d_out2) {
  const TpPlan tp{4, {0, 1, 2, 3}, {2, 6, 12, 16}};
  uint32_t* L1 = reinterpret_cast<uint32_t*>(d_mid);  // 128 partials
  k_gt_tab_prod1_rns<<<64, 64 * RC_WAVES, 0, s>>>(reinterpret_cast<const uint32_t*>(d_tab), d_digits, tp, L1);
  TPST_TRY(hipGetLastError());
  k_gt_tab_prod2_rns<<<8, 64 * RC_WAVES, 0, s>>>(L1, tp, reinterpret_cast<uint32_t*>(d_G));
  TPST_TRY(hipGetLastError());
  k_gt_final_rns<<<1, 64 * RC_WAVES, 0, s>>>(reinterpret_cast<const uint32_t*>(d_G), d_out2);
  return hipGetLastError();
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
