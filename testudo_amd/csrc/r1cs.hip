// Spartan R1CS satisfiability sum-checks on gfx950: R1CSProof::prove
// (r1csproof.rs:237-370) minus the Groth16 step -- the live caller of the
// sqrt-PST path.  Every table (z, eq(tau, .), Az, Bz,
// Cz, the phase-two eq(rx, .)-weighted column sums) lives in HBM as Montgomery
// Fr; each sum-check round is one fused kernel (bind the previous challenge +
// the round's evaluation sums, HBM-bound) plus a one-block reduction; the host
// keeps the Poseidon transcript (a few absorbs and one squeeze per round).
//
//   eq tables         EqPolynomial::evals (dense_mlpoly.rs:231-250)
//   Az / Bz / Cz      SparseMatPolynomial::multiply_vec (sparse_mlpoly.rs:462-476): CSR, one lane per row
//   evals_ABC         compute_eval_table_sparse (sparse_mlpoly.rs:478-488): CSC, one lane per column,
//                     the r_A / r_B / r_C combination (r1csproof.rs:326-338) fused
//   phase one         prove_cubic_with_additive_term (sumcheck.rs:67-148), comb tau (A B - C)
//   phase two         prove_quad (sumcheck.rs:387-444), comb A B
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/tpst.h"
#include "ctx.h"
#include "device_util.h"
#include "r1cs_state.h"
#include "scan_sort.h"

using namespace tpst;

const uint32_t* tpst_internal_poly_evals(const tpst_poly* p);  // pst_api.hip

#define TPST_TRY_HIP(x)                \
  do {                                 \
    hipError_t _e = (x);               \
    if (_e != hipSuccess) return _e;   \
  } while (0)

namespace {

inline unsigned grid_for(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// ------------------------------------------------------------ kernels ----
// out[i] = prod_j (bit (ell-1-j) of i ? r_j : 1 - r_j)   (MSB-first, r Montgomery)
__global__ void k_eq_evals(const uint32_t* __restrict__ r, int ell, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr prod = Fr::one();
  for (int j = 0; j < ell; j++) {
    const Fr rj = load_f<Fr>(r + 8 * j);
    prod = mul(prod, ((i >> (ell - 1 - j)) & 1) ? rj : sub(Fr::one(), rj));
  }
  store_f<Fr>(out + 8 * i, prod);
}

// canonical triples -> count per key (row or column)
__global__ void k_count(const uint32_t* __restrict__ key, size_t nnz, uint32_t* __restrict__ cnt) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nnz) atomicAdd(&cnt[key[e]], 1u);
}

// scatter entry e to its key's slot (order inside a key is irrelevant: the
// sums are exact field additions); vals converted to Montgomery
__global__ void k_scatter(const uint32_t* __restrict__ key, const uint32_t* __restrict__ other,
                          const uint32_t* __restrict__ val, size_t nnz, uint32_t* __restrict__ cursor,
                          uint32_t* __restrict__ o_idx, uint32_t* __restrict__ o_val) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const uint32_t pos = atomicAdd(&cursor[key[e]], 1u);
  o_idx[pos] = other[e];
  store_f<Fr>(o_val + 8 * (size_t)pos, to_mont(load_f<Fr>(val + 8 * e)));
}

// y[row] = sum_{e in row} val_e z[col_e]
__global__ void k_spmv(const uint32_t* __restrict__ ptr, const uint32_t* __restrict__ idx,
                       const uint32_t* __restrict__ val, const uint32_t* __restrict__ z, size_t nrows,
                       uint32_t* __restrict__ y) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  Fr acc = Fr::zero();
  for (uint32_t e = ptr[r]; e < ptr[r + 1]; e++)
    acc = add(acc, mul(load_f<Fr>(val + 8 * (size_t)e), load_f<Fr>(z + 8 * (size_t)idx[e])));
  store_f<Fr>(y + 8 * r, acc);
}

struct Csc3 {
  const uint32_t* ptr[3];
  const uint32_t* idx[3];
  const uint32_t* val[3];
};

// out[col] = sum_M coef_M sum_{e in col of M} val_e rx[row_e]
__global__ void k_eval_table(Csc3 m, const uint32_t* __restrict__ rx, const uint32_t* __restrict__ coef,
                             size_t ncols, uint32_t* __restrict__ out) {
  const size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  Fr tot = Fr::zero();
  for (int k = 0; k < 3; k++) {
    Fr acc = Fr::zero();
    for (uint32_t e = m.ptr[k][c]; e < m.ptr[k][c + 1]; e++)
      acc = add(acc, mul(load_f<Fr>(m.val[k] + 8 * (size_t)e), load_f<Fr>(rx + 8 * (size_t)m.idx[k][e])));
    tot = add(tot, mul(acc, load_f<Fr>(coef + 8 * k)));
  }
  store_f<Fr>(out + 8 * c, tot);
}

// z = vars || 1 || inputs || 0 (r1csproof.rs:263-272), canonical -> Montgomery
__global__ void k_make_z(const uint32_t* __restrict__ vars, size_t nv, const uint32_t* __restrict__ in, size_t ni,
                         size_t len, uint32_t* __restrict__ z) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  Fr v = Fr::zero();
  if (i < nv)
    v = to_mont(load_f<Fr>(vars + 8 * i));
  else if (i == nv)
    v = Fr::one();
  else if (i <= nv + ni)
    v = to_mont(load_f<Fr>(in + 8 * (i - nv - 1)));
  store_f<Fr>(z + 8 * i, v);
}

// synthetic instance (r1csinstance.rs:166-242): row i: A (i, i % sz, 1),
// B (i, (i+2) % sz, 1), C (i, c, Z[a] Z[b] / Z[c]) with c = (i+3) % sz, or
// (i, num_vars, Z[a] Z[b]) when Z[c] = 0.  Z canonical; vals canonical.
__global__ void k_synth(const uint32_t* __restrict__ Z, size_t sz, size_t num_vars, size_t num_cons,
                        uint32_t* __restrict__ rows, uint32_t* __restrict__ cols, uint32_t* __restrict__ vals) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num_cons) return;
  const size_t a = i % sz, b = (i + 2) % sz, c = (i + 3) % sz;
  const Fr za = to_mont(load_f<Fr>(Z + 8 * a)), zb = to_mont(load_f<Fr>(Z + 8 * b));
  const Fr zc = to_mont(load_f<Fr>(Z + 8 * c));
  const Fr ab = mul(za, zb);
  Fr one;
  for (int k = 0; k < 8; k++) one.v[k] = k ? 0u : 1u;  // canonical 1
  for (int m = 0; m < 3; m++) rows[m * num_cons + i] = (uint32_t)i;
  cols[i] = (uint32_t)a;
  cols[num_cons + i] = (uint32_t)b;
  store_f<Fr>(vals + 8 * i, one);
  store_f<Fr>(vals + 8 * (num_cons + i), one);
  const bool zero = is_zero(zc);
  cols[2 * num_cons + i] = (uint32_t)(zero ? num_vars : c);
  store_f<Fr>(vals + 8 * (2 * num_cons + i), from_mont(zero ? ab : mul(ab, inv(zc))));
}

constexpr int SC_BS = 256;

// One sum-check round over K tables of length 2h (before binding): optionally
// bind the previous challenge r (X'[i] = X[i] + r (X[i+2h'] - X[i]) with h' = h)
// in place, then the round's evaluation sums over i < h/2 at t = 0, 2, 3
// (cubic, K = 4, comb tau (A B - C)) or t = 0, 2 (quad, K = 2, comb A B).
//   bind: tables have length 2h, binding produces length h; sums over h/2.
//   no bind (first round): tables have length h; sums over h/2.
template <int K>
__global__ void __launch_bounds__(SC_BS) k_sc_round(uint32_t* t0, uint32_t* t1, uint32_t* t2, uint32_t* t3,
                                                    size_t h, const uint32_t* __restrict__ r, int do_sum,
                                                    uint32_t* __restrict__ partial) {
  __shared__ Fr sh[3][SC_BS];
  uint32_t* tab[4] = {t0, t1, t2, t3};
  const size_t half = h >> 1;
  const size_t i = (size_t)blockIdx.x * SC_BS + threadIdx.x;
  Fr s0 = Fr::zero(), s2 = Fr::zero(), s3 = Fr::zero();
  const bool bind = r != nullptr;
  const Fr rr = bind ? load_f<Fr>(r) : Fr::zero();
  if (i < (half ? half : 1) && (half || i < h)) {
    Fr lo[K], hi[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      uint32_t* X = tab[k];
      if (bind) {
        const size_t j0 = i, j1 = i + half;
        const Fr a0 = load_f<Fr>(X + 8 * j0), b0 = load_f<Fr>(X + 8 * (j0 + h));
        lo[k] = add(a0, mul(rr, sub(b0, a0)));
        store_f<Fr>(X + 8 * j0, lo[k]);
        if (half) {
          const Fr a1 = load_f<Fr>(X + 8 * j1), b1 = load_f<Fr>(X + 8 * (j1 + h));
          hi[k] = add(a1, mul(rr, sub(b1, a1)));
          store_f<Fr>(X + 8 * j1, hi[k]);
        }
      } else {
        lo[k] = load_f<Fr>(X + 8 * i);
        if (half) hi[k] = load_f<Fr>(X + 8 * (i + half));
      }
    }
    if (do_sum && half) {
      if (K == 4) {
        s0 = mul(lo[0], sub(mul(lo[1], lo[2]), lo[3]));
        Fr p[4], q[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const Fr d = sub(hi[k], lo[k]);
          p[k] = add(hi[k], d);  // 2 hi - lo
          q[k] = add(p[k], d);   // 3 hi - 2 lo
        }
        s2 = mul(p[0], sub(mul(p[1], p[2]), p[3]));
        s3 = mul(q[0], sub(mul(q[1], q[2]), q[3]));
      } else {
        s0 = mul(lo[0], lo[1]);
        const Fr p0 = sub(dbl(hi[0]), lo[0]), p1 = sub(dbl(hi[1]), lo[1]);
        s2 = mul(p0, p1);
      }
    }
  }
  if (!do_sum) return;
  sh[0][threadIdx.x] = s0;
  sh[1][threadIdx.x] = s2;
  sh[2][threadIdx.x] = s3;
  __syncthreads();
  for (int w = SC_BS / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int k = 0; k < 3; k++) sh[k][threadIdx.x] = add(sh[k][threadIdx.x], sh[k][threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x < 3) store_f<Fr>(partial + 8 * (3 * (size_t)blockIdx.x + threadIdx.x), sh[threadIdx.x][0]);
}

// sum nblk partial triples -> out[3] (canonical)
__global__ void __launch_bounds__(SC_BS) k_sc_reduce(const uint32_t* __restrict__ partial, size_t nblk,
                                                     uint32_t* __restrict__ out) {
  __shared__ Fr sh[3][SC_BS];
  Fr a[3] = {Fr::zero(), Fr::zero(), Fr::zero()};
  for (size_t b = threadIdx.x; b < nblk; b += SC_BS)
    for (int k = 0; k < 3; k++) a[k] = add(a[k], load_f<Fr>(partial + 8 * (3 * b + k)));
  for (int k = 0; k < 3; k++) sh[k][threadIdx.x] = a[k];
  __syncthreads();
  for (int w = SC_BS / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int k = 0; k < 3; k++) sh[k][threadIdx.x] = add(sh[k][threadIdx.x], sh[k][threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x < 3) store_f<Fr>(out + 8 * threadIdx.x, from_mont(sh[threadIdx.x][0]));
}

// ---------------------------------------------- SPARK dense representation --
// (SparseMatPolynomial::multi_sparse_to_dense_rep, sparse_mlpoly.rs:358-437)
// addresses of the batch's ops, instance after instance, each padded to N with
// address 0 (sparse_to_dense_vecs); pos = position in that sequence
__global__ void k_ops_addr(const uint32_t* __restrict__ a0, const uint32_t* __restrict__ a1,
                           const uint32_t* __restrict__ a2, uint32_t n0, uint32_t n1, uint32_t n2, size_t N,
                           uint32_t* __restrict__ addr, uint32_t* __restrict__ pos) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * N) return;
  const size_t b = i / N, e = i % N;
  const uint32_t* src = b == 0 ? a0 : b == 1 ? a1 : a2;
  const uint32_t nn = b == 0 ? n0 : b == 1 ? n1 : n2;
  addr[i] = e < nn ? src[e] : 0u;
  pos[i] = (uint32_t)i;
}

// over the stably sorted (addr, pos): the read timestamp of position pos is
// its rank among the earlier accesses of the same cell (AddrTimestamps::new,
// sparse_mlpoly.rs:227-261); the audit timestamp of a cell = its access count
__global__ void k_timestamps(const uint32_t* __restrict__ skey, const uint32_t* __restrict__ spos, size_t m,
                             uint32_t* __restrict__ read_ts, uint32_t* __restrict__ audit) {
  const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= m) return;
  const uint32_t k = skey[s];
  // segment start by binary search (the keys are sorted)
  size_t lo = 0, hi = s;
  while (lo < hi) {
    const size_t mid = (lo + hi) >> 1;
    if (skey[mid] < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  read_ts[spos[s]] = (uint32_t)(s - lo);
  if (s + 1 == m || skey[s + 1] != k) audit[k] = (uint32_t)(s + 1 - lo);
}

// Fr (canonical) out[i] = small integer in[i]
__global__ void k_u32_to_fr(const uint32_t* __restrict__ in, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4* o = reinterpret_cast<uint4*>(out + 8 * i);
  o[0] = make_uint4(in[i], 0u, 0u, 0u);
  o[1] = make_uint4(0u, 0u, 0u, 0u);
}

// padded values of instance b (canonical Fr) -> out[b N + e]
__global__ void k_vals_padded(const uint32_t* __restrict__ v0, const uint32_t* __restrict__ v1,
                              const uint32_t* __restrict__ v2, uint32_t n0, uint32_t n1, uint32_t n2, size_t N,
                              uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * N) return;
  const size_t b = i / N, e = i % N;
  const uint32_t* src = b == 0 ? v0 : b == 1 ? v1 : v2;
  const uint32_t nn = b == 0 ? n0 : b == 1 ? n1 : n2;
  uint4* o = reinterpret_cast<uint4*>(out + 8 * i);
  if (e < nn) {
    const uint4* q = reinterpret_cast<const uint4*>(src + 8 * e);
    o[0] = q[0];
    o[1] = q[1];
  } else {
    o[0] = make_uint4(0u, 0u, 0u, 0u);
    o[1] = o[0];
  }
}

// ------------------------------------------------------ host Fr helpers ----
Fr fr_small(uint32_t v) {
  Fr a = Fr::zero();
  a.v[0] = v;
  return to_mont(a);
}

// UniPoly::from_evals (unipoly.rs:15-45), Montgomery in/out
void from_evals(const Fr* e, int n, Fr* cs) {
  static const Fr i2 = inv(fr_small(2)), i6 = inv(fr_small(6));
  if (n == 3) {
    const Fr c = e[0];
    const Fr a = mul(i2, add(sub(sub(e[2], e[1]), e[1]), c));
    cs[0] = c;
    cs[1] = sub(sub(e[1], c), a);
    cs[2] = a;
    return;
  }
  const Fr d = e[0];
  const Fr a = mul(i6, sub(add(sub(e[3], mul(fr_small(3), e[2])), mul(fr_small(3), e[1])), e[0]));
  const Fr b = mul(i2, sub(add(sub(dbl(e[0]), mul(fr_small(5), e[1])), mul(fr_small(4), e[2])), e[3]));
  cs[0] = d;
  cs[1] = sub(sub(sub(e[1], d), a), b);
  cs[2] = b;
  cs[3] = a;
}

Fr uni_eval(const Fr* cs, int n, const Fr& r) {
  Fr out = cs[0], pw = r;
  for (int i = 1; i < n; i++) {
    out = add(out, mul(pw, cs[i]));
    pw = mul(pw, r);
  }
  return out;
}

}  // namespace

// CSR (by key = rows) or CSC (by key = cols) of one matrix from device triples
static hipError_t build_compressed(hipStream_t s, const uint32_t* key, const uint32_t* other, const uint32_t* val,
                                   size_t nnz, size_t nkeys, Buf& ptr, Buf& idx, Buf& vout) {
  TPST_TRY_HIP(ptr.alloc((nkeys + 1) * 4));
  TPST_TRY_HIP(idx.alloc(nnz ? nnz * 4 : 4));
  TPST_TRY_HIP(vout.alloc(nnz ? nnz * 32 : 32));
  Buf cnt, cursor, tmp;
  TPST_TRY_HIP(cnt.alloc((nkeys + 1) * 4));
  TPST_TRY_HIP(cursor.alloc((nkeys + 1) * 4));
  TPST_TRY_HIP(hipMemsetAsync(cnt.p, 0, (nkeys + 1) * 4, s));
  if (nnz) k_count<<<grid_for(nnz, 256), 256, 0, s>>>(key, nnz, cnt.u());
  TPST_TRY_HIP(hipGetLastError());
  TPST_TRY_HIP(tmp.alloc(scan_sort::scan_scratch(nkeys + 1) * 4 + 4));
  TPST_TRY_HIP(scan_sort::scan_excl_u32(s, cnt.u(), ptr.u(), nkeys + 1, tmp.u()));
  TPST_TRY_HIP(hipMemcpyAsync(cursor.p, ptr.p, (nkeys + 1) * 4, hipMemcpyDeviceToDevice, s));
  if (nnz) k_scatter<<<grid_for(nnz, 256), 256, 0, s>>>(key, other, val, nnz, cursor.u(), idx.u(), vout.u());
  TPST_TRY_HIP(hipGetLastError());
  return hipStreamSynchronize(s);  // the scratch buffers are freed on return
}

// device triples (rows[3][nnz], cols, vals canonical) -> instance tables
static int r1cs_from_device(tpst_ctx* ctx, tpst_r1cs* R, const uint32_t* const rows[3], const uint32_t* const cols[3],
                            const uint32_t* const vals[3]) {
  for (int m = 0; m < 3; m++) {
    const size_t k = R->nnz[m];
    TPST_HIP(ctx, R->orow[m].alloc(k * 4 + 4));
    TPST_HIP(ctx, R->ocol[m].alloc(k * 4 + 4));
    TPST_HIP(ctx, R->oval[m].alloc(k * 32 + 32));
    if (k) {
      TPST_HIP(ctx, hipMemcpyAsync(R->orow[m].p, rows[m], k * 4, hipMemcpyDeviceToDevice, ctx->stream));
      TPST_HIP(ctx, hipMemcpyAsync(R->ocol[m].p, cols[m], k * 4, hipMemcpyDeviceToDevice, ctx->stream));
      TPST_HIP(ctx, hipMemcpyAsync(R->oval[m].p, vals[m], k * 32, hipMemcpyDeviceToDevice, ctx->stream));
    }
    TPST_HIP(ctx, build_compressed(ctx->stream, rows[m], cols[m], vals[m], R->nnz[m], R->num_cons, R->rptr[m],
                                   R->ridx[m], R->rval[m]));
    TPST_HIP(ctx, build_compressed(ctx->stream, cols[m], rows[m], vals[m], R->nnz[m], R->ncols, R->cptr[m],
                                   R->cidx[m], R->cval[m]));
  }
  return TPST_OK;
}

static int r1cs_dims(tpst_ctx* ctx, size_t num_cons, size_t num_vars, size_t num_inputs) {
  if (log2_exact(num_cons) < 1 || log2_exact(num_vars) < 2) return fail(ctx, TPST_E_ARG, "num_cons / num_vars must be powers of two (num_vars >= 4)");
  if (num_inputs >= num_vars) return fail(ctx, TPST_E_ARG, "num_inputs + 1 must be <= num_vars");
  if (num_cons > ((size_t)1 << 31) || num_vars > ((size_t)1 << 30)) return fail(ctx, TPST_E_ARG, "instance too large");
  return TPST_OK;
}

extern "C" int tpst_r1cs_load(tpst_ctx* ctx, size_t num_cons, size_t num_vars, size_t num_inputs,
                              const size_t* nnz, const uint32_t* const* rows, const uint32_t* const* cols,
                              const uint64_t* const* vals, tpst_r1cs** out) {
  if (!ctx || !nnz || !rows || !cols || !vals || !out) return fail(ctx, TPST_E_ARG, "null argument");
  if (int rc = r1cs_dims(ctx, num_cons, num_vars, num_inputs)) return rc;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  std::unique_ptr<tpst_r1cs> R(new tpst_r1cs());
  R->owner = ctx;
  R->num_cons = num_cons;
  R->num_vars = num_vars;
  R->num_inputs = num_inputs;
  R->ncols = 2 * num_vars;
  Buf dr[3], dc[3], dv[3];
  const uint32_t *pr[3], *pc[3], *pv[3];
  for (int m = 0; m < 3; m++) {
    R->nnz[m] = nnz[m];
    if (nnz[m] && (!rows[m] || !cols[m] || !vals[m])) return fail(ctx, TPST_E_ARG, "null matrix");
    for (size_t e = 0; e < nnz[m]; e++) {
      if (rows[m][e] >= num_cons || cols[m][e] >= R->ncols) return fail(ctx, TPST_E_ARG, "entry out of range");
      if (!fr_ok_host(vals[m] + 4 * e)) return fail(ctx, TPST_E_ARG, "matrix value >= r");
    }
    TPST_HIP(ctx, dr[m].alloc(nnz[m] * 4 + 4));
    TPST_HIP(ctx, dc[m].alloc(nnz[m] * 4 + 4));
    TPST_HIP(ctx, dv[m].alloc(nnz[m] * 32 + 32));
    if (nnz[m]) {
      TPST_HIP(ctx, hipMemcpyAsync(dr[m].p, rows[m], nnz[m] * 4, hipMemcpyHostToDevice, ctx->stream));
      TPST_HIP(ctx, hipMemcpyAsync(dc[m].p, cols[m], nnz[m] * 4, hipMemcpyHostToDevice, ctx->stream));
      TPST_HIP(ctx, hipMemcpyAsync(dv[m].p, vals[m], nnz[m] * 32, hipMemcpyHostToDevice, ctx->stream));
    }
    pr[m] = dr[m].u();
    pc[m] = dc[m].u();
    pv[m] = dv[m].u();
  }
  if (int rc = r1cs_from_device(ctx, R.get(), pr, pc, pv)) return rc;
  *out = R.release();
  return TPST_OK;
}

extern "C" int tpst_r1cs_synthetic(tpst_ctx* ctx, size_t num_cons, size_t num_vars, size_t num_inputs,
                                   uint64_t seed, tpst_r1cs** out, uint64_t* vars, uint64_t* inputs) {
  if (!ctx || !out || !vars || (num_inputs && !inputs)) return fail(ctx, TPST_E_ARG, "null argument");
  if (int rc = r1cs_dims(ctx, num_cons, num_vars, num_inputs)) return rc;
  const size_t sz = num_vars + num_inputs + 1;
  std::vector<uint64_t> Z(4 * sz);
  tpst_fr_stream(seed, sz, 0, Z.data());
  memset(&Z[4 * num_vars], 0, 32);
  Z[4 * num_vars] = 1;  // the constant term
  memcpy(vars, Z.data(), num_vars * 32);
  if (num_inputs) memcpy(inputs, &Z[4 * (num_vars + 1)], num_inputs * 32);
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  std::unique_ptr<tpst_r1cs> R(new tpst_r1cs());
  R->owner = ctx;
  R->num_cons = num_cons;
  R->num_vars = num_vars;
  R->num_inputs = num_inputs;
  R->ncols = 2 * num_vars;
  Buf dZ, rows, cols, vals;
  TPST_HIP(ctx, dZ.alloc(sz * 32));
  TPST_HIP(ctx, rows.alloc(3 * num_cons * 4));
  TPST_HIP(ctx, cols.alloc(3 * num_cons * 4));
  TPST_HIP(ctx, vals.alloc(3 * num_cons * 32));
  TPST_HIP(ctx, hipMemcpyAsync(dZ.p, Z.data(), sz * 32, hipMemcpyHostToDevice, ctx->stream));
  k_synth<<<grid_for(num_cons, 256), 256, 0, ctx->stream>>>(dZ.u(), sz, num_vars, num_cons, rows.u(), cols.u(),
                                                            vals.u());
  TPST_HIP(ctx, hipGetLastError());
  const uint32_t* pr[3] = {rows.u(), rows.u() + num_cons, rows.u() + 2 * num_cons};
  const uint32_t* pc[3] = {cols.u(), cols.u() + num_cons, cols.u() + 2 * num_cons};
  const uint32_t* pv[3] = {vals.u(), vals.u() + 8 * num_cons, vals.u() + 16 * num_cons};
  for (int m = 0; m < 3; m++) R->nnz[m] = num_cons;
  if (int rc = r1cs_from_device(ctx, R.get(), pr, pc, pv)) return rc;
  *out = R.release();
  return TPST_OK;
}

extern "C" void tpst_r1cs_free(tpst_r1cs* r) { delete r; }

// UniPoly::from_evals (unipoly.rs:15-45) as the sum-check rounds use it: n = 3
// (quad) or 4 (cubic) evaluations at 0..n-1 -> coefficients, constant first
extern "C" int tpst_unipoly_from_evals(const uint64_t* evals, int n, uint64_t* coeffs) {
  if (!evals || !coeffs || (n != 3 && n != 4)) return TPST_E_ARG;
  Fr e[4], cs[4];
  for (int i = 0; i < n; i++) {
    if (!fr_ok_host(evals + 4 * i)) return TPST_E_ARG;
    e[i] = frc(evals + 4 * i);
  }
  from_evals(e, n, cs);
  for (int i = 0; i < n; i++) fro(cs[i], coeffs + 4 * i);
  return TPST_OK;
}

// EqPolynomial::evals (dense_mlpoly.rs:231-250) on the device: the MSB-first
// chi table of r (ell <= 30), the kernel the phase-one tau table uses
extern "C" int tpst_eq_evals(tpst_ctx* ctx, const uint64_t* r, int ell, uint64_t* out) {
  if (!ctx || !r || !out || ell < 0 || ell > 30) return fail(ctx, TPST_E_ARG, "eq_evals: bad argument");
  std::vector<Fr> rm(ell ? ell : 1);
  for (int j = 0; j < ell; j++) {
    if (!fr_ok_host(r + 4 * j)) return fail(ctx, TPST_E_ARG, "eq_evals: r_j >= r");
    rm[j] = frc(r + 4 * j);
  }
  const size_t n = (size_t)1 << ell;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  Buf dr, dt;
  TPST_HIP(ctx, dr.alloc(rm.size() * 32));
  TPST_HIP(ctx, dt.alloc(n * 32));
  TPST_HIP(ctx, hipMemcpyAsync(dr.p, rm.data(), rm.size() * 32, hipMemcpyHostToDevice, s));
  k_eq_evals<<<grid_for(n, 256), 256, 0, s>>>(dr.u(), ell, n, dt.u());
  TPST_HIP(ctx, hipGetLastError());
  std::vector<Fr> h(n);
  TPST_HIP(ctx, hipMemcpyAsync(h.data(), dt.p, n * 32, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  for (size_t i = 0; i < n; i++) fro(h[i], out + 4 * i);
  return TPST_OK;
}

// one sum-check (K = 4 cubic with additive term, K = 2 quad) over device
// tables of length 2^rounds; transcript on the host between rounds
template <int K>
static int sumcheck(tpst_ctx* ctx, void* pin, uint32_t* const* tabs, int rounds, Fr claim, tpst_transcript* tr,
                    uint64_t* polys, Fr* rs, Fr* finals) {
  hipStream_t s = ctx->stream;
  const size_t n0 = (size_t)1 << rounds;
  const size_t nblk0 = grid_for(n0 / 2, SC_BS);
  Buf partial, sums, dr;
  TPST_HIP(ctx, partial.alloc(nblk0 * 3 * 32));
  TPST_HIP(ctx, sums.alloc(3 * 32));
  TPST_HIP(ctx, dr.alloc(32));
  // pinned staging (the instance's, allocated once): the round sums down, the
  // challenge up -- one round trip per round
  if (!pin) return fail(ctx, TPST_E_HIP, "hipHostMalloc");
  uint64_t(*hs)[4] = reinterpret_cast<uint64_t(*)[4]>(pin);
  uint32_t* rpin = reinterpret_cast<uint32_t*>((char*)pin + 1024);
  uint32_t* t[4] = {tabs[0], tabs[1], K == 4 ? tabs[2] : nullptr, K == 4 ? tabs[3] : nullptr};
  Fr e = claim;
  constexpr int NC = K == 4 ? 4 : 3;  // coefficients per round polynomial
  for (int j = 0; j < rounds; j++) {
    const size_t h = n0 >> j;  // table length after binding the previous challenge
    const size_t nblk = grid_for(h / 2, SC_BS);
    k_sc_round<K><<<(unsigned)nblk, SC_BS, 0, s>>>(t[0], t[1], t[2], t[3], h, j ? dr.u() : nullptr, 1,
                                                   partial.u());
    TPST_HIP(ctx, hipGetLastError());
    k_sc_reduce<<<1, SC_BS, 0, s>>>(partial.u(), nblk, sums.u());
    TPST_HIP(ctx, hipGetLastError());
    TPST_HIP(ctx, hipMemcpyAsync(hs, sums.p, 96, hipMemcpyDeviceToHost, s));
    TPST_HIP(ctx, hipStreamSynchronize(s));
    // evals at 0, 1 (= e - eval(0)), 2, 3 (sumcheck.rs:127-128, 427)
    Fr ev[4] = {frc(hs[0]), Fr::zero(), frc(hs[1]), frc(hs[2])};
    ev[1] = sub(e, ev[0]);
    Fr cs[4];
    from_evals(ev, NC, cs);
    for (int c = 0; c < NC; c++) {
      uint64_t* out = polys + 4 * ((size_t)j * NC + c);
      fro(cs[c], out);
      if (tpst_transcript_append_fr(tr, out) != TPST_OK) return fail(ctx, TPST_E_ARG, "transcript append");
    }
    uint64_t rc[4];
    tpst_transcript_challenge(tr, rc);
    rs[j] = frc(rc);
    e = uni_eval(cs, NC, rs[j]);
    memcpy(rpin, rs[j].v, 32);
    TPST_HIP(ctx, hipMemcpyAsync(dr.p, rpin, 32, hipMemcpyHostToDevice, s));
  }
  // bind the last challenge: length 2 -> 1; the finals are the tables' [0]
  k_sc_round<K><<<1, SC_BS, 0, s>>>(t[0], t[1], t[2], t[3], 1, dr.u(), 0, partial.u());
  TPST_HIP(ctx, hipGetLastError());
  for (int k = 0; k < K; k++) TPST_HIP(ctx, hipMemcpyAsync(finals[k].v, t[k], 32, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  return TPST_OK;
}

static void fr_copy_out(const Fr& a, uint64_t* o) { fro(a, o); }

// R1CSProof::prove (r1csproof.rs:237-370) without prove_verifier: the
// polynomial commitment of the witness (sqrt-PST commit, its GT appended),
// both sum-checks on the device, then the PST opening at ry[1..].
extern "C" int tpst_r1cs_prove(tpst_ctx* ctx, tpst_r1cs* R, const uint64_t* vars, const uint64_t* inputs,
                               tpst_transcript* tr, tpst_r1cs_proof* out) {
  if (!ctx || !R || !vars || (R->num_inputs && !inputs) || !tr || !out) return fail(ctx, TPST_E_ARG, "null argument");
  if (R->owner != ctx) return fail(ctx, TPST_E_ARG, "instance belongs to another context");
  memset(out, 0, sizeof(*out));
  const int nvar_bits = log2_exact(R->num_vars);
  const int rx_n = log2_exact(R->num_cons), ry_n = nvar_bits + 1;
  if (rx_n > TPST_R1CS_MAX_ROUNDS || ry_n > TPST_R1CS_MAX_ROUNDS || nvar_bits > 2 * TPST_MAX_VARS)
    return fail(ctx, TPST_E_ARG, "instance too large for tpst_r1cs_proof");
  for (size_t i = 0; i < R->num_vars; i++)
    if (!fr_ok_host(vars + 4 * i)) return fail(ctx, TPST_E_ARG, "witness value >= r");
  for (size_t i = 0; i < R->num_inputs; i++)
    if (!fr_ok_host(inputs + 4 * i)) return fail(ctx, TPST_E_ARG, "input value >= r");
  out->rounds_x = rx_n;
  out->rounds_y = ry_n;
  out->num_vars_log = nvar_bits;
  // ---- commitment to the witness polynomial (sqrt_pst.rs:117-149)
  tpst_poly* pl = nullptr;
  if (int rc = tpst_poly_from_evaluations(ctx, vars, nvar_bits, &pl)) return rc;
  std::unique_ptr<tpst_poly, void (*)(tpst_poly*)> guard(pl, tpst_poly_free);
  const int m_col = nvar_bits / 2;
  std::vector<uint64_t> comms(((size_t)1 << m_col) * 12);
  if (int rc = tpst_poly_commit(ctx, pl, comms.data(), out->T)) return rc;
  tpst_transcript_append_gt(tr, out->T);
  tpst_transcript_challenge(tr, out->initial_state);
  tpst_transcript_reset_fr(tr, out->initial_state);
  for (size_t i = 0; i < R->num_inputs; i++) tpst_transcript_append_fr(tr, inputs + 4 * i);
  std::vector<Fr> tau(rx_n), rx(rx_n), ry(ry_n);
  for (int j = 0; j < rx_n; j++) {
    uint64_t c[4];
    tpst_transcript_challenge(tr, c);
    tau[j] = frc(c);
  }
  Fr fin1[4], fin2[2];
  Fr rA, rB, rC;
  {
    std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
    TPST_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t M = R->num_cons, Nz = R->ncols;
    Buf dins, z, tabs[4], dtau, drx, coef, abc;
    const uint32_t* d_vars = tpst_internal_poly_evals(pl);  // uploaded once, by from_evaluations
    if (!d_vars) return fail(ctx, TPST_E_STATE, "witness polynomial not resident");
    TPST_HIP(ctx, dins.alloc(R->num_inputs * 32 + 32));
    TPST_HIP(ctx, z.alloc(Nz * 32));
    TPST_HIP(ctx, dtau.alloc(rx_n * 32));
    for (auto& b : tabs) TPST_HIP(ctx, b.alloc(M * 32));
    if (R->num_inputs) TPST_HIP(ctx, hipMemcpyAsync(dins.p, inputs, R->num_inputs * 32, hipMemcpyHostToDevice, s));
    k_make_z<<<grid_for(Nz, 256), 256, 0, s>>>(d_vars, R->num_vars, dins.u(), R->num_inputs, Nz, z.u());
    TPST_HIP(ctx, hipGetLastError());
    TPST_HIP(ctx, hipMemcpyAsync(dtau.p, tau.data(), rx_n * 32, hipMemcpyHostToDevice, s));
    k_eq_evals<<<grid_for(M, 256), 256, 0, s>>>(dtau.u(), rx_n, M, tabs[0].u());
    TPST_HIP(ctx, hipGetLastError());
    for (int m = 0; m < 3; m++) {
      k_spmv<<<grid_for(M, 256), 256, 0, s>>>(R->rptr[m].u(), R->ridx[m].u(), R->rval[m].u(), z.u(), M,
                                              tabs[1 + m].u());
      TPST_HIP(ctx, hipGetLastError());
    }
    uint32_t* t4[4] = {tabs[0].u(), tabs[1].u(), tabs[2].u(), tabs[3].u()};
    if (int rc = sumcheck<4>(ctx, R->pinned(), t4, rx_n, Fr::zero(), tr, &out->sc1[0][0][0], rx.data(), fin1)) return rc;
    // claims_phase2 = (Az, Bz, Cz, Az Bz) at rx (r1csproof.rs:299-306)
    const Fr az = fin1[1], bz = fin1[2], cz = fin1[3];
    fr_copy_out(az, out->claims_phase2[0]);
    fr_copy_out(bz, out->claims_phase2[1]);
    fr_copy_out(cz, out->claims_phase2[2]);
    fr_copy_out(mul(az, bz), out->claims_phase2[3]);
    uint64_t c[4];
    tpst_transcript_challenge(tr, c);
    rA = frc(c);
    tpst_transcript_challenge(tr, c);
    rB = frc(c);
    tpst_transcript_challenge(tr, c);
    rC = frc(c);
    const Fr claim2 = add(add(mul(rA, az), mul(rB, bz)), mul(rC, cz));
    // evals_ABC (r1csproof.rs:326-338) into tabs[1]; eq(rx, .) into tabs[0]
    TPST_HIP(ctx, drx.alloc(rx_n * 32));
    TPST_HIP(ctx, coef.alloc(3 * 32));
    TPST_HIP(ctx, abc.alloc(Nz * 32));
    TPST_HIP(ctx, hipMemcpyAsync(drx.p, rx.data(), rx_n * 32, hipMemcpyHostToDevice, s));
    const Fr cf[3] = {rA, rB, rC};
    TPST_HIP(ctx, hipMemcpyAsync(coef.p, cf, 96, hipMemcpyHostToDevice, s));
    k_eq_evals<<<grid_for(M, 256), 256, 0, s>>>(drx.u(), rx_n, M, tabs[0].u());
    TPST_HIP(ctx, hipGetLastError());
    Csc3 csc;
    for (int m = 0; m < 3; m++) {
      csc.ptr[m] = R->cptr[m].u();
      csc.idx[m] = R->cidx[m].u();
      csc.val[m] = R->cval[m].u();
    }
    k_eval_table<<<grid_for(Nz, 256), 256, 0, s>>>(csc, tabs[0].u(), coef.u(), Nz, abc.u());
    TPST_HIP(ctx, hipGetLastError());
    uint32_t* t2[2] = {z.u(), abc.u()};
    if (int rc = sumcheck<2>(ctx, R->pinned(), t2, ry_n, claim2, tr, &out->sc2[0][0][0], ry.data(), fin2)) return rc;
    fr_copy_out(fin2[0], out->claims_phase2_z_abc[0]);
    fr_copy_out(fin2[1], out->claims_phase2_z_abc[1]);
  }
  for (int j = 0; j < rx_n; j++) fro(rx[j], out->rx[j]);
  for (int j = 0; j < ry_n; j++) fro(ry[j], out->ry[j]);
  fro(rA, out->r_abc[0]);
  fro(rB, out->r_abc[1]);
  fro(rC, out->r_abc[2]);
  tpst_transcript_challenge(tr, out->transcript_sat_state);
  tpst_transcript_reset_fr(tr, out->transcript_sat_state);
  // ---- PST opening of the witness at ry[1..] (r1csproof.rs:349-357)
  const uint64_t* point = &out->ry[1][0];
  if (int rc = tpst_poly_eval(ctx, pl, point, out->eval_vars_at_ry)) return rc;
  if (int rc = tpst_poly_open(ctx, pl, tr, comms.data(), point, out->T, &out->open)) return rc;
  return TPST_OK;
}

// R1CSInstance::commit -> SparseMatPolynomial::multi_commit over (A, B, C)
// (r1csinstance.rs:313-344, sparse_mlpoly.rs:490-517): the SPARK dense
// representation (row / col addresses and memory-checking timestamps, values)
// built on the device, merged into comb_ops (16 N) and comb_mem (2 cells), each
// committed with DensePolynomial::commit (Hyrax rows, zero blinds) over the
// generators PolyCommitmentGens::setup(num_vars, label) derives
// (DotProductProofGens: the first R of MultiCommitGens::new(R + 1, label)).
extern "C" int tpst_r1cs_commit(tpst_ctx* ctx, tpst_r1cs* R, const uint8_t* label, size_t label_len,
                                uint64_t* comm_ops, size_t* ops_rows, uint64_t* comm_mem, size_t* mem_rows) {
  if (!ctx || !R || !ops_rows || !mem_rows || (label_len && !label)) return fail(ctx, TPST_E_ARG, "null argument");
  if (R->owner != ctx) return fail(ctx, TPST_E_ARG, "instance belongs to another context");
  size_t maxnz = 1;
  for (int m = 0; m < 3; m++) maxnz = R->nnz[m] > maxnz ? R->nnz[m] : maxnz;
  size_t N = 1;
  while (N < maxnz) N <<= 1;
  const int vx = log2_exact(R->num_cons), vy = log2_exact(R->ncols);
  const int vmax = vx > vy ? vx : vy;
  const size_t cells = (size_t)1 << vmax;
  const int ell_ops = log2_exact(N) + 4, ell_mem = vmax + 1;  // batch 3: (3 * 5).next_power_of_two() = 16
  const size_t L_ops = (size_t)1 << (ell_ops / 2), R_ops = (size_t)1 << (ell_ops - ell_ops / 2);
  const size_t L_mem = (size_t)1 << (ell_mem / 2), R_mem = (size_t)1 << (ell_mem - ell_mem / 2);
  *ops_rows = L_ops;
  *mem_rows = L_mem;
  if (!comm_ops || !comm_mem) return TPST_OK;  // size query
  if (3 * N >= ((size_t)1 << 31)) return fail(ctx, TPST_E_ARG, "instance too large");
  Buf ops, mem;
  {
    std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
    TPST_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t M3 = 3 * N;
    TPST_HIP(ctx, ops.alloc(16 * N * 32));
    TPST_HIP(ctx, mem.alloc(2 * cells * 32));
    TPST_HIP(ctx, hipMemsetAsync(ops.p, 0, 16 * N * 32, s));
    Buf addr, pos, skey, spos, rts, audit, tmp;
    TPST_HIP(ctx, addr.alloc(M3 * 4));
    TPST_HIP(ctx, pos.alloc(M3 * 4));
    TPST_HIP(ctx, skey.alloc(M3 * 4));
    TPST_HIP(ctx, spos.alloc(M3 * 4));
    TPST_HIP(ctx, rts.alloc(M3 * 4));
    TPST_HIP(ctx, audit.alloc(cells * 4));
    TPST_HIP(ctx, tmp.alloc(scan_sort::sort_scratch(M3) * 4));
    for (int rc = 0; rc < 2; rc++) {  // rows, then columns
      const Buf* o = rc ? R->ocol : R->orow;
      k_ops_addr<<<grid_for(M3, 256), 256, 0, s>>>(o[0].u(), o[1].u(), o[2].u(), (uint32_t)R->nnz[0],
                                                   (uint32_t)R->nnz[1], (uint32_t)R->nnz[2], N, addr.u(), pos.u());
      TPST_HIP(ctx, hipGetLastError());
      // stable by address: equal addresses keep position order (the timestamps' rank)
      TPST_HIP(ctx, scan_sort::stable_sort_pairs(s, addr.u(), pos.u(), skey.u(), spos.u(), M3, vmax + 1, tmp.u()));
      TPST_HIP(ctx, hipMemsetAsync(audit.p, 0, cells * 4, s));
      k_timestamps<<<grid_for(M3, 256), 256, 0, s>>>(skey.u(), spos.u(), M3, rts.u(), audit.u());
      TPST_HIP(ctx, hipGetLastError());
      // comb_ops segments: row.ops_addr | row.read_ts | col.ops_addr | col.read_ts | val | 0
      uint32_t* base = ops.u() + 8 * (size_t)(rc * 2) * M3;
      k_u32_to_fr<<<grid_for(M3, 256), 256, 0, s>>>(addr.u(), M3, base);
      k_u32_to_fr<<<grid_for(M3, 256), 256, 0, s>>>(rts.u(), M3, base + 8 * M3);
      // comb_mem = row.audit_ts | col.audit_ts
      k_u32_to_fr<<<grid_for(cells, 256), 256, 0, s>>>(audit.u(), cells, mem.u() + 8 * (size_t)rc * cells);
      TPST_HIP(ctx, hipGetLastError());
    }
    k_vals_padded<<<grid_for(M3, 256), 256, 0, s>>>(R->oval[0].u(), R->oval[1].u(), R->oval[2].u(),
                                                    (uint32_t)R->nnz[0], (uint32_t)R->nnz[1], (uint32_t)R->nnz[2], N,
                                                    ops.u() + 8 * 4 * M3);
    TPST_HIP(ctx, hipGetLastError());
    TPST_HIP(ctx, hipStreamSynchronize(s));
  }
  // the two Hyrax commitments (the library calls below take the context lock)
  struct Job {
    const Buf* buf;
    size_t L, Rn;
    uint64_t* out;
  } jobs[2] = {{&ops, L_ops, R_ops, comm_ops}, {&mem, L_mem, R_mem, comm_mem}};
  for (const Job& j : jobs) {
    std::vector<uint64_t> G((j.Rn + 1) * 12), h(12);
    if (int rc = tpst_gens_new(ctx, j.Rn + 1, label, label_len, G.data(), h.data(), nullptr)) return rc;
    tpst_gens* gens = nullptr;
    if (int rc = tpst_gens_load(ctx, G.data(), j.Rn, h.data(), &gens)) return rc;
    std::unique_ptr<tpst_gens, void (*)(tpst_gens*)> gg(gens, tpst_gens_free);
    Buf dout;
    TPST_HIP(ctx, dout.alloc(j.L * 96));
    if (int rc = tpst_g1_msm_batch_dev(ctx, gens, j.buf->p, j.L, j.Rn, j.Rn, 1, dout.p)) return rc;
    TPST_HIP(ctx, hipMemcpyAsync(j.out, dout.p, j.L * 96, hipMemcpyDeviceToHost, ctx->stream));
    TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return TPST_OK;
}
