// Groth16 over BLS12-377 for an R1CS instance on gfx950 (SURVEY.md §8(f)
// rank 4): the prover behind R1CSProof::prove_verifier (r1csproof.rs:374-434,
// `Groth16::<E>::prove` at :421), i.e. ark-groth16's create_proof with the
// LibsnarkReduction QAP, plus the matching key generation and verifier.
//
//   witness map   LibsnarkReduction::witness_map_from_matrices: a, b, c = A z,
//                 B z, C z on the domain (a also carries the instance copy rows),
//                 iFFT, coset FFT (offset = Fr generator 22), (a b - c) / Z_H(g),
//                 coset iFFT -> h (n - 1 coefficients)
//   key           generate_parameters_with_qap: Lagrange coefficients at tau,
//                 a/b/c(tau) per variable (CSC column sums), the query scalars,
//                 then k * G for every query point (one lane per point)
//   prove         A = alpha + sum z_i A_i + r delta          (G1 MSM, N + 2 points)
//                 B = beta + sum z_i B_i + s delta            (G2 MSM and G1 MSM)
//                 C = sum w_i L_i + sum h_i H_i + s A + r B1 - r s delta   (G1 MSM)
//                 every constant term is a base appended to its MSM, so the
//                 prover is four msm_var calls and no lone scalar multiplication
//
// The domain lives in HBM as Montgomery Fr; the NTT is a bit reversal plus
// log2(n) radix-2 butterfly passes (HBM-bound, ~3 ms at n = 2^21 -- small next
// to the MSMs).  Variables are kept in the Spartan z order (vars, 1, inputs):
// the instance variables are z[num_vars .. num_vars + num_inputs], the witness
// z[0 .. num_vars); the proof is independent of the order.  Randomness (the
// toxic waste and r, s) is an argument, not thread_rng, so runs reproduce.
//
// The circuit the reference proves (R1CSVerificationCircuit, constraints.rs)
// is out of scope; this prover runs on any tpst_r1cs instance.
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/tpst.h"
#include "ctx.h"
#include "device_util.h"
#include "msm.h"
#include "pst_kernels.h"
#include "r1cs_state.h"

using namespace tpst;

#define TPST_TRY(x)                \
  do {                             \
    hipError_t _e = (x);           \
    if (_e != hipSuccess) return _e; \
  } while (0)

namespace {

inline unsigned grid_for(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

struct FrArg {  // an Fr passed by value to a kernel
  uint32_t v[8];
};
FrArg arg(const Fr& a) {
  FrArg r;
  memcpy(r.v, a.v, 32);
  return r;
}
__device__ __forceinline__ Fr val(const FrArg& a) { return Fr::from_limbs(a.v); }

__device__ Fr fr_pow(Fr b, uint64_t e) {
  Fr r = Fr::one();
  while (e) {
    if (e & 1) r = mul(r, b);
    b = mul(b, b);
    e >>= 1;
  }
  return r;
}

// out[i] = scale * base^i
__global__ void k_pow_table(FrArg base, FrArg scale, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_f<Fr>(out + 8 * i, mul(val(scale), fr_pow(val(base), i)));
}

__global__ void k_bitrev(uint32_t* __restrict__ a, size_t n, int lg) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t j = __brevll((unsigned long long)i) >> (64 - lg);
  if (i < j) {
    const Fr x = load_f<Fr>(a + 8 * i), y = load_f<Fr>(a + 8 * j);
    store_f<Fr>(a + 8 * i, y);
    store_f<Fr>(a + 8 * j, x);
  }
}

// one radix-2 decimation-in-time pass over butterflies of span 2 half;
// tw[k] = w^k for k < n/2, the pass uses w^(j n / (2 half))
__global__ void k_ntt_pass(uint32_t* __restrict__ a, size_t n, size_t half, const uint32_t* __restrict__ tw) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n / 2) return;
  const size_t j = t & (half - 1);
  const size_t i0 = ((t - j) << 1) + j, i1 = i0 + half;
  const Fr w = load_f<Fr>(tw + 8 * (j * (n / (2 * half))));
  const Fr u = load_f<Fr>(a + 8 * i0);
  const Fr v = mul(load_f<Fr>(a + 8 * i1), w);
  store_f<Fr>(a + 8 * i0, add(u, v));
  store_f<Fr>(a + 8 * i1, sub(u, v));
}

// a[i] *= tab[i] for i < n (Montgomery); canon: also write from_mont to out
__global__ void k_mul_table(uint32_t* __restrict__ a, const uint32_t* __restrict__ tab, size_t n,
                            uint32_t* __restrict__ canon_out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr x = mul(load_f<Fr>(a + 8 * i), load_f<Fr>(tab + 8 * i));
  if (canon_out)
    store_f<Fr>(canon_out + 8 * i, from_mont(x));
  else
    store_f<Fr>(a + 8 * i, x);
}

// (a b - c) / Z_H(g) on the coset
__global__ void k_qap(uint32_t* __restrict__ a, const uint32_t* __restrict__ b, const uint32_t* __restrict__ c,
                      FrArg vinv, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr x = sub(mul(load_f<Fr>(a + 8 * i), load_f<Fr>(b + 8 * i)), load_f<Fr>(c + 8 * i));
  store_f<Fr>(a + 8 * i, mul(x, val(vinv)));
}

// y[row] = sum_{e in row} val_e z[col_e]  (CSR; one lane per constraint)
__global__ void k_rows(const uint32_t* __restrict__ ptr, const uint32_t* __restrict__ idx,
                       const uint32_t* __restrict__ v, const uint32_t* __restrict__ z, size_t nrows,
                       uint32_t* __restrict__ y) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  Fr acc = Fr::zero();
  for (uint32_t e = ptr[r]; e < ptr[r + 1]; e++)
    acc = add(acc, mul(load_f<Fr>(v + 8 * (size_t)e), load_f<Fr>(z + 8 * (size_t)idx[e])));
  store_f<Fr>(y + 8 * r, acc);
}

// out[col] = sum_{e in col} val_e u[row_e] for col < ncols  (CSC; a/b/c(tau))
__global__ void k_cols(const uint32_t* __restrict__ ptr, const uint32_t* __restrict__ idx,
                       const uint32_t* __restrict__ v, const uint32_t* __restrict__ u, size_t ncols,
                       uint32_t* __restrict__ out) {
  const size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  Fr acc = Fr::zero();
  for (uint32_t e = ptr[c]; e < ptr[c + 1]; e++)
    acc = add(acc, mul(load_f<Fr>(v + 8 * (size_t)e), load_f<Fr>(u + 8 * (size_t)idx[e])));
  store_f<Fr>(out + 8 * c, acc);
}

// z = vars || 1 || inputs || 0 in Montgomery form, and the canonical copies the
// MSMs take: sA = sB = z[0 .. nq), sC = z[0 .. nv)
__global__ void k_assign(const uint32_t* __restrict__ vars, size_t nv, const uint32_t* __restrict__ in, size_t ni,
                         size_t ncols, uint32_t* __restrict__ zm, uint32_t* __restrict__ sA,
                         uint32_t* __restrict__ sB, uint32_t* __restrict__ sC) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ncols) return;
  Fr c = Fr::zero();
  if (i < nv)
    c = load_f<Fr>(vars + 8 * i);
  else if (i == nv)
    c.v[0] = 1;
  else if (i <= nv + ni)
    c = load_f<Fr>(in + 8 * (i - nv - 1));
  store_f<Fr>(zm + 8 * i, to_mont(c));
  if (i <= nv + ni) {
    store_f<Fr>(sA + 8 * i, c);
    store_f<Fr>(sB + 8 * i, c);
  }
  if (i < nv) store_f<Fr>(sC + 8 * i, c);
}

// the instance copy constraints (r1cs_to_qap.rs: a[num_cons + k] = instance k)
__global__ void k_instance_rows(const uint32_t* __restrict__ zm, size_t nv, size_t ni, size_t num_cons,
                                uint32_t* __restrict__ a) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > ni) return;
  store_f<Fr>(a + 8 * (num_cons + k), load_f<Fr>(zm + 8 * (nv + k)));
}

struct Tails {  // up to 4 canonical scalars written into the MSM scalar arrays
  uint32_t v[4][8];
  uint32_t* dst[4];
  int n;
};
__global__ void k_tails(Tails t) {
  const int k = threadIdx.x;
  if (k >= t.n) return;
  for (int j = 0; j < 8; j++) t.dst[k][j] = t.v[k][j];
}

// ---- key generation
// Lagrange coefficients at tau (evaluate_all_lagrange_coefficients):
// u_i = (tau^n - 1) / n * w^i / (tau - w^i)
__global__ void k_lagrange(FrArg tau, FrArg omega, FrArg ztn, size_t n, uint32_t* __restrict__ u) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr wi = fr_pow(val(omega), i);
  store_f<Fr>(u + 8 * i, mul(mul(val(ztn), wi), inv(sub(val(tau), wi))));
}

__global__ void k_instance_cols(uint32_t* __restrict__ at, const uint32_t* __restrict__ u, size_t nv, size_t ni,
                                size_t num_cons) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > ni) return;
  store_f<Fr>(at + 8 * (nv + k), add(load_f<Fr>(at + 8 * (nv + k)), load_f<Fr>(u + 8 * (num_cons + k))));
}

// out[j] = canonical((beta a + alpha b + c)[off + j] * scale), j < cnt
__global__ void k_lin3(const uint32_t* __restrict__ at, const uint32_t* __restrict__ bt,
                       const uint32_t* __restrict__ ct, size_t off, size_t cnt, FrArg beta, FrArg alpha,
                       FrArg scale, uint32_t* __restrict__ out) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cnt) return;
  const size_t i = off + j;
  const Fr x = add(add(mul(val(beta), load_f<Fr>(at + 8 * i)), mul(val(alpha), load_f<Fr>(bt + 8 * i))),
                   load_f<Fr>(ct + 8 * i));
  store_f<Fr>(out + 8 * j, from_mont(mul(x, val(scale))));
}

// out[i] = canonical(in[i]) (Montgomery -> canonical), i < n
__global__ void k_canon(const uint32_t* __restrict__ in, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_f<Fr>(out + 8 * i, from_mont(load_f<Fr>(in + 8 * i)));
}

// h query scalars: canonical(zt / delta * tau^i)
__global__ void k_hquery(FrArg tau, FrArg scale, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_f<Fr>(out + 8 * i, from_mont(mul(val(scale), fr_pow(val(tau), i))));
}

// out[i] = k_i * G (affine, Montgomery), k canonical
template <class F>
__global__ void __launch_bounds__(64, 1) k_gen_mul(const uint32_t* __restrict__ k, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<F> g;
  if constexpr (sizeof(F) == sizeof(Fq))
    g = {Fq::from_limbs(params::G1_GEN_X), Fq::from_limbs(params::G1_GEN_Y)};
  else
    g = {fq2_const(params::G2_GEN_X), fq2_const(params::G2_GEN_Y)};
  uint32_t s[8];
#pragma unroll
  for (int j = 0; j < 8; j++) s[j] = k[8 * i + j];
  store_affine(out, i, to_affine(scalar_mul(g, s, 253)));
}

// two-adic root of unity of Fr (GENERATOR^((r - 1) / 2^47), GENERATOR = 22), canonical
constexpr uint64_t FR_ROOT47[4] = {0x476ef4a4ec2a895eull, 0x9b506ee363e3f04aull, 0x60c69477d1a8a12full,
                                   0x11d4b7f60cb92cc1ull};
constexpr int FR_TWO_ADICITY = 47;
constexpr uint32_t FR_GENERATOR = 22;

Fr fr_u64(uint64_t v) {
  Fr a = Fr::zero();
  a.v[0] = (uint32_t)v;
  a.v[1] = (uint32_t)(v >> 32);
  return to_mont(a);
}
Fr fr_pow_host(Fr b, uint64_t e) {
  Fr r = Fr::one();
  while (e) {
    if (e & 1) r = mul(r, b);
    b = mul(b, b);
    e >>= 1;
  }
  return r;
}
void fr_canon(const Fr& a, uint32_t* o) {
  const Fr c = from_mont(a);
  memcpy(o, c.v, 32);
}

}  // namespace

// ================================================================ state ==
struct tpst_groth16_pk {
  const tpst_ctx* owner = nullptr;  // the context whose device, stream and arena the key uses
  size_t num_cons = 0, nv = 0, ni = 0, ncols = 0;
  size_t nq = 0;      // variables in the QAP: nv witness + 1 + ni instance
  size_t n = 0;       // domain size
  int lg = 0;
  size_t nC = 0;      // C-MSM length: nv + (n - 1) + 3
  Fr vinv;            // 1 / (g^n - 1)
  Buf twf, twi;       // w^k, w^-k (k < n/2)
  Buf cosf, cosi;     // n^-1 g^i, n^-1 g^-i
  Buf bA, bB1, bB2, bC;  // MSM bases (affine, Montgomery) with the constant points appended
  Buf gamma_abc;      // ni + 1 G1 points (Montgomery)
  Buf vk;             // alpha_g1 | beta_g2 | gamma_g2 | delta_g2 (Montgomery)
  // prove-time scratch
  Buf a, b, c, zm, sA, sB, sC, in, out_x, out_aff;
  // the G2 MSM runs on its own stream + scratch arena, beside the G1 MSMs
  Arena ar2;
  hipStream_t s2 = nullptr;
  hipEvent_t ev_in = nullptr, ev_b2 = nullptr;
  hipError_t side_init() {
    if (s2) return hipSuccess;
    TPST_TRY(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    TPST_TRY(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    return hipEventCreateWithFlags(&ev_b2, hipEventDisableTiming);
  }
  ~tpst_groth16_pk() {
    if (s2) (void)hipStreamSynchronize(s2);
    ar2.release();
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_b2) (void)hipEventDestroy(ev_b2);
    if (s2) (void)hipStreamDestroy(s2);
  }
};

static int setup_fail(tpst_ctx* ctx, const char* m) { return fail(ctx, TPST_E_ARG, m); }

// NTT of `a` in place: natural order in, natural order out; tw = w^k table
static hipError_t ntt(hipStream_t s, uint32_t* a, size_t n, int lg, const uint32_t* tw) {
  k_bitrev<<<grid_for(n, 256), 256, 0, s>>>(a, n, lg);
  TPST_TRY(hipGetLastError());
  for (size_t half = 1; half < n; half <<= 1) {
    k_ntt_pass<<<grid_for(n / 2, 256), 256, 0, s>>>(a, n, half, tw);
    TPST_TRY(hipGetLastError());
  }
  return hipSuccess;
}

extern "C" int tpst_groth16_setup(tpst_ctx* ctx, tpst_r1cs* R, const uint64_t* toxic, tpst_groth16_pk** out) {
  if (!ctx || !R || !toxic || !out) return setup_fail(ctx, "null argument");
  if (R->owner != ctx) return setup_fail(ctx, "instance belongs to another context");
  *out = nullptr;
  for (int k = 0; k < 5; k++) {
    if (!fr_ok_host(toxic + 4 * k)) return setup_fail(ctx, "toxic waste value >= r");
    const uint64_t* t = toxic + 4 * k;
    if (!(t[0] | t[1] | t[2] | t[3])) return setup_fail(ctx, "toxic waste value is zero");
  }
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  std::unique_ptr<tpst_groth16_pk> P(new tpst_groth16_pk());
  P->owner = ctx;
  P->num_cons = R->num_cons;
  P->nv = R->num_vars;
  P->ni = R->num_inputs;
  P->ncols = R->ncols;
  P->nq = P->nv + P->ni + 1;
  const size_t dom = P->num_cons + P->ni + 1;  // constraints + instance copy rows
  P->lg = 1;
  while (((size_t)1 << P->lg) < dom) P->lg++;
  if (P->lg > 28) return setup_fail(ctx, "domain too large");
  const size_t n = P->n = (size_t)1 << P->lg;
  P->nC = P->nv + (n - 1) + 3;
  if (P->nC > MSM_MAX_POINTS) return setup_fail(ctx, "instance too large");
  const Fr tau = frc(toxic), alpha = frc(toxic + 4), beta = frc(toxic + 8), gamma = frc(toxic + 12),
           delta = frc(toxic + 16);
  // domain constants
  Fr omega = frc(FR_ROOT47);
  for (int k = P->lg; k < FR_TWO_ADICITY; k++) omega = mul(omega, omega);
  const Fr omega_inv = inv(omega), n_inv = inv(fr_u64(n)), g = fr_u64(FR_GENERATOR), g_inv = inv(g);
  P->vinv = inv(sub(fr_pow_host(g, n), Fr::one()));
  const Fr zt = sub(fr_pow_host(tau, n), Fr::one());
  if (is_zero(zt)) return setup_fail(ctx, "tau lies in the evaluation domain");
  const Fr delta_inv = inv(delta), gamma_inv = inv(gamma);
  // tables
  TPST_HIP(ctx, P->twf.alloc(n / 2 * 32));
  TPST_HIP(ctx, P->twi.alloc(n / 2 * 32));
  TPST_HIP(ctx, P->cosf.alloc(n * 32));
  TPST_HIP(ctx, P->cosi.alloc(n * 32));
  k_pow_table<<<grid_for(n / 2, 256), 256, 0, s>>>(arg(omega), arg(Fr::one()), n / 2, P->twf.u());
  k_pow_table<<<grid_for(n / 2, 256), 256, 0, s>>>(arg(omega_inv), arg(Fr::one()), n / 2, P->twi.u());
  k_pow_table<<<grid_for(n, 256), 256, 0, s>>>(arg(g), arg(n_inv), n, P->cosf.u());
  k_pow_table<<<grid_for(n, 256), 256, 0, s>>>(arg(g_inv), arg(n_inv), n, P->cosi.u());
  TPST_HIP(ctx, hipGetLastError());
  // a, b, c at tau per variable
  Buf u, at, bt, ct, sc;
  TPST_HIP(ctx, u.alloc(n * 32));
  k_lagrange<<<grid_for(n, 256), 256, 0, s>>>(arg(tau), arg(omega), arg(mul(zt, n_inv)), n, u.u());
  TPST_HIP(ctx, hipGetLastError());
  Buf* tabs[3] = {&at, &bt, &ct};
  for (int m = 0; m < 3; m++) {
    TPST_HIP(ctx, tabs[m]->alloc(P->ncols * 32));
    k_cols<<<grid_for(P->ncols, 256), 256, 0, s>>>(R->cptr[m].u(), R->cidx[m].u(), R->cval[m].u(), u.u(), P->ncols,
                                                   tabs[m]->u());
    TPST_HIP(ctx, hipGetLastError());
  }
  k_instance_cols<<<grid_for(P->ni + 1, 64), 64, 0, s>>>(at.u(), u.u(), P->nv, P->ni, P->num_cons);
  TPST_HIP(ctx, hipGetLastError());
  // query scalars (canonical) -> points.  Layouts:
  //   bA  = a(tau)[0..nq) | alpha | delta        bB1 = b(tau)[0..nq) | beta | delta   (G1)
  //   bB2 = b(tau)[0..nq) | beta | delta  (G2)
  //   bC  = L[0..nv) | H[0..n-1) | A slot | B1 slot | delta
  const size_t nA = P->nq + 2;
  TPST_HIP(ctx, sc.alloc(std::max(nA, P->nC) * 32));
  TPST_HIP(ctx, P->bA.alloc(nA * 96));
  TPST_HIP(ctx, P->bB1.alloc(nA * 96));
  TPST_HIP(ctx, P->bB2.alloc(nA * 192));
  TPST_HIP(ctx, P->bC.alloc(P->nC * 96));
  TPST_HIP(ctx, P->gamma_abc.alloc((P->ni + 1) * 96));
  TPST_HIP(ctx, P->vk.alloc(96 + 3 * 192));
  auto tails = [&](uint32_t* base, size_t at_idx, std::initializer_list<Fr> vals) -> hipError_t {
    Tails t{};
    t.n = 0;
    for (const Fr& v : vals) {
      fr_canon(v, t.v[t.n]);
      t.dst[t.n] = base + 8 * (at_idx + t.n);
      t.n++;
    }
    k_tails<<<1, 64, 0, s>>>(t);
    return hipGetLastError();
  };
  // A
  k_canon<<<grid_for(P->nq, 256), 256, 0, s>>>(at.u(), P->nq, sc.u());
  TPST_HIP(ctx, tails(sc.u(), P->nq, {alpha, delta}));
  k_gen_mul<Fq><<<grid_for(nA, 64), 64, 0, s>>>(sc.u(), nA, P->bA.u());
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, hipStreamSynchronize(s));  // sc is reused
  // B (G1 and G2)
  k_canon<<<grid_for(P->nq, 256), 256, 0, s>>>(bt.u(), P->nq, sc.u());
  TPST_HIP(ctx, tails(sc.u(), P->nq, {beta, delta}));
  k_gen_mul<Fq><<<grid_for(nA, 64), 64, 0, s>>>(sc.u(), nA, P->bB1.u());
  k_gen_mul<Fq2><<<grid_for(nA, 64), 64, 0, s>>>(sc.u(), nA, P->bB2.u());
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, hipStreamSynchronize(s));
  // C: L (witness), H, two slots filled by the prover, delta
  k_lin3<<<grid_for(P->nv, 256), 256, 0, s>>>(at.u(), bt.u(), ct.u(), 0, P->nv, arg(beta), arg(alpha),
                                              arg(delta_inv), sc.u());
  k_hquery<<<grid_for(n - 1, 256), 256, 0, s>>>(arg(tau), arg(mul(zt, delta_inv)), n - 1, sc.u() + 8 * P->nv);
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, tails(sc.u(), P->nv + n - 1, {Fr::zero(), Fr::zero(), delta}));
  k_gen_mul<Fq><<<grid_for(P->nC, 64), 64, 0, s>>>(sc.u(), P->nC, P->bC.u());
  TPST_HIP(ctx, hipGetLastError());
  TPST_HIP(ctx, hipStreamSynchronize(s));
  // verifying key: gamma_abc over the instance variables, alpha_g1, beta/gamma/delta_g2
  k_lin3<<<grid_for(P->ni + 1, 64), 64, 0, s>>>(at.u(), bt.u(), ct.u(), P->nv, P->ni + 1, arg(beta),
                                                          arg(alpha), arg(gamma_inv), sc.u());
  TPST_HIP(ctx, hipGetLastError());
  k_gen_mul<Fq><<<grid_for(P->ni + 1, 64), 64, 0, s>>>(sc.u(), P->ni + 1, P->gamma_abc.u());
  TPST_HIP(ctx, tails(sc.u(), 0, {alpha, beta, gamma, delta}));
  k_gen_mul<Fq><<<1, 64, 0, s>>>(sc.u(), 1, P->vk.u());
  k_gen_mul<Fq2><<<1, 64, 0, s>>>(sc.u() + 8, 3, P->vk.u() + 24);
  TPST_HIP(ctx, hipGetLastError());
  // prove-time scratch
  TPST_HIP(ctx, P->a.alloc(n * 32));
  TPST_HIP(ctx, P->b.alloc(n * 32));
  TPST_HIP(ctx, P->c.alloc(n * 32));
  TPST_HIP(ctx, P->zm.alloc(P->ncols * 32));
  TPST_HIP(ctx, P->sA.alloc(nA * 32));
  TPST_HIP(ctx, P->sB.alloc(nA * 32));
  TPST_HIP(ctx, P->sC.alloc(P->nC * 32));
  TPST_HIP(ctx, P->in.alloc((P->nv + P->ni + 1) * 32));
  TPST_HIP(ctx, P->out_x.alloc(4 * sizeof(Xyzz<Fq2>)));
  TPST_HIP(ctx, P->out_aff.alloc(4 * 192));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  *out = P.release();
  return TPST_OK;
}

extern "C" void tpst_groth16_pk_free(tpst_groth16_pk* pk) { delete pk; }

extern "C" int tpst_groth16_domain(const tpst_groth16_pk* pk, size_t* n) {
  if (!pk || !n) return TPST_E_ARG;
  *n = pk->n;
  return TPST_OK;
}

extern "C" int tpst_groth16_vk(tpst_ctx* ctx, const tpst_groth16_pk* pk, uint64_t* alpha_g1, uint64_t* beta_g2,
                               uint64_t* gamma_g2, uint64_t* delta_g2, uint64_t* gamma_abc_g1) {
  if (!ctx || !pk || !alpha_g1 || !beta_g2 || !gamma_g2 || !delta_g2 || !gamma_abc_g1)
    return fail(ctx, TPST_E_ARG, "null argument");
  if (pk->owner != ctx) return fail(ctx, TPST_E_ARG, "proving key belongs to another context");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  Buf o;
  const size_t ng = pk->ni + 1;
  TPST_HIP(ctx, o.alloc(96 + 3 * 192 + ng * 96));
  TPST_HIP(ctx, affine_from_mont<Fq>(s, pk->vk.u(), o.u(), 1));
  TPST_HIP(ctx, affine_from_mont<Fq2>(s, pk->vk.u() + 24, o.u() + 24, 3));
  TPST_HIP(ctx, affine_from_mont<Fq>(s, pk->gamma_abc.u(), o.u() + 24 + 144, ng));
  std::vector<uint64_t> h((96 + 3 * 192 + ng * 96) / 8);
  TPST_HIP(ctx, hipMemcpyAsync(h.data(), o.p, h.size() * 8, hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  memcpy(alpha_g1, h.data(), 96);
  memcpy(beta_g2, h.data() + 12, 192);
  memcpy(gamma_g2, h.data() + 36, 192);
  memcpy(delta_g2, h.data() + 60, 192);
  memcpy(gamma_abc_g1, h.data() + 84, ng * 96);
  return TPST_OK;
}

// the QAP witness map: a/b/c on the domain -> h on the coset -> h coefficients
// (first n - 1, canonical) into pk->sC[nv ..]
static hipError_t witness_map(tpst_groth16_pk* P, const tpst_r1cs* R, hipStream_t s) {
  const size_t n = P->n;
  uint32_t* tabs[3] = {P->a.u(), P->b.u(), P->c.u()};
  for (int m = 0; m < 3; m++) {
    TPST_TRY(hipMemsetAsync(tabs[m] + 8 * P->num_cons, 0, (n - P->num_cons) * 32, s));
    k_rows<<<grid_for(P->num_cons, 256), 256, 0, s>>>(R->rptr[m].u(), R->ridx[m].u(), R->rval[m].u(), P->zm.u(),
                                                      P->num_cons, tabs[m]);
    TPST_TRY(hipGetLastError());
  }
  k_instance_rows<<<grid_for(P->ni + 1, 64), 64, 0, s>>>(P->zm.u(), P->nv, P->ni, P->num_cons, P->a.u());
  TPST_TRY(hipGetLastError());
  for (int m = 0; m < 3; m++) {
    TPST_TRY(ntt(s, tabs[m], n, P->lg, P->twi.u()));  // coefficients (times n)
    k_mul_table<<<grid_for(n, 256), 256, 0, s>>>(tabs[m], P->cosf.u(), n, nullptr);
    TPST_TRY(hipGetLastError());
    TPST_TRY(ntt(s, tabs[m], n, P->lg, P->twf.u()));  // evaluations on the coset g H
  }
  k_qap<<<grid_for(n, 256), 256, 0, s>>>(P->a.u(), P->b.u(), P->c.u(), arg(P->vinv), n);
  TPST_TRY(hipGetLastError());
  TPST_TRY(ntt(s, P->a.u(), n, P->lg, P->twi.u()));
  k_mul_table<<<grid_for(n - 1, 256), 256, 0, s>>>(P->a.u(), P->cosi.u(), n - 1, P->sC.u() + 8 * P->nv);
  return hipGetLastError();
}

static int check_inputs(tpst_ctx* ctx, const tpst_groth16_pk* P, const tpst_r1cs* R, const uint64_t* vars,
                        const uint64_t* inputs) {
  if (P->owner != ctx || R->owner != ctx) return fail(ctx, TPST_E_ARG, "key or instance belongs to another context");
  if (R->num_cons != P->num_cons || R->num_vars != P->nv || R->num_inputs != P->ni)
    return fail(ctx, TPST_E_ARG, "proving key does not match the instance");
  for (size_t i = 0; i < P->nv; i++)
    if (!fr_ok_host(vars + 4 * i)) return fail(ctx, TPST_E_ARG, "witness value >= r");
  for (size_t i = 0; i < P->ni; i++)
    if (!fr_ok_host(inputs + 4 * i)) return fail(ctx, TPST_E_ARG, "input value >= r");
  return TPST_OK;
}

static int upload_assignment(tpst_ctx* ctx, tpst_groth16_pk* P, const uint64_t* vars, const uint64_t* inputs) {
  hipStream_t s = ctx->stream;
  TPST_HIP(ctx, hipMemcpyAsync(P->in.p, vars, P->nv * 32, hipMemcpyHostToDevice, s));
  if (P->ni)
    TPST_HIP(ctx, hipMemcpyAsync(P->in.u() + 8 * P->nv, inputs, P->ni * 32, hipMemcpyHostToDevice, s));
  k_assign<<<grid_for(P->ncols, 256), 256, 0, s>>>(P->in.u(), P->nv, P->in.u() + 8 * P->nv, P->ni, P->ncols,
                                                   P->zm.u(), P->sA.u(), P->sB.u(), P->sC.u());
  TPST_HIP(ctx, hipGetLastError());
  return TPST_OK;
}

extern "C" int tpst_groth16_witness_map(tpst_ctx* ctx, tpst_groth16_pk* pk, tpst_r1cs* R, const uint64_t* vars,
                                        const uint64_t* inputs, uint64_t* h) {
  if (!ctx || !pk || !R || !vars || (R->num_inputs && !inputs) || !h) return fail(ctx, TPST_E_ARG, "null argument");
  if (int rc = check_inputs(ctx, pk, R, vars, inputs)) return rc;
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  if (int rc = upload_assignment(ctx, pk, vars, inputs)) return rc;
  TPST_HIP(ctx, witness_map(pk, R, ctx->stream));
  TPST_HIP(ctx, hipMemcpyAsync(h, pk->sC.u() + 8 * pk->nv, (pk->n - 1) * 32, hipMemcpyDeviceToHost, ctx->stream));
  TPST_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return TPST_OK;
}

extern "C" int tpst_groth16_prove(tpst_ctx* ctx, tpst_groth16_pk* pk, tpst_r1cs* R, const uint64_t* vars,
                                  const uint64_t* inputs, const uint64_t* rs, uint64_t* A, uint64_t* B,
                                  uint64_t* C) {
  if (!ctx || !pk || !R || !vars || (R->num_inputs && !inputs) || !rs || !A || !B || !C)
    return fail(ctx, TPST_E_ARG, "null argument");
  if (int rc = check_inputs(ctx, pk, R, vars, inputs)) return rc;
  if (!fr_ok_host(rs) || !fr_ok_host(rs + 4)) return fail(ctx, TPST_E_ARG, "r or s >= r");
  std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
  TPST_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  tpst_groth16_pk* P = pk;
  const Fr r = frc(rs), sv = frc(rs + 4);
  if (int rc = upload_assignment(ctx, P, vars, inputs)) return rc;
  // constant terms of each MSM (canonical scalars after the variables)
  const size_t nA = P->nq + 2, tc = P->nv + P->n - 1;
  {
    Tails t{};
    const Fr one = Fr::one(), mrs = neg(mul(r, sv));
    const Fr v[4] = {one, r, one, sv};
    uint32_t* d[4] = {P->sA.u() + 8 * P->nq, P->sA.u() + 8 * (P->nq + 1), P->sB.u() + 8 * P->nq,
                      P->sB.u() + 8 * (P->nq + 1)};
    t.n = 4;
    for (int k = 0; k < 4; k++) {
      fr_canon(v[k], t.v[k]);
      t.dst[k] = d[k];
    }
    k_tails<<<1, 64, 0, s>>>(t);
    Tails t2{};
    const Fr v2[3] = {sv, r, mrs};
    t2.n = 3;
    for (int k = 0; k < 3; k++) {
      fr_canon(v2[k], t2.v[k]);
      t2.dst[k] = P->sC.u() + 8 * (tc + k);
    }
    k_tails<<<1, 64, 0, s>>>(t2);
    TPST_HIP(ctx, hipGetLastError());
  }
  Xyzz<Fq>* xA = (Xyzz<Fq>*)P->out_x.p;
  Xyzz<Fq>* xB1 = xA + 1;
  Xyzz<Fq>* xC = xA + 2;
  Xyzz<Fq2>* xB2 = (Xyzz<Fq2>*)(xA + 3);
  // B in G2 on the side stream once its scalars are in place (the G2 bucket
  // accumulation runs at low occupancy: the witness map and the G1 MSMs fill
  // the rest of the chip)
  TPST_HIP(ctx, P->side_init());
  TPST_HIP(ctx, hipEventRecord(P->ev_in, s));
  TPST_HIP(ctx, hipStreamWaitEvent(P->s2, P->ev_in, 0));
  TPST_HIP(ctx, msm_var<Fq2>(P->ar2, P->s2, P->bB2.u(), P->sB.u(), nA, xB2));
  TPST_HIP(ctx, hipEventRecord(P->ev_b2, P->s2));
  TPST_HIP(ctx, witness_map(P, R, s));
  TPST_HIP(ctx, msm_var<Fq>(ctx->arena, s, P->bA.u(), P->sA.u(), nA, xA));
  TPST_HIP(ctx, msm_var<Fq>(ctx->arena, s, P->bB1.u(), P->sB.u(), nA, xB1));
  // A and B1 become bases of the C MSM (slots after L and H)
  TPST_HIP(ctx, xyzz_to_affine_mont<Fq>(s, xA, P->bC.u() + 24 * tc, 2));
  TPST_HIP(ctx, msm_var<Fq>(ctx->arena, s, P->bC.u(), P->sC.u(), P->nC, xC));
  TPST_HIP(ctx, hipStreamWaitEvent(s, P->ev_b2, 0));
  uint32_t* o = P->out_aff.u();
  TPST_HIP(ctx, xyzz_to_affine_canonical<Fq>(s, xA, o, 1));
  TPST_HIP(ctx, xyzz_to_affine_canonical<Fq>(s, xC, o + 24, 1));
  TPST_HIP(ctx, xyzz_to_affine_canonical<Fq2>(s, xB2, o + 48, 1));
  uint64_t h[12 + 12 + 24];
  TPST_HIP(ctx, hipMemcpyAsync(h, o, sizeof(h), hipMemcpyDeviceToHost, s));
  TPST_HIP(ctx, hipStreamSynchronize(s));
  memcpy(A, h, 96);
  memcpy(C, h + 12, 96);
  memcpy(B, h + 24, 192);
  return TPST_OK;
}

// Groth16::verify_proof (ark-groth16 verifier.rs, r1csproof.rs verifier side):
// every element is validated first -- canonical coordinates, on the curve, in
// the r-torsion subgroup, inputs < r -- as arkworks' deserialisation with
// Validate::Yes would; then e(A, B) == e(alpha, beta) e(IC, gamma) e(C, delta)
// with IC = gamma_abc[0] + sum_i inputs_i gamma_abc[i + 1] (device MSM), as one
// device multi-pairing of (A, B), (-alpha, beta), (-IC, gamma), (-C, delta).
bool tpst_internal_g1_valid(const uint64_t* p);  // pst_api.hip
bool tpst_internal_g2_valid(const uint64_t* p);

extern "C" int tpst_groth16_verify(tpst_ctx* ctx, const uint64_t* alpha_g1, const uint64_t* beta_g2,
                                   const uint64_t* gamma_g2, const uint64_t* delta_g2, const uint64_t* gamma_abc_g1,
                                   size_t n_abc, const uint64_t* inputs, size_t n_inputs, const uint64_t* A,
                                   const uint64_t* B, const uint64_t* C) {
  if (!ctx || !alpha_g1 || !beta_g2 || !gamma_g2 || !delta_g2 || !gamma_abc_g1 || (n_inputs && !inputs) || !A ||
      !B || !C)
    return fail(ctx, TPST_E_ARG, "null argument");
  if (n_abc != n_inputs + 1) return fail(ctx, TPST_E_ARG, "wrong number of public inputs");
  for (size_t i = 0; i < n_inputs; i++)
    if (!fr_ok_host(inputs + 4 * i)) return fail(ctx, TPST_E_VERIFY, "public input >= r");
  if (!tpst_internal_g1_valid(A) || !tpst_internal_g2_valid(B) || !tpst_internal_g1_valid(C))
    return fail(ctx, TPST_E_VERIFY, "malformed proof element");
  if (!tpst_internal_g1_valid(alpha_g1) || !tpst_internal_g2_valid(beta_g2) || !tpst_internal_g2_valid(gamma_g2) ||
      !tpst_internal_g2_valid(delta_g2))
    return fail(ctx, TPST_E_VERIFY, "malformed verifying key");
  for (size_t i = 0; i < n_abc; i++)
    if (!tpst_internal_g1_valid(gamma_abc_g1 + 12 * i)) return fail(ctx, TPST_E_VERIFY, "malformed verifying key");
  std::vector<uint64_t> sc(4 * n_abc, 0);
  sc[0] = 1;
  if (n_inputs) memcpy(sc.data() + 4, inputs, n_inputs * 32);
  uint64_t ic[12];
  if (int rc = tpst_g1_msm(ctx, gamma_abc_g1, n_abc, sc.data(), n_abc, ic)) return rc;
  // -P of an affine point: y -> p - y (infinity, all-zero, stays)
  auto neg = [](const uint64_t* p, uint64_t* o) {
    memcpy(o, p, 96);
    bool inf = true;
    for (int k = 0; k < 12; k++) inf = inf && !p[k];
    if (inf) return;
    static const uint64_t P6[6] = {0x8508c00000000001ull, 0x170b5d4430000000ull, 0x1ef3622fba094800ull,
                                   0x1a22d9f300f5138full, 0xc63b05c06ca1493bull, 0x01ae3a4617c510eaull};
    unsigned __int128 borrow = 0;
    for (int k = 0; k < 6; k++) {
      const unsigned __int128 d = (unsigned __int128)P6[k] - p[6 + k] - borrow;
      o[6 + k] = (uint64_t)d;
      borrow = (d >> 64) ? 1 : 0;
    }
  };
  uint64_t g1[4 * 12], g2[4 * 24];
  memcpy(g1, A, 96);
  neg(alpha_g1, g1 + 12);
  neg(ic, g1 + 24);
  neg(C, g1 + 36);
  memcpy(g2, B, 192);
  memcpy(g2 + 24, beta_g2, 192);
  memcpy(g2 + 48, gamma_g2, 192);
  memcpy(g2 + 72, delta_g2, 192);
  uint64_t gt[72];
  if (int rc = tpst_multi_pairing(ctx, g1, g2, 4, gt)) return rc;
  bool one = gt[0] == 1;
  for (int k = 1; k < 72; k++) one = one && !gt[k];
  return one ? TPST_OK : fail(ctx, TPST_E_VERIFY, "pairing check failed");
}
