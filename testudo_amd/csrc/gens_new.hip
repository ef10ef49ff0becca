// MultiCommitGens::new (commitments.rs:17-39) on the device: the Pedersen /
// Hyrax generators of a label.
//
//   sponge = PoseidonSponge<Fr>(poseidon_params())   (parameters.rs:156-186)
//   sponge.absorb(label); sponge.absorb(G1 generator, compressed)
//   G_i = Affine::rand(StdRng::from_seed(sponge.squeeze_bytes(32)))  i = 0..n
//
// The sponge is sequential and cheap (one permutation per generator): host.
// Each generator's StdRng (= ChaCha12) stream, Fq::rand rejection sampling,
// square root and cofactor clearing are independent: one device lane each
// (a 2^12-generator set costs milliseconds instead of seconds on the host).
// Algorithms restated from the published crates (rand 0.8 / rand_chacha 0.3 /
// ark 0.4, not vendored here) -- see oracle/py/gens.py; parity unpinned.
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/tpst.h"
#include "ctx.h"
#include "device_util.h"

using namespace tpst;

#include "poseidon_constants.inc"

namespace {

inline unsigned grid_for(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// ------------------------------------------------------------ host sponge --
const uint64_t FR_P64[4] = {0x0a11800000000001ull, 0x59aa76fed0000001ull, 0x60b44d1e5c37b001ull,
                            0x12ab655e9a2ca556ull};

bool ge_r(const uint64_t* v) {
  for (int k = 3; k >= 0; k--)
    if (v[k] != FR_P64[k]) return v[k] > FR_P64[k];
  return true;
}

// a < 2^256 canonical -> Montgomery Fr (reduced mod r)
Fr fr_from_u256(const uint64_t* a) {
  uint64_t v[4] = {a[0], a[1], a[2], a[3]};
  while (ge_r(v)) {
    unsigned __int128 br = 0;
    for (int k = 0; k < 4; k++) {
      const unsigned __int128 d = (unsigned __int128)v[k] - FR_P64[k] - (uint64_t)br;
      v[k] = (uint64_t)d;
      br = (d >> 64) & 1;
    }
  }
  Fr f;
  memcpy(f.v, v, 32);
  return to_mont(f);
}

struct FrPoseidon {
  Fr ark[39][3], mds[3][3];
  FrPoseidon() {
    for (int r = 0; r < 39; r++)
      for (int i = 0; i < 3; i++) ark[r][i] = fr_from_u256(POSEIDON_ARK[r][i]);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) mds[i][j] = fr_from_u256(POSEIDON_MDS[i][j]);
  }
};

const FrPoseidon& frp() {
  static FrPoseidon p;
  return p;
}

// PoseidonSponge<Fr>: rate 2, capacity 1, alpha 17, 8 full + 31 partial rounds
struct FrSponge {
  Fr st[3] = {Fr::zero(), Fr::zero(), Fr::zero()};
  bool squeezing = false;
  int idx = 0;
  void permute() {
    const FrPoseidon& P = frp();
    for (int r = 0; r < 39; r++) {
      for (int i = 0; i < 3; i++) st[i] = add(st[i], P.ark[r][i]);
      const bool full = r < 4 || r >= 35;
      for (int i = 0; i < (full ? 3 : 1); i++) {
        const Fr x = st[i], x2 = mul(x, x), x4 = mul(x2, x2), x8 = mul(x4, x4), x16 = mul(x8, x8);
        st[i] = mul(x16, x);
      }
      Fr ns[3];
      for (int i = 0; i < 3; i++) ns[i] = add(add(mul(P.mds[i][0], st[0]), mul(P.mds[i][1], st[1])), mul(P.mds[i][2], st[2]));
      for (int i = 0; i < 3; i++) st[i] = ns[i];
    }
  }
  void absorb(const std::vector<Fr>& e) {
    if (squeezing || idx == 2) {
      permute();
      idx = 0;
    }
    for (const Fr& x : e) {
      if (idx == 2) {
        permute();
        idx = 0;
      }
      st[1 + idx] = add(st[1 + idx], x);
      idx++;
    }
    squeezing = false;
  }
  // Absorb for byte slices: u64 LE length prefix, 31-byte LE chunks
  void absorb_bytes(const uint8_t* d, size_t n) {
    std::vector<uint8_t> buf(8 + n);
    const uint64_t len = n;
    memcpy(buf.data(), &len, 8);
    if (n) memcpy(buf.data() + 8, d, n);
    std::vector<Fr> e;
    for (size_t o = 0; o < buf.size(); o += 31) {
      uint64_t l[4] = {0, 0, 0, 0};
      memcpy(l, buf.data() + o, buf.size() - o < 31 ? buf.size() - o : 31);
      e.push_back(fr_from_u256(l));
    }
    absorb(e);
  }
  Fr squeeze1() {
    if (!squeezing || idx == 2) {
      permute();
      idx = 0;
    }
    squeezing = true;
    return st[1 + idx++];
  }
  // squeeze_bytes(32): two native elements, 31 LE bytes of each, truncated
  void squeeze32(uint8_t* out) {
    uint8_t b[62];
    for (int k = 0; k < 2; k++) {
      const Fr c = from_mont(squeeze1());
      memcpy(b + 31 * k, c.v, 31);
    }
    memcpy(out, b, 32);
  }
};

// ----------------------------------------------------------- device side --
struct SqrtConsts {
  uint32_t e[12];   // (q - 1) / 2, q = (p - 1) / 2^46
  uint32_t zq[12];  // z^q (Montgomery), z the least non-residue
};

__device__ Fq fq_pow_dev(const Fq& a, const uint32_t* e, int nbits) {
  Fq r = Fq::one();
  for (int b = nbits - 1; b >= 0; b--) {
    r = mul(r, r);
    if ((e[b >> 5] >> (b & 31)) & 1) r = mul(r, a);
  }
  return r;
}

// Tonelli-Shanks (2-adicity 46); false for a non-residue
__device__ bool fq_sqrt_dev(const Fq& a, const SqrtConsts& K, Fq& out) {
  if (is_zero(a)) {
    out = a;
    return true;
  }
  const Fq w = fq_pow_dev(a, K.e, 330);
  Fq r = mul(a, w), t = mul(r, w), c = Fq::from_limbs(K.zq);
  int m = 46;
  while (!eq(t, Fq::one())) {
    int i = 0;
    Fq t2 = t;
    while (!eq(t2, Fq::one())) {
      t2 = mul(t2, t2);
      if (++i == m) return false;
    }
    Fq b = c;
    for (int k = 0; k < m - i - 1; k++) b = mul(b, b);
    m = i;
    c = mul(b, b);
    t = mul(t, c);
    r = mul(r, b);
  }
  out = r;
  return true;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }

// ChaCha12 keystream (rand_chacha 0.3 ChaCha12Rng: key = seed, counter from 0,
// nonce 0), consumed word by word
struct ChaChaDev {
  uint32_t key[8];
  uint32_t ctr = 0;
  uint32_t buf[16];
  int pos = 16;
  __device__ void refill() {
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4],      key[5],      key[6],      key[7],      ctr,    0u,     0u,     0u};
    uint32_t s[16];
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = x[i];
#define QR(a, b, c, d)                \
  x[a] += x[b];                       \
  x[d] = rotl32(x[d] ^ x[a], 16);     \
  x[c] += x[d];                       \
  x[b] = rotl32(x[b] ^ x[c], 12);     \
  x[a] += x[b];                       \
  x[d] = rotl32(x[d] ^ x[a], 8);      \
  x[c] += x[d];                       \
  x[b] = rotl32(x[b] ^ x[c], 7);
    for (int r = 0; r < 6; r++) {
      QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
      QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
    }
#undef QR
#pragma unroll
    for (int i = 0; i < 16; i++) buf[i] = x[i] + s[i];
    ctr++;
    pos = 0;
  }
  __device__ uint32_t next_u32() {
    if (pos == 16) refill();
    return buf[pos++];
  }
};

__device__ bool lt_p_words(const uint32_t* w) {
  for (int i = 11; i >= 0; i--)
    if (w[i] != params::FQ_P[i]) return w[i] < params::FQ_P[i];
  return false;
}

__device__ int cmp_canon(const Fq& a, const Fq& b) {
  const Fq x = from_mont(a), y = from_mont(b);
  for (int i = 11; i >= 0; i--)
    if (x.v[i] != y.v[i]) return x.v[i] < y.v[i] ? -1 : 1;
  return 0;
}

// G1 cofactor (x - 1)^2 / 3 = 0x170b5d44300000000000000000000000 (125 bits)
__constant__ uint32_t G1_COFACTOR[4] = {0x00000000u, 0x00000000u, 0x30000000u, 0x170b5d44u};

// one lane per generator: Affine::rand over ChaCha12(seed); canonical x || y out
__global__ void __launch_bounds__(64) k_gens_from_seeds(const uint8_t* __restrict__ seeds, size_t n, SqrtConsts K,
                                                       uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ChaChaDev rng;
  for (int k = 0; k < 8; k++) {
    const uint8_t* s = seeds + 32 * i + 4 * k;
    rng.key[k] = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
  }
  G1A pt;
  for (;;) {
    Fq x;  // Fq::rand: 6 u64 limbs = the Montgomery form, top limb to 57 bits, < p
    for (;;) {
      for (int k = 0; k < 12; k++) x.v[k] = rng.next_u32();
      x.v[11] &= (1u << 25) - 1;
      if (lt_p_words(x.v)) break;
    }
    const bool greatest = (rng.next_u32() >> 31) != 0;
    Fq y;
    if (!fq_sqrt_dev(add(mul(mul(x, x), x), Fq::one()), K, y)) continue;
    const Fq ny = neg(y);
    const bool y_larger = cmp_canon(y, ny) > 0;
    pt = {x, (greatest == y_larger) ? y : ny};
    break;
  }
  const G1A r = to_affine(scalar_mul(pt, G1_COFACTOR, 125));
  store_f<Fq>(out + 24 * i, from_mont(r.x));
  store_f<Fq>(out + 24 * i + 12, from_mont(r.y));
}

SqrtConsts sqrt_consts() {
  // e = (q - 1) / 2 with q = (p - 1) >> 46 (p - 1 = p with limb 0 cleared: p's low word is 1)
  uint32_t pm1[12];
  for (int i = 0; i < 12; i++) pm1[i] = params::FQ_P[i];
  pm1[0] -= 1;
  auto shr = [](uint32_t* a, int s) {
    for (int k = 0; k < s; k++)
      for (int i = 0; i < 12; i++) a[i] = (a[i] >> 1) | (i < 11 ? a[i + 1] << 31 : 0);
  };
  SqrtConsts K;
  uint32_t q[12];
  memcpy(q, pm1, 48);
  shr(q, 46);
  memcpy(K.e, q, 48);
  K.e[0] -= 1;  // q odd
  shr(K.e, 1);
  // z = least quadratic non-residue: z^((p-1)/2) = -1
  uint32_t half[12];
  memcpy(half, pm1, 48);
  shr(half, 1);
  auto powh = [](const Fq& a, const uint32_t* e, int nb) {
    Fq r = Fq::one();
    for (int b = nb - 1; b >= 0; b--) {
      r = mul(r, r);
      if ((e[b >> 5] >> (b & 31)) & 1) r = mul(r, a);
    }
    return r;
  };
  Fq z = Fq::one();
  const Fq minus1 = neg(Fq::one());
  do {
    z = add(z, Fq::one());
  } while (!eq(powh(z, half, 377), minus1));
  const Fq zq = powh(z, q, 331);
  memcpy(K.zq, zq.v, 48);
  return K;
}

// compressed G1 generator (48 bytes): canonical x with the YIsNegative flag
// (params hold the generator in Montgomery form)
void g1_gen_compressed(uint8_t* b) {
  const Fq xm = Fq::from_limbs(params::G1_GEN_X), ym = Fq::from_limbs(params::G1_GEN_Y);
  const Fq xc = from_mont(xm), yc = from_mont(ym), nyc = from_mont(neg(ym));
  memcpy(b, xc.v, 48);
  bool negf = false;
  for (int i = 11; i >= 0; i--)
    if (yc.v[i] != nyc.v[i]) {
      negf = yc.v[i] > nyc.v[i];
      break;
    }
  if (negf) b[47] |= 0x80;
}

}  // namespace

// the n + 1 StdRng seeds of MultiCommitGens::new (host only)
static void gens_seeds(size_t n, const uint8_t* label, size_t label_len, uint8_t* seeds) {
  FrSponge sp;
  sp.absorb_bytes(label, label_len);
  uint8_t gb[48];
  g1_gen_compressed(gb);
  sp.absorb_bytes(gb, 48);
  for (size_t i = 0; i <= n; i++) sp.squeeze32(seeds + 32 * i);
}

extern "C" int tpst_gens_seeds(size_t n, const uint8_t* label, size_t label_len, uint8_t* seeds) {
  if (!seeds || (label_len && !label)) return TPST_E_ARG;
  gens_seeds(n, label, label_len, seeds);
  return TPST_OK;
}

extern "C" int tpst_gens_new(tpst_ctx* ctx, size_t n, const uint8_t* label, size_t label_len, uint64_t* G_out,
                             uint64_t* h_out, tpst_gens** out) {
  if (!ctx || !G_out || !h_out || (label_len && !label)) return fail(ctx, TPST_E_ARG, "null argument");
  if (n == 0 || n > ((size_t)1 << 26)) return fail(ctx, TPST_E_ARG, "n out of range");
  std::vector<uint8_t> seeds(32 * (n + 1));
  gens_seeds(n, label, label_len, seeds.data());
  static const SqrtConsts K = sqrt_consts();
  std::vector<uint64_t> pts(12 * (n + 1));
  {
    std::lock_guard<tpst::CtxMutex> lk(ctx->mu);
    TPST_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    void *d_seeds = nullptr, *d_out = nullptr;
    TPST_HIP(ctx, hipMalloc(&d_seeds, seeds.size()));
    if (hipMalloc(&d_out, pts.size() * 8) != hipSuccess) {
      (void)hipFree(d_seeds);
      return fail(ctx, TPST_E_HIP, "hipMalloc");
    }
    hipError_t e = hipMemcpyAsync(d_seeds, seeds.data(), seeds.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
      k_gens_from_seeds<<<grid_for(n + 1, 64), 64, 0, s>>>((const uint8_t*)d_seeds, n + 1, K, (uint32_t*)d_out);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(pts.data(), d_out, pts.size() * 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d_seeds);
    (void)hipFree(d_out);
    if (e != hipSuccess) return hip_fail(ctx, e, "gens_new");
  }
  memcpy(G_out, pts.data(), n * 96);
  memcpy(h_out, &pts[12 * n], 96);
  if (out) return tpst_gens_load(ctx, G_out, n, h_out, out);
  return TPST_OK;
}
