/*
 * tpst.h -- C ABI of the MI355X-native sqrt-PST engine (libtpst.so).
 *
 * Drop-in boundary for the BLS12-377 hot path of Testudo's sqrt-PST
 * polynomial commitment (reference: rosariocannavo/testudo).  The reference
 * has no FFI of its own; every entry point below replaces one Rust call
 * site (file:line under the reference tree), see INTEGRATION.md.
 *
 * Conventions
 *  - Field elements are CANONICAL (non-Montgomery) little-endian u64 limbs:
 *      Fr  = 4 x u64 (value < r),  Fq = 6 x u64 (value < p).
 *  - G1 affine = x || y (12 u64, 96 bytes); G2 affine = x.c0 || x.c1 ||
 *    y.c0 || y.c1 (24 u64, 192 bytes).  The point at infinity is all zero
 *    (x = y = 0 lies on neither curve), i.e. arkworks' Affine with the
 *    `infinity` flag mapped to (0, 0).
 *  - GT / Fq12 = 12 Fq in arkworks order c0.c0.c0, c0.c0.c1, c0.c1.c0, ...,
 *    c1.c2.c1 (72 u64, 576 bytes).
 *  - Caller owns every host buffer; the library reads inputs and writes
 *    outputs only.  `_dev` entry points take device pointers (hipMalloc /
 *    torch allocations on the context's device) and run on the context's
 *    stream; bases passed to `_dev` calls are in Montgomery form (the same
 *    bytes as arkworks' in-memory G1Affine x/y), scalars canonical (what
 *    arkworks' msm_bigint consumes).
 *  - Return 0 (TPST_OK) or a negative TPST_E_* code; tpst_last_error()
 *    gives the message.  No exceptions or aborts cross the ABI.  One call
 *    in flight per context (internally serialised by a mutex).
 */
#ifndef TPST_H
#define TPST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPST_OK 0
#define TPST_E_ARG -1     /* bad length / null pointer / out-of-range value */
#define TPST_E_NODEV -2   /* no HIP device */
#define TPST_E_HIP -3     /* HIP runtime failure */
#define TPST_E_STATE -4   /* e.g. no SRS loaded */
#define TPST_E_VERIFY -5  /* verification failed */

typedef struct tpst_ctx tpst_ctx;

/* ---- context ---------------------------------------------------------- */
int tpst_device_count(void);
int tpst_create(int device, tpst_ctx** out);
void tpst_destroy(tpst_ctx* ctx);
const char* tpst_last_error(const tpst_ctx* ctx);
/* hipStream_t of the context, for callers that order their own work */
void* tpst_stream(tpst_ctx* ctx);
int tpst_synchronize(tpst_ctx* ctx);
/* Ordering against a caller's stream (e.g. the framework stream that wrote a
 * device buffer handed to a _dev call, or will read one a _dev call fills).
 * The library's stream is non-blocking, so without these the two streams are
 * unordered.  tpst_wait_stream: work the library queues from now on starts
 * after everything queued on `stream` so far.  tpst_join_stream: work queued
 * on `stream` from now on starts after everything the library queued so far.
 * Both are asynchronous (one event each); stream == NULL is the legacy
 * default stream. */
int tpst_wait_stream(tpst_ctx* ctx, void* stream);
int tpst_join_stream(tpst_ctx* ctx, void* stream);

/* ---- K2: variable-base MSM ---------------------------------------------
 * sum_i scalars[i] * bases[i] over min(n_bases, n_scalars) terms.
 * Replaces <G1 as VariableBaseMSM>::msm_unchecked (sqrt_pst.rs:198,
 * mipp.rs:393 via multiexponentiation mipp.rs:385-394) and msm_bigint inside
 * MultilinearPC::commit / open. */
int tpst_g1_msm(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                size_t n_scalars, uint64_t* out);
int tpst_g2_msm(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                size_t n_scalars, uint64_t* out);
/* device-resident form: d_bases Montgomery affine (24 u32 each), d_scalars
 * canonical Fr (8 u32 each), d_out one canonical affine G1.  Stream-ordered:
 * the call starts after the work already queued on tpst_stream and the MSM's
 * end is ordered before anything queued on tpst_stream after it (the host
 * returns at once; consecutive calls run one after another on the device). */
int tpst_g1_msm_dev(tpst_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n, void* d_out);
/* Pipelined form (opt-in): consecutive calls overlap on the library's
 * internal streams (call i+1 decomposes and sorts while call i accumulates).
 * The call starts after the work already queued on tpst_stream, but its work
 * is NOT ordered before work the caller queues directly on tpst_stream
 * afterwards.  LIFETIME RULE: d_bases, d_scalars and d_out must stay
 * allocated and unmodified (and d_out unread) until tpst_synchronize,
 * tpst_join_stream or the next call of any other tpst_* entry point (each of
 * which waits for every pending pipelined MSM) -- a framework's caching
 * allocator must not recycle them before that. */
int tpst_g1_msm_dev_async(tpst_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n, void* d_out);
/* One MSM split over ranks (sqrt_pst.rs:198 / mipp.rs:393 at 1/2/4/8 GPUs):
 * each rank's share of the points as the raw XYZZ sum (192 B: X, Y, ZZ, ZZZ,
 * Montgomery u64 limbs; no per-rank affine inversion), gathered as bytes,
 * then summed on one device to one canonical affine G1 (k shares, stride_bytes
 * apart in d_parts; d_parts and stride_bytes 16-byte aligned, else TPST_E_ARG). */
int tpst_g1_msm_xyzz_dev(tpst_ctx* ctx, const void* d_bases, const void* d_scalars, size_t n, void* d_out_xyzz);
int tpst_g1_xyzz_sum_dev(tpst_ctx* ctx, const void* d_parts, size_t k, size_t stride_bytes, void* d_out);

/* Length-checked form: mipp.rs:385-394 `multiexponentiation` returns
 * Err(InvalidIPVectorLength) when the lengths differ -> TPST_E_ARG here. */
int tpst_g1_multiexp(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                     size_t n_scalars, uint64_t* out);
int tpst_g2_multiexp(tpst_ctx* ctx, const uint64_t* bases, size_t n_bases, const uint64_t* scalars,
                     size_t n_scalars, uint64_t* out);

/* ---- shared-base batch MSM and Pedersen/Hyrax commitments -----------------
 * A generator set = MultiCommitGens {n, G[n], h} (commitments.rs:9-15),
 * uploaded once (K1 window tables built here).  h may be NULL when only the
 * batch MSM is used. */
typedef struct tpst_gens tpst_gens;
int tpst_gens_load(tpst_ctx* ctx, const uint64_t* G, size_t n, const uint64_t* h, tpst_gens** out);
void tpst_gens_free(tpst_gens* gens);
/* out[r] = sum_{j < cols} scalars[r*row_stride + j*col_stride] * G[j] for
 * r < rows (canonical affine G1 each); cols must equal gens->n.  The strides
 * let one call consume a row split of Z without a host transpose: this is
 * the whole par_iter row loop of sqrt_pst.rs:121-125 / dense_mlpoly.rs:323-327
 * in one launch. */
int tpst_g1_msm_batch(tpst_ctx* ctx, const tpst_gens* gens, const uint64_t* scalars, size_t rows, size_t cols,
                      size_t row_stride, size_t col_stride, uint64_t* out);
int tpst_g1_msm_batch_dev(tpst_ctx* ctx, const tpst_gens* gens, const void* d_scalars, size_t rows, size_t cols,
                          size_t row_stride, size_t col_stride, void* d_out);
/* MultiCommitGens::new (commitments.rs:17-39): Poseidon<Fr> over label || the
 * compressed G1 generator, 32 squeezed bytes per generator -> StdRng (ChaCha12)
 * -> Affine::rand (Fq::rand rejection sampling, square root, cofactor
 * clearing; one device lane per generator).  Writes G_out (n G1) and h_out
 * (the (n+1)-th), canonical affine; with out != NULL also loads them as a
 * generator set (tpst_gens_load). */
int tpst_gens_new(tpst_ctx* ctx, size_t n, const uint8_t* label, size_t label_len, uint64_t* G_out,
                  uint64_t* h_out, tpst_gens** out);
/* its n + 1 32-byte StdRng seeds (host only; the squeezed sponge bytes) */
int tpst_gens_seeds(size_t n, const uint8_t* label, size_t label_len, uint8_t* seeds);
/* PedersenCommit::commit_slice (commitments.rs:79-86): msm(G, scalars) + h * blind;
 * n must equal gens->n (the reference assert_eq!s, here TPST_E_ARG). */
int tpst_pedersen_commit_slice(tpst_ctx* ctx, const tpst_gens* gens, const uint64_t* scalars, size_t n,
                               const uint64_t* blind, uint64_t* out);
/* DensePolynomial::commit_inner (dense_mlpoly.rs:314-329): n_rows = |blinds|
 * rows of R = n_z / n_rows contiguous evaluations, row i -> commit_slice(Z[R i ..
 * R (i+1)], blinds[i]); out = n_rows canonical affine G1. */
int tpst_pedersen_commit_rows(tpst_ctx* ctx, const tpst_gens* gens, const uint64_t* Z, size_t n_z,
                              const uint64_t* blinds, size_t n_rows, uint64_t* out);

/* ---- fixed-base grouped MSM (csrc/fbt.h) --------------------------------
 * Builds the 64-window x 8-multiple lookup table of the n bases, then
 * out[g] = sum over k in group g of scalars[k] * bases[k] for L/D groups,
 * k(g, m) = (m / D) * L + g * D + m % D  (n % L == 0, L % D == 0).
 * L = D = n is a plain MSM; D = 1 is the MIPP fold a_i + sum_t w_t a_{i+tL}
 * (mipp.rs:124-136 applied over all rounds at once). */
int tpst_g1_msm_fixed(tpst_ctx* ctx, const uint64_t* bases, size_t n, const uint64_t* scalars, size_t L, size_t D,
                      uint64_t* out);
int tpst_g2_msm_fixed(tpst_ctx* ctx, const uint64_t* bases, size_t n, const uint64_t* scalars, size_t L, size_t D,
                      uint64_t* out);

/* ---- K4: multi-pairing ---------------------------------------------------
 * prod_i e(g1[i], g2[i]) after final exponentiation (ark-ec
 * Pairing::multi_pairing(...).0; sqrt_pst.rs:143, mipp.rs:397). */
int tpst_multi_pairing(tpst_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* out_gt);
/* Valid::check of a canonical affine point (ark-serialize Validate::Yes):
 * coordinates < p, on the curve, in the r-torsion subgroup (infinity = all
 * zero is valid).  TPST_OK or TPST_E_VERIFY; host only, no context. */
int tpst_g1_check(const uint64_t* p);
int tpst_g2_check(const uint64_t* p);


/* ---- sqrt-PST protocol ----------------------------------------------------
 * Mirrors sqrt_pst.rs:14-265 (Polynomial), mipp.rs:21-320 (MippProof) and
 * the ark-poly-commit fork's MultilinearPC keys.  n = number of variables,
 * m_col = n/2, m_row = n - m_col. */
#define TPST_MAX_VARS 20

/* Poseidon sponge state of PoseidonTranscript<Fq> (poseidon_transcript.rs:12-15):
 * state = capacity || rate (3 canonical Fq), duplex mode and index. */
typedef struct {
  uint64_t state[3][6];
  uint32_t squeezing; /* 0 = absorbing, 1 = squeezing */
  uint32_t index;     /* next absorb / squeeze position in the rate */
} tpst_transcript;

/* (Commitment U, Proof{m_row G2}, MippProof) returned by Polynomial::open */
typedef struct {
  int32_t m_col, m_row;
  uint64_t U[12];                              /* c_u, sqrt_pst.rs:198 */
  uint64_t pst_proof[TPST_MAX_VARS][24];       /* PST proof of q (G2) */
  uint64_t comms_t[TPST_MAX_VARS][2][72];      /* MippProof.comms_t */
  uint64_t comms_u[TPST_MAX_VARS][2][12];      /* MippProof.comms_u */
  uint64_t final_a[12];                        /* MippProof.final_a */
  uint64_t final_h[24];                        /* MippProof.final_h */
  uint64_t pst_proof_h[TPST_MAX_VARS][12];     /* MippProof.pst_proof_h (G1) */
} tpst_open_proof;

typedef struct tpst_poly tpst_poly;

/* Poseidon transcript (host): new / append(G1 | GT) / challenge_scalar */
void tpst_transcript_init(tpst_transcript* t);
int tpst_transcript_append_g1(tpst_transcript* t, const uint64_t* g1);
int tpst_transcript_append_gt(tpst_transcript* t, const uint64_t* gt);
int tpst_transcript_challenge(tpst_transcript* t, uint64_t* out_fr);

/* SRS / CommitterKey + VerifierKey of MultilinearPC (setup + trim to nv vars).
 * Flat canonical layout: g | h | for i < nv: powers_of_g[i] (2^(nv-i) G1) |
 * powers_of_h[i] (2^(nv-i) G2) | g_mask (nv G1) | h_mask (nv G2). */
size_t tpst_srs_flat_len(int nv);
int tpst_srs_setup(tpst_ctx* ctx, int nv, uint64_t seed);   /* seeded trapdoor, on the GPU */
int tpst_srs_load(tpst_ctx* ctx, int nv, const uint64_t* flat);
int tpst_srs_export(tpst_ctx* ctx, uint64_t* flat);
/* SplitMix64 uniform-Fr stream used for synthetic inputs; returns next index */
uint64_t tpst_fr_stream(uint64_t seed, size_t n, uint64_t start, uint64_t* out);

/* Polynomial::from_evaluations (sqrt_pst.rs:32-75): Z = 2^n canonical Fr.
 * The row split is a strided view of Z on the device (no host transpose). */
int tpst_poly_from_evaluations(tpst_ctx* ctx, const uint64_t* Z, int n, tpst_poly** out);
int tpst_poly_from_evaluations_dev(tpst_ctx* ctx, const void* d_Z, int n, tpst_poly** out);
/* Rank-local shard: upload only the columns [c0, c1) of the
 * strided view (for every j: Z[j 2^m_col + c0 .. j 2^m_col + c1), one 2D copy).
 * Such a handle serves tpst_poly_commit_rows[_partial] for rows inside
 * [c0, c1); eval / commit / open need the whole polynomial (TPST_E_STATE). */
int tpst_poly_from_evaluations_cols(tpst_ctx* ctx, const uint64_t* Z, int n, size_t c0, size_t c1,
                                    tpst_poly** out);
void tpst_poly_free(tpst_poly* p);
/* Polynomial::eval (sqrt_pst.rs:105-115); computes and caches q, chi(b) */
int tpst_poly_eval(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point, uint64_t* out_v);
/* Polynomial::commit (sqrt_pst.rs:117-149): comms = 2^m_col G1, T = GT */
int tpst_poly_commit(tpst_ctx* ctx, tpst_poly* p, uint64_t* comms, uint64_t* T);
int tpst_poly_commit_dev(tpst_ctx* ctx, tpst_poly* p, void* d_comms, void* d_T);
/* Row-sharded commit (multi-GPU): the MSMs of rows [r0, r1)
 * of the sqrt_pst.rs:121-125 loop -> (r1-r0) canonical G1; and the IPP of a
 * gathered commitment list (sqrt_pst.rs:128-143) -> T. */
int tpst_poly_commit_rows(tpst_ctx* ctx, tpst_poly* p, size_t r0, size_t r1, uint64_t* comms);
int tpst_poly_ipp(tpst_ctx* ctx, int n, const uint64_t* comms, uint64_t* T);
/* Same row range with the IPP split across ranks: also returns this share's
 * Miller-loop product prod_{r0<=i<r1} ml(C_i, h_i) BEFORE final
 * exponentiation (canonical Fq12, 72 u64).  T = FE(product of every rank's
 * partial) via tpst_gt_final_exp_product (sqrt_pst.rs:128-143 split by rows). */
int tpst_poly_commit_rows_partial(tpst_ctx* ctx, tpst_poly* p, size_t r0, size_t r1, uint64_t* comms,
                                  uint64_t* miller);
int tpst_gt_final_exp_product(tpst_ctx* ctx, const uint64_t* partials, size_t k, uint64_t* T);
/* Device-resident variants for the RCCL path (no host round trip): the share
 * [comms (R x 12) | Miller partial (72)] written into a device buffer of
 * R * 96 + 576 bytes; k partials read from device memory `stride_bytes` apart
 * (an all-gather of those buffers). */
int tpst_poly_commit_rows_partial_dev(tpst_ctx* ctx, tpst_poly* p, size_t r0, size_t r1, void* d_out);
int tpst_gt_final_exp_product_dev(tpst_ctx* ctx, const void* d_partials, size_t stride_bytes, size_t k, uint64_t* T);

/* Row-sharded opening (sqrt_pst.rs:81-101, 198).  Rank g
 * (rows [r0, r1) resident, e.g. a from_evaluations_cols handle) computes its
 * share of get_q, zq_g[j] = sum_{r0 <= i < r1} Z_i[j] chi_i(b) (2^m_row
 * canonical Fr), and of c_u = sum_{r0 <= i < r1} chi_i(b) C_i (canonical
 * affine, from its own row commitments).  The shares are summed on rank 0
 * (tpst_fr_sum_dev: k device vectors of n canonical Fr, mod r; c_u: a G1 sum),
 * which opens from an opening-only handle: tpst_poly_from_q_dev (q on the
 * device, chi(b) from the point, c_u optional -- NULL computes it) serves
 * tpst_poly_eval and tpst_poly_open without the evaluations. */
int tpst_poly_get_q_partial(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point, size_t r0, size_t r1, uint64_t* zq);
int tpst_poly_get_q_partial_dev(tpst_ctx* ctx, tpst_poly* p, const uint64_t* point, size_t r0, size_t r1, void* d_zq);
int tpst_fr_sum_dev(tpst_ctx* ctx, const void* d_parts, size_t k, size_t n, void* d_out);
int tpst_poly_cu_partial(tpst_ctx* ctx, int n, const uint64_t* point, size_t r0, size_t r1, const uint64_t* comms,
                         uint64_t* out);
int tpst_poly_from_q_dev(tpst_ctx* ctx, int n, const uint64_t* point, const void* d_zq, const uint64_t* U,
                         tpst_poly** out);
/* Polynomial::open (sqrt_pst.rs:168-230); the transcript is updated in place.
 * U = MSM(comms, chi(b)) over the caller's comm_list (sqrt_pst.rs:198). */
int tpst_poly_open(tpst_ctx* ctx, tpst_poly* p, tpst_transcript* tr, const uint64_t* comms,
                   const uint64_t* point, const uint64_t* T, tpst_open_proof* proof);
/* Row-sharded Polynomial::open (the MIPP rounds of
 * mipp.rs:58-120 split across `world` ranks, one process per GPU).  Rank g
 * owns the rows i = g mod world of comm_list (and of h, y): while a round's
 * length is >= 4 world its cross MSMs, folds, h preparations and look-ahead
 * pairings run on the rank's own rows, and one all-gather per product
 * combines them (cross partials summed, Miller partials multiplied before
 * the final exponentiation); every rank replays the transcript.  At the first
 * shorter round the folded a-vector (2 world points) is gathered to rank 0,
 * which finishes the rounds and the epilogue alone.  Same proof bytes as
 * tpst_poly_open on the same inputs.
 *
 * The library does no communication: `allgather` is the caller's transport
 * (RCCL, gloo, MPI, ...).  It must gather `bytes` from d_arena + send_off of
 * every rank into d_arena + recv_off (world x bytes, rank-major) ordered
 * after the work queued on `stream` (a hipStream_t of the library) and before
 * work queued on it afterwards -- e.g. an RCCL all-gather enqueued on that
 * stream; return 0 on success.  Every rank issues the same gathers in the
 * same order.  d_arena: device memory of arena_bytes >=
 * tpst_open_sharded_arena_bytes(n, world), reachable by the transport.
 *
 * rank 0: p = the opening handle (tpst_poly_from_q_dev, or a whole
 * polynomial) and `proof`; other ranks: p and proof may be NULL.  Every
 * rank: the whole comm_list, the point, U = c_u (canonical affine, e.g. the
 * combined tpst_poly_cu_partial shares) and its own transcript copy.  With
 * fewer than 4 world rows rank 0 opens alone (the others return at once).
 *
 * After the call only rank 0's transcript is the reference's end state: the
 * other ranks stop at the hand-over round and leave theirs mid-protocol (a
 * prover that keeps using the transcript on every rank must take rank 0's).
 * The allgather callback runs while the context's lock is held: it must not
 * call back into libtpst on the same context.  A rank that returns an error
 * stops issuing gathers, so its peers would wait in their next collective:
 * on any non-OK return the caller must abort the whole group (e.g.
 * ncclCommAbort / destroying the process group), not retry the call. */
typedef int (*tpst_allgather_fn)(void* user, size_t send_off, size_t recv_off, size_t bytes, void* stream);
typedef struct {
  int world, rank;
  tpst_allgather_fn allgather;
  void* user;
  void* d_arena;
  size_t arena_bytes;
} tpst_exchange;
size_t tpst_open_sharded_arena_bytes(int n, int world);
int tpst_poly_open_sharded(tpst_ctx* ctx, tpst_poly* p, tpst_transcript* tr, int n, const uint64_t* comms,
                           const uint64_t* point, const uint64_t* U, const tpst_exchange* x, tpst_open_proof* proof);
/* Polynomial::verify (sqrt_pst.rs:232-264): TPST_OK if valid, TPST_E_VERIFY if
 * not, including any proof element that is non-canonical, off its curve or
 * outside the prime-order subgroup (checked before the transcript absorbs it). */
int tpst_pst_verify(tpst_ctx* ctx, tpst_transcript* tr, int n, const uint64_t* point, const uint64_t* v,
                    const uint64_t* T, const tpst_open_proof* proof);

/* ---- MultilinearPC single calls (ark-poly-commit fork) --
 * Against the loaded SRS; a polynomial of nv <= ck.nv variables uses level
 * ck.nv - nv.  evals: 2^nv canonical Fr (to_evaluations order); point: nv Fr,
 * LSB-first (as MultilinearPC takes it, cf. a_rev at sqrt_pst.rs:218-225).
 * commit  (sqrt_pst.rs:124)  -> g_product (G1)
 * commit_g2 (mipp.rs:133)     -> h_product (G2)
 * open    (sqrt_pst.rs:225)   -> nv G2 proofs;  open_g1 (mipp.rs:144) -> nv G1
 * check   (sqrt_pst.rs:261)   -> TPST_OK / TPST_E_VERIFY
 * check_2 (mipp.rs:307)       -> TPST_OK / TPST_E_VERIFY
 * The checks reject non-canonical, off-curve or non-subgroup inputs. */
int tpst_mlpc_commit(tpst_ctx* ctx, const uint64_t* evals, int nv, uint64_t* g_product);
int tpst_mlpc_commit_g2(tpst_ctx* ctx, const uint64_t* evals, int nv, uint64_t* h_product);
int tpst_mlpc_open(tpst_ctx* ctx, const uint64_t* evals, int nv, const uint64_t* point, uint64_t* proofs);
int tpst_mlpc_open_g1(tpst_ctx* ctx, const uint64_t* evals, int nv, const uint64_t* point, uint64_t* proofs);
int tpst_mlpc_check(tpst_ctx* ctx, int nv, const uint64_t* comm, const uint64_t* point, const uint64_t* value,
                    const uint64_t* proofs);
int tpst_mlpc_check_2(tpst_ctx* ctx, int nv, const uint64_t* comm_h, const uint64_t* point, const uint64_t* value,
                      const uint64_t* proofs);

/* Transcript calls of the R1CS prover (poseidon_transcript.rs:55-60, 83-85):
 * append_scalar -- an Fr absorbed as one Fq element of the same value;
 * new_from_state2 -- a fresh sponge that absorbs the 32-byte uncompressed Fr. */
int tpst_transcript_append_fr(tpst_transcript* t, const uint64_t* fr);
int tpst_transcript_reset_fr(tpst_transcript* t, const uint64_t* fr);
/* append_bytes (poseidon_transcript.rs:67-69): absorb a byte vector (u64
 * length prefix, 47-byte chunks); `append` of any value = this over its
 * Compress::No serialisation (poseidon_transcript.rs:22-28). */
int tpst_transcript_append_bytes(tpst_transcript* t, const uint8_t* bytes, size_t n);

/* ---- Spartan R1CS sum-checks (csrc/r1cs.hip) ------
 * R1CSInstance (r1csinstance.rs): num_cons x (2 num_vars) sparse A, B, C;
 * z = vars || 1 || inputs || 0.  Matrices as (row u32, col u32, canonical Fr)
 * triples, any order; kept on the device as CSR (multiply_vec) + CSC
 * (compute_eval_table_sparse). */
typedef struct tpst_r1cs tpst_r1cs;
int tpst_r1cs_load(tpst_ctx* ctx, size_t num_cons, size_t num_vars, size_t num_inputs, const size_t* nnz /*[3]*/,
                   const uint32_t* const* rows /*[3]*/, const uint32_t* const* cols /*[3]*/,
                   const uint64_t* const* vals /*[3]*/, tpst_r1cs** out);
/* produce_synthetic_r1cs (r1csinstance.rs:166-242) over the SplitMix64 Fr
 * stream of `seed` (the reference draws thread_rng): also returns the
 * satisfying vars (num_vars Fr) and inputs (num_inputs Fr) */
int tpst_r1cs_synthetic(tpst_ctx* ctx, size_t num_cons, size_t num_vars, size_t num_inputs, uint64_t seed,
                        tpst_r1cs** out, uint64_t* vars, uint64_t* inputs);
void tpst_r1cs_free(tpst_r1cs* r);
/* UniPoly::from_evals (unipoly.rs:15-45): n = 3 or 4 canonical evaluations at
 * 0..n-1 -> n coefficients, constant first (host; the sum-check round encoding). */
int tpst_unipoly_from_evals(const uint64_t* evals, int n, uint64_t* coeffs);
/* EqPolynomial::evals (dense_mlpoly.rs:231-250): the MSB-first chi table of
 * r[0..ell) (ell <= 30), computed on the device; out = 2^ell canonical Fr. */
int tpst_eq_evals(tpst_ctx* ctx, const uint64_t* r, int ell, uint64_t* out);

/* R1CSInstance::commit (r1csinstance.rs:313-344) = SparseMatPolynomial::
 * multi_commit over (A, B, C) (sparse_mlpoly.rs:490-517): the SPARK dense
 * representation (addresses, memory-checking read / audit timestamps, values)
 * built on the device, comb_ops and comb_mem each committed with
 * DensePolynomial::commit (Hyrax rows, zero blinds) over the generators of
 * PolyCommitmentGens::setup(num_vars, label).  ops_rows / mem_rows receive the
 * row counts (the G1 points of each PolyCommitment); with comm_ops or
 * comm_mem NULL only the sizes are reported. */
int tpst_r1cs_commit(tpst_ctx* ctx, tpst_r1cs* r1cs, const uint8_t* label, size_t label_len, uint64_t* comm_ops,
                     size_t* ops_rows, uint64_t* comm_mem, size_t* mem_rows);

#define TPST_R1CS_MAX_ROUNDS 48
/* R1CSProof (r1csproof.rs:24-38) without the Groth16 part; canonical Fr.
 * sc1: cubic round polynomials (4 coefficients, constant first), sc2: quad
 * (3); claims_phase2 = (Az, Bz, Cz, Az Bz)(rx); claims_phase2_z_abc = the
 * phase-two finals (z(ry), ABC(ry)); open = (comm U, proof_eval_vars_at_ry,
 * mipp_proof) of the witness polynomial at ry[1..]. */
typedef struct {
  int32_t rounds_x, rounds_y, num_vars_log, pad;
  uint64_t T[72];
  uint64_t initial_state[4];
  uint64_t sc1[TPST_R1CS_MAX_ROUNDS][4][4];
  uint64_t claims_phase2[4][4];
  uint64_t claims_phase2_z_abc[2][4];
  uint64_t r_abc[3][4];
  uint64_t sc2[TPST_R1CS_MAX_ROUNDS][3][4];
  uint64_t rx[TPST_R1CS_MAX_ROUNDS][4];
  uint64_t ry[TPST_R1CS_MAX_ROUNDS][4];
  uint64_t transcript_sat_state[4];
  uint64_t eval_vars_at_ry[4];
  tpst_open_proof open;
} tpst_r1cs_proof;
/* R1CSProof::prove (r1csproof.rs:237-370) minus prove_verifier: needs the SRS
 * loaded for ceil(log2(num_vars) / 2) variables; `tr` is updated in place. */
int tpst_r1cs_prove(tpst_ctx* ctx, tpst_r1cs* r1cs, const uint64_t* vars, const uint64_t* inputs,
                    tpst_transcript* tr, tpst_r1cs_proof* out);

/* ---- Groth16 over BLS12-377 (csrc/groth16.hip) ----
 * The prover behind R1CSProof::prove_verifier (r1csproof.rs:374-434,
 * Groth16::<E>::prove at :421): ark-groth16 create_proof with the
 * LibsnarkReduction QAP, over any tpst_r1cs instance (variables in the
 * Spartan z order: witness z[0..num_vars), instance (1, inputs)).  The
 * reference's thread_rng draws are arguments here. */
typedef struct tpst_groth16_pk tpst_groth16_pk;
/* generate_random_parameters_with_reduction: toxic = (tau, alpha, beta,
 * gamma, delta) canonical Fr (5 x 4 u64, nonzero, tau outside the domain).
 * Keeps the proving key (query points) on the device. */
int tpst_groth16_setup(tpst_ctx* ctx, tpst_r1cs* r1cs, const uint64_t* toxic, tpst_groth16_pk** out);
void tpst_groth16_pk_free(tpst_groth16_pk* pk);
/* QAP domain size n = next_pow2(num_cons + num_inputs + 1) */
int tpst_groth16_domain(const tpst_groth16_pk* pk, size_t* n);
/* VerifyingKey: alpha_g1 (12 u64), beta_g2 / gamma_g2 / delta_g2 (24 u64
 * each), gamma_abc_g1 (num_inputs + 1 points), affine canonical */
int tpst_groth16_vk(tpst_ctx* ctx, const tpst_groth16_pk* pk, uint64_t* alpha_g1, uint64_t* beta_g2,
                    uint64_t* gamma_g2, uint64_t* delta_g2, uint64_t* gamma_abc_g1);
/* LibsnarkReduction::witness_map: the first n - 1 coefficients of h (canonical) */
int tpst_groth16_witness_map(tpst_ctx* ctx, tpst_groth16_pk* pk, tpst_r1cs* r1cs, const uint64_t* vars,
                             const uint64_t* inputs, uint64_t* h);
/* create_proof_with_reduction: rs = (r, s) canonical; Proof { a: G1, b: G2, c: G1 } */
int tpst_groth16_prove(tpst_ctx* ctx, tpst_groth16_pk* pk, tpst_r1cs* r1cs, const uint64_t* vars,
                       const uint64_t* inputs, const uint64_t* rs, uint64_t* A, uint64_t* B, uint64_t* C);
/* Groth16::verify_proof (ark-groth16 verifier.rs): TPST_OK if the proof
 * verifies, TPST_E_VERIFY if it does not or if any element is malformed
 * (coordinate >= p, off the curve, outside the r-torsion subgroup, input >= r:
 * what Validate::Yes deserialisation rejects); TPST_E_ARG if n_abc !=
 * n_inputs + 1.  Canonical affine points, vk as tpst_groth16_vk returns it. */
int tpst_groth16_verify(tpst_ctx* ctx, const uint64_t* alpha_g1, const uint64_t* beta_g2, const uint64_t* gamma_g2,
                        const uint64_t* delta_g2, const uint64_t* gamma_abc_g1, size_t n_abc, const uint64_t* inputs,
                        size_t n_inputs, const uint64_t* A, const uint64_t* B, const uint64_t* C);

/* ---- arkworks wire format (csrc/serialize.hip; host only, no context) ------
 * CanonicalSerialize with Compress::Yes (ark-serialize 0.4): G1 48 B, G2 96 B
 * (x with SWFlags in the top bits of the last byte: 0x80 y negative, 0x40
 * infinity), GT 576 B, usize / Vec length as u64 LE.  The byte strings of
 * benches/pst.rs:43-46,64-74 (commiter_key_size, proof_size = |Proof| +
 * |MippProof|).  Writers: out == NULL only reports the length in *len;
 * TPST_E_ARG if cap is too small or an element is not canonical.  Readers
 * validate like Validate::Yes (canonical, on curve, prime-order subgroup). */
int tpst_ser_g1(const uint64_t* p, uint8_t* out48);
int tpst_ser_g2(const uint64_t* p, uint8_t* out96);
int tpst_de_g1(const uint8_t* in48, uint64_t* p);
int tpst_de_g2(const uint8_t* in96, uint64_t* p);
/* Commitment { nv, g_product } (sqrt_pst.rs:201 U, :121-125 comm_list entries) */
int tpst_ser_commitment(int nv, const uint64_t* g1, uint8_t* out, size_t cap, size_t* len);
/* Proof { proofs: Vec<G2> } -- the pst_proof of Polynomial::open (sqrt_pst.rs:225) */
int tpst_ser_pst_proof(const tpst_open_proof* p, uint8_t* out, size_t cap, size_t* len);
/* MippProof (mipp.rs:21-28) */
int tpst_ser_mipp_proof(const tpst_open_proof* p, uint8_t* out, size_t cap, size_t* len);
/* both back into a tpst_open_proof (U left zero) */
int tpst_de_open_proof(const uint8_t* pst, size_t pst_len, const uint8_t* mipp, size_t mipp_len,
                       tpst_open_proof* out);
/* CommitterKey { nv, powers_of_g, powers_of_h, g, h } from the flat SRS of
 * tpst_srs_export (benches/pst.rs:43-46) */
int tpst_ser_committer_key(int nv, const uint64_t* srs_flat, size_t flat_len, uint8_t* out, size_t cap,
                           size_t* len);  /* flat_len == tpst_srs_flat_len(nv) */

/* ---- utilities ----------------------------------------------------------- */
/* out[i] = scalars[i] * G1 generator (affine, canonical); synthetic bases */
int tpst_g1_mul_generator(tpst_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out);
int tpst_g2_mul_generator(tpst_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out);
/* device forms: d_out Montgomery (for _dev MSM bases) */
int tpst_g1_mul_generator_dev(tpst_ctx* ctx, const void* d_scalars, size_t n, void* d_out_mont);

/* Field microbenchmark (measured peak for the roofline's compute column):
 * kind 0 = Fq Montgomery multiply, 1 = G1 XYZZ mixed add, 2 = Fq inverse, 3 / 4 = Fq multiply
 * variants (two interleaved accumulation chains / independent columns), 5 = G1 XYZZ doubling, 15 = Fq inverse
 * by a whole wave (csrc/inv_wave.h; one chain per 64 threads), 16 + op = one wave
 * running `iters` stages of wave-engine op `op` (csrc/wave_ops.inc).  Runs `threads`
 * threads x `iters` dependent ops each; returns kernel milliseconds. */
int tpst_microbench(tpst_ctx* ctx, int kind, size_t threads, int iters, double* ms);
/* shader-clock cycles of the parts of `iters` stages of wave op `op` (forms,
 * product, product store, output forms, output reduce/store) */
int tpst_microbench_wave_phases(tpst_ctx* ctx, int op, int iters, uint64_t* cycles5);
/* Self-test of the two device Fq inverses: n Montgomery-form values (6 words
 * each) -> their inverses by the lone-lane routine and by the wave routine. */
int tpst_selftest_inv(tpst_ctx* ctx, size_t n, const uint64_t* in, uint64_t* out_lane, uint64_t* out_wave);

/* Per-stage HIP-event timing of the MSM pipeline on the context's stream.
 * stage: 0 decompose, 1 sort, 2 bucket bounds, 3 bucket accumulation (the
 * dominant kernel), 4 bucket reduction, 5 window combine, 6 K1 row sort. */
int tpst_profile_enable(tpst_ctx* ctx, int on);
int tpst_profile_reset(tpst_ctx* ctx);
int tpst_profile_read(tpst_ctx* ctx, int stage, double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* TPST_H */
