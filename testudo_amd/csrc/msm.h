// Pippenger multi-scalar multiplication engine for CDNA4 (host-side API of
// msm.hip).  Two shapes, matching the reference hot loops:
//
//  K2  variable-base MSM  sum_i s_i * P_i            (sqrt_pst.rs:198,
//      mipp.rs:393, config 2 of BASELINE.json)
//  K1  batched shared-base MSM  C_r = sum_j Z[r][j] * B_j  over R rows with
//      one SRS-fixed base vector (sqrt_pst.rs:121-125 par_iter of
//      MultilinearPC::commit), using precomputed window tables
//      T[w][j] = 2^(c w) B_j so every row is ONE bucket set.
//
// Both run the same pipeline of kernels:
//   signed-digit decomposition -> (bucket key, point index|sign) pairs
//   -> radix sort by key -> bucket bounds -> bucket accumulation (XYZZ
//   mixed adds, one thread per bucket) -> segmented weighted bucket
//   reduction -> per-group (window / row) tree reduction -> combine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <vector>
#include "curve.h"

namespace tpst {

// Optional per-stage HIP-event timing of the MSM pipeline (the bench's
// roofline needs the dominant kernel's own duration on the stream it runs on).
// The sqrt-PST stages carry the reference's Timer labels (sqrt_pst.rs:33-262):
// build_q, sqrt_commit = comm_list + ipp, sqrt_open = msm (U) + mipp_prove +
// pst_open; their device spans (first command to last, across the opening's
// streams) are recorded here, and the same names are roctx host ranges
// (trace.h) for rocprofv3 --marker-trace.
enum MsmStage {
  ST_DECOMPOSE = 0, ST_SORT, ST_BOUNDS, ST_BUCKET_ACC, ST_REDUCE, ST_COMBINE, ST_BATCH_SORT,
  ST_BUILD_Q, ST_SQRT_COMMIT, ST_COMM_LIST, ST_IPP, ST_SQRT_OPEN, ST_MSM_U, ST_MIPP_PROVE, ST_PST_OPEN,
  N_STAGES
};

struct Profiler {
  bool on = false;
  std::vector<hipEvent_t> ev[N_STAGES];  // begin/end pairs
  size_t used[N_STAGES] = {};
  double total_ms[N_STAGES] = {};
  uint64_t count[N_STAGES] = {};
  void begin(int st, hipStream_t s);
  void end(int st, hipStream_t s);
  void collect();  // caller synchronised the stream
  void reset();
  ~Profiler();
};

// grow-only device scratch arena; reset() per call, never freed mid-call
struct Arena {
  Profiler* prof = nullptr;
  char* base = nullptr;
  size_t cap = 0;
  size_t off = 0;
  // auxiliary streams + events of the window-grouped MSM (msm_var): the
  // latency-bound reduction / doubling chain of one window group runs on an
  // aux stream while the next group's bucket accumulation fills the chip.
  // Created on first use on the current device, destroyed by release().
  static constexpr int N_AUX = 2, N_AUX_EV = 16;
  hipStream_t aux[N_AUX] = {};
  hipEvent_t aux_ev[N_AUX_EV] = {};
  bool aux_ready = false;
  Arena* aux_from = nullptr;  // borrow that arena's aux streams (own events only)
  hipError_t aux_init();
  hipError_t reserve(size_t bytes);
  void reset() { off = 0; }
  template <class T>
  T* take(size_t count) {
    size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base + off);
    off += bytes;
    return p;
  }
  static size_t need(size_t count, size_t elem) { return (count * elem + 255) & ~size_t(255); }
  void release();
};

// Longest variable-base MSM one call accepts: the sort runs over
// m = 2 W n < 2^31 (key, value) entries (int-sized for hipCUB, u32 bucket
// bounds).  msm_var returns hipErrorInvalidValue beyond it.
constexpr size_t MSM_MAX_POINTS = (size_t)1 << 27;

// window size used for a variable-base MSM of n points
int msm_window_bits(size_t n);

// Variable-base MSM over device buffers.  bases: n affine points,
// Montgomery form (24 / 48 u32 each); scalars: n canonical Fr (8 u32 each).
// Writes one XYZZ point to d_out.  Returns hipSuccess or the first error.
// tail != nullptr: the last window group's fixup, reduction and window chain
// (the latency-bound tail) may run on `tail` instead of s -- then *on_tail is
// set and d_out is final in `tail`'s order (s is free for the next call's
// decomposition and accumulation; the caller keeps the arena until then).
// front != nullptr: the scalar decomposition and the sort run on `front`
// (ordered before s's accumulation by an event) -- so a pipelining caller's
// next call sorts while this one accumulates.
template <class F>
hipError_t msm_var(Arena& ar, hipStream_t s, const uint32_t* d_bases, const uint32_t* d_scalars,
                   size_t n, Xyzz<F>* d_out, hipStream_t tail = nullptr, bool* on_tail = nullptr,
                   hipStream_t front = nullptr);

// Fixed-base tables for K1: T[w][j] = 2^(c w) * B_j (affine, Montgomery).
struct BatchTables {
  uint32_t* d_table = nullptr;  // W * N points T[w][j], 128-byte radix-2^29 records (msm.hip fetch_rec29)
  size_t N = 0;
  int c = 0;
  int W = 0;
};

hipError_t batch_tables_build(hipStream_t s, const uint32_t* d_bases, size_t N, int c, BatchTables& t);
void batch_tables_free(BatchTables& t);
int batch_window_bits(size_t N);

// K1: rows x N scalar matrix; scalar (r, j) is at d_scalars + 8*(r*row_stride + j*col_stride)
// (canonical Fr).  Writes `rows` XYZZ points.
hipError_t msm_batch(Arena& ar, hipStream_t s, const BatchTables& t, const uint32_t* d_scalars,
                     size_t rows, size_t row_stride, size_t col_stride, Xyzz<Fq>* d_out);

// elementwise helpers
template <class F>
hipError_t points_to_mont(hipStream_t s, const uint32_t* d_in, uint32_t* d_out, size_t n);
template <class F>
hipError_t xyzz_to_affine_canonical(hipStream_t s, const Xyzz<F>* d_in, uint32_t* d_out, size_t n);
template <class F>
hipError_t affine_from_mont(hipStream_t s, const uint32_t* d_in, uint32_t* d_out, size_t n);

}  // namespace tpst
