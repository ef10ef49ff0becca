// Internal state behind the opaque tpst_ctx handle.
#pragma once
#include <hip/hip_runtime.h>
#include <mutex>
#include <string>
#include <vector>
#include "msm.h"
#include "pairing_kernels.h"

namespace tpst {
// The per-context lock.  lock() also orders the context stream after any
// work a previous call left running off it (the pipelined device MSM's tail,
// tpst_g1_msm_dev): every entry point sees the results of every earlier call
// in stream order, as if it had all run on `stream`.  lock_keep() (the
// pipelined MSM itself) leaves that work pending.
struct CtxMutex {
  std::mutex m;
  hipStream_t* stream = nullptr;
  std::vector<hipEvent_t> pending;
  void lock() {
    m.lock();
    if (stream && *stream)
      for (hipEvent_t e : pending) (void)hipStreamWaitEvent(*stream, e, 0);
    pending.clear();
  }
  void lock_keep() { m.lock(); }
  void unlock() { m.unlock(); }
};
struct CtxKeep {  // lock_guard of lock_keep()
  CtxMutex& mu;
  explicit CtxKeep(CtxMutex& m) : mu(m) { mu.lock_keep(); }
  ~CtxKeep() { mu.unlock(); }
};
}  // namespace tpst

struct tpst_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  tpst::CtxMutex mu;
  // pipelined device MSMs (tpst_g1_msm_dev): three arenas used in turn;
  // call i+1 decomposes and sorts on side[0] while call i accumulates on
  // side[1], and call i's latency-bound tail (last window group's fixup,
  // reduction, window chain, affine output) runs on msm_tail.  (The side
  // streams are shared with the opening: two more streams of their own cost
  // the commit's IPP 0.7 ms at 2^20 -- more HIP streams than hardware queues.)
  static constexpr int MSM_SLOTS = 3;  // call i+1's sort must not wait for call i-1's tail
  tpst::Arena arena_msm[MSM_SLOTS];
  hipStream_t msm_tail = nullptr;
  hipEvent_t msm_in[MSM_SLOTS] = {};  // the caller's inputs ready (on `stream`)
  hipEvent_t msm_done[MSM_SLOTS] = {};
  void* msm_out[MSM_SLOTS] = {};  // each slot's XYZZ result
  bool msm_done_set[MSM_SLOTS] = {};
  int msm_slot = 0;
  std::string err;
  tpst::Arena arena;   // kernel scratch (reset per primitive)
  tpst::Arena io;      // staging for host-pointer entry points
  tpst::Arena arena2;  // scratch for nested primitives (open / MIPP)
  tpst::Profiler prof; // stage timing (tpst_profile_*)
  // the opening runs four streams concurrently (pst_api.hip tpst_poly_open):
  // `stream` + side[0..2], each with its own scratch arena; created on first use
  hipStream_t side[3] = {nullptr, nullptr, nullptr};
  tpst::Arena arena_side[3];
  hipStream_t comm = nullptr;      // the row-sharded opening's all-gathers (tpst_poly_open_sharded)
  hipStream_t side_c = nullptr;    // the opening's per-round h preparation (greatest priority)
  std::vector<hipEvent_t> events;  // timing-free event pool of the opening
  hipEvent_t ev_wait = nullptr;    // tpst_wait_stream / tpst_join_stream
  hipEvent_t ev_join = nullptr;
  void* pinned = nullptr;          // pinned host staging of the opening
  size_t pinned_cap = 0;
};

void tpst_release_pst_state(tpst_ctx* ctx);

namespace tpst {

// record an error message and return code
int fail(tpst_ctx* ctx, int code, const std::string& msg);
int hip_fail(tpst_ctx* ctx, hipError_t e, const char* where);

}  // namespace tpst

#define TPST_HIP(ctx, x)                                            \
  do {                                                              \
    hipError_t _e = (x);                                            \
    if (_e != hipSuccess) return tpst::hip_fail((ctx), _e, #x);     \
  } while (0)
