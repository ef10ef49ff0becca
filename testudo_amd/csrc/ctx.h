// Internal state behind the opaque tpst_ctx handle.
#pragma once
#include <hip/hip_runtime.h>
#include <mutex>
#include <string>
#include <vector>
#include "msm.h"
#include "pairing_kernels.h"

struct tpst_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
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
