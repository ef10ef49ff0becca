// roctx host ranges named after the reference's Timer labels (timer.rs:15-68,
// sqrt_pst.rs:33-262): poly_list_build, build_q, sqrt_commit, comm_list, ipp,
// sqrt_open, msm, mipp_prove, pst_open, mipp_verify, pst_verify.  Visible in
// `rocprofv3 --marker-trace`; a no-op without a profiler attached.  The
// device-side spans of the same stages are hipEvent pairs (msm.h MsmStage).
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace tpst {

struct TraceRange {
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace tpst
