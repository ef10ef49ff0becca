// G2 (Fq2) instantiations of the MSM pipeline, compiled as a separate
// translation unit so the build parallelises.  The G2 variable-base MSM only
// serves the verifier and tpst_g2_msm (the opening's G2 MSMs run on fixed-base
// tables, fbt.hip), so its Fq2 products are out of line (see field.h).
#define TPST_MSM_G2_ONLY
#define TPST_FQ2_ATTR __host__ __device__ inline __attribute__((noinline))
#include "msm.hip"
