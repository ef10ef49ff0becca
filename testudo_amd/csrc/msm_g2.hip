// G2 (Fq2) instantiations of the MSM pipeline, compiled as a separate
// translation unit so the build parallelises.  The G2 variable-base MSM
// serves the verifier, tpst_g2_msm and Groth16's B (groth16.hip; the opening's
// G2 MSMs run on fixed-base tables, fbt.hip).  Its Fq2 products stay out of
// line (see field.h): inlined, the XYZZ mixed addition spills ~420 VGPRs and
// the unit takes ~9 min to compile.
#define TPST_MSM_G2_ONLY
#define TPST_FQ2_ATTR __host__ __device__ inline __attribute__((noinline))
#include "msm.hip"
