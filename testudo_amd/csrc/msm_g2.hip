// G2 (Fq2) instantiations of the MSM pipeline, compiled as a separate
// translation unit so the build parallelises.
#define TPST_MSM_G2_ONLY
#include "msm.hip"
