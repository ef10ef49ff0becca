// Compile-only lab for the accumulation kernels (register / spill / ISA
// checks in ~1 minute instead of msm.hip's ~3.5): msm.hip's kernels without
// its host side, with only the variants named here instantiated.
//   hipcc -std=c++17 -O3 --offload-arch=gfx950 --cuda-device-only -c \
//     -Rpass-analysis=kernel-resource-usage -I testudo_amd/csrc -I include \
//     [-DTPST_K2_MINW=3 -DTPST_K2_NBUF=1 ...] tools/lab/acc_lab.hip -o /tmp/lab.o
#define TPST_MSM_LAB
#include "msm.hip"

namespace tpst {
template __global__ void k_bucket_acc_short_lds<TPST_K2_MINW, true>(
    const uint32_t* __restrict__, const uint32_t* __restrict__, const uint32_t* __restrict__, int, int, uint32_t,
    const uint32_t* __restrict__, const uint32_t* __restrict__, const uint32_t* __restrict__,
    const uint32_t* __restrict__, uint32_t, int, Xyzz<Fq>* __restrict__, Xyzz<Fq>* __restrict__);
#ifdef LAB_K1
template __global__ void k_bucket_acc_chunk_lds<TPST_K1_MINW>(const uint32_t* __restrict__, const uint32_t* __restrict__, size_t,
                                                   const uint32_t* __restrict__, uint32_t, const uint32_t* __restrict__,
                                                   const uint32_t* __restrict__, const uint32_t* __restrict__, int,
                                                   Xyzz<Fq>* __restrict__, Xyzz<Fq>* __restrict__, Xyzz<Fq>* __restrict__);
#endif
}  // namespace tpst
