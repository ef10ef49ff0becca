// GLV scalar decomposition on G1 (and, with beta^2, on G2): shared by the
// variable-base MSM (msm.hip) and the GLV fixed-base tables (fbt.hip).
#pragma once
#include "device_util.h"

namespace tpst {

// GLV split k = k1 + k2 * lambda (lambda = x^2 - 1, 127 bits), both halves
// < 2^127: k2 = floor(k * mu / 2^256) (+1 correction), k1 = k - k2 * lambda
__device__ __forceinline__ void glv_split(const uint32_t* k, uint32_t* k1, uint32_t* k2) {
  uint32_t prod[13];
#pragma unroll
  for (int i = 0; i < 13; i++) prod[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const uint64_t t = (uint64_t)k[i] * params::GLV_MU[j] + prod[i + j] + carry;
      prod[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    prod[i + 5] = (uint32_t)carry;
  }
  uint32_t q[4] = {prod[8], prod[9], prod[10], prod[11]};
  uint32_t ql[8];
#pragma unroll
  for (int i = 0; i < 8; i++) ql[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t t = (uint64_t)q[i] * params::GLV_LAMBDA[j] + ql[i + j] + carry;
      ql[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    ql[i + 4] = (uint32_t)carry;
  }
  uint32_t r[4];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {  // k - q*lambda < 2*lambda < 2^128
    const int64_t d = (int64_t)k[i] - ql[i] + br;
    r[i] = (uint32_t)d;
    br = d >> 32;
  }
  // r >= lambda ?  -> subtract once more
  uint32_t s[4];
  br = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int64_t d = (int64_t)r[i] - params::GLV_LAMBDA[i] + br;
    s[i] = (uint32_t)d;
    br = d >> 32;
  }
  const bool ge = (br == 0);
  uint64_t c = ge ? 1 : 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    k1[i] = ge ? s[i] : r[i];
    c += q[i];
    k2[i] = (uint32_t)c;
    c >>= 32;
  }
}

}  // namespace tpst
