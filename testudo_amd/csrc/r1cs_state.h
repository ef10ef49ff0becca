// Device-resident R1CS instance shared by the Spartan sum-checks (r1cs.hip)
// and the Groth16 prover (groth16.hip), plus their small host Fr helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/tpst.h"
#include "field.h"

namespace tpst {

struct Buf {  // owning device allocation
  void* p = nullptr;
  ~Buf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t bytes) {
    if (p) (void)hipFree(p);
    p = nullptr;
    return bytes ? hipMalloc(&p, bytes) : hipSuccess;
  }
  uint32_t* u() const { return (uint32_t*)p; }
};

// ------------------------------------------------------ host Fr helpers ----
inline Fr frc(const uint64_t* c) {  // canonical -> Montgomery
  Fr a;
  memcpy(a.v, c, 32);
  return to_mont(a);
}
inline void fro(const Fr& a, uint64_t* c) {
  const Fr r = from_mont(a);
  memcpy(c, r.v, 32);
}
inline bool fr_ok_host(const uint64_t* v) {
  static const uint64_t rp[4] = {0x0a11800000000001ull, 0x59aa76fed0000001ull, 0x60b44d1e5c37b001ull,
                                 0x12ab655e9a2ca556ull};
  for (int k = 3; k >= 0; k--)
    if (v[k] != rp[k]) return v[k] < rp[k];
  return false;
}

inline int log2_exact(size_t n) {
  int l = 0;
  while (((size_t)1 << l) < n) l++;
  return ((size_t)1 << l) == n ? l : -1;
}


}  // namespace tpst

// ================================================================ state ==
struct tpst_r1cs {
  const tpst_ctx* owner = nullptr;  // the context whose device holds the tables
  size_t num_cons = 0, num_vars = 0, num_inputs = 0, ncols = 0;
  size_t nnz[3] = {0, 0, 0};
  tpst::Buf rptr[3], ridx[3], rval[3];  // CSR over rows (multiply_vec)
  tpst::Buf cptr[3], cidx[3], cval[3];  // CSC over the 2 num_vars columns of z (eval table)
  tpst::Buf orow[3], ocol[3], oval[3];  // the entries in the caller's order (SPARK dense rep)
  void* pin = nullptr;            // 4 KiB pinned host staging of the sum-check rounds
  void* pinned() {
    if (!pin && hipHostMalloc(&pin, 4096, hipHostMallocDefault) != hipSuccess) pin = nullptr;
    return pin;
  }
  ~tpst_r1cs() {
    if (pin) (void)hipHostFree(pin);
  }
};

