// Host check of host_mont_adx.inc (MULX / ADCX / ADOX Montgomery product)
// against poseidon_host.h's C++ hmul<true> on random inputs below 2p, and a
// timing of both (tests/test_host_field.py).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "poseidon_host.h"

using namespace tpst;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 200000;
  if (!(__builtin_cpu_supports("adx") && __builtin_cpu_supports("bmi2"))) {
    printf("skip: no ADX/BMI2\n");
    return 0;
  }
  const HostP64& P = hp64();
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  uint64_t p2[6];  // 2p
  for (int j = 0; j < 6; j++) p2[j] = (P.p[j] << 1) | (j ? P.p[j - 1] >> 63 : 0);
  auto rand2p = [&](Fq& x) {  // uniform below 2p (378-bit draws, rejected at >= 2p)
    for (;;) {
      uint64_t w[6];
      for (int i = 0; i < 6; i++) w[i] = rnd();
      w[5] &= (1ull << 58) - 1;
      int j = 5;
      while (j > 0 && w[j] == p2[j]) j--;
      if (w[j] < p2[j]) {
        memcpy(x.v, w, 48);
        return;
      }
    }
  };
  int bad = 0;
  for (int it = 0; it < n; it++) {
    Fq a, b;
    rand2p(a);
    rand2p(b);
    if (it == 0) memset(a.v, 0, 48);
    if (it == 1 || it == 2) {  // 2p - 1 (the largest lazy value) against itself / p - 1
      uint64_t w[6];
      memcpy(w, p2, 48);
      w[0] -= 1;
      memcpy(a.v, w, 48);
      memcpy(w, P.p, 48);
      w[0] -= 1;
      memcpy(b.v, it == 1 ? a.v : (const uint32_t*)w, 48);
    }
    const Fq ref = hmul_cxx<true>(a, b);
    uint64_t r[6];
    mont_mul_adx(r, (const uint64_t*)a.v, (const uint64_t*)b.v, P.p, P.inv);
    // both < 2p and congruent: compare canonical forms
    Fq got;
    memcpy(got.v, r, 48);
    if (memcmp(hcanon(got).v, hcanon(ref).v, 48)) bad++;
  }
  Fq a, b;
  rand2p(a);
  rand2p(b);
  const int reps = 2000000;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; i++) a = hmul_cxx<true>(a, b);
  auto t1 = std::chrono::steady_clock::now();
  uint64_t x[6];
  memcpy(x, a.v, 48);
  for (int i = 0; i < reps; i++) mont_mul_adx(x, x, (const uint64_t*)b.v, P.p, P.inv);
  auto t2 = std::chrono::steady_clock::now();
  printf("mismatches %d of %d; hmul_cxx %.1f ns, mont_mul_adx %.1f ns (check %llx %llx)\n", bad, n,
         std::chrono::duration<double, std::nano>(t1 - t0).count() / reps,
         std::chrono::duration<double, std::nano>(t2 - t1).count() / reps, (unsigned long long)a.v[0],
         (unsigned long long)x[0]);
  return bad != 0;
}
