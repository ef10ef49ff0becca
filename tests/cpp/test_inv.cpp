// Host check of field.h's constant-flow inverse (Fq and Fr): a * inv(a) == 1
// for random and edge inputs; inv(0) == 0.  Built and run by tests/test_abi.py.
#include <cstdio>
#include <cstdlib>
#include <random>
#include "field.h"

using namespace tpst;

template <class C>
static int check(std::mt19937_64& rng, int n) {
  int bad = 0;
  for (int k = 0; k < n; k++) {
    Fp<C> a;
    for (int i = 0; i < C::N; i++) a.v[i] = (uint32_t)rng();
    if (k == 0) a = Fp<C>::one();
    if (k == 1) a = sub(Fp<C>::zero(), Fp<C>::one());
    if (k == 2) { a = Fp<C>::zero(); a.v[0] = 1; }
    a.v[C::N - 1] &= C::p(C::N - 1);  // keep below the modulus' top limb
    reduce_once(a);
    if (is_zero(a)) continue;
    const Fp<C> r = mul(a, inv(a));
    if (!eq(r, Fp<C>::one())) bad++;
  }
  if (!is_zero(inv(Fp<C>::zero()))) bad++;
  return bad;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 20000;
  std::mt19937_64 rng(377);
  const int bq = check<FqCfg>(rng, n), br = check<FrCfg>(rng, n);
  printf("fq_bad %d fr_bad %d of %d\n", bq, br, n);
  return (bq || br) ? 1 : 0;
}
