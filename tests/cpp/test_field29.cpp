// Host check of field29.h (radix-2^29 Fq, R = 2^377) against Python integers
// (tests/test_field29.py): per input line "a b" (field.h Montgomery words,
// 12 x u32 hex, possibly unreduced below 64 p) print
//   mul, sqr, add, sub, to_std(from_std(a)), inv(a),
//   mul_sum(a, b, a, a) = ab + a^2, mul_sub(a, b, b, b) = ab - b^2,
//   pack377(a) (= a 2^377 mod p as a plain integer), unpack377(pack377(a)),
//   cneg(a, 1) = -a, cneg(a, 0) = a  for reduced a, b
//   the wave engine's stage product / square               for wide a, b
#include <cstdio>
#include <cstring>
#include "field.h"

using namespace tpst;

static void put(const Fq& r) {
  for (int i = 0; i < 12; i++) printf("%08x ", r.v[i]);
  printf("\n");
}

int main() {
  int n;
  if (scanf("%d", &n) != 1) return 1;
  for (int t = 0; t < n; t++) {
    int wide;
    Fq a, b;
    if (scanf("%d", &wide) != 1) return 1;
    for (int i = 0; i < 12; i++)
      if (scanf("%x", &a.v[i]) != 1) return 1;
    for (int i = 0; i < 12; i++)
      if (scanf("%x", &b.v[i]) != 1) return 1;
    const Fq29 x = from_std(a), y = from_std(b);
    if (wide) {  // wave_tower.h stage_mul / stage_sqr
      Fq29 m = mul(x, y);
      reduce_once(m);
      put(to_std(m));
      put(to_std(sqr(x)));
    } else {
      put(to_std(mul(x, y)));
      put(to_std(sqr(x)));
      put(to_std(add(x, y)));
      put(to_std(sub(x, y)));
      put(to_std(x));
      put(inv(a));
      put(to_std(mul_sum(x, y, x, x)));
      put(to_std(mul_sub(x, y, y, y)));
      Fq w;  // the accumulation kernels' packed bucket format and back
      pack377(x, w.v);
      put(w);
      put(to_std(unpack377(w.v)));
      put(to_std(cneg(x, true)));
      put(to_std(cneg(x, false)));
    }
  }
  return 0;
}
