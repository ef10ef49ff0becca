// Host Poseidon A/B: the transcript permutation as the sponge runs it
// (poseidon_host.h: squarings, constants and sparse matrices of the
// equivalent form) against the textbook round structure, plus the field
// operations it is built from.  Checks the two permutations agree.
//   tools/build_host_bench.sh -> tools/bin/host_poseidon_bench
#include <chrono>
#include <cstdio>
#include "../testudo_amd/csrc/poseidon_host.h"
#include "../testudo_amd/csrc/field29.h"
#include "../testudo_amd/csrc/host_curve.h"

using namespace tpst;

static double now_ns() {
  return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// textbook permutation: full ark, x^17 by multiplications, dense MDS
static void permute_plain(Fq* st) {
  static Fq ark[39][3], mds[3][3];
  static bool init = false;
  if (!init) {
    for (int r = 0; r < 39; r++)
      for (int i = 0; i < 3; i++) ark[r][i] = fq_canon(POSEIDON_ARK[r][i]);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) mds[i][j] = fq_canon(POSEIDON_MDS[i][j]);
    init = true;
  }
  for (int r = 0; r < 39; r++) {
    for (int i = 0; i < 3; i++) st[i] = add(st[i], ark[r][i]);
    const bool full = r < 4 || r >= 35;
    for (int i = 0; i < (full ? 3 : 1); i++) {
      const Fq x = st[i], x2 = hmul(x, x), x4 = hmul(x2, x2), x8 = hmul(x4, x4), x16 = hmul(x8, x8);
      st[i] = hmul(x16, x);
    }
    Fq ns[3];
    for (int i = 0; i < 3; i++) ns[i] = hmul3(mds[i][0], st[0], mds[i][1], st[1], mds[i][2], st[2]);
    for (int i = 0; i < 3; i++) st[i] = ns[i];
  }
}

int main() {
  Sponge sp;
  uint64_t seed[6] = {0x1234, 0x5678, 0x9abc, 0xdef0, 0x1111, 0x0022};
  for (int i = 0; i < 3; i++) {
    seed[0] += 7;
    sp.st[i] = fq_canon(seed);
  }
  Fq ref[3] = {sp.st[0], sp.st[1], sp.st[2]};
  for (int k = 0; k < 4; k++) {
    sp.permute();
    permute_plain(ref);
  }
  for (int i = 0; i < 3; i++)
    if (memcmp(sp.st[i].v, ref[i].v, 48)) {
      printf("MISMATCH\n");
      return 1;
    }
  const int N = 2000;
  double t0 = now_ns();
  for (int k = 0; k < N; k++) sp.permute();
  double t1 = now_ns();
  for (int k = 0; k < N; k++) permute_plain(ref);
  double t2 = now_ns();
  Fq a = sp.st[0], b = sp.st[1];
  const int M = 200000;
  double t3 = now_ns();
  for (int k = 0; k < M; k++) a = hmul(a, b);
  double t4 = now_ns();
  for (int k = 0; k < M; k++) a = hsqr(a);
  double t5 = now_ns();
  for (int k = 0; k < M; k++) a = hmul3(a, b, b, a, a, b);
  double t6 = now_ns();
  for (int k = 0; k < M; k++) a = add(a, b);
  double t7 = now_ns();
  double t8 = now_ns();
  host::HFq h = host::HFq::from(a);
  for (int k = 0; k < 2000; k++) {
    h = host::inv(h);
    h.v[1] ^= 1;
  }
  double t9 = now_ns();
  Fq g = a;
  for (int k = 0; k < 2000; k++) {
    g = inv(g);
    g.v[1] ^= 1;
  }
  double t10 = now_ns();
  printf("inverse: host::inv %.2f us, tpst::inv (field29 binary GCD) %.2f us (check %llx)\n", (t9 - t8) / 2000 * 1e-3,
         (t10 - t9) / 2000 * 1e-3, (unsigned long long)(h.v[0] ^ g.v[0]));
  printf("permute (sponge form) %.2f us, textbook %.2f us; hmul %.1f ns, hsqr %.1f ns, hmul3 %.1f ns, add %.1f ns"
         " (check %llx)\n",
         (t1 - t0) / N * 1e-3, (t2 - t1) / N * 1e-3, (t4 - t3) / M, (t5 - t4) / M, (t6 - t5) / M, (t7 - t6) / M,
         (unsigned long long)(a.v[0] ^ ref[0].v[0]));
  printf("host products: %s\n", host_adx() ? "MULX/ADCX/ADOX assembly" : "C++ __int128");
  return 0;
}
