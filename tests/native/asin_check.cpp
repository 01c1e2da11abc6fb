// Host check: asin_go_sel (the select form the kernels use) == asin_go (Go's math.Asin
// restated) bit for bit, over edge values and random inputs in [-1, 1].
#include <cstdio>
#include <cstring>
#include <random>

#include "../../veneur_amd/csrc/gomath.h"

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 rng(12345);
  long bad = 0;
  auto check = [&](double x) {
    double a = vn::asin_go(x), b = vn::asin_go_sel(x);
    uint64_t ua, ub;
    memcpy(&ua, &a, 8);
    memcpy(&ub, &b, 8);
    if (ua != ub && !(a != a && b != b)) {
      if (bad < 5) printf("mismatch x=%.17g go=%.17g sel=%.17g\n", x, a, b);
      bad++;
    }
  };
  const double edges[] = {0.0, -0.0, 1.0, -1.0, 0.7, -0.7, 0.66, 2.41421356237309504880, 1e-300, 5e-324,
                          0.5, -0.5, 0.9999999999999999, 1.0000000000000002, 0.70000000000000007};
  for (double e : edges) check(e);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (long i = 0; i < n; i++) check(u(rng));
  // dense sweeps around the branch points (in the argument and in satan's argument)
  for (double c : {0.7, 0.66 / sqrt(1 + 0.66 * 0.66), 2.41421356237309504880 / sqrt(1 + 2.41421356237309504880 * 2.41421356237309504880)}) {
    double x = c;
    for (int i = 0; i < 20000; i++) { check(x); check(-x); x = nextafter(x, 2.0); }
    x = c;
    for (int i = 0; i < 20000; i++) { check(x); x = nextafter(x, -2.0); }
  }
  // k-scale arguments 2q-1 for q = W/T with integer W, T (what indexEstimate sees)
  for (long T = 1; T < 3000; T += 7)
    for (long W = 0; W <= T; W++) check(vn::dsub(vn::dmul(2.0, vn::ddiv((double)W, (double)T)), 1.0));
  printf("%ld mismatches\n", bad);
  return bad != 0;
}
