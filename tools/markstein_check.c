// markstein_check.c -- the shared-divisor quotient of bmpc_core.h (div_rcp) against the IEEE
// division: q0 = x * r, q = fma(fma(-q0, y, x), r, q0) with r = 1 / y correctly rounded gives the
// correctly rounded x / y (Markstein's theorem) -- checked here on 2e8 random pairs over 2^+-60,
// powers-of-two divisors and zero numerators.  build: gcc -O2 -mfma -o /tmp/mk tools/markstein_check.c -lm
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rnd(int emin, int emax) {
  double m = 1.0 + (double)(xr() >> 11) / 9007199254740992.0;
  int e = emin + (int)(xr() % (uint64_t)(emax - emin + 1));
  double v = ldexp(m, e);
  return (xr() & 1) ? -v : v;
}
int main(int argc, char** argv) {
  long bad = 0, n = argc > 1 ? atol(argv[1]) : 200000000;
  for (long i = 0; i < n; ++i) {
    double x = rnd(-60, 60), y = rnd(-60, 60);
    if (i % 7 == 0) y = ldexp(1.0, (int)(xr() % 40) - 20);   // powers of two
    if (i % 11 == 0) x = 0.0;
    double r = 1.0 / y;
    double q0 = x * r;
    double e = fma(-q0, y, x);
    double q = fma(e, r, q0);
    double ref = x / y;
    if (q != ref || signbit(q) != signbit(ref)) {
      if (bad < 5) printf("x=%.17g y=%.17g ref=%.17g got=%.17g\n", x, y, ref, q);
      ++bad;
    }
  }
  printf("mismatches %ld of %ld\n", bad, n);
  return 0;
}
