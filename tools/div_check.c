/* Host check of the corrected-reciprocal division the XZ keys use (gm_keys.hpp div_span / div_time):
 *   q = RN(a * y), y = RN(1 / b);  r = fma(-q, b, a) (exact);  RN(q + r * y) == RN(a / b) ?
 * for the spans b the kernels divide by: 360, 180 (lon / lat) and BinnedTime.maxOffset of the four periods
 * (the XZ3 time span).  Random a in [0, b], random significands over every exponent the kernels can see,
 * +-1..3 ulp around every j b / 2^20, and every integer offset below min(b, 5e7).
 *   gcc -O2 -march=native -o /tmp/div_check tools/div_check.c -lm && /tmp/div_check [draws]   ->  "bad 0"
 * (tests/test_div_check.py runs a reduced count on every CPU test run)
 * (Not part of the library: a proof aid; x86 fma is IEEE-exact.) */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t s = 88172645463325252ull;
static inline uint64_t nx(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline double fdiv(double a, double b, double y) {
  const double q = a * y;
  return fma(fma(-q, b, a), y, q);
}

int main(int argc, char** argv) {
  const long N = argc > 1 ? atol(argv[1]) : 200000000;   /* random draws per kind and span */
  const double bs[6] = {360.0, 180.0, 86400000.0, 604800.0, 2678400.0, 527050.0};
  const int emin[6] = {-45, -45, -900, -900, -900, -900};   /* lon / lat: a = v + 180 is 0 or >= 2^-45 */
  long bad = 0, tot = 0;
  for (int k = 0; k < 6; k++) {
    const double b = bs[k], y = 1.0 / b;
    for (long i = 0; i < N; i++) {
      const double a = (double)(nx() >> 11) * 0x1p-53 * b;
      if (fdiv(a, b, y) != a / b) { if (bad < 5) printf("bad %a / %a\n", a, b); bad++; }
      tot++;
    }
    for (long i = 0; i < N; i++) {
      const uint64_t m = nx();
      const int e = (int)(m % (uint64_t)(40 - emin[k])) + emin[k];
      const double a = ldexp(1.0 + (double)((m >> 12) & ((1ull << 52) - 1)) * 0x1p-52, e);
      if (a > b) continue;
      if (fdiv(a, b, y) != a / b) { if (bad < 5) printf("bad %a / %a\n", a, b); bad++; }
      tot++;
    }
    for (long j = 0; j <= (N < (1L << 20) ? N : (1L << 20)); j++) {
      const double a0 = ldexp((double)j, -20) * b;
      for (int d = -3; d <= 3; d++) {
        double a = a0;
        for (int u = 0; u < (d < 0 ? -d : d); u++) a = nextafter(a, d < 0 ? -1.0 : 1e300);
        if (a < 0 || a > b) continue;
        if (fdiv(a, b, y) != a / b) { if (bad < 5) printf("bad %a / %a\n", a, b); bad++; }
        tot++;
      }
    }
    for (long i = 0; i < (long)b && i < N / 4; i++) {
      const double a = (double)i;
      if (fdiv(a, b, y) != a / b) { if (bad < 5) printf("bad %a / %a\n", a, b); bad++; }
      tot++;
    }
  }
  printf("checked %ld quotients, bad %ld\n", tot, bad);
  return bad != 0;
}
