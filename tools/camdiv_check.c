/* camdiv_check.c — the camera's x / n as one correction step on x * RN(1 / n) (rt_device.h
 * pixel_coord_div) against the IEEE division, on the CPU: every image size n <= 4096 and every 97th up to
 * 65536, jittered pixel coordinates x = px + U (U with 53 random bits) plus x = 0, x = px and
 * x = px + (1 - 2^-53).  Exit status 0 when every quotient is bit-identical.
 * Build: gcc -O2 -ffp-contract=off camdiv_check.c -lm (tests/test_divisions.py). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t nx(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(int argc, char** argv) {
  long long n = argc > 1 ? atoll(argv[1]) : 10000000, bad = 0, tot = 0;
  for (int W = 1; W <= 65536; W = (W < 4096 ? W + 1 : W + 97)) {
    const double w = (double)W, r = 1.0 / w;
    const long long per = W < 4096 ? n / 4096 : n / 700;
    for (long long i = 0; i < per; ++i) {
      const double px = (double)(nx() % (uint64_t)W), u = (double)(nx() >> 11) * 0x1p-53;
      double x = px + u;
      if (i == 0) x = 0.0; else if (i == 1) x = px; else if (i == 2) x = px + (1.0 - 0x1p-53);
      const double q0 = x * r, q = fma(fma(-w, q0, x), r, q0);
      ++tot;
      if (q != x / w) { if (bad < 5) printf("W %d x %.17g: %.17g vs %.17g\n", W, x, q, x / w); ++bad; }
    }
  }
  printf("%lld of %lld differ\n", bad, tot);
  return bad != 0;
}
