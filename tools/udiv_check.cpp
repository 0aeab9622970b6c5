// Host check of the launch-invariant unsigned division (rt_layout.h make_udiv; the device applies it
// with udiv() in the megakernel's unit fetch): q = (t + ((n - t) >> s1)) >> s2, t = mulhi(m, n), must
// equal n / d.  Every divisor 1..4999 against 2000 dividends (0..9, 2^32 - 1, random), then 2 M random
// (divisor, dividend) pairs.  Prints "bad=<count>" and exits 1 on any mismatch.
#include <cstdint>
#include <cstdio>
#include <random>

#include "../shirley-raytracing-rs_amd/csrc/rt/rt_layout.h"

using rt::UDiv;
static uint32_t apply(uint32_t n, UDiv D) {
  const uint32_t t = (uint32_t)(((uint64_t)D.m * n) >> 32);
  return (t + ((n - t) >> D.s1)) >> D.s2;
}

int main() {
  std::mt19937_64 g(1);
  long bad = 0;
  for (uint32_t d = 1; d < 5000; ++d) {
    const UDiv D = rt::make_udiv(d);
    for (int k = 0; k < 2000; ++k) {
      uint32_t n = (uint32_t)g();
      if (k < 10) n = (uint32_t)k;
      if (k == 10) n = 0xffffffffu;
      if (apply(n, D) != n / d) ++bad;
    }
  }
  for (int k = 0; k < 2000000; ++k) {
    uint32_t d = (uint32_t)g() | 1u;
    if (k & 1) d = (uint32_t)(g() % 100000) + 1;
    if (k % 7 == 0) d = 1u << (k % 32);
    const uint32_t n = (uint32_t)g();
    if (apply(n, rt::make_udiv(d)) != n / d) ++bad;
  }
  printf("bad=%ld\n", bad);
  return bad ? 1 : 0;
}
