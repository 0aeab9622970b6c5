// portable_libm.h — sin, log, atan2, acos and x^5 written in plain IEEE binary64 operations (+, -, *, /,
// sqrt, rint, fma on exact-by-construction terms), so that a CPU build (gcc, -ffp-contract=off) and a
// gfx950 build (hipcc, -ffp-contract=off) return the same bits for every argument.
//
// Diagnostic only ("libm isolation"): the product kernels call the device libm (ocml) and
// the oracle calls glibc — the reference's own libm — and the two differ in the last bit for a small share
// of arguments, which is where the frames' non-identical channels come from.  A kernel build with
// RT_PORTABLE_LIBM and an oracle build with OR_PORTABLE_LIBM both call these instead; their frames must
// then agree bit for bit (tests/test_gpu_libm_isolation.py), which separates libm ulps from any semantic
// slip.  Accuracy is ~1e-15 relative (fdlibm-style kernels): good enough for a plausible image, and only
// determinism across the two builds matters here.
#pragma once

#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define PL_FN __host__ __device__ static inline
#else
#define PL_FN static inline
#endif

PL_FN uint64_t pl_bits(double x) {
  uint64_t u;
  __builtin_memcpy(&u, &x, sizeof u);
  return u;
}
PL_FN double pl_from_bits(uint64_t u) {
  double x;
  __builtin_memcpy(&x, &u, sizeof x);
  return x;
}

// sin: k = rint(x 2/pi), r = x - k pi/2 in three parts (Cody-Waite), then the sin / cos kernel of
// quadrant k mod 4 (fdlibm's minimax coefficients)
PL_FN double pl_sin(double x) {
  if (!(fabs(x) <= 1e9)) return (x - x) * 0.0;  // NaN for inf / NaN; 0 beyond the reduction's range
  const double invpio2 = 6.36619772367581382433e-01;
  const double p1 = 1.57079632673412561417e+00, p2 = 6.07710050630396597660e-11, p3 = 2.02226624871116645580e-21;
  const double k = rint(x * invpio2);
  const double r = ((x - k * p1) - k * p2) - k * p3;
  const double z = r * r;
  const double s = r + (r * z) * (-1.66666666666666324348e-01 +
                                  z * (8.33333333332248946124e-03 +
                                       z * (-1.98412698298579493134e-04 +
                                            z * (2.75573137070700676789e-06 +
                                                 z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)))));
  const double c = (1.0 - 0.5 * z) + (z * z) * (4.16666666666666019037e-02 +
                                                z * (-1.38888888888741095749e-03 +
                                                     z * (2.48015872894767294178e-05 +
                                                          z * (-2.75573143513906633035e-07 +
                                                               z * (2.08757232129817482790e-09 +
                                                                    z * -1.13596475577881948265e-11)))));
  const int q = (int)((long long)k & 3);
  return q == 0 ? s : q == 1 ? c : q == 2 ? -s : -c;
}

// log: x = m 2^e with m in [sqrt(2)/2, sqrt(2)), log m = f - f^2/2 + s (f^2/2 + R(s^2)), s = f / (2 + f)
PL_FN double pl_log(double x) {
  if (x == 0.0) return -INFINITY;
  if (!(x > 0.0)) return (x - x) / 0.0;  // NaN for x < 0 and NaN
  if (x == INFINITY) return x;
  int e = 0;
  if (x < 0x1p-1022) {  // subnormal: scale into the normal range (exact)
    x *= 0x1p54;
    e = -54;
  }
  const uint64_t b = pl_bits(x);
  e += (int)((b >> 52) & 0x7ff) - 1023;
  double m = pl_from_bits((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);  // [1, 2)
  if (m > 1.41421356237309504880) {
    m *= 0.5;
    e += 1;
  }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (3.999999999940941908e-01 + w * (2.222219843214978396e-01 + w * 1.531383769920937332e-01));
  const double t2 = z * (6.666666666666735130e-01 +
                         w * (2.857142874366239149e-01 + w * (1.818357216161805012e-01 + w * 1.479819860511658591e-01)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)e;
  return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
}

// atan for t in [0, 1]: t > 2 - sqrt(3) folded by atan t = pi/6 + atan((sqrt(3) t - 1) / (sqrt(3) + t)),
// then the odd series to t^25 (|t| <= 0.268: the next term is < 1e-16 of the sum)
PL_FN double pl_atan01(double t) {
  double base = 0.0;
  if (t > 0.26794919243112270) {
    const double sq3 = 1.73205080756887719318;
    t = (sq3 * t - 1.0) / (sq3 + t);
    base = 5.23598775598298815658e-01;  // pi / 6
  }
  const double z = t * t;
  double p = 1.0 / 25.0;
  p = 1.0 / 23.0 - z * p;
  p = 1.0 / 21.0 - z * p;
  p = 1.0 / 19.0 - z * p;
  p = 1.0 / 17.0 - z * p;
  p = 1.0 / 15.0 - z * p;
  p = 1.0 / 13.0 - z * p;
  p = 1.0 / 11.0 - z * p;
  p = 1.0 / 9.0 - z * p;
  p = 1.0 / 7.0 - z * p;
  p = 1.0 / 5.0 - z * p;
  p = 1.0 / 3.0 - z * p;
  return base + (t - (t * z) * p);
}

PL_FN double pl_atan2(double y, double x) {
  const double pi = 3.14159265358979311600e+00, pio2 = 1.57079632679489655800e+00;
  if (x != x || y != y) return x + y;
  const double ax = fabs(x), ay = fabs(y);
  if (ax == 0.0 && ay == 0.0) return (signbit(x) ? pi : 0.0) * (signbit(y) ? -1.0 : 1.0);
  double a;  // atan(ay / ax) in [0, pi/2]
  if (ay <= ax) a = pl_atan01(ay / ax);
  else a = pio2 - pl_atan01(ax / ay);
  if (signbit(x)) a = pi - a;
  return signbit(y) ? -a : a;
}

PL_FN double pl_acos(double x) {
  if (!(fabs(x) <= 1.0)) return (x - x) / 0.0;
  return pl_atan2(sqrt((1.0 - x) * (1.0 + x)), x);
}

// x^5 as the megakernel's double-double product (rt_device.h pow5) for every x
PL_FN double pl_pow5(double x) {
  const double x2 = x * x;
  const double x2l = fma(x, x, -x2);
  const double x4 = x2 * x2;
  const double x4l = fma(x2, x2, -x4) + (2.0 * x2) * x2l;
  const double x5 = x4 * x;
  const double x5l = fma(x4, x, -x5) + x4l * x;
  return x5 + x5l;
}
