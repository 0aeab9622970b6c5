// Bit-identity check of the shared-reciprocal division (rt_device.h: recip / div_recip / unit_fast)
// against the compiler's binary64 division, and of sqrt_rn against the compiler's sqrt, on the GPU.  Usage: divcheck [log2 pairs per launch] [launches]
// Pairs: random signs, random 52-bit mantissas (a share with all-ones / all-zeros / near-one patterns),
// exponents uniform in [-300, 300]; vectors likewise with independent component exponents in a
// +-40 window.  Prints the mismatch counts; exit code 1 if any.
#include "../shirley-raytracing-rs_amd/csrc/rt/rt_device.h"
#include <cstdio>
#include <cstdlib>

using namespace rt;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}
__device__ __forceinline__ double make(uint64_t h, int e) {
  uint64_t m = h & ((1ull << 52) - 1);
  switch ((h >> 52) & 15) {  // special mantissas now and then
    case 0: m = (1ull << 52) - 1; break;
    case 1: m = 0; break;
    case 2: m = ((1ull << 52) - 1) ^ (h >> 58); break;
    case 3: m = (h >> 58); break;
    default: break;
  }
  const uint64_t bits = ((uint64_t)(h >> 63) << 63) | ((uint64_t)(e + 1023) << 52) | m;
  return __longlong_as_double((long long)bits);
}

__global__ void check(uint64_t base, unsigned long long* bad) {
  const uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t h1 = mix(i * 2 + 1), h2 = mix(i * 2 + 2), h3 = mix(i * 7 + 3);
  const int e1 = (int)(h3 % 601) - 300, e2 = (int)((h3 >> 16) % 601) - 300;
  const double a = make(h1, e1), b = make(h2, e2);
  const double q = a / b;
  const double f = div_recip(a, recip(b));
  if (__double_as_longlong(q) != __double_as_longlong(f)) atomicAdd(&bad[0], 1ull);
  // Markstein's correction with the correctly rounded reciprocal 1.0 / b (the traversal's 1/d: rect and
  // box faces divide through it, rt_device.h rect_t<.., INV>)
  const double g = div_recip(a, Recip{b, 1.0 / b});
  if (__double_as_longlong(q) != __double_as_longlong(g)) atomicAdd(&bad[3], 1ull);
  // face planes (rt_device.h face_div): numerators with exponents in [-310, 700] (every numerator of a
  // quotient >= t_min = 0.001 with |d| >= 2^-300, up to face_div's 2^700 bound) over the same divisors
  const int ef = (int)((h3 >> 40) % 1011) - 310;
  const double af = make(h1, ef);
  if (__double_as_longlong(af / b) != __double_as_longlong(face_div(af, b, 1.0 / b, true))) atomicAdd(&bad[5], 1ull);
  // the traversal's 1 / d (rt_device.h inv_dir): the compiler's 1.0 / b against div_recip(1, recip(b))
  // for |b| in [2^-300, 2^300] (inv_dir's fast path), special values included through inv_dir itself
  const unsigned sp = (unsigned)(h3 >> 58) & 15u;  // special components now and then (inv_dir's fallback)
  const double bs = sp == 0 ? 0.0 : sp == 1 ? -0.0 : sp == 2 ? __builtin_inf() : sp == 3 ? 1e-310 : sp == 4 ? 0x1p-301 : b;
  const v3 iv = inv_dir(V(bs, a, b));
  if (__double_as_longlong(1.0 / bs) != __double_as_longlong(iv.x) || __double_as_longlong(1.0 / a) != __double_as_longlong(iv.y) ||
      __double_as_longlong(1.0 / b) != __double_as_longlong(iv.z))
    atomicAdd(&bad[4], 1ull);
  // unit vectors: component exponents within +-40 of a common one
  const int ec = (int)((h3 >> 32) % 521) - 260;
  const uint64_t g1 = mix(i * 5 + 11), g2 = mix(i * 5 + 12), g3 = mix(i * 5 + 13);
  const v3 v = V(make(g1, ec + (int)(g1 % 81) - 40), make(g2, ec + (int)(g2 % 81) - 40), make(g3, ec + (int)(g3 % 81) - 40));
  const v3 u0 = V(v.x / sqrt(len2(v)), v.y / sqrt(len2(v)), v.z / sqrt(len2(v))), u1 = unit_fast(v);
  if (__double_as_longlong(u0.x) != __double_as_longlong(u1.x) || __double_as_longlong(u0.y) != __double_as_longlong(u1.y) ||
      __double_as_longlong(u0.z) != __double_as_longlong(u1.z))
    atomicAdd(&bad[1], 1ull);
  // sqrt_rn against the compiler's sqrt: positive x over the whole exponent range (denormals, the
  // 2^-767 scaling edge, huge values) plus the special values now and then
  const uint64_t hs = mix(i * 3 + 17);
  const int es = (int)(hs % 2100) - 1075;  // exponents -1075 .. 1024: denormals .. inf / NaN patterns
  double x = es < -1022 ? __longlong_as_double((long long)(hs >> 12)) : make(hs & ~(1ull << 63), es < 1024 ? es : 1023);
  switch ((hs >> 56) & 63) {
    case 0: x = 0.0; break;
    case 1: x = -0.0; break;
    case 2: x = __builtin_inf(); break;
    case 3: x = -1.0; break;
    case 4: x = __builtin_nan(""); break;
    case 5: x = 0x1p-767; break;
    case 6: x = __longlong_as_double(0x1000000000000000ll - 1); break;  // just below 2^-767
    default: break;
  }
  const double s0 = sqrt(x), s1 = sqrt_rn(x);
  if (__double_as_longlong(s0) != __double_as_longlong(s1) && !(s0 != s0 && s1 != s1)) atomicAdd(&bad[2], 1ull);
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 26;
  const int launches = argc > 2 ? atoi(argv[2]) : 16;
  unsigned long long* bad;
  if (hipMalloc(&bad, 48) != hipSuccess) return 2;
  (void)hipMemset(bad, 0, 48);
  const uint64_t per = 1ull << lg;
  for (int l = 0; l < launches; ++l)
    hipLaunchKernelGGL(check, dim3((unsigned)(per / 256)), dim3(256), 0, 0, (uint64_t)l * per, bad);
  unsigned long long h[6];
  if (hipMemcpy(h, bad, 48, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("divcheck: %llu pairs, %llu division mismatches, %llu unit mismatches, %llu sqrt mismatches, "
         "%llu inverse-division mismatches, %llu reciprocal mismatches, %llu face-division mismatches\n",
         (unsigned long long)(per * launches), h[0], h[1], h[2], h[3], h[4], h[5]);
  return (h[0] || h[1] || h[2] || h[3] || h[4] || h[5]) ? 1 : 0;
}
