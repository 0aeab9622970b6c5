// Bit-identity check of the shared-reciprocal division (rt_device.h: recip / div_recip / unit_fast)
// against the compiler's binary64 division, on the GPU.  Usage: divcheck [log2 pairs per launch] [launches]
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
  // unit vectors: component exponents within +-40 of a common one
  const int ec = (int)((h3 >> 32) % 521) - 260;
  const uint64_t g1 = mix(i * 5 + 11), g2 = mix(i * 5 + 12), g3 = mix(i * 5 + 13);
  const v3 v = V(make(g1, ec + (int)(g1 % 81) - 40), make(g2, ec + (int)(g2 % 81) - 40), make(g3, ec + (int)(g3 % 81) - 40));
  const v3 u0 = unit(v), u1 = unit_fast(v);
  if (__double_as_longlong(u0.x) != __double_as_longlong(u1.x) || __double_as_longlong(u0.y) != __double_as_longlong(u1.y) ||
      __double_as_longlong(u0.z) != __double_as_longlong(u1.z))
    atomicAdd(&bad[1], 1ull);
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 26;
  const int launches = argc > 2 ? atoi(argv[2]) : 16;
  unsigned long long* bad;
  if (hipMalloc(&bad, 16) != hipSuccess) return 2;
  (void)hipMemset(bad, 0, 16);
  const uint64_t per = 1ull << lg;
  for (int l = 0; l < launches; ++l)
    hipLaunchKernelGGL(check, dim3((unsigned)(per / 256)), dim3(256), 0, 0, (uint64_t)l * per, bad);
  unsigned long long h[2];
  if (hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("divcheck: %llu pairs, %llu division mismatches, %llu unit mismatches\n",
         (unsigned long long)(per * launches), h[0], h[1]);
  return (h[0] || h[1]) ? 1 : 0;
}
