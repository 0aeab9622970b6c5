// rt_device.h — device functions of the hot path shared by the megakernel (trace.hip) and the
// wavefront kernels (wavefront.hip): f64 vector algebra in nalgebra's order, the counter RNG,
// intersection, BVH traversal, textures, materials, camera.  Semantics follow the reference line by
// line (citations inline); compiled with -ffp-contract=off (Rust never fuses a*b+c).
#pragma once

// The transcendental functions of the path: the device libm, or (RT_PORTABLE_LIBM, a diagnostic build
// only) portable_libm.h's, which the oracle's OR_PORTABLE_LIBM build shares
#ifdef RT_PORTABLE_LIBM
#include "portable_libm.h"
#define RT_SIN pl_sin
#define RT_LOG pl_log
#define RT_ACOS pl_acos
#define RT_ATAN2 pl_atan2
#define RT_POW5_LIBM(x) pl_pow5(x)
#else
#define RT_SIN sin
#define RT_LOG log
#define RT_ACOS acos
#define RT_ATAN2 atan2
#define RT_POW5_LIBM(x) pow(x, 5.0)
#endif
#include <hip/hip_runtime.h>

#include "../../../include/shirley_rt.h"
#include "rt_layout.h"

namespace rt {


// ------------------------------------------------------------------------------------------
// f64 vector algebra in nalgebra's evaluation order (core/vec3.rs over nalgebra 0.31)
// ------------------------------------------------------------------------------------------
struct v3 {
  double x, y, z;
};
__device__ __forceinline__ v3 V(double x, double y, double z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 hmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 scale(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ double dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ double len2(v3 a) { return dot(a, a); }
// Correctly rounded binary64 sqrt with a shorter common path.  hipcc lowers sqrt(x) on gfx950 to:
// x' = x < 2^-767 ? x * 2^256 : x, r = rsq(x'), g = x' r, h = r / 2, e = fma(-h, g, 0.5),
// g = fma(g, e, g), d = fma(-g, g, x'), h = fma(h, e, h), g = fma(d, h, g), d = fma(-g, g, x'),
// g = fma(d, h, g), result = scale g back by 2^-128, and x' itself when x' is +-0 or +inf.  For x in
// [2^-767, DBL_MAX] neither the scaling nor the pass-through applies, so the same rsq + Newton
// sequence alone gives the same bits (checked on the GPU by tools/divcheck.hip); other x take sqrt().
__device__ __forceinline__ double sqrt_rn(double x) {
  if (!(x >= 0x1p-767 && x <= 1.7976931348623157e308)) return sqrt(x);
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r, h = r * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  double d = __builtin_fma(-g, g, x);
  h = __builtin_fma(h, e, h);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double len(v3 a) { return sqrt_rn(len2(a)); }
__device__ __forceinline__ v3 unit(v3 a) {
  double n = len(a);
  return V(a.x / n, a.y / n, a.z / n);
}
// Exact division by a shared reciprocal.  The compiler lowers a / b (binary64, correctly rounded)
// to: b' = div_scale(b), r0 = rcp(b'), two Newton steps r = fma(r, fma(-b', r, 1), r), a' =
// div_scale(a), q0 = a' r, e = fma(-b', q0, a'), q = div_fmas(e, r, q0), div_fixup(q).  With |a| and
// |b| in [2^-300, 2^300] both div_scale steps are the identity (no exponent gap >= 768, no denormal
// or tiny operand or quotient), div_fmas is a plain fma and div_fixup only re-applies the quotient's
// sign — so a / b = fma(fma(-b, a r, a), r, a r) with r from b alone, and divisions by one b can share
// r (the rcp and the Newton steps) at a mul and two fmas each.  Bit-identity is checked by
// tools/divcheck.hip (tests/test_gpu_divcheck.py).
struct Recip {
  double b, r;
};
__device__ __forceinline__ Recip recip(double b) {
  double r = __builtin_amdgcn_rcp(b);  // v_rcp_f64
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  return Recip{b, r};
}
// a / R.b for |a|, |R.b| in [2^-300, 2^300] (the caller checks)
__device__ __forceinline__ double div_recip(double a, const Recip& R) {
  const double q0 = a * R.r;
  return __builtin_fma(__builtin_fma(-R.b, q0, a), R.r, q0);
}
// unit() with the three divisions by |a| sharing one reciprocal when every operand is in range
// (|components| >= 2^-300 and |a| <= 2^300; |components| <= |a| up to rounding); else unit()'s own
// divisions.  Same bits as unit() either way.
__device__ __forceinline__ v3 unit_fast(v3 a) {
  const double n = len(a);
  const double mn = fmin(fmin(fabs(a.x), fabs(a.y)), fabs(a.z));
  if (mn >= 0x1p-300 && n <= 0x1p300) {
    const Recip R = recip(n);
    return V(div_recip(a.x, R), div_recip(a.y, R), div_recip(a.z, R));
  }
  return V(a.x / n, a.y / n, a.z / n);
}
// 1.0 / d per component, bit-identical to the IEEE division (aabb.rs:66 `1.0 / r.direction[a]`): with
// every |d_i| in [2^-300, 2^300] the compiler's own division sequence reduces to div_recip(1, recip(d_i))
// (see Recip; checked on the GPU by tools/divcheck.hip), 7 instructions instead of 11; one range test
// for the three components, the division itself otherwise (0, inf, NaN, extreme magnitudes).
__device__ __forceinline__ v3 inv_dir(v3 d, bool& in_range) {
  const double lo = fmin(fmin(fabs(d.x), fabs(d.y)), fabs(d.z));
  const double hi = fmax(fmax(fabs(d.x), fabs(d.y)), fabs(d.z));
  in_range = lo >= 0x1p-300 && hi <= 0x1p300;
  if (in_range) return V(div_recip(1.0, recip(d.x)), div_recip(1.0, recip(d.y)), div_recip(1.0, recip(d.z)));
  return V(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
}
__device__ __forceinline__ v3 inv_dir(v3 d) {
  bool in_range;
  return inv_dir(d, in_range);
}
__device__ __forceinline__ double comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// vec3.rs:129-132
__device__ __forceinline__ bool near_zero(v3 a) {
  return fabs(a.x) < 1e-8 && fabs(a.y) < 1e-8 && fabs(a.z) < 1e-8;
}
// vec3.rs:134-137
__device__ __forceinline__ v3 reflect(v3 v, v3 n) { return v - scale(n, 2.0 * dot(v, n)); }
// fp.rs:3-11 fmin (NaN-aware) specialised to fmin(x, 1.0) = math.rs:16-19 fmin_one
__device__ __forceinline__ double fmin_one(double x) { return (x < 1.0) ? x : 1.0; }
// vec3.rs:139-145
__device__ __forceinline__ v3 refract(v3 uv, v3 n, double eta) {
  double cos_theta = fmin_one(dot(scale(uv, -1.0), n));
  v3 r_out_perp = scale(scale(n, cos_theta) + uv, eta);
  double r_out_parallel_mag = sqrt_rn(fabs(1.0 - len2(r_out_perp))) * -1.0;
  return r_out_perp + scale(n, r_out_parallel_mag);
}

// ------------------------------------------------------------------------------------------
// counter-based RNG: Philox4x32-10 keyed by seed, counter (draw/2, sample, pixel, 0).
// A draw is converted like rand 0.8's Standard f64: (u64 >> 11) * 2^-53.
// ------------------------------------------------------------------------------------------
struct Rng {
  uint32_t pixel, sample, draw, c2, c3;
};
// n / d with the launch's UDiv of d (rt_layout.h make_udiv)
__device__ __forceinline__ uint32_t udiv(uint32_t n, const UDiv& D) {
  const uint32_t t = __umulhi(D.m, n);
  return (t + ((n - t) >> D.s1)) >> D.s2;
}
// a ^ b ^ c in one instruction (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
#ifndef RT_PHILOX_ROUNDS  // (timing experiments only: the oracle and every test use 10)
#define RT_PHILOX_ROUNDS 10
#endif
__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                         uint32_t k1) {
#pragma unroll
  for (int r = 0; r < RT_PHILOX_ROUNDS; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    // the round keys are recomputed here (two s_add per round) rather than hoisted out of every loop
    // as 20 live SGPRs, which the kernel would spill to VGPR lanes and reload with v_readlane
    asm volatile("" : "+s"(k0), "+s"(k1));
    // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of separate mul_lo / mul_hi
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    uint32_t n0 = xor3(hi1, c1, k0), n2 = xor3(hi0, c3, k1);
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
}
__device__ __forceinline__ double rng_next(Rng& r, uint64_t seed) {
  uint64_t v;
  if ((r.draw & 1u) == 0u) {
    uint32_t c0 = r.draw >> 1, c1 = r.sample, c2 = r.pixel, c3 = 0u;
    philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
    v = (uint64_t)c0 | ((uint64_t)c1 << 32);
    r.c2 = c2;
    r.c3 = c3;
  } else {
    v = (uint64_t)r.c2 | ((uint64_t)r.c3 << 32);
  }
  r.draw++;
  return (double)(v >> 11) * (1.0 / 9007199254740992.0);
}
// core/math.rs:22-25
__device__ __forceinline__ double random_real(Rng& r, uint64_t seed, double mn, double mx) {
  return mn + (mx - mn) * rng_next(r, seed);
}
// core/math.rs:32-45 (+ vec3.rs:104-110)
__device__ __forceinline__ v3 random_in_unit_sphere(Rng& r, uint64_t seed) {
  for (;;) {
    double x = random_real(r, seed, -1.0, 1.0);
    double y = random_real(r, seed, -1.0, 1.0);
    double z = random_real(r, seed, -1.0, 1.0);
    v3 p = V(x, y, z);
    if (len2(p) <= 1.0) return p;
  }
}
// core/math.rs:70-81
__device__ __forceinline__ v3 random_in_unit_disk(Rng& r, uint64_t seed) {
  for (;;) {
    double x = random_real(r, seed, -1.0, 1.0);
    double y = random_real(r, seed, -1.0, 1.0);
    v3 p = V(x, y, 0.0);
    if (len2(p) <= 1.0) return p;
  }
}

// One draw of a side stream (book-2 extensions): Philox4x32-10 at counter
// (c0, sample, pixel, stream) with stream >= 2^30 — disjoint from the path streams (word 3 = 0) and
// the scene streams (word 2 = 0xFFFFFFFF, small stream ids), so side draws never shift the
// reference-order draws of a path.  The seed is the launch's (uniform), so the round keys are pinned to
// SGPRs as in philox10: hoisted, they were 18 of the book-2 instances' spilled SGPRs.
constexpr uint32_t kStreamTime = 0x40000000u;    // the ray time of (pixel, sample)
constexpr uint32_t kStreamMedium = 0x80000000u;  // | prim: a medium's free-flight draw, c0 = path draw index
__device__ __forceinline__ double side_draw(uint64_t seed, uint32_t c0, uint32_t sample, uint32_t pixel,
                                         uint32_t stream) {
  uint32_t c1 = sample, c2 = pixel, c3 = stream;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    asm volatile("" : "+s"(k0), "+s"(k1));
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0), n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
  }
  const uint64_t v = (uint64_t)c0 | ((uint64_t)c1 << 32);
  return (double)(v >> 11) * (1.0 / 9007199254740992.0);
}

// ------------------------------------------------------------------------------------------
// intersection (t only during traversal; the full hit record is rebuilt for the winner)
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// aabb.rs:62-79 hit2, per axis: t0 = (min - o) * inv, t1 = (max - o) * inv, swapped when inv < 0,
// t_min = t0 > t_min ? t0 : t_min, t_max = t1 < t_max ? t1 : t_max, miss when t_max <= t_min
// (evaluated without the per-axis early exit: t_min only grows and t_max only shrinks, so the final
// test equals the reference's early return).
// Implemented with the swap hoisted out: RaySigns = (1/d < 0) per axis, computed once per ray, to
// pick the near / far plane, so t0, t1 are the values the reference's swap produces; the updates
// `t0 > t_min ? t0 : t_min` and `t1 < t_max ? t1 : t_max` become v_max_f64 / v_min_f64, which also
// return the non-NaN operand (a NaN t0 or t1 leaves the bound as the reference does), and differ
// only on equal values (signed zeros), which no later comparison distinguishes.
struct RaySigns {
  bool x, y, z;
};
__device__ __forceinline__ RaySigns ray_signs(v3 inv) { return RaySigns{inv.x < 0.0, inv.y < 0.0, inv.z < 0.0}; }

__device__ __forceinline__ bool slab_axis(double lo, double hi, bool neg, double o, double iv, double& t_min,
                                          double& t_max) {
  const double pn = neg ? hi : lo, pf = neg ? lo : hi;
  const double t0 = (pn - o) * iv, t1 = (pf - o) * iv;
  t_min = fmax(t0, t_min);
  t_max = fmin(t1, t_max);
  return true;
}

__device__ __forceinline__ bool slab_s(const double* b, v3 o, v3 inv, RaySigns ns, double t_min, double t_max,
                                       double& t_enter) {
  slab_axis(b[0], b[3], ns.x, o.x, inv.x, t_min, t_max);
  slab_axis(b[1], b[4], ns.y, o.y, inv.y, t_min, t_max);
  slab_axis(b[2], b[5], ns.z, o.z, inv.z, t_min, t_max);
  t_enter = t_min;
  return !(t_max <= t_min);
}
__device__ __forceinline__ bool slab_s(const double* b, v3 o, v3 inv, RaySigns ns, double t_min, double t_max,
                                       double& t_enter, double& t_exit) {
  slab_axis(b[0], b[3], ns.x, o.x, inv.x, t_min, t_max);
  slab_axis(b[1], b[4], ns.y, o.y, inv.y, t_min, t_max);
  slab_axis(b[2], b[5], ns.z, o.z, inv.z, t_min, t_max);
  t_enter = t_min;
  t_exit = t_max;
  return !(t_max <= t_min);
}

// slab_s on a sphere's bounding box (c - r, c + r) (sphere.rs:54-60), with the near / far plane of
// each axis formed as c + rn and c - rn, rn = (1/d < 0) ? r : -r: the same two sums slab_s selects
// between (x - y == x + (-y) in IEEE arithmetic), for one sign flip instead of four selects per axis.
__device__ __forceinline__ double sel_neg(bool neg, double r) {
  // r with its sign bit flipped unless neg (the low word is shared)
  const int hi = __double2hiint(r);
  return __hiloint2double(neg ? hi : (hi ^ (int)0x80000000), __double2loint(r));
}
__device__ __forceinline__ bool slab_sphere(const double* p, v3 o, v3 inv, RaySigns ns, double t_min, double t_max) {
  const double r = p[3];
  double rn = sel_neg(ns.x, r);
  t_min = fmax(((p[0] + rn) - o.x) * inv.x, t_min);
  t_max = fmin(((p[0] - rn) - o.x) * inv.x, t_max);
  rn = sel_neg(ns.y, r);
  t_min = fmax(((p[1] + rn) - o.y) * inv.y, t_min);
  t_max = fmin(((p[1] - rn) - o.y) * inv.y, t_max);
  rn = sel_neg(ns.z, r);
  t_min = fmax(((p[2] + rn) - o.z) * inv.z, t_min);
  t_max = fmin(((p[2] - rn) - o.z) * inv.z, t_max);
  return !(t_max <= t_min);
}

// sphere.rs:28-46 (t only)
__device__ __forceinline__ bool sphere_t(const double* p, v3 o, v3 d, double a, double t_min, double t_max,
                                         double& t) {
  v3 oc = o - V(p[0], p[1], p[2]);
  double half_b = dot(oc, d);
  double c = len2(oc) - p[3] * p[3];
  double disc = half_b * half_b - a * c;
  if (disc < 0.0) return false;
  double sqrt_d = sqrt_rn(disc);
  double root = (-half_b - sqrt_d) / a;
  if (root < t_min || t_max < root) {
    root = (-half_b + sqrt_d) / a;
    if (root < t_min || t_max < root) return false;
  }
  t = root;
  return true;
}

// (k - o) / d of a face plane, bit-identical to the IEEE quotient: with every |d_i| in [2^-300, 2^300] (`ok`,
// traverse4) and inv = the ray's 1/d (each component the correctly rounded reciprocal, inv_dir), Markstein's
// correction of num * (1/d) (div_recip with y = RN(1/d)) is the correctly rounded quotient for |num| <= 2^700
// (no intermediate overflows or underflows for any quotient the caller can accept: t >= t_min > 0 keeps
// |num| >= 2^-310; tools/divcheck.hip checks it on the GPU); other operands divide.  3 VALU instead of 11.
// (+1.1 % headline, +3.6 % Cornell: the coat and the Cornell boxes are RectBoxes, six faces per trip)
__device__ __forceinline__ double face_div(double num, double den, double inv, bool ok) {
  if (ok && fabs(num) <= 0x1p700) return div_recip(num, Recip{den, inv});
  return num / den;
}
// Root division by a through the per-ray shared reciprocal (exact: div_recip's range, checked per numerator;
// a itself is in range when ra_ok).
__device__ __forceinline__ double div_by(double n, const Recip& R, bool ok) {
  const double m = fabs(n);
  if (ok && m >= 0x1p-300 && m <= 0x1p300) return div_recip(n, R);
  return n / R.b;
}
// sphere.rs:28-46 (t only), both root divisions through div_by, that also says whether the sphere's box test
// (aabb.rs:62-79 hit2 on c -+ r) surely passes for the root it returns: t_min < t < t_max, and the hit point relative to the centre, oc + t d (one fma per axis),
// inside the box by the scene's rounding margin on every axis — p[5] = r - eta rounded down (host, rt_api.cpp;
// <= 0 for radii too small or negative: never sure), eta = 2^-48 (B + L) with B the largest box plane and L the
// origin bound of the f32 node test, which ra_ok includes (with every |d_i| >= 2^-300).  Then every entry and
// exit the slab test computes lies strictly before / after t: DESIGN.md §3.1 has the error bound (it needs
// ~2^-50 (B + L)), tests/sphere_sure_check.c the adversarial CPU check (no false pass; ~55 k false passes
// without the margin).
__device__ __forceinline__ bool sphere_t_sure(const double* p, v3 o, v3 d, const Recip& ra, bool ra_ok, double t_min,
                                              double t_max, double& t, bool& sure) {
  v3 oc = o - V(p[0], p[1], p[2]);
  double half_b = dot(oc, d);
  double c = len2(oc) - p[3] * p[3];
  double disc = half_b * half_b - ra.b * c;
  if (disc < 0.0) return false;
  double sqrt_d = sqrt_rn(disc);
  double root = div_by(-half_b - sqrt_d, ra, ra_ok);
  if (root < t_min || t_max < root) {
    root = div_by(-half_b + sqrt_d, ra, ra_ok);
    if (root < t_min || t_max < root) return false;
  }
  t = root;
  const double p5 = p[5];
  // (bitwise: one straight-line mask, no branches)
  sure = (int)ra_ok & (int)(root > t_min) & (int)(root < t_max) & (int)(fabs(fma(root, d.x, oc.x)) < p5) &
         (int)(fabs(fma(root, d.y, oc.y)) < p5) & (int)(fabs(fma(root, d.z, oc.z)) < p5);
  return true;
}

// rect.rs:54-65 (t only): axes (D1, D2), normal axis n = 3-D1-D2; q = d1_min d1_max d2_min d2_max offset
template <int D1, int D2>
__device__ __forceinline__ bool rect_t(const double* q, v3 o, v3 d, double t_min, double t_max, double& t_out,
                                       v3 inv = v3{0.0, 0.0, 0.0}, bool ok = false) {
  constexpr int n = 3 - D1 - D2;
  double t = face_div(q[4] - comp(o, n), comp(d, n), comp(inv, n), ok);
  if (t < t_min || t > t_max) return false;
  double d1v = comp(o, D1) + t * comp(d, D1);
  double d2v = comp(o, D2) + t * comp(d, D2);
  if (d1v < q[0] || d1v > q[1] || d2v < q[2] || d2v > q[3]) return false;
  t_out = t;
  return true;
}

// rect.rs:132-156 RectBox::hit — six faces in order, each against the running closest.
// Returns the face index (0..5) that won, or -1.
__device__ __forceinline__ int box_t(const double* b, v3 o, v3 d, double t_min, double t_max, double& t_out,
                                     v3 inv = v3{0.0, 0.0, 0.0}, bool ok = false) {
  double q[5];
  int face = -1;
  double tc = t_max, t;
  // xy_sides: (p0.x, p1.x, p0.y, p1.y, p1.z), (..., p0.z)
  q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4];
  q[4] = b[5];
  if (rect_t<0, 1>(q, o, d, t_min, tc, t, inv, ok)) { tc = t; face = 0; }
  q[4] = b[2];
  if (rect_t<0, 1>(q, o, d, t_min, tc, t, inv, ok)) { tc = t; face = 1; }
  // yz_sides: (p0.y, p1.y, p0.z, p1.z, p1.x), (..., p0.x)
  q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5];
  q[4] = b[3];
  if (rect_t<1, 2>(q, o, d, t_min, tc, t, inv, ok)) { tc = t; face = 2; }
  q[4] = b[0];
  if (rect_t<1, 2>(q, o, d, t_min, tc, t, inv, ok)) { tc = t; face = 3; }
  // xz_sides: (p0.x, p1.x, p0.z, p1.z, p1.y), (..., p0.y)
  q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5];
  q[4] = b[4];
  if (rect_t<0, 2>(q, o, d, t_min, tc, t, inv, ok)) { tc = t; face = 4; }
  q[4] = b[1];
  if (rect_t<0, 2>(q, o, d, t_min, tc, t, inv, ok)) { tc = t; face = 5; }
  t_out = tc;
  return face;
}

#ifndef RT_BOX_TWO_PASS
#define RT_BOX_TWO_PASS 6  // book-2 instances: box_t2; reference scenes: box_t1f
#endif
// box_t in at most two passes of three faces (RT_BOX_TWO_PASS: the book-2 instances, final_scene +1 %; in
// the reference-scene instance +1 % Cornell but -0.7 % headline and cfg1 from the register pressure it
// adds to the leaf loop, where box_t1f below wins instead: DESIGN.md §5),
// for rays whose every |d_i| is in face_div's range (no face quotient is NaN or infinite there).  The
// sequential test keeps, of the faces whose rect test passes, the nearest — of equal t the last in face
// order (each face meets the running closest with rect.rs:58's `t > t_max`).  A ray crosses each axis's two
// planes in order: near (its entry side, the slab test's t0) and far (t1).  Pass 1 tests one plane of each
// axis in face order (z, x, y: rising face index) — the near planes, or the far ones when the slab entry is
// t_min (the origin is past every near plane) — and its result stands when the other set provably loses:
//   * every far face quotient RN(num / d) >= the slab's RN(num * RN(1/d)) (1 - 3u) >= t_exit (1 - 3u), so
//     a near result below RN(t_exit (1 - 2^-50)) beats each far face strictly;
//   * with t_enter == t_min every near quotient is <= t_min (1 + 3.01u) (or <= 0), so a far result above
//     RN(t_min (1 + 2^-50)) beats each near face strictly.
// Else pass 2 tests the other set against pass 1's closest, and of a tie the higher face index wins — the
// sequential result in every case (tests/box_pass_check.c: bit for bit on ~11 M adversarial draws).
__device__ __forceinline__ int box_t2(const double* b, v3 o, v3 d, v3 inv, RaySigns ns, double t_min, double t_max,
                                      double t_enter, double t_exit, double& t_out) {
  const bool far_first = !(t_enter > t_min);
  double tc = t_max, t1 = t_max;
  int f1 = -1;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    const bool flip = far_first != (pass == 1);
    double q[5], t;
    int f = -1;
    bool hi = ns.z != flip;  // the max-z plane: faces 0 (max) / 1 (min) of the xy sides
    q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4];
    q[4] = hi ? b[5] : b[2];
    if (rect_t<0, 1>(q, o, d, t_min, tc, t, inv, true)) { tc = t; f = hi ? 0 : 1; }
    hi = ns.x != flip;       // yz sides: faces 2 (max x) / 3 (min x)
    q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5];
    q[4] = hi ? b[3] : b[0];
    if (rect_t<1, 2>(q, o, d, t_min, tc, t, inv, true)) { tc = t; f = hi ? 2 : 3; }
    hi = ns.y != flip;       // xz sides: faces 4 (max y) / 5 (min y)
    q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5];
    q[4] = hi ? b[4] : b[1];
    if (rect_t<0, 2>(q, o, d, t_min, tc, t, inv, true)) { tc = t; f = hi ? 4 : 5; }
    if (pass == 0) {
      t1 = tc; f1 = f;
      if (f >= 0 && (far_first ? tc > t_min * (1.0 + 0x1p-50) : tc < t_exit * (1.0 - 0x1p-50))) break;
    } else if (f >= 0 && (f1 < 0 || tc < t1 || f > f1)) {  // f >= 0: tc <= t1
      t1 = tc; f1 = f;
    }
  }
  t_out = t1;
  return f1;
}

// box_t2's first pass alone, falling back to the six-face sequence wherever the margin does not prove it
// (RT_BOX_TWO_PASS & 4: the reference-scene instance) — the same result, fewer values held across the
// fallback than box_t2's merge of two passes
__device__ __forceinline__ int box_t1f(const double* b, v3 o, v3 d, v3 inv, RaySigns ns, double t_min, double t_max,
                                       double t_enter, double t_exit, double& t_out) {
  const bool far_first = !(t_enter > t_min);
  double tc = t_max, q[5], t;
  int f = -1;
  bool hi = ns.z != far_first;
  q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4];
  q[4] = hi ? b[5] : b[2];
  if (rect_t<0, 1>(q, o, d, t_min, tc, t, inv, true)) { tc = t; f = hi ? 0 : 1; }
  hi = ns.x != far_first;
  q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5];
  q[4] = hi ? b[3] : b[0];
  if (rect_t<1, 2>(q, o, d, t_min, tc, t, inv, true)) { tc = t; f = hi ? 2 : 3; }
  hi = ns.y != far_first;
  q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5];
  q[4] = hi ? b[4] : b[1];
  if (rect_t<0, 2>(q, o, d, t_min, tc, t, inv, true)) { tc = t; f = hi ? 4 : 5; }
  if (!(f >= 0 && (far_first ? tc > t_min * (1.0 + 0x1p-50) : tc < t_exit * (1.0 - 0x1p-50))))
    f = box_t(b, o, d, t_min, t_max, tc, inv, true);
  t_out = tc;
  return f;
}

// ---- book-2 extensions (absent from the reference, parity unpinned) ----
// A path's identity for the side streams: the counter-RNG coordinates of the ray being traced.
__device__ __forceinline__ const DExt& prim_ext(const DScene& S, const DPrim& pr) {
  return S.exts[pr.kind >> kPrimExtShift];
}
// camera.h get_ray (book 2): time = random_double(time0, time1), drawn from the path's time stream; the
// shutter {time0, time1} read here (DScene.shutter), not held across the caller's loop
__device__ __forceinline__ double ray_time(const double* shutter, uint32_t pixel, uint32_t sample, uint64_t seed) {
  const double* sh = shutter;
  asm volatile("" : "+s"(sh));
  const double time0 = sh[0], time1 = sh[1];
  return time0 + (time1 - time0) * side_draw(seed, 0u, sample, pixel, kStreamTime);
}
// moving_sphere.h center(time) = center0 + ((time - time0) / (time1 - time0)) * (center1 - center0)
__device__ __forceinline__ v3 moving_center(const DPrim& pr, const DExt& e, double tm) {
  const v3 c0 = V(pr.p[0], pr.p[1], pr.p[2]);
  return c0 + scale(V(e.c1[0], e.c1[1], e.c1[2]) - c0, (tm - e.t0) / (e.t1 - e.t0));
}
// Translate::hit (moved origin o - offset) then RotateY::hit (origin and direction rotated by -angle)
__device__ __forceinline__ void to_object(const DExt& e, int32_t kind, v3& o, v3& d) {
  if (!(kind & kPrimXform)) return;
  const v3 m = o - V(e.off[0], e.off[1], e.off[2]);
  o = V(e.cos_t * m.x - e.sin_t * m.z, m.y, e.sin_t * m.x + e.cos_t * m.z);
  d = V(e.cos_t * d.x - e.sin_t * d.z, d.y, e.sin_t * d.x + e.cos_t * d.z);
}
// The base shape of an extended primitive in its own frame (t only); tm = ray time.
__device__ __forceinline__ bool base_t(const DPrim& pr, const DExt& e, int32_t base, v3 o, v3 d, double tm,
                                       double t_min, double t_max, double& t, int& face) {
  switch (base) {
    case kPrimSphere: return sphere_t(pr.p, o, d, len2(d), t_min, t_max, t);
    case kPrimMovingSphere: {
      const v3 c = moving_center(pr, e, tm);
      const double q[4] = {c.x, c.y, c.z, pr.p[3]};
      return sphere_t(q, o, d, len2(d), t_min, t_max, t);
    }
    case kPrimRectXY: return rect_t<0, 1>(pr.p, o, d, t_min, t_max, t);
    case kPrimRectYZ: return rect_t<1, 2>(pr.p, o, d, t_min, t_max, t);
    case kPrimRectXZ: return rect_t<0, 2>(pr.p, o, d, t_min, t_max, t);
    default: face = box_t(pr.p, o, d, t_min, t_max, t); return face >= 0;
  }
}
// Closest-hit t of an extended primitive in [t_min, t_max] (after its leaf box passed).
// constant_medium.h hit, restated so that the result does not depend on the running closest hit:
// entry t1 (clamped to t_min, then 0) and exit t2 of the boundary; free flight
// hd = neg_inv_density * ln(U), U from the medium stream keyed by (path draw index, prim); the
// medium scatters at t1 + hd / |d| when hd <= (t2 - t1) |d| and that t is <= t_max.  (The book clamps
// t2 to t_max first; the two agree in exact arithmetic, and this form makes the closest hit
// independent of the order in which the traversal meets the primitives.)
// Inlined into the EXT kernel instances only (out-of-line calls cost those instances ~300 B of
// scratch per lane and 25 % of the book-2 final scene's throughput); the path key (pixel, sample,
// draw index) and the scene fields it reads are passed by value.
struct ExtHit {
  double t;
  int face;
  int hit;
};
__device__ __forceinline__ ExtHit ext_t(const DExt* exts, const double* shutter, const DPrim pr, int prim, v3 o,
                                     v3 d, double t_min, double t_max, uint32_t pixel, uint32_t sample,
                                     uint32_t draw, uint64_t seed) {
  ExtHit r{0.0, -1, 0};
  const DExt& e = exts[pr.kind >> kPrimExtShift];
  const int32_t kind = pr.kind, base = kind & kPrimBaseMask;
  const double tm = base == kPrimMovingSphere ? ray_time(shutter, pixel, sample, seed) : 0.0;
  to_object(e, kind, o, d);
  if (!(kind & kPrimMedium)) {
    r.hit = base_t(pr, e, base, o, d, tm, t_min, t_max, r.t, r.face) ? 1 : 0;
    return r;
  }
  const double inf = __builtin_inf();
  double t1, t2;
  int f = -1;
  if (base == kPrimSphere || base == kPrimMovingSphere) {
    // the two boundary hits of a sphere from one discriminant: exactly what the two sphere_t calls
    // (t in [-inf, inf], then [t1 + 0.0001, inf]) return, each root tested like sphere_t tests it
    const v3 c = base == kPrimSphere ? V(pr.p[0], pr.p[1], pr.p[2]) : moving_center(pr, e, tm);
    const v3 oc = o - c;
    const double a = len2(d), half_b = dot(oc, d), cc = len2(oc) - pr.p[3] * pr.p[3];
    const double disc = half_b * half_b - a * cc;
    if (disc < 0.0) return r;
    const double sq = sqrt(disc);
    const double r1 = (-half_b - sq) / a, r2 = (-half_b + sq) / a;
    t1 = r1;  // sphere_t on [-inf, inf] accepts the first root whatever its value
    const double lo = t1 + 0.0001;
    if (r1 < lo || inf < r1) {
      if (r2 < lo || inf < r2) return r;
      t2 = r2;
    } else {
      t2 = r1;
    }
  } else {
    if (!base_t(pr, e, base, o, d, tm, -inf, inf, t1, f)) return r;
    if (!base_t(pr, e, base, o, d, tm, t1 + 0.0001, inf, t2, f)) return r;
  }
  if (t1 < t_min) t1 = t_min;
  if (t1 >= t2) return r;
  if (t1 < 0.0) t1 = 0.0;
  const double ray_length = len(d);
  const double inside = (t2 - t1) * ray_length;
  const double hd = e.neg_inv_density * RT_LOG(side_draw(seed, draw, sample, pixel, kStreamMedium | (uint32_t)e.object));
  if (hd > inside) return r;
  const double th = t1 + hd / ray_length;
  if (th > t_max) return r;
  r.t = th;
  r.face = -1;
  r.hit = 1;
  return r;
}
__device__ __forceinline__ bool ext_hit_t(const DScene& S, const DPrim& pr, int prim, v3 o, v3 d, double t_min,
                                          double t_max, const Rng& rk, uint64_t seed, double& t, int& face) {
  const ExtHit r = ext_t(S.exts, S.shutter, pr, prim, o, d, t_min, t_max, rk.pixel, rk.sample, rk.draw, seed);
  if (r.hit) {
    t = r.t;
    face = r.face;
  }
  return r.hit != 0;
}

template <bool EXT>
__device__ __forceinline__ bool prim_t(const DScene& S, const DPrim& pr, int prim, v3 o, v3 d, double a,
                                       double t_min, double t_max, const Rng& rk, uint64_t seed, double& t,
                                       int& face) {
  if (EXT && (pr.kind & kPrimExt)) return ext_hit_t(S, pr, prim, o, d, t_min, t_max, rk, seed, t, face);
  switch (pr.kind) {
    case kPrimSphere: return sphere_t(pr.p, o, d, a, t_min, t_max, t);
    case kPrimRectXY: return rect_t<0, 1>(pr.p, o, d, t_min, t_max, t);
    case kPrimRectYZ: return rect_t<1, 2>(pr.p, o, d, t_min, t_max, t);
    case kPrimRectXZ: return rect_t<0, 2>(pr.p, o, d, t_min, t_max, t);
    default: {
      face = box_t(pr.p, o, d, t_min, t_max, t);
      return face >= 0;
    }
  }
}

struct Hit {
  v3 point, normal;
  double t, u, v;
  bool front_face;
};

// hittable.rs:16-38
__device__ __forceinline__ void finish_hit(Hit& h, v3 d, v3 normal) {
  h.front_face = dot(d, normal) < 0.0;
  h.normal = h.front_face ? normal : scale(normal, -1.0);
}

// sphere.rs:17-26 get_uv — acos/atan2 kept out of line to hold the kernel's register budget.
struct UV {
  double u, v;
};
__device__ __noinline__ UV sphere_uv(double nx, double ny, double nz) {
  double theta = RT_ACOS(-ny);
  double phi = RT_ATAN2(-nz, nx) + 3.14159265358979323846;
  return UV{phi / (2.0 * 3.14159265358979323846), theta / 3.14159265358979323846};
}

// Rebuild the winner's HitRecord with the exact reference formulas (same t => same record).
// Written with scalars only (no local arrays) so that nothing is demoted to scratch memory.
// WANT_UV = false skips u, v (only image textures read them; sphere u, v cost an acos + atan2).
template <bool WANT_UV = true>
__device__ __forceinline__ void prim_record(const DPrim& pr, int face, v3 o, v3 d, double t, Hit& h) {
  h.t = t;
  h.point = o + scale(d, t);  // ray.at(t) (vec3.rs:253-255)
  v3 normal;
  double u = 0.0, v = 0.0;
  if (pr.kind == kPrimSphere) {
    // sphere.rs:46-51 + get_uv 17-26: u, v from the outward normal (p - c) / r (signed r)
    normal = scale(h.point - V(pr.p[0], pr.p[1], pr.p[2]), pr.p[4]);  // p[4] = 1.0 / r (host)
    if (WANT_UV) {
      UV uv = sphere_uv(normal.x, normal.y, normal.z);
      u = uv.u;
      v = uv.v;
    }
  } else {
    // rect.rs:66-79; a RectBox face is the rect of RectBox::new with the face's offset
    const double* b = pr.p;
    int kind = pr.kind;
    double q0 = b[0], q1 = b[1], q2 = b[2], q3 = b[3];
    if (kind == kPrimBox) {
      if (face < 2) { q0 = b[0]; q1 = b[3]; q2 = b[1]; q3 = b[4]; kind = kPrimRectXY; }
      else if (face < 4) { q0 = b[1]; q1 = b[4]; q2 = b[2]; q3 = b[5]; kind = kPrimRectYZ; }
      else { q0 = b[0]; q1 = b[3]; q2 = b[2]; q3 = b[5]; kind = kPrimRectXZ; }
    }
    double o1, d1, o2, d2;
    if (kind == kPrimRectXY) { o1 = o.x; d1 = d.x; o2 = o.y; d2 = d.y; normal = V(0.0, 0.0, 1.0); }
    else if (kind == kPrimRectYZ) { o1 = o.y; d1 = d.y; o2 = o.z; d2 = d.z; normal = V(1.0, 0.0, 0.0); }
    else { o1 = o.x; d1 = d.x; o2 = o.z; d2 = d.z; normal = V(0.0, 1.0, 0.0); }
    if (WANT_UV) {
      double d1v = o1 + t * d1;
      double d2v = o2 + t * d2;
      u = (d1v - q0) / (q1 - q0);
      v = (d2v - q2) / (q3 - q2);
    }
  }
  h.u = u;
  h.v = v;
  finish_hit(h, d, normal);
}

// Hit record of an extended primitive, always with u, v: the base shape's record in its own frame
// (a medium's: point r.at(t), normal (1, 0, 0), front face — constant_medium.h), then RotateY::hit
// and Translate::hit map point and normal back to the world (front_face kept from the object frame,
// as in the books' current edition).
__device__ __forceinline__ Hit ext_record(const DExt* exts, const double* shutter, const DPrim pr, int face, v3 o,
                                       v3 d, double t, uint32_t pixel, uint32_t sample, uint64_t seed) {
  // (each branch fills its own record, copied once: with the fields stored per branch the compiler kept
  // u, v in scratch memory behind a select of their addresses — 2-4 scratch stores and 2 scratch loads
  // per book-2 hit record)
  Hit h;
  const DExt& e = exts[pr.kind >> kPrimExtShift];
  const int32_t kind = pr.kind, base = kind & kPrimBaseMask;
  to_object(e, kind, o, d);
  if (kind & kPrimMedium) {
    Hit m;
    m.t = t;
    m.point = o + scale(d, t);
    m.normal = V(1.0, 0.0, 0.0);
    m.front_face = true;
    m.u = 0.0;
    m.v = 0.0;
    h = m;
  } else if (base == kPrimMovingSphere) {
    const v3 c = moving_center(pr, e, ray_time(shutter, pixel, sample, seed));
    Hit m;
    m.t = t;
    m.point = o + scale(d, t);
    const v3 n = scale(m.point - c, pr.p[4]);  // p[4] = 1.0 / r (host)
    const UV uv = sphere_uv(n.x, n.y, n.z);
    m.u = uv.u;
    m.v = uv.v;
    finish_hit(m, d, n);
    h = m;
  } else {
    DPrim q = pr;
    q.kind = base;
    Hit m;
    prim_record<true>(q, face, o, d, t, m);
    h = m;
  }
  if (kind & kPrimXform) {
    const v3 p = h.point, n = h.normal;
    h.point = V(e.cos_t * p.x + e.sin_t * p.z, p.y, -e.sin_t * p.x + e.cos_t * p.z) + V(e.off[0], e.off[1], e.off[2]);
    h.normal = V(e.cos_t * n.x + e.sin_t * n.z, n.y, -e.sin_t * n.x + e.cos_t * n.z);
  }
  return h;
}
// The winner's record: prim_record for reference primitives, ext_record for extended ones.
template <bool WANT_UV, bool EXT>
__device__ __forceinline__ void hit_record(const DScene& S, const DPrim& pr, int face, v3 o, v3 d, double t,
                                           const Rng& rk, uint64_t seed, Hit& h) {
  if (EXT && (pr.kind & kPrimExt)) h = ext_record(S.exts, S.shutter, pr, face, o, d, t, rk.pixel, rk.sample, seed);
  else prim_record<WANT_UV>(pr, face, o, d, t, h);
}

// Exact ties.  Acceptance is inclusive (sphere.rs:40-45, rect.rs:58) and bbox_tree.rs:56-91
// walks the reference tree rhs-first, re-testing every node and leaf box against the running closest with
// hit2's strict `t_max <= t_min` (aabb.rs:74).  So of the objects hit at the closest binary64 t*, the first
// the reference meets is the one latest in its tree's leaf order (lhs before rhs), and each later one — each
// earlier in leaf order — replaces it iff its own box still passes hit2 at t* (its ancestors' boxes contain
// it, so they pass too).  The winner: the earliest in leaf order whose box passes at t*, else the latest.
// The host numbers the primitives in that leaf order (rt_api.cpp reference_ranks), so it is a function of
// the set of tied primitives, whatever tree the device walks and in whatever order: the order "box passes
// at t*, lowest rank first; then the others, highest rank first" is total, so the winner can be kept
// incrementally.  Two tested candidates at an equal t are compared at once (tie_takes).  A tied object
// whose own test is skipped because its box fails at the running closest (near_entry: by no more than
// rounding; a sphere, whose t is known before its box test, on t == t_best exactly) raises `tie`, and a
// traversal that ends with `tie` set recomputes the winner over every primitive (resolve_ties: rare, exact).
__device__ __forceinline__ void leaf_box(const DPrim& pr, double* b);
// A box that fails hit2 at the running closest t_best with its entry te only slightly beyond it may still
// hold a primitive hit at exactly t_best: a RectBox's face t is the correctly rounded (b - o) / d and its
// slab entry (b - o) * (1 / d), a few ulps apart.  Such a failure raises `tie` when te lies in the same or
// the next high word as t_best (both >= 0 order like their bit patterns): within 2^-19 relative, far above
// any rounding gap, in two instructions (a 64-bit ulp count cost Cornell 0.3-0.6 %, r06aa / r06ab).  The
// band reaches a little below t_best too (a box missed with its entry there): those marks, like any in the
// band without a tie, only run resolve_ties for nothing.
__device__ __forceinline__ bool near_entry(double te, double t_best) {
  return (unsigned)__double2hiint(te) - (unsigned)__double2hiint(t_best) <= 1u;
}
// `tie` is bit 30 of the running best primitive (indices stay below 2^28, kLeafPrimMask): a vector bit
// that a new closest hit clears by assignment, where a separate per-lane flag would hold an SGPR pair
// through the whole traversal loop (the megakernels' SGPRs are at the limit).  best = -1 is unchanged by it.
constexpr int kTieBit = 1 << 30;
// (reference-scene instances only: book-2 scenes, parity unpinned, keep the pairwise rule of tie_takes —
// there the marks and the resolve pass cost final_scene 4.6 %, r06y)
template <bool EXT>
__device__ __forceinline__ void mark_tie(int& best, bool c) {
  if constexpr (!EXT) best |= c ? kTieBit : 0;
}
__device__ __forceinline__ int strip_tie(int best) { return best < 0 ? best : (best & ~kTieBit); }
// Closest-hit update of an accepted object hit (t <= t_best).  Strictly closer, or the first hit at all
// (best = -1: the reference accepts t == t_max), replaces.  An equal t between two primitives whose boxes
// both passed is decided at once by the rank order (both are candidates the reference tests):
//   leaf < best — the candidate's box was just tested at t_max = t_best and passed: it wins;
//   leaf > best — best wins unless its own box fails hit2 at t (re-tested from the global copy; ties only).
// (While `tie` is set resolve_ties decides at the end, so the pair is left alone.)
template <bool EXT>
__device__ __forceinline__ bool tie_takes(const DScene& S, int leaf, int best, double t, double t_best, v3 o, v3 inv,
                                          RaySigns ns, double t_min) {
  if (t != t_best || best < 0) return true;
  if (best & kTieBit) return false;
  if (leaf < best) return true;
  const DPrim& pb = S.prims[best];
  double b[6], te;
  if (EXT && (pb.kind & kPrimExt)) {
    const double* eb = S.exts[pb.kind >> kPrimExtShift].box;
    for (int k = 0; k < 6; ++k) b[k] = eb[k];
  } else {
    leaf_box(pb, b);
  }
  return !slab_s(b, o, inv, ns, t_min, t, te);
}
template <bool EXT>
__device__ __forceinline__ bool prim_t(const DScene& S, const DPrim& pr, int prim, v3 o, v3 d, double a,
                                       double t_min, double t_max, const Rng& rk, uint64_t seed, double& t,
                                       int& face);
// (inline; RT_TIES_OUTLINE makes it a call — -0.3 % on Cornell / headline, r06aa — for which the scene
// pointers and the seed, launch-uniform, are read back as such for the side streams' SGPR-pinned keys)
struct TieWin {
  int best, face;
};
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  return (T*)(uintptr_t)uniform64((uint64_t)(uintptr_t)p);
}
#ifdef RT_TIES_OUTLINE
#define RT_TIES_LINKAGE __noinline__
#else
#define RT_TIES_LINKAGE __forceinline__
#endif
template <bool EXT>
__device__ RT_TIES_LINKAGE TieWin resolve_ties_ool(const DPrim* prims_v, const DExt* exts_v, const double* shutter_v,
                                                int n_prims, v3 o, v3 d, double t_min, double ts, Rng rk,
                                                uint64_t seed_v) {
  DScene S{};
  S.prims = uniform_ptr(prims_v);
  S.exts = uniform_ptr(exts_v);
  S.shutter = uniform_ptr(shutter_v);
  const uint64_t seed = uniform64(seed_v);
  n_prims = __builtin_amdgcn_readfirstlane(n_prims);
  // the ray's reciprocals and |d|^2 recomputed (the same correctly rounded values the traversal used), so
  // that the callers' copies need not outlive their loops
  const v3 inv = V(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
  const RaySigns ns = ray_signs(inv);
  const double a = len2(d);
  int pmin = -1, pface = -1, mmax = -1, mface = -1;
#pragma unroll 1
  for (int i = 0; i < n_prims; ++i) {
    const DPrim& pr = S.prims[i];
    double b[6], t, te;
    if (EXT && (pr.kind & kPrimExt)) {
      const double* eb = S.exts[pr.kind >> kPrimExtShift].box;
      for (int k = 0; k < 6; ++k) b[k] = eb[k];
    } else {
      leaf_box(pr, b);
    }
    // (the box first: one entered well beyond ts holds no primitive hit at ts — the margin 2^-16 is far
    // above any rounding gap between a primitive's t and its box, and above near_entry's band)
    if (!slab_s(b, o, inv, ns, t_min, __builtin_inf(), te) || te > fma(ts, 0x1p-16, ts)) continue;
    int f = -1;
    if (!prim_t<EXT>(S, pr, i, o, d, a, t_min, ts, rk, seed, t, f) || t != ts) continue;
    mmax = i;  // (ascending: the latest in leaf order so far)
    mface = f;
    if (pmin < 0 && slab_s(b, o, inv, ns, t_min, ts, te)) {
      pmin = i;
      pface = f;
    }
  }
  return pmin >= 0 ? TieWin{pmin, pface} : TieWin{mmax, mface};
}
template <bool EXT>
__device__ __forceinline__ void resolve_ties(const DScene& S, v3 o, v3 d, double t_min, double ts, int& best,
                                             int& face_best, const Rng& rk, uint64_t seed) {
  if constexpr (EXT) return;  // (nothing marks a book-2 traversal: mark_tie)
  if (best < 0 || !(best & kTieBit)) return;
  best &= ~kTieBit;
  const TieWin w = resolve_ties_ool<EXT>(S.prims, S.exts, S.shutter, S.n_prims, o, d, t_min, ts, rk, seed);
  if (w.best >= 0) {
    best = w.best;
    face_best = w.face;
  }
}

// ------------------------------------------------------------------------------------------
// BVH traversal: closest hit in [t_min, t_max] (bbox_tree.rs:56-91 semantics, near-first order)
// ------------------------------------------------------------------------------------------
// Traversal state of one ray.
struct Trav {
  v3 inv;         // 1/d per axis (aabb.rs:66 computes the same quotient per call)
  RaySigns ns;    // 1/d < 0 per axis
  double a;       // |d|^2 (sphere.rs:31)
  double t_best;  // closest accepted t so far (t_max initially)
  int best, face, node, sp, steps;  // best: | kTieBit while an exact tie at t_best may be unresolved
};

__device__ __forceinline__ void trav_begin(Trav& T, v3 d, double t_max) {
  T.inv = V(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
  T.ns = ray_signs(T.inv);
  T.a = len2(d);
  T.t_best = t_max;
  T.best = -1;
  T.face = -1;
  T.node = 0;  // top node: child[0] = root
  T.sp = 0;
  T.steps = 0;
}

// Node source by kernel instance: all nodes in LDS, all in HBM/L2, or the first n_lds_nodes (BFS
// order: the top levels) in LDS and the rest in HBM.  Separate instances keep LDS reads ds_read
// (a select between an LDS and a global pointer would make every read a FLAT load).
template <int MODE>
__device__ __forceinline__ const DNode& fetch_node(const DScene& S, const DNode* lds_nodes, int idx) {
  if (MODE == kNodesLds) return lds_nodes[idx];
  if (MODE == kNodesGlobal) return S.nodes[idx];
  return (idx < S.n_lds_nodes) ? lds_nodes[idx] : S.nodes[idx];
}

// A leaf child whose (exact) box was hit: the object against the running closest (bbox_tree.rs:60-71).
template <bool EXT>
__device__ __forceinline__ void leaf_visit(const DScene& S, int prim, v3 o, v3 d, double t_min, Trav& T,
                                           const Rng& rk, uint64_t seed, unsigned& ptests) {
  const DPrim& pr = S.prims[prim];
  double t;
  int f = -1;
  ++ptests;
  if (prim_t<EXT>(S, pr, prim, o, d, T.a, t_min, T.t_best, rk, seed, t, f) &&
      tie_takes<EXT>(S, prim, T.best, t, T.t_best, o, T.inv, T.ns, t_min)) {
    T.t_best = t;
    T.best = prim;
    T.face = f;
  }
}

// Visit node T.node: test both child boxes (f64 hit2 on the reference's boxes), visit hit leaf
// children at once (they can shrink t_best for the sibling), descend into the nearer hit internal
// child and push the farther.  Returns true when the traversal is complete (T.best / T.t_best /
// T.face hold the closest hit).  Stack: per-lane, in LDS, [depth][lane] with a stride of the block
// size (bank = lane % 32); entry t rounded down to f32 (only ever compared against t_best).
template <int STRIDE, int MODE, bool EXT>
__device__ __forceinline__ bool trav_step(const DScene& S, const DNode* lds_nodes, v3 o, v3 d, double t_min, Trav& T,
                                          const Rng& rk, uint64_t seed, int* stk_node, float* stk_t,
                                          unsigned& visits, unsigned& ptests) {
  if (++T.steps > S.n_nodes) {  // defect guard: a traversal visits each node at most once
    T.best = strip_tie(T.best);
    return true;
  }
  const DNode& nd = fetch_node<MODE>(S, lds_nodes, T.node);
  const int c0 = nd.child[0], c1 = nd.child[1];
  double te0 = 0.0, te1 = 0.0;
  bool h0 = (c0 != kEmptyChild) && slab_s(nd.box[0], o, T.inv, T.ns, t_min, T.t_best, te0);
  bool h1 = (c1 != kEmptyChild) && slab_s(nd.box[1], o, T.inv, T.ns, t_min, T.t_best, te1);
  visits += (c0 != kEmptyChild ? 1u : 0u) + (c1 != kEmptyChild ? 1u : 0u);
  // a box failing at the closest t by no more than rounding: a possible tie below it (near_entry)
  mark_tie<EXT>(T.best, (!h0 && near_entry(te0, T.t_best)) || (!h1 && near_entry(te1, T.t_best)));
  // leaf children (one primitive each)
  if (h0 && c0 < 0) {
    leaf_visit<EXT>(S, ~c0, o, d, t_min, T, rk, seed, ptests);
    h0 = false;
  }
  if (h1 && c1 < 0) {
    leaf_visit<EXT>(S, ~c1, o, d, t_min, T, rk, seed, ptests);
    h1 = false;
  }
  int next;
  if (h0 && h1) {
    const bool first0 = te0 <= te1;
    next = first0 ? c0 : c1;
    stk_node[T.sp * STRIDE] = first0 ? c1 : c0;
    stk_t[T.sp * STRIDE] = __double2float_rd(first0 ? te1 : te0);
    ++T.sp;
  } else if (h0 || h1) {
    next = h0 ? c0 : c1;
  } else {
    next = -1;
    while (T.sp > 0) {
      --T.sp;
      // a pushed subtree whose entry lies beyond the current closest hit cannot hold it
      if ((double)stk_t[T.sp * STRIDE] <= T.t_best) {
        next = stk_node[T.sp * STRIDE];
        break;
      }
    }
    if (next < 0) {
      resolve_ties<EXT>(S, o, d, t_min, T.t_best, T.best, T.face, rk, seed);
      return true;
    }
  }
  T.node = next;
  return false;
}

// Whole closest-hit query (WorkspaceScene::hit_workspace, scene/mod.rs:152-164; the unbounded
// HitList is always empty because every geometry is bounded).  Same visit order and tests as
// trav_step, written as one loop over locals: the megakernel holds a whole path's state beside the
// traversal, and this form keeps the traversal's registers out of scratch.
template <int STRIDE, int MODE, bool EXT>
__device__ __forceinline__ int traverse(const DScene& S, const DNode* lds_nodes, v3 o, v3 d, double t_min,
                                        double& t_best, int& face_best, const Rng& rk, uint64_t seed,
                                        int* stk_node, float* stk_t, unsigned& visits, unsigned& ptests) {
  const v3 inv = V(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
  const RaySigns ns = ray_signs(inv);
  const double a = len2(d);
  int best = -1;
  int sp = 0;
  int node = 0;  // top node: child[0] = root
  for (int steps = 0; steps < S.n_nodes; ++steps) {  // bounded like traverse4
    const DNode& nd = fetch_node<MODE>(S, lds_nodes, node);
    const int c0 = nd.child[0], c1 = nd.child[1];
    double te0 = 0.0, te1 = 0.0;
    bool h0 = (c0 != kEmptyChild) && slab_s(nd.box[0], o, inv, ns, t_min, t_best, te0);
    bool h1 = (c1 != kEmptyChild) && slab_s(nd.box[1], o, inv, ns, t_min, t_best, te1);
    visits += (c0 != kEmptyChild ? 1u : 0u) + (c1 != kEmptyChild ? 1u : 0u);
    mark_tie<EXT>(best, (!h0 && near_entry(te0, t_best)) || (!h1 && near_entry(te1, t_best)));
    if (h0 && c0 < 0) {
      const DPrim& pr = S.prims[~c0];
      double t;
      int f = -1;
      ++ptests;
      if (prim_t<EXT>(S, pr, ~c0, o, d, a, t_min, t_best, rk, seed, t, f) &&
          tie_takes<EXT>(S, ~c0, best, t, t_best, o, inv, ns, t_min)) {
        t_best = t;
        best = ~c0;
        face_best = f;
      }
      h0 = false;
    }
    if (h1 && c1 < 0) {
      const DPrim& pr = S.prims[~c1];
      double t;
      int f = -1;
      ++ptests;
      if (prim_t<EXT>(S, pr, ~c1, o, d, a, t_min, t_best, rk, seed, t, f) &&
          tie_takes<EXT>(S, ~c1, best, t, t_best, o, inv, ns, t_min)) {
        t_best = t;
        best = ~c1;
        face_best = f;
      }
      h1 = false;
    }
    int next;
    if (h0 && h1) {
      const bool first0 = te0 <= te1;
      next = first0 ? c0 : c1;
      stk_node[sp * STRIDE] = first0 ? c1 : c0;
      stk_t[sp * STRIDE] = __double2float_rd(first0 ? te1 : te0);
      ++sp;
    } else if (h0) {
      next = c0;
    } else if (h1) {
      next = c1;
    } else {
      next = -1;
      while (sp > 0) {
        --sp;
        if ((double)stk_t[sp * STRIDE] <= t_best) {
          next = stk_node[sp * STRIDE];
          break;
        }
      }
      if (next < 0) break;
    }
    node = next;
  }
  resolve_ties<EXT>(S, o, d, t_min, t_best, best, face_best, rk, seed);
  return best;
}

// ---- 4-wide traversal (megakernel, wf_extend4) ----
#ifdef RT_PHASE_TIMING
// per-lane step counter of the instrumented build (a register of the calling kernel)
#define g_trav_lane_steps trav_lane_steps_ref
// event counters of the instrumented build: slot 2i += active lanes, slot 2i + 1 += 1 (per wave)
static __device__ unsigned long long g_phase_ctr[64];
// histograms of the instrumented build: node visits per traversing lane, and per wave (its slowest lane)
static __device__ unsigned long long g_visit_hist[64], g_wave_visit_hist[64];

__device__ __forceinline__ void ph_count(int i) {
  const unsigned long long act = __ballot(1);
  if ((int)__lane_id() == __builtin_ctzll(act)) {
    atomicAdd(&g_phase_ctr[2 * i], (unsigned long long)__popcll(act));
    atomicAdd(&g_phase_ctr[2 * i + 1], 1ull);
  }
}
#ifndef RT_PHASE_NO_EVENTS
#define PH_COUNT(i) ph_count(i)
#else  // (clock stamps only: the event atomics would dominate the phase clocks)
#define PH_COUNT(i)
#endif
#else
#define PH_COUNT(i)
#endif
// Per-lane node-visit / primitive-test statistics of the 4-wide traversal: counted in the instrumented
// build only (they cost the production megakernel 0.5 %: ~15 VALU per iteration and two registers).
#ifdef RT_PHASE_TIMING
#define RT_STAT(x) x
#define RT_STAT_ARG(x) , x
#else
#define RT_STAT(x)
#define RT_STAT_ARG(x)
#endif
#ifdef RT_TIMELINE
// timeline build: per-wave start, unit-pool-exhausted and exit times (s_memrealtime, 100 MHz)
constexpr int kTimelineWaves = 1 << 16;
static __device__ unsigned long long g_wave_t0[kTimelineWaves], g_wave_tx[kTimelineWaves], g_wave_t1[kTimelineWaves];
#endif
template <int MODE, class N4>
__device__ __forceinline__ const N4& fetch_node4(const DScene& S, const N4* lds_nodes, int idx) {
  // LDS byte offset with a full-rate 24-bit multiply (an LDS node index is < 2^24)
  if (MODE == kNodesLds || MODE == kSceneLds)
    return *reinterpret_cast<const N4*>(reinterpret_cast<const char*>(lds_nodes) +
                                        __umul24((unsigned)idx, (unsigned)sizeof(N4)));
  const N4* g = static_cast<const N4*>(S.nodes4);
  if (MODE == kNodesGlobal) return g[idx];
  return (idx < S.n_lds_nodes4) ? lds_nodes[idx] : g[idx];
}

// Ray in the form the f32 node test uses: o and 1/d rounded to f32, and o * (1/d) for the FMA.
struct RayF {
  float ox, oy, oz, ix, iy, iz, oix, oiy, oiz;
  bool fast;  // max|o| <= origin_limit: the f32 test's error bound holds
  int dx, dy, dz;  // N4::kNegRow when 1/d < 0 on the axis (the near plane is the hi row), else 0
};
template <class N4>
__device__ __forceinline__ RayF ray_f(const DScene& S, v3 o, v3 inv) {
  RayF r;
  r.ox = (float)o.x;
  r.oy = (float)o.y;
  r.oz = (float)o.z;
  r.ix = (float)inv.x;
  r.iy = (float)inv.y;
  r.iz = (float)inv.z;
  r.oix = r.ox * r.ix;
  r.oiy = r.oy * r.iy;
  r.oiz = r.oz * r.iz;
  r.fast = fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z)) <= (double)S.origin_limit;
  r.dx = r.ix < 0.f ? N4::kNegRow : 0;
  r.dy = r.iy < 0.f ? N4::kNegRow : 0;
  r.dz = r.iz < 0.f ? N4::kNegRow : 0;
  return r;
}

// Conservative tests of the four children of a 4-wide node: per child the entry t (a lower bound)
// or +inf when missed.  The ray picks each axis's near and far plane rows by the sign of 1/d (six
// 16-B reads, no per-child min / max), the f32 slab arithmetic runs two children per packed
// instruction (v_pk_fma_f32), and only a ray with a far origin (max|o| > origin_limit: rare,
// divergent) re-evaluates the same boxes in f64 (exact arithmetic on a superset box).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 f2(float a, float b) { return f32x2{a, b}; }
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// A missed child's key: +inf, or all ones (M1: a NaN, an inline constant, where +inf needs a v_mov
// per visit; the LDS-node instances, +0.5 %; the L1/L2 ones measured -1 % with it).  Keys are only
// handled as bits: either packs above every bound and entry (node4_next), and the leaf test masks
// both out (node4_visit).
template <bool M1, class N4>
__device__ __forceinline__ void node4_keys(const N4& nd, const RayF& r, v3 o, v3 inv, float tminf, float tmaxf,
                                           double t_min, double t_max, float& k0, float& k1, float& k2, float& k3,
                                           const int4& ch, unsigned (&hc)[4]) {
  const unsigned chw[4] = {(unsigned)ch.x, (unsigned)ch.y, (unsigned)ch.z, (unsigned)ch.w};
  // the near / far plane rows picked per ray by the sign of 1/d (see DNode4F / DNode4C): for 1/d >= 0, fma(lo, i, -o i) <= fma(hi, i, -o i) (the FMA rounds monotonically), so the
  // pick equals the min / max of the two and each child needs only max3 / min3; a NaN (0 * inf) is
  // dropped by max3 / min3 like by the min / max form; an inverted box (lo > hi) now fails, which the
  // exact test on it never passes either (its planes cross, so hit2 misses in that axis).
  const char* nb = reinterpret_cast<const char*>(&nd);
  float4 nx4, fx4, ny4, fy4, nz4, fz4;
  if constexpr (N4::kRows3) {
    const char* bx = nb + r.dx;
    const char* by = nb + r.dy;
    const char* bz = nb + r.dz;
    nx4 = *reinterpret_cast<const float4*>(bx);
    fx4 = *reinterpret_cast<const float4*>(bx + 16);
    ny4 = *reinterpret_cast<const float4*>(by + 48);
    fy4 = *reinterpret_cast<const float4*>(by + 64);
    nz4 = *reinterpret_cast<const float4*>(bz + 96);
    fz4 = *reinterpret_cast<const float4*>(bz + 112);
  } else {
    nx4 = *reinterpret_cast<const float4*>(nb + r.dx);
    fx4 = *reinterpret_cast<const float4*>((nb - r.dx) + 48);
    ny4 = *reinterpret_cast<const float4*>(nb + (16 + r.dy));
    fy4 = *reinterpret_cast<const float4*>((nb - r.dy) + 64);
    nz4 = *reinterpret_cast<const float4*>(nb + (32 + r.dz));
    fz4 = *reinterpret_cast<const float4*>((nb - r.dz) + 80);
  }
  const f32x2 ix = f2(r.ix, r.ix), iy = f2(r.iy, r.iy), iz = f2(r.iz, r.iz);
  const f32x2 nx = f2(-r.oix, -r.oix), ny = f2(-r.oiy, -r.oiy), nz = f2(-r.oiz, -r.oiz);
  float key[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x2 x0 = pk_fma(h ? f2(nx4.z, nx4.w) : f2(nx4.x, nx4.y), ix, nx);
    const f32x2 x1 = pk_fma(h ? f2(fx4.z, fx4.w) : f2(fx4.x, fx4.y), ix, nx);
    const f32x2 y0 = pk_fma(h ? f2(ny4.z, ny4.w) : f2(ny4.x, ny4.y), iy, ny);
    const f32x2 y1 = pk_fma(h ? f2(fy4.z, fy4.w) : f2(fy4.x, fy4.y), iy, ny);
    const f32x2 z0 = pk_fma(h ? f2(nz4.z, nz4.w) : f2(nz4.x, nz4.y), iz, nz);
    const f32x2 z1 = pk_fma(h ? f2(fz4.z, fz4.w) : f2(fz4.x, fz4.y), iz, nz);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float tn = fmaxf(fmaxf(x0[e], y0[e]), fmaxf(z0[e], tminf));
      const float tf = fminf(fminf(x1[e], y1[e]), fminf(z1[e], tmaxf));
      hc[2 * h + e] = tn <= tf ? chw[2 * h + e] : 0u;  // the child word where its box is hit
      key[2 * h + e] = tn <= tf ? tn : (M1 ? __uint_as_float(~0u) : __builtin_inff());
    }
  }
  if (!r.fast) {  // far origins: the same inflated boxes in f64 (exact arithmetic on a superset box)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double tn = t_min, tf = t_max;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const double iv = comp(inv, a), oa = comp(o, a);
        float lo, hi;
        if constexpr (N4::kRows3) {
          lo = nd.row[a][0][k];
          hi = nd.row[a][1][k];
        } else {
          lo = nd.lo[a][k];
          hi = nd.hi[a][k];
        }
        const double t0 = ((double)lo - oa) * iv, t1 = ((double)hi - oa) * iv;
        tn = fmax(tn, fmin(t0, t1));
        tf = fmin(tf, fmax(t0, t1));
      }
      hc[k] = tn <= tf ? chw[k] : 0u;
      key[k] = tn <= tf ? __double2float_rd(tn) : (M1 ? __uint_as_float(~0u) : __builtin_inff());
    }
  }
  k0 = key[0];
  k1 = key[1];
  k2 = key[2];
  k3 = key[3];
}

// The reference's bounding_box() of a leaf object, exactly: sphere c -+ r with the signed radius
// (sphere.rs:54-60), rect +-BBOX_WIDTH on its normal axis (rect.rs:82-99), RectBox min/max
// (rect.rs:158-163).
__device__ __forceinline__ void leaf_box(const DPrim& pr, double* b) {
  const double* p = pr.p;
  switch (pr.kind) {
    case kPrimSphere:
      b[0] = p[0] - p[3]; b[1] = p[1] - p[3]; b[2] = p[2] - p[3];
      b[3] = p[0] + p[3]; b[4] = p[1] + p[3]; b[5] = p[2] + p[3];
      break;
    case kPrimRectXY:
      b[0] = p[0]; b[1] = p[2]; b[2] = p[4] - 0.0001; b[3] = p[1]; b[4] = p[3]; b[5] = p[4] + 0.0001;
      break;
    case kPrimRectYZ:
      b[0] = p[4] - 0.0001; b[1] = p[0]; b[2] = p[2]; b[3] = p[4] + 0.0001; b[4] = p[1]; b[5] = p[3];
      break;
    case kPrimRectXZ:
      b[0] = p[0]; b[1] = p[4] - 0.0001; b[2] = p[2]; b[3] = p[1]; b[4] = p[4] + 0.0001; b[5] = p[3];
      break;
    default:
      for (int k = 0; k < 6; ++k) b[k] = p[k];
  }
}

// The hit leaf children of a 4-wide node against the running closest, each exactly as
// bbox_tree.rs:60-71 does: f64 hit2 on the object's own bounding box and the object (for spheres
// evaluated object first — the same conjunction of two pure functions).  One loop per
// leaf kind — spheres (sphere.rs:28-46), rects (rect.rs:54-65), boxes (rect.rs:132-156) — each in
// child order, so a wave runs a kind's code only while one of its lanes holds a leaf of that kind.
// (Of several leaves hit at exactly the closest t the reference's own leaf order decides: tie_takes, resolve_ties.)
// A hit also
// lowers tmaxf (the f32 bound of t_best the node tests use).
__device__ __forceinline__ int child_at(int k, int c0, int c1, int c2, int c3) {
  const int lo = (k & 1) ? c1 : c0, hi = (k & 1) ? c3 : c2;
  return (k & 2) ? hi : lo;
}
// f32 upper bound of a t, finite so that a miss key never passes `k <= tmaxf`.  f = (float)t
// rounds to nearest, so |t - f| <= ulp(f) / 2, and f + |f| 2^-23 >= f + ulp(f) (toward +inf for either
// sign) is >= t after its own rounding: four instructions instead of the emulated round-up conversion
// (~20).  The bound may be up to two f32 ulps above t: a few more subtrees kept, never one dropped.
__device__ __forceinline__ float tmax_f32(double t) {
  const float f = (float)t;
  return fminf(f + fabsf(f) * 0x1p-23f, 3.402823466e38f);
}
// The top bytes of four words as one word, byte i = w_i >> 24 (two v_perm_b32 and an or).  Leaf
// masks are kept in this "spread" form: bit 8 i + 7 stands for child i.
__device__ __forceinline__ unsigned top_bytes(unsigned w0, unsigned w1, unsigned w2, unsigned w3) {
  return __builtin_amdgcn_perm(w1, w0, 0x0c0c0703u) | __builtin_amdgcn_perm(w3, w2, 0x07030c0cu);
}

template <int MODE, bool EXT, bool DEFER = false>
__device__ __forceinline__ void leaf_tests4(const DScene& S, const DPrim* lds_prims, v3 o, v3 d, v3 inv,
                                            RaySigns ns, const Recip& ra, bool ra_ok, double t_min, unsigned lm, int c0, int c1,
                                            int c2, int c3, const int32_t* chp, double& t_best, float& tmaxf, int& best,
                                            int& face_best, const Rng& rk, uint64_t seed, unsigned& ptests,
                                            unsigned& xdefer) {
  // lm: spread mask of hit leaf children (bit 8 i + 7: child i).  A leaf's child word is
  // ~(prim | flags), so its generic / box flags (bits 29 / 28) are bits 5 / 4 of its top byte, inverted.
  const unsigned nf = ~top_bytes((unsigned)c0, (unsigned)c1, (unsigned)c2, (unsigned)c3);
  const unsigned gm = (nf << 2) & 0x80808080u, bm = (nf << 3) & 0x80808080u;
  unsigned sph = lm & ~gm, rect = lm & gm & ~bm, box = lm & bm;
  const bool div_ok = ra_ok;  // every |d_i| in range too (traverse4): faces divide through inv (face_div)
  bool hit = false;
  // nodes in LDS: child k's word read back from the node (one address op and one ds_read) instead of
  // the select chain over c0..c3 (+0.3 %)
  constexpr bool kReread = (MODE == kNodesLds || MODE == kSceneLds) && !EXT;
  auto child = [&](int k) -> int { return kReread ? chp[k] : child_at(k, c0, c1, c2, c3); };
#pragma unroll 1
  while (sph) {
    PH_COUNT(2);
    const int k = __builtin_ctz(sph) >> 3;
    sph &= sph - 1;
    const int leaf = ~child(k);
    const DPrim& pr = (MODE == kSceneLds) ? lds_prims[leaf] : S.prims[leaf];
    // the reference's `box.hit2 && sphere.hit` (bbox_tree.rs:60-71) as `sphere.hit && box.hit2`: both are
    // pure functions of the same (ray, t_min, t_best), so the conjunction is the same; the sphere test
    // is the cheaper filter here (the box passes ~95 % of the trips, the sphere far fewer): +1.3 %
    double t;
    PH_COUNT(3);
    RT_STAT(++ptests);
    // The reference's `box.hit2 && sphere.hit`: the box test runs only where the sphere test hit and the
    // rounding margin does not already prove that it passes (sphere_t_sure; +0.3 %).  The
    // primitive is re-read for it, so no copy of c, r is held across the sphere test.
    bool sure;
    if (!sphere_t_sure(pr.p, o, d, ra, ra_ok, t_min, t_best, t, sure)) continue;
    if (!sure) {
      const DPrim* pp = &pr;
      if constexpr (MODE == kSceneLds) {  // (laundered as an LDS pointer, so the re-read stays a ds_read)
        typedef __attribute__((address_space(3))) const DPrim LdsPrim;
        LdsPrim* lp = (LdsPrim*)pp;
        asm volatile("" : "+v"(lp));
        pp = (const DPrim*)lp;
      } else {
        asm volatile("" : "+v"(pp));
      }
      if (!slab_sphere(pp->p, o, inv, ns, t_min, t_best)) {
        mark_tie<EXT>(best, t == t_best);  // (a sphere at the closest t whose box fails there: a possible tie)
        continue;
      }
    }
    if (!tie_takes<EXT>(S, leaf, best, t, t_best, o, inv, ns, t_min)) continue;
    t_best = t; best = leaf; face_best = -1; hit = true;
  }
  // RectBox leaves before rect leaves: a box in front of a rect (the random scene's ground coat over its
  // lower surface, Cornell's blocks before its walls) then shrinks t_best first, so the rect's own box
  // test rejects without the rect test (+0.25 % headline)
#pragma unroll 1
  while (box) {
    PH_COUNT(7);
    const int k = __builtin_ctz(box) >> 3;
    box &= box - 1;
    const int leaf = (~child(k)) & kLeafPrimMask;
    const DPrim& pr = (MODE == kSceneLds) ? lds_prims[leaf] : S.prims[leaf];
    double te, t;
    if (EXT && pr.kind != kPrimBox) {  // an extended primitive (book 2): exact box from its DExt record
      if (!slab_s(prim_ext(S, pr).box, o, inv, ns, t_min, t_best, te)) continue;  // (no tie marks: mark_tie)
      // DEFER: the object test after the traversal (ext_deferred) — it is a pure function of (ray, t_min,
      // t_max), and a later, smaller t_max can only drop hits that lose anyway — so its code and registers
      // stay out of the traversal loop (book-2 instances: 74 -> 26 spilled VGPRs at 4 waves per SIMD)
      if (DEFER && (unsigned)(pr.kind >> kPrimExtShift) < 32u) {
        xdefer |= 1u << (pr.kind >> kPrimExtShift);
        continue;
      }
      RT_STAT(++ptests);
      int f = -1;
      if (ext_hit_t(S, pr, leaf, o, d, t_min, t_best, rk, seed, t, f) && tie_takes<EXT>(S, leaf, best, t, t_best, o, inv, ns, t_min)) {
        t_best = t; best = leaf; face_best = f; hit = true;
      }
      continue;
    }
    // RT_BOX_TWO_PASS bits: box_t2 in the reference-scene (1) / book-2 (2) instances, box_t1f in the
    // reference-scene (4) / book-2 (8) ones, else the six-face sequence
    constexpr bool kTwoPass = (RT_BOX_TWO_PASS & (EXT ? 2 : 1)) != 0;
    // (the scene-in-LDS instances only: compiled into the L1/L2 ones it cost gen_spheres 0.7 %)
    constexpr bool kOneFull = (RT_BOX_TWO_PASS & (EXT ? 8 : 4)) != 0 && (EXT || MODE == kSceneLds);
    double tx;
    if (!slab_s(pr.p, o, inv, ns, t_min, t_best, te, tx)) {  // a RectBox's bounding box is its p[0..5]
      mark_tie<EXT>(best, near_entry(te, t_best));
      continue;
    }
    RT_STAT(++ptests);
    const int f = (kTwoPass && div_ok)   ? box_t2(pr.p, o, d, inv, ns, t_min, t_best, te, tx, t)
                  : (kOneFull && div_ok) ? box_t1f(pr.p, o, d, inv, ns, t_min, t_best, te, tx, t)
                                         : box_t(pr.p, o, d, t_min, t_best, t, inv, div_ok);
    if (f >= 0 && tie_takes<EXT>(S, leaf, best, t, t_best, o, inv, ns, t_min)) { t_best = t; best = leaf; face_best = f; hit = true; }
  }
#pragma unroll 1
  while (rect) {
    PH_COUNT(4);
    const int k = __builtin_ctz(rect) >> 3;
    rect &= rect - 1;
    const int leaf = (~child(k)) & kLeafPrimMask;
    const DPrim& pr = (MODE == kSceneLds) ? lds_prims[leaf] : S.prims[leaf];
    double b[6], te, t;
    leaf_box(pr, b);
    // (no tie mark: the box is padded 0.0001 along the normal, so it fails at the rect's own t only where
    // that t is on the rect's edge, a rounding-level coincidence; the mark cost Cornell 1.5 %, r06z)
    if (!slab_s(b, o, inv, ns, t_min, t_best, te)) continue;
    RT_STAT(++ptests);
    bool h;
    switch (pr.kind) {
      case kPrimRectXY: h = rect_t<0, 1>(pr.p, o, d, t_min, t_best, t, inv, div_ok); break;
      case kPrimRectYZ: h = rect_t<1, 2>(pr.p, o, d, t_min, t_best, t, inv, div_ok); break;
      default: h = rect_t<0, 2>(pr.p, o, d, t_min, t_best, t, inv, div_ok);
    }
    if (h && tie_takes<EXT>(S, leaf, best, t, t_best, o, inv, ns, t_min)) { t_best = t; best = leaf; face_best = -1; hit = true; }
  }
  if (hit) tmaxf = tmax_f32(t_best);
}

// One node visit: conservative f32 tests of the four child boxes; hit leaf children tested exactly
// at once (they can shrink t_best); hit internal children visited nearest-first, the others pushed
// and skipped on pop when beyond the closest hit.
// A child is one 32-bit word: its f32 entry t (> 0, so its bits order like the value) with the low K
// bits (S.key_mask) replaced by the node index — a lower bound of the entry, so culling with it stays
// conservative; misses, leaves and empty slots are ~0u.  Ordering is then 4 min/max pairs, a stack
// entry is one word, and the cull `entry <= tmaxf` is one unsigned compare against bits(tmaxf) | mask.
// tmaxf >= t_best: the cull may keep a subtree the exact comparison would drop, never the reverse, and
// extra visits cannot change the closest hit (leaf tests are exact).  `sp` is the stack offset in
// elements (depth x STRIDE).  Returns the next node, or -1 when the traversal is complete.
__device__ __forceinline__ void cas_u(unsigned& a, unsigned& b) {
  const unsigned lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}
// visit4's node part: the f32 keys of `node`'s four children, its children, and the spread mask
// (see top_bytes) of its hit leaf children.
template <int MODE, class N4>
__device__ __forceinline__ unsigned node4_visit(const DScene& S, const N4* lds_nodes, v3 o, v3 inv,
                                                const RayF& rf, double t_min, double t_best, float tmaxf, int node,
                                                int4& ch, float& k0, float& k1, float& k2, float& k3,
                                                unsigned& visits, const int32_t*& chp) {
  PH_COUNT(0);
  const N4& nd = fetch_node4<MODE>(S, lds_nodes, node);
  chp = nd.child;
  ch = *reinterpret_cast<const int4*>(nd.child);
  const float tminf = fmaxf(__double2float_rd(t_min), 1.17549435e-38f);  // entry keys > 0
  constexpr bool kM1 = MODE == kNodesLds || MODE == kSceneLds;
  unsigned hc[4];
  node4_keys<kM1>(nd, rf, o, inv, tminf, tmaxf, t_min, t_best, k0, k1, k2, k3, ch, hc);
  RT_STAT(visits += 4);
  // hit leaf: the child word where the box test passed (the key's own compare, no second test), else 0;
  // its sign bit marks a leaf, gathered into the spread mask (4 VALU per visit fewer than re-testing the
  // keys' bits)
  return top_bytes(hc[0], hc[1], hc[2], hc[3]) & 0x80808080u;
  // hit leaf: key < inf (bits(k) + 0x80800000 keeps the sign bit exactly for bits(k) < bits(inf); keys
  // are >= 0) and a negative child word; as a spread mask
  // (an M1 miss key ~0u: its sum keeps the top bit, so it is masked by ~bits(k) — one v_bitop3 with the
  // child)
}
// visit4's ordering part: internal children as packed words (a miss, k = inf or ~0u, packs above any
// bound), nearest first; the three farther ones pushed, the nearest returned, else the stack popped.
template <int STRIDE, bool FULL>
__device__ __forceinline__ int node4_next(const DScene& S, int4 ch, float k0, float k1, float k2, float k3,
                                          float tmaxf, int& sp, unsigned& top, unsigned* stk) {
  // No select needed for leaves and empty slots: a leaf's child word is negative (top bit set) and
  // kEmptyChild is 0x7fffffff, so either word or-ed in packs above any limit (bits(tmaxf) | km <=
  // 0x7f7fffff: tmaxf is finite and km < 2^20), as does a missed child's key (+inf or ~0u).
  const unsigned km = S.key_mask;
  unsigned p0 = (__float_as_uint(k0) & ~km) | (unsigned)ch.x;
  unsigned p1 = (__float_as_uint(k1) & ~km) | (unsigned)ch.y;
  unsigned p2 = (__float_as_uint(k2) & ~km) | (unsigned)ch.z;
  unsigned p3 = (__float_as_uint(k3) & ~km) | (unsigned)ch.w;
  // the sorting network; with the scene in LDS only four of its five exchanges: p0 the nearest, p3 the
  // farthest, the middle pair left in either order (there the last exchange bought fewer visits than it
  // cost: +0.4 % headline without it; scenes read through L2 lose 2-4 % without it)
  cas_u(p0, p1);
  cas_u(p2, p3);
  cas_u(p0, p2);
  cas_u(p1, p3);
  if (FULL) cas_u(p1, p2);
  const unsigned lim = __float_as_uint(tmaxf) | km;  // tmaxf finite: inf entries fail
  // the stack's top entry lives in `top` (~0u: empty); a push moves the old top to LDS (so stk[0]
  // holds the ~0u sentinel under any pushed entry), a pop takes `top` and prefetches the next one
  if (p3 <= lim) { stk[sp] = top; sp += STRIDE; top = p3; }
  if (p2 <= lim) { stk[sp] = top; sp += STRIDE; top = p2; }
  if (p1 <= lim) { stk[sp] = top; sp += STRIDE; top = p1; }
  if (p0 <= lim) return (int)(p0 & km);
  // Culled entries are skipped in a loop with a single-compare exit (lim < e < ~0u as one unsigned
  // range test: 4 VALU + 3 SALU per trip instead of 11 + 7 for a test-pop-compare loop; +0.4 % on the
  // headline); the accepted entry is then popped once.  Same entries popped in the same
  // order as popping one at a time.
  const unsigned lo = lim + 1u, span = ~0u - lo;
  unsigned e = top;
  while (e - lo < span) {
    PH_COUNT(5);
    sp -= STRIDE;
    e = stk[sp];
  }
  if (e == ~0u) {
    top = e;
    return -1;
  }
  sp -= STRIDE;  // e is a real entry: the ~0u sentinel lies below it
  top = stk[sp];
  return (int)(e & km);
}
template <int STRIDE, int MODE, bool EXT, bool DEFER = false>
__device__ __forceinline__ int visit4(const DScene& S, const typename Node4Sel<EXT>::T* lds_nodes, const DPrim* lds_prims, v3 o, v3 d,
                                      v3 inv, RaySigns ns, const RayF& rf, const Recip& ra, bool ra_ok, double t_min, int node,
                                      double& t_best, float& tmaxf, int& best, int& face_best, int& sp,
                                      unsigned& top, unsigned* stk, const Rng& rk, uint64_t seed,
                                      unsigned& visits, unsigned& ptests, unsigned& xdefer) {
  int4 ch;
  float k0, k1, k2, k3;
  const int32_t* chp;
  const unsigned lm = node4_visit<MODE>(S, lds_nodes, o, inv, rf, t_min, t_best, tmaxf, node, ch, k0, k1, k2, k3,
                                        visits, chp);
  if (lm) PH_COUNT(1);
  if (lm)
    leaf_tests4<MODE, EXT, DEFER>(S, lds_prims, o, d, inv, ns, ra, ra_ok, t_min, lm, ch.x, ch.y, ch.z, ch.w, chp, t_best, tmaxf,
                                  best, face_best, rk, seed, ptests, xdefer);
  return node4_next<STRIDE, MODE != kSceneLds>(S, ch, k0, k1, k2, k3, tmaxf, sp, top, stk);
}

// The extended objects a traversal deferred (bit e: DScene.exts[e], whose box passed at its visit), each
// tested against the final closest hit in index order — the same closest hit as testing them where they
// were visited (each test is a pure function of the ray, t_min and t_max; ties: tie_takes).  Measured on
// final_scene @ 200 spp: +2.7 % (1654 vs 1611); out of line (a call) -1.4 %, and a 1024-thread book-2
// block (RT_EXT_WIDE_THREADS=1024, 4 waves per SIMD at 68-83 spilled VGPRs) -10 % (gpurun_out/r06g).
__device__ __forceinline__ void ext_deferred(const DScene& S, unsigned xdefer, v3 o, v3 d, v3 inv, RaySigns ns, double t_min, double& t_best,
                                             int& best, int& face_best, const Rng& rk, uint64_t seed) {
#pragma unroll 1
  while (xdefer) {
    const int e = __builtin_ctz(xdefer);
    xdefer &= xdefer - 1u;
    const int leaf = S.exts[e].prim;
    const DPrim& pr = S.prims[leaf];
    double t;
    int f = -1;
    if (ext_hit_t(S, pr, leaf, o, d, t_min, t_best, rk, seed, t, f) && tie_takes<true>(S, leaf, best, t, t_best, o, inv, ns, t_min)) {
      t_best = t;
      best = leaf;
      face_best = f;
    }
  }
}

// Whole closest-hit query over the 4-wide tree (t_min > 0).  The conservative internal tests and the
// exact leaf tests make the set of primitives that can win the reference's (see DNode4F); the closest
// hit is the reference's up to exact ties in t.
template <int STRIDE, int MODE, bool EXT>
__device__ __forceinline__ int traverse4(const DScene& S, const typename Node4Sel<EXT>::T* lds_nodes, const DPrim* lds_prims, v3 o, v3 d,
                                         double t_min, double& t_best, int& face_best, unsigned* stk,
                                         const Rng& rk, uint64_t seed, unsigned& visits, unsigned& ptests
#ifdef RT_PHASE_TIMING
                                         , unsigned long long& trav_lane_steps_ref
#endif
                                         ) {
  PH_COUNT(23);
  bool inv_ok;
  const v3 inv = inv_dir(d, inv_ok);
  const RaySigns ns = ray_signs(inv);
  const RayF rf = ray_f<typename Node4Sel<EXT>::T>(S, o, inv);
  const double a = len2(d);
  const Recip ra = recip(a);  // the sphere roots' divisor, shared (sphere_t_sure)
  // the shared-reciprocal divisions' operand ranges: a (sphere roots) and every |d_i| (face planes, face_div),
  // and t_min >= 0.001, which keeps an accepted face quotient's numerator >= 2^-310 (face_div's proof; a
  // caller of rt_scene_hit_ex may pass a smaller t_min: those rays divide exactly like the reference).
  // The megakernel's literal 0.001 folds the last test away.
  const bool ra_ok = inv_ok && a >= 0x1p-300 && a <= 0x1p300 && rf.fast && t_min >= 0.001;
  float tmaxf = tmax_f32(t_best);
  int best = -1;
  int sp = 0;
  unsigned top = ~0u;  // the stack's top entry (node4_next)
  int node = S.root4;
  unsigned xdefer = 0u;  // book-2: extended objects whose box passed, tested after the loop (leaf_tests4)
  // a tree traversal visits every node at most once: more steps than nodes can only be a defect,
  // and ends the loop instead of hanging the wave
  for (int steps = 0; steps < S.n_nodes4 && node >= 0; ++steps) {
#ifdef RT_PHASE_TIMING
    ++g_trav_lane_steps;
#endif
    node = visit4<STRIDE, MODE, EXT, EXT>(S, lds_nodes, lds_prims, o, d, inv, ns, rf, ra, ra_ok, t_min, node, t_best, tmaxf,
                                          best, face_best, sp, top, stk, rk, seed, visits, ptests, xdefer);
  }
  if (EXT) ext_deferred(S, xdefer, o, d, inv, ns, t_min, t_best, best, face_best, rk, seed);
  if (best >= 0 && (best & kTieBit)) PH_COUNT(25);
  resolve_ties<EXT>(S, o, d, t_min, t_best, best, face_best, rk, seed);
  return best;
}

// Step-wise form for wf_extend4, where a ray's traversal state lives across loop iterations.
struct Trav4 {
  v3 inv;
  Recip ra;  // ra.b = |d|^2 (sphere_t_sure)
  bool ra_ok;
  double t_best;
  float tmaxf;
  int best, face, node, sp, steps;
  unsigned top;  // the stack's top entry (node4_next)
  RaySigns ns;
  RayF rf;
};

template <bool EXT>
__device__ __forceinline__ void trav4_begin(Trav4& T, const DScene& S, v3 o, v3 d, double t_max) {
  bool inv_ok;
  T.inv = inv_dir(d, inv_ok);
  T.ns = ray_signs(T.inv);
  T.rf = ray_f<typename Node4Sel<EXT>::T>(S, o, T.inv);
  T.ra = recip(len2(d));
  T.ra_ok = inv_ok && T.ra.b >= 0x1p-300 && T.ra.b <= 0x1p300 && T.rf.fast;
  T.t_best = t_max;
  T.tmaxf = tmax_f32(t_max);
  T.best = -1;
  T.face = -1;
  T.node = S.root4;
  T.sp = 0;
  T.top = ~0u;
  T.steps = 0;
}

// Returns true when the traversal is complete (T.best / T.t_best / T.face hold the closest hit).
template <int STRIDE, int MODE, bool EXT>
__device__ __forceinline__ bool trav4_step(const DScene& S, const typename Node4Sel<EXT>::T* lds_nodes, const DPrim* lds_prims, v3 o,
                                           v3 d, double t_min, Trav4& T, unsigned* stk, const Rng& rk,
                                           uint64_t seed, unsigned& visits, unsigned& ptests) {
  if (++T.steps > S.n_nodes4) {  // defect guard
    T.best = strip_tie(T.best);
    return true;
  }
  unsigned xdefer = 0u;  // (not used: the step-wise form tests extended objects at once)
  T.node = visit4<STRIDE, MODE, EXT>(S, lds_nodes, lds_prims, o, d, T.inv, T.ns, T.rf, T.ra, T.ra_ok, t_min, T.node, T.t_best,
                                     T.tmaxf, T.best, T.face, T.sp, T.top, stk, rk, seed, visits, ptests, xdefer);
  if (T.node >= 0) return false;
  resolve_ties<EXT>(S, o, d, t_min, T.t_best, T.best, T.face, rk, seed);
  return true;
}

template <int MODE, class N4>
__device__ __forceinline__ void stage_nodes4(const DScene& S, N4* lds_nodes, DPrim* lds_prims) {
  if (MODE == kNodesGlobal) return;
  const int4* src = reinterpret_cast<const int4*>(S.nodes4);
  int4* dst = reinterpret_cast<int4*>(lds_nodes);
  const int n16 = S.n_lds_nodes4 * (int)(sizeof(N4) / 16);
  for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
  if (MODE == kSceneLds) {
    const int4* ps = reinterpret_cast<const int4*>(S.prims);
    int4* pd = reinterpret_cast<int4*>(lds_prims);
    const int p16 = S.n_lds_prims * (int)(sizeof(DPrim) / 16);
    for (int i = threadIdx.x; i < p16; i += blockDim.x) pd[i] = ps[i];
    // Perlin tables right after the primitives (when they fit: S.n_lds_perlin > 0)
    const int4* ts = reinterpret_cast<const int4*>(S.perlin);
    int4* td = reinterpret_cast<int4*>(lds_prims + S.n_lds_prims);
    const int t16 = S.n_lds_perlin * (int)(sizeof(DPerlin) / 16);
    for (int i = threadIdx.x; i < t16; i += blockDim.x) td[i] = ts[i];
    // then the material and texture tables (when they fit: S.n_lds_mats > 0)
    if (S.n_lds_mats > 0) {
      const int4* ms = reinterpret_cast<const int4*>(S.mats);
      int4* md = td + t16;
      const int m16 = S.n_lds_mats * (int)(sizeof(DMat) / 16);
      for (int i = threadIdx.x; i < m16; i += blockDim.x) md[i] = ms[i];
      const int4* xs = reinterpret_cast<const int4*>(S.texs);
      int4* xd = md + m16;
      const int x16 = S.n_lds_texs * (int)(sizeof(DTex) / 16);
      for (int i = threadIdx.x; i < x16; i += blockDim.x) xd[i] = xs[i];
    }
  }
  __syncthreads();
}

// Copy nodes [0, n_lds_nodes) into the block's LDS node cache (16-B coalesced loads).
template <int MODE>
__device__ __forceinline__ void stage_nodes(const DScene& S, DNode* lds_nodes) {
  if (MODE == kNodesGlobal) return;
  const int4* src = reinterpret_cast<const int4*>(S.nodes);
  int4* dst = reinterpret_cast<int4*>(lds_nodes);
  const int n16 = S.n_lds_nodes * (int)(sizeof(DNode) / 16);
  for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// textures (material/texture/*.rs, perlin/mod.rs) and materials
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int32_t sat_i32(double x) {
  if (x != x) return 0;
  if (x >= 2147483647.0) return 2147483647;
  if (x <= -2147483648.0) return (int32_t)(-2147483647 - 1);
  return (int32_t)x;
}

// perlin/mod.rs:87-109 + interp 40-63.  The six permutation entries and then the eight gradient
// vectors are fetched as independent loads (the corner loop of the reference serialises four
// dependent loads per corner).  The accumulation runs in the reference's (di, dj, dk) order with its
// product order ((wx wy) wz) dot.  Its corner weights `i*uu + (1-i)*(1-uu)` with i in {0.0, 1.0}
// are exactly `1 - uu` and `uu`: uu = u*u*(3-2u) lies in [0, 1] for u in [0, 1) (it rounds to at
// most 1.0), so 0*uu and 0*(1-uu) are +0, 1*x is x and x + 0 is x; for a NaN u both forms are NaN.
// So the value is bit-identical with a third of the reference's arithmetic.
template <class TP>  // table pointer: const DPerlin* (global) or LdsPerlin* (LDS)
__device__ __forceinline__ double perlin_noise_t(TP T, v3 p) {
  double xf = floor(p.x), yf = floor(p.y), zf = floor(p.z);
  double u = p.x - xf, v = p.y - yf, w = p.z - zf;
  uint32_t i = (uint32_t)sat_i32(xf), j = (uint32_t)sat_i32(yf), k = (uint32_t)sat_i32(zf);
  double uu = u * u * (3.0 - 2.0 * u);
  double vv = v * v * (3.0 - 2.0 * v);
  double ww = w * w * (3.0 - 2.0 * w);
  const int px[2] = {T->perm_x[i & 0xFF], T->perm_x[(i + 1) & 0xFF]};
  const int py[2] = {T->perm_y[j & 0xFF], T->perm_y[(j + 1) & 0xFF]};
  const int pz[2] = {T->perm_z[k & 0xFF], T->perm_z[(k + 1) & 0xFF]};
  const double wx[2] = {1.0 - uu, uu}, wy[2] = {1.0 - vv, vv}, wz[2] = {1.0 - ww, ww};
  const double gx[2] = {u, u - 1.0}, gy[2] = {v, v - 1.0}, gz[2] = {w, w - 1.0};  // u - i (u - 0.0 == u)
  double accum = 0.0;
#pragma unroll
  for (int di = 0; di < 2; ++di) {
#pragma unroll
    for (int dj = 0; dj < 2; ++dj) {
      const int pxy = px[di] ^ py[dj];
      const double wxy = wx[di] * wy[dj];
#pragma unroll
      for (int dk = 0; dk < 2; ++dk) {
        const int idx = pxy ^ pz[dk];
        const v3 c = V(T->ranfloat[idx][0], T->ranfloat[idx][1], T->ranfloat[idx][2]);
        accum += (wxy * wz[dk]) * dot(c, V(gx[di], gy[dj], gz[dk]));
      }
    }
  }
  return accum;
}

__device__ __forceinline__ double perlin_noise_inl(const DPerlin* T, v3 p) { return perlin_noise_t(T, p); }
__device__ __noinline__ double perlin_noise(const DPerlin* T, v3 p) { return perlin_noise_t(T, p); }

// A Perlin table in LDS, typed so that out-of-line code reads it with ds_read (a generic pointer
// would make every gather a FLAT load).
typedef __attribute__((address_space(3))) const DPerlin LdsPerlin;

// perlin/mod.rs:162-183 NoiseTexture::value ("marble"): 0.5 (1 + sin(scale p.z + 10 turb(p, 7)));
// the x/y terms of the reference's dot with (0,0,1) contribute exactly 0.  NOISE = the octave's
// noise function (out-of-line in the megakernel to hold its registers, inline in wf_texture).
template <class TP>
__device__ __forceinline__ double marble_t(TP T, double sc, v3 p) {
  double accum = 0.0;
  v3 tp = p;
  double weight = 1.0;
#pragma unroll 1
  for (int i = 0; i < 7; ++i) {  // turbulence, perlin/mod.rs:111-124
    accum += weight * perlin_noise_t(T, tp);
    weight *= 0.5;
    tp = scale(tp, 2.0);
  }
  double turb = 10.0 * fabs(accum);
  double total_noise = RT_SIN(sc * p.z + turb);
  return 0.5 * (1.0 + total_noise);
}

// out of line in the megakernel (holds its register budget), inline in wf_texture
__device__ __noinline__ double marble(const DPerlin* T, double sc, v3 p) { return marble_t(T, sc, p); }
__device__ __noinline__ double marble_lds(LdsPerlin* T, double sc, v3 p) { return marble_t(T, sc, p); }
__device__ __forceinline__ double marble_inl(const DPerlin* T, double sc, v3 p) { return marble_t(T, sc, p); }

__device__ __forceinline__ unsigned long long lanes_below() {
  const unsigned lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull) >> (64 - lane);
}

// Lane of the j-th (0-based) set bit of `mask` (binary search on prefix popcounts).
__device__ __forceinline__ int select_lane(unsigned long long mask, int j) {
  int lo = 0;
  for (int w = 32; w > 0; w >>= 1) {
    const unsigned long long below = (lo + w >= 64) ? mask : (mask & ((1ull << (lo + w)) - 1ull));
    if (__popcll(below) <= j) lo += w;
  }
  return lo;
}
// The inverse of the rank map of `mask`, for the whole wave in one forward permute: lane j (j <
// popcount(mask)) receives the lane of mask's j-th set bit.  Every lane pushes its id (ds_permute:
// dst[addr / 4] = src) — a set lane to slot rank, an unset lane to slot k + (its rank among the unset
// lanes) — so the slots form a permutation and no two lanes write one slot.  Replaces a per-lane
// binary search (select_lane, ~50 VALU) by a handful of instructions.  Wave-uniform control flow.
__device__ __forceinline__ int rank_owners(unsigned long long mask) {
  const int lane = __lane_id();
  const int below = __popcll(mask & lanes_below());
  const int k = __popcll(mask);
  const int slot = ((mask >> lane) & 1ull) ? below : k + (lane - below);
  return __builtin_amdgcn_ds_permute(slot << 2, lane);
}

// v from lane L - 1 on lane L (lane 0: 0), a whole-wave DPP shift (wave_shr:1) of both halves
__device__ __forceinline__ double lane_shift_up(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// perlin/mod.rs:162-183 marble for every lane with `need`, computed by the whole wave: a round serves
// 9 needing lanes, needing lane j's 7 octaves being lanes 7j .. 7j + 6, so a wave needs ceil(k / 9)
// noise evaluations instead of 7 (the octave loop otherwise runs for all lanes while any one needs
// it).  Octave i's input p * 2^i is the reference's tp after i doublings (scaling by 2 is exact), its
// weight 0.5^i likewise; the octaves are then summed in the reference's order along the 7 lanes (six
// one-lane DPP shifts of the running sums) — the value is bit-identical.  Must be called in wave-uniform control flow (it shuffles).
template <class TP>
__device__ __forceinline__ double marble_coop(TP tables, bool need, int tab, double sc, v3 p) {
  const unsigned long long mask = __ballot(need);
  if (mask == 0ull) return 0.0;
  const int k = __popcll(mask);
  const int lane = __lane_id();
  const int rank = __popcll(mask & lanes_below());
  const int owners = rank_owners(mask);  // lane j < k: the lane of the j-th needing lane
  const int jl = lane / 7, oct = lane - 7 * jl;
  const double w = __builtin_amdgcn_ldexp(1.0, -oct);  // the reference's weight after oct halvings
  double accum = 0.0;
  for (int base = 0; base < k; base += 9) {
    PH_COUNT(8);
    const bool valid = lane < 63 && base + jl < k;
    const int owner = __shfl(owners, valid ? base + jl : 0);
    const double qx = __shfl(p.x, owner), qy = __shfl(p.y, owner), qz = __shfl(p.z, owner);
    const int qt = __shfl(tab, owner);
    double nv = 0.0;
    if (valid) {
      const double f = (double)(1 << oct);  // 2^oct, exact
      nv = perlin_noise_t(tables + qt, V(qx * f, qy * f, qz * f));
    }
    // accum = 0.0; accum += weight * noise, in octave order.  Every lane adds what the lane below held
    // one step earlier, so at step s lane 7j + s holds octaves 0 .. s of lane j (by induction: it read
    // lane 7j + s - 1 after step s - 1); what the other lanes hold then is never read.
    const double term = w * nv;
    double run = 0.0 + term;
#pragma unroll
    for (int st = 1; st < 7; ++st) run = lane_shift_up(run) + term;
    const bool mine = need && rank >= base && rank < base + 9;
    const double v = __shfl(run, mine ? 7 * (rank - base) + 6 : 0);
    if (mine) accum = v;
  }
  const double turb = 10.0 * fabs(accum);
  if (need) PH_COUNT(14);
  return need ? 0.5 * (1.0 + RT_SIN(sc * p.z + turb)) : 0.0;
}

// One Philox block of a lane's stream: draws 2c (c0, c1) and 2c + 1 (c2, c3) of (seed, pixel, sample).
__device__ __forceinline__ void philox_block(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t c, uint64_t& even,
                                             uint64_t& odd) {
  uint32_t c0 = c, c1 = sample, c2 = pixel, c3 = 0u;
  philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
  even = (uint64_t)c0 | ((uint64_t)c1 << 32);
  odd = (uint64_t)c2 | ((uint64_t)c3 << 32);
}
// A draw's 53 random bits, v >> 11 (< 2^53), as an exact double: the high 21 bits times 2^32 plus the
// low 32 bits in one FMA (every term exact).  rand 0.8's Standard f64 is draw_bits(v) * 2^-53.
__device__ __forceinline__ double draw_bits(uint64_t v) {
  const uint64_t m = v >> 11;
  return fma((double)(uint32_t)(m >> 32), 4294967296.0, (double)(uint32_t)m);
}
__device__ __forceinline__ double unit_draw(uint64_t v) { return __builtin_amdgcn_ldexp(draw_bits(v), -53); }
// a + s * gen::<f64>() for s = 2^k (core/math.rs:22-25 random_real(-1, 1): a = -1, s = 2; the camera jitter
// i + U, render.rs:60-63: a = i, s = 1): s * U is exact, so the reference rounds once, at the sum — the
// single rounding of one FMA on the exact draw bits (2^(k-53) scales them exactly).
__device__ __forceinline__ double affine_draw(uint64_t v, double pow2_over_2_53, double a) {
  return fma(draw_bits(v), pow2_over_2_53, a);
}
constexpr double kTwoOver2p53 = 0x1p-52;  // random_real(-1, 1): (1 - -1) * 2^-53
constexpr double kOneOver2p53 = 0x1p-53;

// core/math.rs:32-45 random_in_unit_sphere for every lane with `need`, by the whole wave.  Each such
// lane first makes its own attempt (the serial loop's first iteration, 52 % accepted).  The lanes it
// rejected are then served together: all 64 lanes evaluate one later attempt each — attempt i of the
// pending lane of rank q sits on lane q + i·n (n pending lanes) — and every owner takes its first
// accepted attempt.  An attempt is a pure function of (seed, pixel, sample, draw index) (Philox is
// counter-based): attempt at draw t uses draws t, t+1, t+2 = halves of blocks t/2 and t/2 + 1.  So
// the point, the draw counter after it (t + 3) and the cached odd half (block t/2 + 1's) are exactly
// the serial loop's, while a wave runs ~3 rounds instead of the ~6 iterations its unluckiest lane
// needs.  Must be called in wave-uniform control flow (it shuffles).
__device__ __forceinline__ v3 random_in_unit_sphere_coop(Rng& r, uint64_t seed, bool need) {
  v3 p = V(0.0, 0.0, 0.0);
  bool pending = false;
  // A lane's own first attempt, with two Philox evaluations per wave instead of three: draws d, d+1,
  // d+2 are halves of blocks d/2 and d/2 + 1, and an odd d takes its first draw from the cached odd
  // half of block d/2 (three rng_next calls would each run Philox for the lanes at an even draw).
  if (need) {
    const bool odd = (r.draw & 1u) != 0u;
    uint64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
    if (!odd) philox_block(seed, r.pixel, r.sample, r.draw >> 1, a0, a1);
    philox_block(seed, r.pixel, r.sample, (r.draw >> 1) + 1u, b0, b1);
    const uint64_t cached = (uint64_t)r.c2 | ((uint64_t)r.c3 << 32);
    const double x = affine_draw(odd ? cached : a0, kTwoOver2p53, -1.0);  // random_real(-1, 1)
    const double y = affine_draw(odd ? b0 : a1, kTwoOver2p53, -1.0);
    const double z = affine_draw(odd ? b1 : b0, kTwoOver2p53, -1.0);
    r.draw += 3u;
    r.c2 = (uint32_t)b1;  // the odd half of block d/2 + 1, as the serial draws leave it
    r.c3 = (uint32_t)(b1 >> 32);
    p = V(x, y, z);
    pending = !(len2(p) <= 1.0);
  }
  unsigned long long mask = __ballot(pending);
  if (mask == 0ull) return p;
  const int lane = __lane_id();
  while (mask != 0ull) {
    PH_COUNT(9);
    const int n = __popcll(mask);
    const int rank = __popcll(mask & lanes_below());  // meaningful for pending lanes
    const int q = lane % n, i = lane / n;
    const int owner = __shfl(rank_owners(mask), q);
    const uint32_t t = (uint32_t)__shfl((int)r.draw, owner) + 3u * (uint32_t)i;
    const uint32_t pix = (uint32_t)__shfl((int)r.pixel, owner), smp = (uint32_t)__shfl((int)r.sample, owner);
    uint64_t a0, a1, b0, b1;
    philox_block(seed, pix, smp, t >> 1, a0, a1);
    philox_block(seed, pix, smp, (t >> 1) + 1u, b0, b1);
    const bool odd = (t & 1u) != 0u;
    const double x = affine_draw(odd ? a1 : a0, kTwoOver2p53, -1.0);  // random_real(-1, 1)
    const double y = affine_draw(odd ? b0 : a1, kTwoOver2p53, -1.0);
    const double z = affine_draw(odd ? b1 : b0, kTwoOver2p53, -1.0);
    const unsigned long long acc = __ballot(len2(V(x, y, z)) <= 1.0);
    // owners' first accepted attempt, level by level (wave-uniform masks of n bits)
    const unsigned long long owners = (n == 64) ? ~0ull : ((1ull << n) - 1ull);
    unsigned long long found = 0ull;
    int src = -1, lvl = 0;
    for (int base = 0; base < 64 && found != owners; base += n, ++lvl) {
      const unsigned long long bits = (acc >> base) & owners;
      if (pending && ((bits & ~found) >> rank) & 1ull) src = lvl;
      found |= bits;
    }
    const int sl = src >= 0 ? src * n + rank : 0;
    const double sx = __shfl(x, sl), sy = __shfl(y, sl), sz = __shfl(z, sl);
    const uint32_t s2 = (uint32_t)__shfl((int)(uint32_t)b1, sl), s3 = (uint32_t)__shfl((int)(uint32_t)(b1 >> 32), sl);
    if (pending) {
      if (src >= 0) {
        p = V(sx, sy, sz);
        r.draw += 3u * (uint32_t)src + 3u;
        r.c2 = s2;
        r.c3 = s3;
        pending = false;
      } else {
        r.draw += 3u * (uint32_t)((64 - rank + n - 1) / n);  // this round's attempts of this owner
      }
    }
    mask = __ballot(pending);
  }
  return p;
}

// All random draws of one megakernel iteration, by the whole wave at once.  A lane asks for one of:
//   kDrawSphere — random_in_unit_sphere for its scatter (lambertian / metal / fairy light / isotropic),
//                 draws d, d+1, d+2 per attempt (core/math.rs:32-45);
//   kDrawDiel   — the dielectric's uniform (dielectric.rs:41), draw d — drawn speculatively: the
//                 shader consumes it (advances the counter) only when there is no total internal
//                 reflection, exactly like the reference's conditional draw;
//   kDrawCam    — a new sample's camera draws: jitter x, y = draws 0, 1 (render.rs:60-63), then
//                 random_in_unit_disk (camera/mod.rs:99-106, core/math.rs:70-81) from draw 2 on when
//                 the camera has a lens, 2 draws per attempt.
// First attempts: every lane's needs fit two Philox evaluations (block A, block B): a sphere attempt
// at an even d takes blocks d/2 and d/2 + 1, at an odd d the cached odd half of block (d-1)/2 and block
// (d+1)/2 = d/2 + 1; the dielectric's draw is block d/2's even half or the cache; the camera takes block
// 0 (jitter) and block 1 (first disk attempt).  So two call sites serve the whole wave instead of
// separate ones per material and a serial lens loop per new sample.  Rejected attempts (sphere or disk)
// are then served together as in random_in_unit_sphere_coop, each pending lane getting a block of
// consecutive lanes per round; a disk item evaluates two consecutive disk attempts (one per block).  Every
// attempt is a pure function of (seed, pixel, sample, draw index), so the points, the draw counters and
// the cached odd halves are exactly the serial loops'.  Must be called in wave-uniform control flow.
// Returns: kDrawSphere -> the point; kDrawCam -> (disk x, disk y, 0) (lens) with the jitter in jx, jy;
// kDrawDiel -> (uniform, bits of the cache after the draw, 0).
enum : int { kDrawNone = 0, kDrawSphere = 1, kDrawDiel = 2, kDrawCam = 3 };
__device__ __forceinline__ double u64_as_double(uint64_t v) { return __longlong_as_double((long long)v); }
__device__ __forceinline__ uint64_t double_as_u64(double v) { return (uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ v3 draws_coop(Rng& r, uint64_t seed, int kind, bool lens, uint32_t pxy, double& jx,
                                         double& jy) {
  const bool cam = kind == kDrawCam;
  const bool even = (r.draw & 1u) == 0u;
  uint64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
  if (cam || ((kind == kDrawSphere || kind == kDrawDiel) && even)) {
    PH_COUNT(12);
    philox_block(seed, r.pixel, r.sample, cam ? 0u : (r.draw >> 1), a0, a1);
  }
  if (kind == kDrawSphere || (cam && lens)) {
    PH_COUNT(13);
    philox_block(seed, r.pixel, r.sample, cam ? 1u : (r.draw >> 1) + 1u, b0, b1);
  }
  const uint64_t cached = (uint64_t)r.c2 | ((uint64_t)r.c3 << 32);
  // the first attempts' draw bits, converted once for every kind: a sphere takes u0 u1 u2 (x y z), a
  // camera u0 u1 (jitter) and u2 u3 (disk), a dielectric u0; each kind then scales them (affine_draw)
  const bool sph = kind == kDrawSphere;
  const double u0 = draw_bits((!even && !cam) ? cached : a0);
  const double u1 = draw_bits((sph && !even) ? b0 : a1);
  const double u2 = draw_bits((sph && !even) ? b1 : b0);
  const double u3 = draw_bits(b1);
  v3 p = V(0.0, 0.0, 0.0);
  bool pending = false;
  if (sph) {
    p = V(fma(u0, kTwoOver2p53, -1.0), fma(u1, kTwoOver2p53, -1.0), fma(u2, kTwoOver2p53, -1.0));  // random_real(-1, 1)
    r.draw += 3u;
    r.c2 = (uint32_t)b1;  // the odd half of block d/2 + 1, as the serial draws leave it
    r.c3 = (uint32_t)(b1 >> 32);
    pending = !(len2(p) <= 1.0);
  } else if (kind == kDrawDiel) {
    p = V(__builtin_amdgcn_ldexp(u0, -53), u64_as_double(even ? a1 : cached), 0.0);
  } else if (cam) {
    jx = fma(u0, kOneOver2p53, (double)(pxy & 0xffffu));  // i + U (render.rs:60-63)
    jy = fma(u1, kOneOver2p53, (double)(pxy >> 16));
    r.draw = 2u;
    if (lens) {
      const double x = fma(u2, kTwoOver2p53, -1.0), y = fma(u3, kTwoOver2p53, -1.0);
      p = V(x, y, 0.0);
      r.draw = 4u;
      pending = !(x * x + y * y <= 1.0);  // len2((x, y, 0)): the + 0*0 term cannot change a sum >= 0
    }
  }
  unsigned long long mask = __ballot(pending);
  if (mask == 0ull) return p;
  const int lane = __lane_id();
  // a pending camera lane rejects disk points; the flag rides in bit 31 of the shared draw counter
  const uint32_t disk_bit = cam ? 0x80000000u : 0u;
  while (mask != 0ull) {
    PH_COUNT(9);
    // the n pending lanes get m = 64 / n consecutive items each: owner q's items are lanes [q m, q m + m)
    // (the 64 - n m others idle), so an owner's first accepted item is the lowest set bit of an m-bit
    // field of the acceptance ballot
    const int n = __popcll(mask);
    const int m = 64 / n;
    const int rank = __popcll(mask & lanes_below());  // meaningful for pending lanes
    // q = lane / m exactly: (lane + 1/2) / m stays >= 1 / (2m) >= 2^-7 away from an integer
    const int q = (int)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)m));
    const int i = lane - q * m;
    const bool valid = q < n;
    const int owner = __shfl(rank_owners(mask), valid ? q : 0);
    const uint32_t tw = (uint32_t)__shfl((int)(r.draw | disk_bit), owner);
    const bool odisk = (tw & 0x80000000u) != 0u;
    const uint32_t t0 = tw & 0x7fffffffu;
    const uint32_t pix = (uint32_t)__shfl((int)r.pixel, owner), smp = (uint32_t)__shfl((int)r.sample, owner);
    // a sphere item is the attempt at draw t0 + 3i; a disk item the two attempts at draws t0 + 4i and
    // t0 + 4i + 2 (t0 even), i.e. blocks t0/2 + 2i and t0/2 + 2i + 1
    const uint32_t t = t0 + 3u * (uint32_t)i;
    const uint32_t c = odisk ? (t0 >> 1) + 2u * (uint32_t)i : (t >> 1);
    uint64_t e0, e1, f0, f1;
    philox_block(seed, pix, smp, c, e0, e1);
    philox_block(seed, pix, smp, c + 1u, f0, f1);
    const double d0 = affine_draw(e0, kTwoOver2p53, -1.0), d1 = affine_draw(e1, kTwoOver2p53, -1.0);
    const double d2 = affine_draw(f0, kTwoOver2p53, -1.0), d3 = affine_draw(f1, kTwoOver2p53, -1.0);
    double x, y, z;
    bool acc;
    uint32_t used;  // draws this item consumed up to its accepted point (disk)
    if (odisk) {
      const bool acc1 = d0 * d0 + d1 * d1 <= 1.0;
      acc = acc1 || d2 * d2 + d3 * d3 <= 1.0;
      x = acc1 ? d0 : d2;
      y = acc1 ? d1 : d3;
      z = 0.0;
      used = acc1 ? 2u : 4u;
    } else {
      const bool odd = (t & 1u) != 0u;
      x = odd ? d1 : d0;
      y = odd ? d2 : d1;
      z = odd ? d3 : d2;
      acc = len2(V(x, y, z)) <= 1.0;
      used = 3u;
    }
    const unsigned long long accm = __ballot(valid && acc);
    const int shift = pending ? rank * m : 0;  // < 64 for a pending lane (rank < n, n m <= 64)
    const unsigned long long field = (m == 64 ? accm : (accm >> shift) & ((1ull << m) - 1ull));
    const int src = (pending && field != 0ull) ? (int)__builtin_ctzll(field) : -1;
    const int sl = src >= 0 ? rank * m + src : 0;
    const double sx = __shfl(x, sl), sy = __shfl(y, sl), sz = __shfl(z, sl);
    const uint32_t s2 = (uint32_t)__shfl((int)(uint32_t)f1, sl), s3 = (uint32_t)__shfl((int)(uint32_t)(f1 >> 32), sl);
    const uint32_t su = (uint32_t)__shfl((int)used, sl);
    if (pending) {
      const uint32_t stride = disk_bit ? 4u : 3u;  // draws per item
      if (src >= 0) {
        p = V(sx, sy, sz);
        r.draw += stride * (uint32_t)src + su;
        r.c2 = s2;  // (a disk point leaves an even counter: the cache is then never read)
        r.c3 = s3;
        pending = false;
      } else {
        r.draw += stride * (uint32_t)m;  // this round's items of this owner
      }
    }
    mask = __ballot(pending);
  }
  return p;
}

// camera/mod.rs:97-132 from the sample's draws: jitter (x, y) and the unit-disk point (lens cameras).
// CAM: a DCamera (reference) or a pointer-like to one (the megakernel's constant-address-space copy).
typedef __attribute__((address_space(4))) const DCamera KCamera;
typedef __attribute__((address_space(4))) const DWork KWork;
typedef __attribute__((address_space(4))) const DScene KScene;
typedef __attribute__((address_space(4))) const KBlock KBlk;
// the pass's KBlock behind an opaque copy of its address (the empty asm keeps the scalar loads from
// being hoisted out of the megakernel's loop)
__device__ __forceinline__ KBlk* kblock(uint64_t a) {
  KBlk* kb = (KBlk*)(uintptr_t)a;
  asm volatile("" : "+s"(kb));
  return kb;
}
// x / n for the camera's jittered pixel coordinate x in [0, n], n = width or height <= 65536, with
// r = RN(1 / n) from the host: q0 = x r is within an ulp of x / n, and one correction step with the
// correctly rounded reciprocal gives the correctly rounded quotient (Markstein, IBM J. Res. Dev. 34,
// 1990) — bit-identical to the IEEE division the reference does (camera/mod.rs:98-99), at a mul and two
// fmas instead of the ~11-instruction division.  Checked on the CPU against x / n for every n <= 4096
// and every 97th n up to 65536, ~76 M jittered coordinates with edge cases (tools/camdiv_check.c,
// tests/test_divisions.py), and on the GPU by every parity test (same bits as the oracle's x / n).
__device__ __forceinline__ double pixel_coord_div(double x, double n, double r) {
  const double q0 = x * r;
  return __builtin_fma(__builtin_fma(-n, q0, x), r, q0);
}
template <class CAM>
__device__ __forceinline__ void camera_ray_drawn(const CAM& C, double x, double y, v3 disk, v3& o, v3& d) {
  const double xp = pixel_coord_div(x, C.wd, C.inv_w);
  const double yp = pixel_coord_div(y, C.hd, C.inv_h);
  const v3 u = V(C.u[0], C.u[1], C.u[2]), v = V(C.v[0], C.v[1], C.v[2]);
  const v3 origin = V(C.origin[0], C.origin[1], C.origin[2]);
  v3 offset = V(0.0, 0.0, 0.0);
  if (C.has_lens) {
    const v3 rd = scale(disk, C.lens_radius);
    offset = scale(u, rd.x) + scale(v, rd.y);
  }
  const v3 ll = V(C.lower_left[0], C.lower_left[1], C.lower_left[2]);
  const v3 hz = V(C.horizontal[0], C.horizontal[1], C.horizontal[2]);
  const v3 vt = V(C.vertical[0], C.vertical[1], C.vertical[2]);
  d = (((ll + scale(hz, xp)) + scale(vt, yp)) - origin) - offset;
  o = origin + offset;
}

// checker.rs:28-30
__device__ __noinline__ double checker_sines(double s, double x, double y, double z) {
  return RT_SIN(s * x) * RT_SIN(s * y) * RT_SIN(s * z);
}

// Sign of sin(y) for a double y, exactly: +1, -1 or 0 — or 2 when this fast path does not decide
// (NaN, |y| < 1e-100, |y| > 3e6, or y within 1e-12 of a multiple of pi).  y is reduced by pi split in
// three parts (P1, P2 with 33 significant bits, so k*P1 and k*P2 are exact for |k| < 2^20, and
// y - k*P1 is exact by Sterbenz): r = y - k*pi to ~2^-100 absolute, and sin(y) = (-1)^k sin(r) with
// |r| < pi, so sign(sin y) = (-1)^k sign(r).  Any faithful sin (glibc's, ocml's) has that sign.
__device__ __forceinline__ int sin_sign(double y) {
  if (y == 0.0) return 0;
  const double ay = fabs(y);
  if (!(ay >= 1e-100 && ay <= 3.0e6)) return 2;
  const double P1 = 0x1.921fb54400000p+1, P2 = 0x1.0b4611a600000p-33, P3 = 0x1.3198a2e037073p-68;
  const double k = rint(y * 0x1.45f306dc9c883p-2);  // y / pi
  double r = fma(-k, P1, y);
  r = fma(-k, P2, r);
  r = fma(-k, P3, r);
  if (fabs(r) < 1e-12) return 2;
  const int sr = r > 0.0 ? 1 : -1;
  return (((long long)k) & 1) ? -sr : sr;
}

// checker.rs:27-37 decides odd/even by `sin(s x) sin(s y) sin(s z) < 0.0` alone.  Each |factor| is
// >= ~1e-100 on the fast path, so the product cannot underflow and its sign is the product of the
// signs; anything the fast path cannot decide evaluates the reference's product.
__device__ __forceinline__ bool checker_odd(double s, double x, double y, double z) {
  const int a = sin_sign(s * x), b = sin_sign(s * y), c = sin_sign(s * z);
  if (a == 2 || b == 2 || c == 2) return checker_sines(s, x, y, z) < 0.0;
  return a * b * c < 0;
}

// The texture a material reads, resolved down to its leaf (checker.rs:27-37 picks odd/even by the
// sign of a sine product).  Returns the leaf index.
__device__ __forceinline__ int resolve_texture_t(const DTex* texs, int ti, v3 p) {
  for (;;) {
    const DTex& t = texs[ti];
    if (t.kind != RT_TEX_CHECKER) return ti;
    PH_COUNT(16);
    ti = checker_odd(t.scale, p.x, p.y, p.z) ? t.odd : t.even;
  }
}

__device__ __forceinline__ int resolve_texture(const DScene& S, int ti, v3 p) { return resolve_texture_t(S.texs, ti, p); }

// image_texture.rs:34-56: clamp, flip v, truncate, /255.
__device__ __forceinline__ v3 image_texel(const DTex& tx, double u, double v) {
  const DTexImage im = tx.img;
  double uu = (u > 0.0) ? ((u < 1.0) ? u : 1.0) : 0.0;
  double vv = 1.0 - ((v > 0.0) ? ((v < 1.0) ? v : 1.0) : 0.0);
  uint32_t ix = (uint32_t)(uu * (double)(im.width - 1));
  uint32_t iy = (uint32_t)(vv * (double)(im.height - 1));
  // (the texels are in global memory: typed so, a texture record read from LDS does not make them FLAT loads)
  typedef __attribute__((address_space(1))) const uint8_t GTexel;
  GTexel* px = (GTexel*)im.texels + ((size_t)iy * (size_t)im.width + ix) * 3;
  const double cs = 1.0 / 255.0;
  return V((double)px[0] * cs, (double)px[1] * cs, (double)px[2] * cs);
}

// u, v of a hit record built without them (prim_record<false>), from the record itself: a sphere's
// outward normal is the record's normal un-flipped (negation is exact), and a rect's o1 + t d1 is
// exactly the record's point component (x*y == y*x); the formulas are then prim_record's.
__device__ __forceinline__ UV hit_uv(const DPrim& pr, int face, const Hit& h) {
  if (pr.kind & kPrimExt) return UV{h.u, h.v};  // ext_record computed them
  if (pr.kind == kPrimSphere) {
    const v3 n = h.front_face ? h.normal : scale(h.normal, -1.0);
    return sphere_uv(n.x, n.y, n.z);
  }
  const double* b = pr.p;
  int kind = pr.kind;
  double q0 = b[0], q1 = b[1], q2 = b[2], q3 = b[3];
  if (kind == kPrimBox) {
    if (face < 2) { q0 = b[0]; q1 = b[3]; q2 = b[1]; q3 = b[4]; kind = kPrimRectXY; }
    else if (face < 4) { q0 = b[1]; q1 = b[4]; q2 = b[2]; q3 = b[5]; kind = kPrimRectYZ; }
    else { q0 = b[0]; q1 = b[3]; q2 = b[2]; q3 = b[5]; kind = kPrimRectXZ; }
  }
  const double a1 = (kind == kPrimRectYZ) ? h.point.y : h.point.x;
  const double a2 = (kind == kPrimRectXY) ? h.point.y : h.point.z;
  return UV{(a1 - q0) / (q1 - q0), (a2 - q2) / (q3 - q2)};
}

// Texture value at a hit (texture.rs Texture::value): checker resolved by the hit point, Perlin
// marble by the hit point, solid directly, image by u, v (computed only for an image leaf).
// Texture value of an already resolved leaf whose marble value (if Perlin) is `pn`.
__device__ __forceinline__ v3 leaf_texture_value(const DScene& S, const DTex* texs, int leaf, double pn, int prim,
                                                 int face, const Hit& h) {
  const DTex& tx = texs[leaf];
  if (tx.kind == RT_TEX_SOLID) return V(tx.color[0], tx.color[1], tx.color[2]);  // solid.rs:17-21
  if (tx.kind == RT_TEX_PERLIN) return V(pn, pn, pn);
  const UV uv = hit_uv(S.prims[prim], face, h);
  return image_texel(tx, uv.u, uv.v);
}

// `lds_perlin`: the block's LDS copy of the Perlin tables, or null (tables read through L1/L2).
__device__ __forceinline__ v3 texture_value(const DScene& S, const DPerlin* lds_perlin, int ti, int prim, int face,
                                            const Hit& h) {
  const int leaf = resolve_texture(S, ti, h.point);
  const DTex& tx = S.texs[leaf];
  if (tx.kind == RT_TEX_SOLID) return V(tx.color[0], tx.color[1], tx.color[2]);  // solid.rs:17-21
  if (tx.kind == RT_TEX_PERLIN) {
    const double n = lds_perlin ? marble_lds((LdsPerlin*)(lds_perlin + tx.table), tx.scale, h.point)
                                : marble(S.perlin + tx.table, tx.scale, h.point);
    return V(n, n, n);
  }
  const UV uv = hit_uv(S.prims[prim], face, h);
  return image_texel(tx, uv.u, uv.v);
}

// x^5 for x in [0, 4] as a double-double product (x^2 and x^4 carried with their FMA-exact
// low parts): within ~2^-100 relative of the exact value before the final rounding, i.e. correctly
// rounded save for values within 2^-100 of a rounding boundary — as glibc's pow(x, 5.0) is (the
// oracle's and the reference's libm).  Other x take pow().
__device__ __forceinline__ double pow5(double x) {
  if (!(x >= 0.0 && x <= 4.0)) return RT_POW5_LIBM(x);
  const double x2 = x * x;
  const double x2l = fma(x, x, -x2);
  const double x4 = x2 * x2;
  const double x4l = fma(x2, x2, -x4) + (2.0 * x2) * x2l;
  const double x5 = x4 * x;
  const double x5l = fma(x4, x, -x5) + x4l * x;
  return x5 + x5l;
}

// dielectric.rs:15-19 (Schlick); only ever compared against a uniform draw (dielectric.rs:41)
__device__ __forceinline__ double reflectance_inl(double cosine, double ref_idx) {
  double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * pow5(1.0 - cosine);
}
__device__ __noinline__ double reflectance(double cosine, double ref_idx) { return reflectance_inl(cosine, ref_idx); }
// reflectance_inl with its r0^2 from the host (DMat: a dielectric's albedo[0] / albedo[1] for the front / back face)
__device__ __noinline__ double pow5_libm(double x) { return RT_POW5_LIBM(x); }
__device__ __forceinline__ double reflectance_r0sq(double cosine, double r0sq) {
  const double x = 1.0 - cosine;
  double p;
  if (!(x >= 0.0 && x <= 4.0)) {
    p = pow5_libm(x);
  } else {
    const double x2 = x * x;
    const double x2l = fma(x, x, -x2);
    const double x4 = x2 * x2;
    const double x4l = fma(x2, x2, -x4) + (2.0 * x2) * x2l;
    const double x5 = x4 * x;
    const double x5l = fma(x4, x, -x5) + x4l * x;
    p = x5 + x5l;
  }
  return r0sq + (1.0 - r0sq) * p;
}

// skybox/mod.rs:5-25
// skybox/mod.rs:18-25 given un = unit(d)
template <class SC>  // a DScene, or the megakernel's constant-address-space copy (KScene)
__device__ __forceinline__ v3 sky_unit(const SC& S, v3 un) {
  if (S.sky == RT_SKY_ABOVE) {
    double t = 0.5 * (un.y + 1.0);
    return scale(V(1.0, 1.0, 1.0), 1.0 - t) + scale(V(0.5, 0.7, 1.0), t);
  }
  if (S.sky == RT_SKY_FLAT) return V(S.sky_color[0], S.sky_color[1], S.sky_color[2]);
  return V(0.0, 0.0, 0.0);
}
__device__ __forceinline__ v3 sky(const DScene& S, v3 d) {
  if (S.sky == RT_SKY_ABOVE) {
    v3 un = unit(d);
    double t = 0.5 * (un.y + 1.0);
    return scale(V(1.0, 1.0, 1.0), 1.0 - t) + scale(V(0.5, 0.7, 1.0), t);
  }
  if (S.sky == RT_SKY_FLAT) return V(S.sky_color[0], S.sky_color[1], S.sky_color[2]);
  return V(0.0, 0.0, 0.0);
}

// One ray_color loop iteration after the hit (render.rs:31-40): emitted, then scatter.
// Returns false when the path ends (material absorbed).  Metal, Lambertian and FairyLight all draw
// random_in_unit_sphere (metal.rs:32, lambertian.rs:23 via random_unit_vector); it has one call site.
// The hit record comes without u, v (prim_record<false>); (prim, face, t) let an image texture
// rebuild them.
__device__ __forceinline__ bool shade(const DScene& S, const DPerlin* lds_perlin, const DMat& m, Rng& rng,
                                      uint64_t seed, v3& o, v3& d, const Hit& h, int prim, int face, v3& att, v3& em) {
  if (m.kind == RT_MAT_DIFFUSE_LIGHT) {  // lighting.rs:21-29: emits, never scatters
    v3 e = texture_value(S, lds_perlin, m.tex, prim, face, h);
    em = em + hmul(att, e);
    return false;
  }
  if (m.kind == RT_MAT_DIELECTRIC) {  // dielectric.rs:21-49
    double ratio = h.front_face ? (1.0 / m.param) : m.param;
    v3 ud = unit(d);
    double cos_theta = fmin_one(dot(scale(ud, -1.0), h.normal));
    double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
    bool refl = ratio * sin_theta > 1.0;
    if (!refl) refl = reflectance(cos_theta, ratio) > rng_next(rng, seed);  // drawn only if not TIR
    o = h.point;
    d = refl ? reflect(ud, h.normal) : refract(ud, h.normal, ratio);
    return true;  // attenuation = Color::ones()
  }
  v3 r = random_in_unit_sphere(rng, seed);
  if (m.kind == RT_MAT_METAL) {  // metal.rs:26-40 — never absorbs
    v3 reflected = reflect(unit(d), h.normal);
    o = h.point;
    d = reflected + scale(r, m.param);
    att = hmul(att, V(m.albedo[0], m.albedo[1], m.albedo[2]));
    return true;
  }
  if (m.kind == RT_MAT_ISOTROPIC) {  // book-2 isotropic (extension): random_in_unit_sphere, albedo
    att = hmul(att, texture_value(S, lds_perlin, m.tex, prim, face, h));
    o = h.point;
    d = r;
    return true;
  }
  // RT_MAT_LAMBERTIAN (lambertian.rs:21-37) / RT_MAT_FAIRY_LIGHT (lighting.rs:42-66)
  v3 a = texture_value(S, lds_perlin, m.tex, prim, face, h);
  if (m.kind == RT_MAT_FAIRY_LIGHT) {
    double s = dot(h.normal, scale(d, -1.0));
    em = em + hmul(att, scale(a, s / len(d)));
    a = unit(a);
  }
  v3 sc = h.normal + unit(r);
  if (near_zero(sc)) sc = h.normal;
  o = h.point;
  d = sc;
  att = hmul(att, a);
  return true;
}

// shade() with the wave-level parts done beforehand: the texture leaf resolved, its marble value
// (if any) and the scatter's random_in_unit_sphere point `r` (lambertian / metal / fairy light)
// computed by the wave (marble_coop, random_in_unit_sphere_coop), and `un` = the one unit vector the
// material needs — unit(r) for lambertian / fairy light, unit(d) for dielectric / metal — computed
// for all lanes at once instead of once per material branch.  Same steps otherwise.
// DRAWN: the dielectric's uniform was drawn ahead by draws_coop (r = (uniform, bits of the cache after
// it, 0)); it is consumed here — the counter advanced — only when the reference draws it (no TIR).
template <bool DRAWN = false>
__device__ __forceinline__ bool shade_pre(const DScene& S, const DMat& m, int leaf, double pn, v3 r, v3 un,
                                          Rng& rng, uint64_t seed, v3& o, v3& d, const Hit& h, int prim,
                                          int face, v3& att, v3& em) {
  const DTex* texs = S.texs;
  if (m.kind == RT_MAT_DIFFUSE_LIGHT) {  // lighting.rs:21-29: emits, never scatters
    PH_COUNT(21);
    v3 e = leaf_texture_value(S, texs, leaf, pn, prim, face, h);
    em = em + hmul(att, e);
    return false;
  }
  if (m.kind == RT_MAT_DIELECTRIC) {  // dielectric.rs:21-49
    PH_COUNT(17);
    double ratio = h.front_face ? m.inv_param : m.param;  // 1.0 / ir, precomputed
    const v3 ud = un;
    double cos_theta = fmin_one(dot(scale(ud, -1.0), h.normal));
    double sin_theta = sqrt_rn(1.0 - cos_theta * cos_theta);
    bool refl = ratio * sin_theta > 1.0;
    if (!refl) {  // drawn only if not TIR
      PH_COUNT(22);
      if (DRAWN) {
        refl = reflectance(cos_theta, ratio) > r.x;
        const uint64_t cb = double_as_u64(r.y);
        rng.draw += 1u;
        rng.c2 = (uint32_t)cb;
        rng.c3 = (uint32_t)(cb >> 32);
      } else {
        refl = reflectance(cos_theta, ratio) > rng_next(rng, seed);
      }
    }
    o = h.point;
    d = refl ? reflect(ud, h.normal) : refract(ud, h.normal, ratio);
    return true;  // attenuation = Color::ones()
  }
  if (m.kind == RT_MAT_METAL) {  // metal.rs:26-40 — never absorbs
    PH_COUNT(18);
    v3 reflected = reflect(un, h.normal);
    o = h.point;
    d = reflected + scale(r, m.param);
    att = hmul(att, V(m.albedo[0], m.albedo[1], m.albedo[2]));
    return true;
  }
  if (m.kind == RT_MAT_ISOTROPIC) {  // book-2 isotropic (extension): random_in_unit_sphere, albedo
    att = hmul(att, leaf_texture_value(S, texs, leaf, pn, prim, face, h));
    o = h.point;
    d = r;
    return true;
  }
  // RT_MAT_LAMBERTIAN (lambertian.rs:21-37) / RT_MAT_FAIRY_LIGHT (lighting.rs:42-66)
  PH_COUNT(19);
  v3 a = leaf_texture_value(S, texs, leaf, pn, prim, face, h);
  if (m.kind == RT_MAT_FAIRY_LIGHT) {
    double s = dot(h.normal, scale(d, -1.0));
    em = em + hmul(att, scale(a, s / len(d)));
    a = unit(a);
  }
  v3 sc = h.normal + un;
  if (near_zero(sc)) sc = h.normal;
  o = h.point;
  d = sc;
  att = hmul(att, a);
  return true;
}

// shade_pre<true> with the path's attenuation and emission left to the caller, so that the megakernel
// reads and writes them once per segment instead of once per material branch: the material's
// attenuation factor goes to `mul` (att = att * mul; 1 for a dielectric, exact) and its emission to
// `emit` with `has_emit` (em = em + att * emit, applied before the factor — the reference's order for
// the fairy light).  Same arithmetic as shade_pre.
__device__ __forceinline__ bool shade_factor(const DScene& S, const DTex* texs, const DMat& m, int leaf, double pn, v3 r, v3 un,
                                             Rng& rng, v3& o, v3& d, const Hit& h, int prim, int face, v3& mul,
                                             v3& emit, bool& has_emit) {
  if (m.kind == RT_MAT_DIFFUSE_LIGHT) {  // lighting.rs:21-29: emits, never scatters
    PH_COUNT(21);
    emit = leaf_texture_value(S, texs, leaf, pn, prim, face, h);
    has_emit = true;
    return false;
  }
  if (m.kind == RT_MAT_DIELECTRIC) {  // dielectric.rs:21-49
    PH_COUNT(17);
    double ratio = h.front_face ? m.inv_param : m.param;  // 1.0 / ir, precomputed
    const v3 ud = un;
    double cos_theta = fmin_one(dot(scale(ud, -1.0), h.normal));
    // ratio * sin_theta > 1 (TIR) needs ratio > 1: sin_theta = sqrt(1 - cos^2) <= 1 (or NaN, which fails the
    // compare) since cos^2 >= 0, so with ratio <= 1 — every front face, and both faces of an ir = 1 coat —
    // the square root is skipped and the decision is the same
    bool refl = ratio > 1.0 && ratio * sqrt_rn(1.0 - cos_theta * cos_theta) > 1.0;
    if (!refl) {  // drawn only if not TIR: the uniform drawn ahead by draws_coop is consumed
      PH_COUNT(22);
      refl = reflectance_r0sq(cos_theta, h.front_face ? m.albedo[0] : m.albedo[1]) > r.x;
      const uint64_t cb = double_as_u64(r.y);
      rng.draw += 1u;
      rng.c2 = (uint32_t)cb;
      rng.c3 = (uint32_t)(cb >> 32);
    }
    o = h.point;
    d = refl ? reflect(ud, h.normal) : refract(ud, h.normal, ratio);
    return true;  // attenuation = Color::ones()
  }
  if (m.kind == RT_MAT_METAL) {  // metal.rs:26-40 — never absorbs
    PH_COUNT(18);
    v3 reflected = reflect(un, h.normal);
    o = h.point;
    d = reflected + scale(r, m.param);
    mul = V(m.albedo[0], m.albedo[1], m.albedo[2]);
    return true;
  }
  if (m.kind == RT_MAT_ISOTROPIC) {  // book-2 isotropic (extension): random_in_unit_sphere, albedo
    mul = leaf_texture_value(S, texs, leaf, pn, prim, face, h);
    o = h.point;
    d = r;
    return true;
  }
  // RT_MAT_LAMBERTIAN (lambertian.rs:21-37) / RT_MAT_FAIRY_LIGHT (lighting.rs:42-66)
  PH_COUNT(19);
  v3 a = leaf_texture_value(S, texs, leaf, pn, prim, face, h);
  if (m.kind == RT_MAT_FAIRY_LIGHT) {
    double s = dot(h.normal, scale(d, -1.0));
    emit = scale(a, s / len(d));
    has_emit = true;
    a = unit(a);
  }
  v3 sc = h.normal + un;
  if (near_zero(sc)) sc = h.normal;
  o = h.point;
  d = sc;
  mul = a;
  return true;
}

// camera/mod.rs:97-132 (horizontal / vertical / lower_left precomputed on the host, same ops)
__device__ __forceinline__ void camera_ray(const DCamera& C, Rng& rng, uint64_t seed, double x, double y, v3& o,
                                           v3& d) {
  double xp = pixel_coord_div(x, C.wd, C.inv_w);
  double yp = pixel_coord_div(y, C.hd, C.inv_h);
  v3 u = V(C.u[0], C.u[1], C.u[2]), v = V(C.v[0], C.v[1], C.v[2]);
  v3 origin = V(C.origin[0], C.origin[1], C.origin[2]);
  v3 offset = V(0.0, 0.0, 0.0);
  if (C.has_lens) {
    v3 rd = scale(random_in_unit_disk(rng, seed), C.lens_radius);
    offset = scale(u, rd.x) + scale(v, rd.y);
  }
  v3 ll = V(C.lower_left[0], C.lower_left[1], C.lower_left[2]);
  v3 hz = V(C.horizontal[0], C.horizontal[1], C.horizontal[2]);
  v3 vt = V(C.vertical[0], C.vertical[1], C.vertical[2]);
  d = (((ll + scale(hz, xp)) + scale(vt, yp)) - origin) - offset;
  o = origin + offset;
}


}  // namespace rt
