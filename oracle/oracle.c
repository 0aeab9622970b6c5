/*
 * oracle.c — f64 CPU restatement of scottschroeder/shirley-raytracing-rs's render hot path.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP path and the timed CPU baseline
 * ("port", bench.py cpu_baseline).  Never linked into the product.  See oracle.h for pinning:
 * pinned by the reference's 25 unit tests + analytic KATs; image-level parity vs a reference run
 * is unpinned (Rust toolchain absent, reference RNG unseedable).
 *
 * Build: gcc -O2 -ffp-contract=off (Rust never contracts a*b+c into an FMA), see oracle/Makefile.
 * Evaluation order follows nalgebra 0.31 (Cargo.lock:619): dot = (x*x'+y*y')+z*z',
 * norm = sqrt(dot(v,v)), normalize = v / norm, cross = (ay*bz-az*by, az*bx-ax*bz, ax*by-ay*bx).
 *
 * RNG: the reference draws from rand::thread_rng() (unseedable, render.rs:61-62, main.rs:98,119).
 * The oracle replaces it with the build's counter-based Philox4x32-10 stream keyed by
 * (seed, pixel, sample, draw#), drawn in the reference's order; each
 * draw is converted exactly like rand 0.8's Standard f64: (u64 >> 11) * 2^-53.
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* The transcendental functions: glibc's (the reference's libm), or (OR_PORTABLE_LIBM, the diagnostic build
 * liboracle_pl.so) the portable ones the kernel's RT_PORTABLE_LIBM build also calls. */
#ifdef OR_PORTABLE_LIBM
#include "portable_libm.h"
#define OR_SIN pl_sin
#define OR_LOG pl_log
#define OR_ACOS pl_acos
#define OR_ATAN2 pl_atan2
#define OR_POW5(x) pl_pow5(x)
#else
#define OR_SIN sin
#define OR_LOG log
#define OR_ACOS acos
#define OR_ATAN2 atan2
#define OR_POW5(x) pow(x, 5.0)
#endif

/* ------------------------------------------------------------------------------------------ */
/* RNG                                                                                          */
/* ------------------------------------------------------------------------------------------ */
void or_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint64_t or_rng_u64(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t draw) {
  uint32_t ctr[4] = {draw >> 1, sample, pixel, 0u};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  or_philox4x32_10(ctr, key, o);
  if ((draw & 1u) == 0u) return (uint64_t)o[0] | ((uint64_t)o[1] << 32);
  return (uint64_t)o[2] | ((uint64_t)o[3] << 32);
}

static inline double u64_to_f64(uint64_t v) { return (double)(v >> 11) * (1.0 / 9007199254740992.0); }

double or_rng_f64(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t draw) {
  return u64_to_f64(or_rng_u64(seed, pixel, sample, draw));
}

typedef struct rng_t {
  uint64_t seed;
  uint32_t pixel, sample, draw;
} rng_t;

/* rng.gen::<f64>() */
static inline double rng_gen(rng_t* r) { return or_rng_f64(r->seed, r->pixel, r->sample, r->draw++); }

/* ------------------------------------------------------------------------------------------ */
/* core/fp.rs:3-28                                                                             */
/* ------------------------------------------------------------------------------------------ */
double or_non_nan(double a, double b) { return isnan(a) ? b : a; }
/* fmin: partial_cmp Less -> a; Equal/Greater -> b; unordered -> non_nan(a, b) */
double or_fmin(double a, double b) {
  if (isnan(a) || isnan(b)) return or_non_nan(a, b);
  return (a < b) ? a : b;
}
double or_fmax(double a, double b) {
  if (isnan(a) || isnan(b)) return or_non_nan(a, b);
  return (a > b) ? a : b;
}

/* ------------------------------------------------------------------------------------------ */
/* core/vec3.rs (nalgebra order)                                                               */
/* ------------------------------------------------------------------------------------------ */
typedef struct v3 {
  double x, y, z;
} v3;
static inline v3 V(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }
static inline double vdot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline double vlen2(v3 a) { return vdot(a, a); }
static inline double vlen(v3 a) { return sqrt(vlen2(a)); }
static inline v3 vunit(v3 a) { double n = vlen(a); return V(a.x / n, a.y / n, a.z / n); }
static inline v3 vcross(v3 a, v3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void vset(v3* a, int i, double s) { if (i == 0) a->x = s; else if (i == 1) a->y = s; else a->z = s; }
/* vec3.rs:129-132 */
static inline int near_zero(v3 a) { return fabs(a.x) < 1e-8 && fabs(a.y) < 1e-8 && fabs(a.z) < 1e-8; }
/* vec3.rs:134-137 */
static inline v3 reflect(v3 v, v3 n) { return vsub(v, vscale(n, 2.0 * vdot(v, n))); }
/* vec3.rs:139-145 */
static inline v3 refract(v3 uv, v3 n, double eta) {
  double cos_theta = or_fmin(vdot(vscale(uv, -1.0), n), 1.0);
  v3 r_out_perp = vscale(vadd(vscale(n, cos_theta), uv), eta);
  double r_out_parallel_mag = sqrt(fabs(1.0 - vlen2(r_out_perp))) * -1.0;
  v3 r_out_parallel = vscale(n, r_out_parallel_mag);
  return vadd(r_out_perp, r_out_parallel);
}

typedef struct ray_t {
  v3 o, d;
} ray_t;
/* vec3.rs:253-255 */
static inline v3 ray_at(const ray_t* r, double t) { return vadd(r->o, vscale(r->d, t)); }

/* core/math.rs:22-25 */
static inline double random_real(rng_t* r, double mn, double mx) { return mn + (mx - mn) * rng_gen(r); }
/* core/math.rs:32-45 (guess and check), vec3.rs:104-110 random_range_with_rng */
static v3 random_in_unit_sphere(rng_t* r) {
  for (;;) {
    double x = random_real(r, -1.0, 1.0);
    double y = random_real(r, -1.0, 1.0);
    double z = random_real(r, -1.0, 1.0);
    v3 p = V(x, y, z);
    if (vlen2(p) <= 1.0) return p;
  }
}
/* core/math.rs:61-68 */
static v3 random_unit_vector(rng_t* r) { return vunit(random_in_unit_sphere(r)); }
/* core/math.rs:70-81 */
static v3 random_in_unit_disk(rng_t* r) {
  for (;;) {
    double x = random_real(r, -1.0, 1.0);
    double y = random_real(r, -1.0, 1.0);
    v3 p = V(x, y, 0.0);
    if (vlen2(p) <= 1.0) return p;
  }
}

/* ------------------------------------------------------------------------------------------ */
/* bvh/aabb.rs                                                                                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct aabb_t {
  v3 mn, mx;
} aabb_t;

static aabb_t box_from(const double b[6]) { aabb_t a = {V(b[0], b[1], b[2]), V(b[3], b[4], b[5])}; return a; }
static void box_to(aabb_t a, double b[6]) {
  b[0] = a.mn.x; b[1] = a.mn.y; b[2] = a.mn.z; b[3] = a.mx.x; b[4] = a.mx.y; b[5] = a.mx.z;
}
/* aabb.rs:18-33 */
static aabb_t surrounding(aabb_t l, aabb_t r) {
  aabb_t o;
  o.mn = V(or_fmin(l.mn.x, r.mn.x), or_fmin(l.mn.y, r.mn.y), or_fmin(l.mn.z, r.mn.z));
  o.mx = V(or_fmax(l.mx.x, r.mx.x), or_fmax(l.mx.y, r.mx.y), or_fmax(l.mx.z, r.mx.z));
  return o;
}
/* aabb.rs:42-61 (unused by the render path; kept for the unit tests) */
static int aabb_hit(aabb_t b, const ray_t* r, double t_min, double t_max) {
  for (int a = 0; a < 3; ++a) {
    double mn = vget(b.mn, a), mx = vget(b.mx, a), o = vget(r->o, a), d = vget(r->d, a);
    double t0 = or_fmin((mn - o) / d, (mx - o) / d);
    double t1 = or_fmax((mn - o) / d, (mx - o) / d);
    t_min = or_fmax(t0, t_min);
    t_max = or_fmin(t1, t_max);
    if (t_max <= t_min) return 0;
  }
  return 1;
}
/* aabb.rs:62-79 — plain > / < comparisons: a NaN slab bound leaves the interval unchanged */
static int aabb_hit2(aabb_t b, const ray_t* r, double t_min, double t_max) {
  for (int a = 0; a < 3; ++a) {
    double inv_d = 1.0 / vget(r->d, a);
    double t0 = (vget(b.mn, a) - vget(r->o, a)) * inv_d;
    double t1 = (vget(b.mx, a) - vget(r->o, a)) * inv_d;
    if (inv_d < 0.0) { double tmp = t0; t0 = t1; t1 = tmp; }
    t_min = (t0 > t_min) ? t0 : t_min;
    t_max = (t1 < t_max) ? t1 : t_max;
    if (t_max <= t_min) return 0;
  }
  return 1;
}
/* aabb.rs:81-86 — named `area` but is the volume */
static double aabb_area(aabb_t b) {
  double x = b.mx.x - b.mn.x, y = b.mx.y - b.mn.y, z = b.mx.z - b.mn.z;
  return x * y * z;
}

/* ------------------------------------------------------------------------------------------ */
/* geometry                                                                                     */
/* ------------------------------------------------------------------------------------------ */
typedef struct hit_t {
  v3 point, normal;
  double t;
  int front_face;
  double u, v;
} hit_t;

/* hittable.rs:16-38 */
static hit_t make_hit(const ray_t* in, v3 point, v3 normal, double t, double u, double v) {
  hit_t h;
  h.front_face = vdot(in->d, normal) < 0.0;
  if (!h.front_face) normal = vscale(normal, -1.0);
  h.point = point; h.normal = normal; h.t = t; h.u = u; h.v = v;
  return h;
}

static const double PI_ = 3.14159265358979323846;

/* statistics hook (tools/sphere_stats.c): outcome k = 0 miss (disc < 0), 1 no root in range, 2 hit */
#ifndef OR_SPHERE_STAT
#define OR_SPHERE_STAT(k, oc, d, half_b, cc, radius, disc)
#endif

/* sphere.rs:28-52 (+ get_uv 17-26) */
static int sphere_hit(const double* p, const ray_t* r, double t_min, double t_max, hit_t* out) {
  v3 c = V(p[0], p[1], p[2]);
  double radius = p[3];
  v3 oc = vsub(r->o, c);
  double a = vlen2(r->d);
  double half_b = vdot(oc, r->d);
  double cc = vlen2(oc) - radius * radius;
  double disc = half_b * half_b - a * cc;
  if (disc < 0.0) {
    OR_SPHERE_STAT(0, oc, r->d, half_b, cc, radius, disc);
    return 0;
  }
  double sqrt_d = sqrt(disc);
  double root = (-half_b - sqrt_d) / a;
  if (root < t_min || t_max < root) {
    root = (-half_b + sqrt_d) / a;
    if (root < t_min || t_max < root) {
      OR_SPHERE_STAT(1, oc, r->d, half_b, cc, radius, disc);
      return 0;
    }
  }
  OR_SPHERE_STAT(2, oc, r->d, half_b, cc, radius, disc);
  v3 point = ray_at(r, root);
  v3 normal = vscale(vsub(point, c), 1.0 / radius);
  double theta = OR_ACOS(-normal.y);
  double phi = OR_ATAN2(-normal.z, normal.x) + PI_;
  double u = phi / (2.0 * PI_);
  double v = theta / PI_;
  *out = make_hit(r, point, normal, root, u, v);
  return 1;
}

/* rect.rs:54-80; Rect<D1,D2> with normal axis n = 3-D1-D2; q = {d1_min,d1_max,d2_min,d2_max,offset} */
static int rect_hit(int D1, int D2, const double* q, const ray_t* r, double t_min, double t_max, hit_t* out) {
  int n = 3 - D1 - D2;
  double t = (q[4] - vget(r->o, n)) / vget(r->d, n);
  if (t < t_min || t > t_max) return 0;
  double d1v = vget(r->o, D1) + t * vget(r->d, D1);
  double d2v = vget(r->o, D2) + t * vget(r->d, D2);
  if (d1v < q[0] || d1v > q[1] || d2v < q[2] || d2v > q[3]) return 0;
  double u = (d1v - q[0]) / (q[1] - q[0]);
  double v = (d2v - q[2]) / (q[3] - q[2]);
  v3 normal = V(0.0, 0.0, 0.0);
  vset(&normal, n, 1.0);
  v3 point = ray_at(r, t);
  *out = make_hit(r, point, normal, t, u, v);
  return 1;
}

static void geom_axes(int kind, int* D1, int* D2) {
  if (kind == RT_GEOM_RECT_XY) { *D1 = 0; *D2 = 1; }
  else if (kind == RT_GEOM_RECT_YZ) { *D1 = 1; *D2 = 2; }
  else { *D1 = 0; *D2 = 2; }
}

/* rect.rs:132-144 check_closer + 146-156 RectBox::hit; sides per RectBox::new (rect.rs:111-129) */
static int rectbox_hit(const double* b, const ray_t* r, double t_min, double t_max, hit_t* out) {
  double p0x = b[0], p0y = b[1], p0z = b[2], p1x = b[3], p1y = b[4], p1z = b[5];
  double sides[6][5] = {
      {p0x, p1x, p0y, p1y, p1z}, {p0x, p1x, p0y, p1y, p0z}, /* xy_sides */
      {p0y, p1y, p0z, p1z, p1x}, {p0y, p1y, p0z, p1z, p0x}, /* yz_sides */
      {p0x, p1x, p0z, p1z, p1y}, {p0x, p1x, p0z, p1z, p0y}, /* xz_sides */
  };
  int kinds[6] = {RT_GEOM_RECT_XY, RT_GEOM_RECT_XY, RT_GEOM_RECT_YZ, RT_GEOM_RECT_YZ, RT_GEOM_RECT_XZ, RT_GEOM_RECT_XZ};
  int have = 0;
  hit_t best;
  for (int s = 0; s < 6; ++s) {
    double t_closest = have ? best.t : t_max;
    int D1, D2;
    geom_axes(kinds[s], &D1, &D2);
    hit_t h;
    if (rect_hit(D1, D2, sides[s], r, t_min, t_closest, &h)) { best = h; have = 1; }
  }
  if (have) *out = best;
  return have;
}

/* ------------------------------------------------------------------------------------------ */
/* book-2 ("The Next Week") extensions — ABSENT from the reference;  */
/* restated from the book's moving_sphere.h / constant_medium.h / rotate_y / translate / camera */
/* time, with the deviations DESIGN.md §10 states.  PARITY UNPINNED (no reference to compare). */
/* ------------------------------------------------------------------------------------------ */
/* the path key of the ray being traced: side streams for the ray time and a medium's free flight */
typedef struct hctx_t {
  uint64_t seed;
  uint32_t pixel, sample, draw;
  double time0, time1;
} hctx_t;

/* side stream: Philox4x32-10 at counter (c0, sample, pixel, stream), stream >= 2^30 */
static double side_draw(uint64_t seed, uint32_t c0, uint32_t sample, uint32_t pixel, uint32_t stream) {
  uint32_t ctr[4] = {c0, sample, pixel, stream};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  or_philox4x32_10(ctr, key, o);
  return u64_to_f64((uint64_t)o[0] | ((uint64_t)o[1] << 32));
}
#define STREAM_TIME 0x40000000u
#define STREAM_MEDIUM 0x80000000u

/* camera.h get_ray: time = random_double(time0, time1) (from the path's time stream) */
static double ray_time(const hctx_t* cx) {
  return cx->time0 + (cx->time1 - cx->time0) * side_draw(cx->seed, 0u, cx->sample, cx->pixel, STREAM_TIME);
}
/* moving_sphere.h center(time) */
static v3 moving_center(const rt_object* o, double tm) {
  v3 c0 = V(o->p[0], o->p[1], o->p[2]), c1 = V(o->q[0], o->q[1], o->q[2]);
  return vadd(c0, vscale(vsub(c1, c0), (tm - o->q[3]) / (o->q[4] - o->q[3])));
}
static int object_hit(const rt_object* o, const ray_t* r, double t_min, double t_max, hit_t* out);
static int sphere_hit(const double* p, const ray_t* r, double t_min, double t_max, hit_t* out);
/* the object's own shape (reference geometry, or moving_sphere.h hit at the ray's time) */
static int shape_hit(const rt_object* o, const ray_t* r, double t_min, double t_max, const hctx_t* cx, hit_t* out) {
  if (o->geometry == RT_GEOM_MOVING_SPHERE) {
    v3 c = moving_center(o, ray_time(cx));
    double p[4] = {c.x, c.y, c.z, o->p[3]};
    return sphere_hit(p, r, t_min, t_max, out);
  }
  return object_hit(o, r, t_min, t_max, out);
}
/* constant_medium.h hit with the shape as boundary (t2 not clamped to t_max; the scatter t is
 * compared with t_max instead — equal in exact arithmetic, order-independent); the free-flight
 * uniform comes from the medium stream keyed by (draw index of the path, object index). */
static int medium_hit(const rt_object* o, int32_t obj, const ray_t* r, double t_min, double t_max,
                      const hctx_t* cx, hit_t* out) {
  hit_t rec1, rec2;
  if (!shape_hit(o, r, -INFINITY, INFINITY, cx, &rec1)) return 0;
  if (!shape_hit(o, r, rec1.t + 0.0001, INFINITY, cx, &rec2)) return 0;
  if (rec1.t < t_min) rec1.t = t_min;
  if (rec1.t >= rec2.t) return 0;
  if (rec1.t < 0) rec1.t = 0;
  double ray_length = vlen(r->d);
  double distance_inside_boundary = (rec2.t - rec1.t) * ray_length;
  double neg_inv_density = -1.0 / o->density;
  double hit_distance = neg_inv_density * OR_LOG(side_draw(cx->seed, cx->draw, cx->sample, cx->pixel,
                                                        STREAM_MEDIUM | (uint32_t)obj));
  if (hit_distance > distance_inside_boundary) return 0;
  double t = rec1.t + hit_distance / ray_length;
  if (t > t_max) return 0;
  out->t = t;
  out->point = ray_at(r, t);
  out->normal = V(1.0, 0.0, 0.0); /* arbitrary */
  out->front_face = 1;            /* also arbitrary */
  out->u = out->v = 0.0;
  return 1;
}
static void rotate_y_cs(const rt_object* o, double* cs, double* sn) {
  double radians = o->rotate_y_deg * PI_ / 180.0;
  *cs = cos(radians);
  *sn = sin(radians);
}
/* translate(rotate_y(inner)): Translate::hit moves the ray by -offset, RotateY::hit rotates it,
 * the inner hit's point and normal are rotated back and translated (front_face kept). */
static int ext_object_hit(const rt_object* o, int32_t obj, const ray_t* r, double t_min, double t_max,
                          const hctx_t* cx, hit_t* out) {
  if (!o->transform) {
    if (o->medium) return medium_hit(o, obj, r, t_min, t_max, cx, out);
    return shape_hit(o, r, t_min, t_max, cx, out);
  }
  v3 off = V(o->offset[0], o->offset[1], o->offset[2]);
  double cs, sn;
  rotate_y_cs(o, &cs, &sn);
  ray_t moved = {vsub(r->o, off), r->d};
  ray_t rot;
  rot.o = V(cs * moved.o.x - sn * moved.o.z, moved.o.y, sn * moved.o.x + cs * moved.o.z);
  rot.d = V(cs * moved.d.x - sn * moved.d.z, moved.d.y, sn * moved.d.x + cs * moved.d.z);
  hit_t h;
  int ok = o->medium ? medium_hit(o, obj, &rot, t_min, t_max, cx, &h) : shape_hit(o, &rot, t_min, t_max, cx, &h);
  if (!ok) return 0;
  v3 p = h.point, n = h.normal;
  h.point = vadd(V(cs * p.x + sn * p.z, p.y, -sn * p.x + cs * p.z), off);
  h.normal = V(cs * n.x + sn * n.z, n.y, -sn * n.x + cs * n.z);
  *out = h;
  return 1;
}
static int is_extended(const rt_object* o) {
  return o->geometry == RT_GEOM_MOVING_SPHERE || o->medium || o->transform;
}

/* object.rs:45-58 */
static int object_hit(const rt_object* o, const ray_t* r, double t_min, double t_max, hit_t* out) {
  switch (o->geometry) {
    case RT_GEOM_SPHERE: return sphere_hit(o->p, r, t_min, t_max, out);
    case RT_GEOM_RECT_XY:
    case RT_GEOM_RECT_YZ:
    case RT_GEOM_RECT_XZ: {
      int D1, D2;
      geom_axes(o->geometry, &D1, &D2);
      return rect_hit(D1, D2, o->p, r, t_min, t_max, out);
    }
    case RT_GEOM_RECT_BOX: return rectbox_hit(o->p, r, t_min, t_max, out);
  }
  return 0;
}

static int reference_bbox(const rt_object* o, aabb_t* out);
/* bounding boxes of book-2 objects: moving_sphere.h (boxes at time0 and time1, surrounded),
 * rotate_y.h (8 rotated corners), translate (+offset), constant_medium.h (the boundary's) */
static int object_bbox(const rt_object* o, aabb_t* out) {
  aabb_t b;
  if (o->geometry == RT_GEOM_MOVING_SPHERE) {
    v3 rr = V(o->p[3], o->p[3], o->p[3]);
    v3 c0 = moving_center(o, o->q[3]), c1 = moving_center(o, o->q[4]);
    aabb_t b0 = {vsub(c0, rr), vadd(c0, rr)}, b1 = {vsub(c1, rr), vadd(c1, rr)};
    b = surrounding(b0, b1);
  } else if (!reference_bbox(o, &b)) {
    return 0;
  }
  if (o->transform) {
    double cs, sn;
    rotate_y_cs(o, &cs, &sn);
    v3 mn = V(INFINITY, INFINITY, INFINITY), mx = V(-INFINITY, -INFINITY, -INFINITY);
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          double x = i * b.mx.x + (1 - i) * b.mn.x;
          double y = j * b.mx.y + (1 - j) * b.mn.y;
          double z = k * b.mx.z + (1 - k) * b.mn.z;
          double newx = cs * x + sn * z;
          double newz = -sn * x + cs * z;
          v3 tester = V(newx, y, newz);
          for (int c = 0; c < 3; c++) {
            vset(&mn, c, fmin(vget(mn, c), vget(tester, c)));
            vset(&mx, c, fmax(vget(mx, c), vget(tester, c)));
          }
        }
    v3 off = V(o->offset[0], o->offset[1], o->offset[2]);
    b.mn = vadd(mn, off);
    b.mx = vadd(mx, off);
  }
  *out = b;
  return 1;
}

/* sphere.rs:54-60 (signed radius), rect.rs:82-99 (BBOX_WIDTH = 1e-4), rect.rs:158-163 */
static int reference_bbox(const rt_object* o, aabb_t* out) {
  switch (o->geometry) {
    case RT_GEOM_SPHERE: {
      v3 c = V(o->p[0], o->p[1], o->p[2]);
      double rr = o->p[3];
      v3 rv = V(rr, rr, rr);
      out->mn = vsub(c, rv);
      out->mx = vadd(c, rv);
      return 1;
    }
    case RT_GEOM_RECT_XY:
    case RT_GEOM_RECT_YZ:
    case RT_GEOM_RECT_XZ: {
      int D1, D2;
      geom_axes(o->geometry, &D1, &D2);
      int n = 3 - D1 - D2;
      v3 mn = V(0, 0, 0), mx = V(0, 0, 0);
      vset(&mn, D1, o->p[0]);
      vset(&mn, D2, o->p[2]);
      vset(&mn, n, o->p[4] - 0.0001);
      vset(&mx, D1, o->p[1]);
      vset(&mx, D2, o->p[3]);
      vset(&mx, n, o->p[4] + 0.0001);
      out->mn = mn;
      out->mx = mx;
      return 1;
    }
    case RT_GEOM_RECT_BOX:
      out->mn = V(o->p[0], o->p[1], o->p[2]);
      out->mx = V(o->p[3], o->p[4], o->p[5]);
      return 1;
  }
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* scene + BBox tree (scene/mod.rs:111-137, bvh/bbox_tree.rs, bvh/bbox_tree/constructor.rs)     */
/* ------------------------------------------------------------------------------------------ */
typedef struct node_t {
  aabb_t bbox;
  int32_t leaf; /* >= 0: NodePointer::Leaf(idx); -1: Branch */
  int32_t lhs, rhs;
} node_t;

struct or_scene {
  rt_scene_desc desc; /* deep copy */
  rt_object* objects;
  rt_material* materials;
  rt_texture* textures;
  rt_perlin_table* perlin;
  rt_image* images;
  uint8_t** image_pixels;
  node_t* tree;
  int32_t n_tree;
  int32_t root; /* -1 = empty tree (BboxTree.root = None) */
};

/* f64::total_cmp (used by sorted_with_idx, constructor.rs:53-57, and split_best's min_by) */
static int total_cmp(double a, double b) {
  int64_t ia, ib;
  memcpy(&ia, &a, 8);
  memcpy(&ib, &b, 8);
  ia ^= (int64_t)(((uint64_t)(ia >> 63)) >> 1);
  ib ^= (int64_t)(((uint64_t)(ib >> 63)) >> 1);
  return (ia < ib) ? -1 : (ia > ib ? 1 : 0);
}

typedef struct iv_t {
  int32_t idx;
  double v;
} iv_t;
/* constructor.rs:53-57 sort_unstable_by total_cmp.  Rust's unstable sort leaves the order of
 * equal keys implementation-defined; the oracle breaks ties by index (documented in DESIGN.md:
 * tree shape under tied keys is unpinned; hits are tree-independent up to measure-zero ties). */
static int iv_cmp(const void* pa, const void* pb) {
  const iv_t* a = (const iv_t*)pa;
  const iv_t* b = (const iv_t*)pb;
  int c = total_cmp(a->v, b->v);
  if (c) return c;
  return (a->idx > b->idx) - (a->idx < b->idx);
}

typedef struct build_t {
  const aabb_t* leaf_box;
  int32_t n;
  iv_t* order[3]; /* x_min, y_min, z_min */
  node_t* tree;
  int32_t n_tree;
  uint8_t* mark; /* scratch membership */
} build_t;

/* set = list of leaf indices; membership tests use `mark` like HashSet::contains */
static double set_volume(const build_t* b, const int32_t* set, int32_t n) {
  /* aabb.rs:6-16 bounding() over the set (order-independent union) + area(); empty -> 0.0 */
  if (n == 0) return 0.0;
  aabb_t acc = b->leaf_box[set[0]];
  for (int32_t i = 1; i < n; ++i) acc = surrounding(acc, b->leaf_box[set[i]]);
  return aabb_area(acc);
}

/* constructor.rs:63-79 split_median */
static void split_median(build_t* b, const iv_t* order, int32_t n_in, int32_t* lhs, int32_t* nl, int32_t* rhs,
                         int32_t* nr) {
  *nl = 0;
  *nr = 0;
  for (int32_t k = 0; k < b->n; ++k) {
    int32_t idx = order[k].idx;
    if (!b->mark[idx]) continue;
    if (*nl < n_in / 2) lhs[(*nl)++] = idx;
    else rhs[(*nr)++] = idx;
  }
}

/* constructor.rs:81-110 split_space */
static void split_space(build_t* b, const iv_t* order, int32_t n_in, int32_t* lhs, int32_t* nl, int32_t* rhs,
                        int32_t* nr, iv_t* avail) {
  int32_t na = 0;
  for (int32_t k = 0; k < b->n; ++k)
    if (b->mark[order[k].idx]) avail[na++] = order[k];
  (void)n_in;
  double mid = (avail[na - 1].v + avail[0].v) / 2.0;
  *nl = 0;
  *nr = 0;
  for (int32_t k = 0; k < na; ++k) {
    if (k == 0) { lhs[(*nl)++] = avail[k].idx; continue; }
    if (avail[k].v < mid) lhs[(*nl)++] = avail[k].idx;
    else rhs[(*nr)++] = avail[k].idx;
  }
}

/* constructor.rs:168-198 partition_nodes (+ split_best 137-166). Returns the node (not pushed). */
static node_t partition_nodes(build_t* b, const int32_t* set, int32_t n) {
  if (n == 1) {
    node_t leaf;
    leaf.bbox = b->leaf_box[set[0]];
    leaf.leaf = set[0];
    leaf.lhs = leaf.rhs = -1;
    return leaf;
  }
  int32_t* cand = (int32_t*)malloc(sizeof(int32_t) * (size_t)n * 12);
  iv_t* avail = (iv_t*)malloc(sizeof(iv_t) * (size_t)n);
  int32_t nl[6], nr[6];
  int32_t* L[6];
  int32_t* R[6];
  for (int s = 0; s < 6; ++s) { L[s] = cand + (size_t)n * (2 * s); R[s] = cand + (size_t)n * (2 * s + 1); }
  for (int32_t i = 0; i < n; ++i) b->mark[set[i]] = 1;
  /* split order: xmin_median, xmin_space, ymin_median, ymin_space, zmin_median, zmin_space */
  for (int a = 0; a < 3; ++a) {
    split_median(b, b->order[a], n, L[2 * a], &nl[2 * a], R[2 * a], &nr[2 * a]);
    split_space(b, b->order[a], n, L[2 * a + 1], &nl[2 * a + 1], R[2 * a + 1], &nr[2 * a + 1], avail);
  }
  for (int32_t i = 0; i < n; ++i) b->mark[set[i]] = 0;
  /* min_by(total_cmp): first minimum wins */
  int best = 0;
  double best_score = 0.0;
  for (int s = 0; s < 6; ++s) {
    double score = set_volume(b, L[s], nl[s]) + set_volume(b, R[s], nr[s]);
    if (s == 0 || total_cmp(score, best_score) < 0) { best = s; best_score = score; }
  }
  free(avail);
  int32_t* ls = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  int32_t nls = nl[best], nrs = nr[best];
  memcpy(ls, L[best], sizeof(int32_t) * (size_t)nls);
  memcpy(ls + nls, R[best], sizeof(int32_t) * (size_t)nrs);
  free(cand);
  node_t lhs = partition_nodes(b, ls, nls);
  node_t rhs = partition_nodes(b, ls + nls, nrs);
  free(ls);
  node_t parent;
  parent.bbox = surrounding(lhs.bbox, rhs.bbox);
  parent.leaf = -1;
  parent.lhs = b->n_tree;
  b->tree[b->n_tree++] = lhs;
  parent.rhs = b->n_tree;
  b->tree[b->n_tree++] = rhs;
  return parent;
}

static void* dupmem(const void* p, size_t n) {
  if (n == 0 || !p) return NULL;
  void* q = malloc(n);
  memcpy(q, p, n);
  return q;
}

/* Does texture ti read the hit's u, v?  Only an image leaf does (image_texture.rs:34-56). */
static int texture_uses_uv(const rt_scene_desc* d, int32_t ti) {
  if (ti < 0 || ti >= d->n_textures) return 0;
  const rt_texture* t = &d->textures[ti];
  if (t->kind == RT_TEX_IMAGE) return 1;
  if (t->kind == RT_TEX_CHECKER) return texture_uses_uv(d, t->odd) || texture_uses_uv(d, t->even);
  return 0;
}
/* Book-2 (extension): Translate(RotateY(sphere)) of a plain sphere is the sphere about the moved
 * centre, so such an instance is flattened into a world-space sphere before anything else reads it —
 * centre (cs cx + sn cz + off.x, cy + off.y, -sn cx + cs cz + off.z), the same formula that maps an
 * instance's hit point back to the world (ext_object_hit) — and takes the reference sphere path.  The
 * host (rt_api.cpp flat_object) flattens by the same rule.  t, point and normal agree with per-ray
 * instancing in real arithmetic (the records differ at the last bit); u, v do not under a
 * rotation, so a rotated sphere is flattened only when its material never reads them, and keeps its
 * angle (transform = 0) for the hit query's u, v (or_scene_hit_at). */
static void flatten_instanced_sphere(const rt_scene_desc* d, rt_object* o) {
  if (o->geometry != RT_GEOM_SPHERE || !o->transform || o->medium) return;
  if (o->rotate_y_deg != 0.0 &&
      (o->material < 0 || o->material >= d->n_materials || texture_uses_uv(d, d->materials[o->material].texture)))
    return;
  double cs, sn;
  rotate_y_cs(o, &cs, &sn);
  const double cx = o->p[0], cy = o->p[1], cz = o->p[2];
  o->p[0] = (cs * cx + sn * cz) + o->offset[0];
  o->p[1] = cy + o->offset[1];
  o->p[2] = (-sn * cx + cs * cz) + o->offset[2];
  o->transform = 0;
  o->offset[0] = o->offset[1] = o->offset[2] = 0.0;
}

or_scene* or_scene_new(const rt_scene_desc* d) {
  if (!d || d->n_objects < 0) return NULL;
  or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
  s->desc = *d;
  s->objects = (rt_object*)dupmem(d->objects, sizeof(rt_object) * (size_t)d->n_objects);
  for (int32_t i = 0; i < d->n_objects; ++i) flatten_instanced_sphere(d, &s->objects[i]);
  s->desc.objects = s->objects;
  s->materials = (rt_material*)dupmem(d->materials, sizeof(rt_material) * (size_t)d->n_materials);
  s->textures = (rt_texture*)dupmem(d->textures, sizeof(rt_texture) * (size_t)d->n_textures);
  s->perlin = (rt_perlin_table*)dupmem(d->perlin, sizeof(rt_perlin_table) * (size_t)d->n_perlin);
  s->images = (rt_image*)dupmem(d->images, sizeof(rt_image) * (size_t)d->n_images);
  if (d->n_images > 0) {
    s->image_pixels = (uint8_t**)calloc((size_t)d->n_images, sizeof(uint8_t*));
    for (int32_t i = 0; i < d->n_images; ++i) {
      size_t nb = (size_t)d->images[i].width * (size_t)d->images[i].height * 3;
      s->image_pixels[i] = (uint8_t*)dupmem(d->images[i].rgb, nb);
      s->images[i].rgb = s->image_pixels[i];
    }
  }
  s->root = -1;
  int32_t n = d->n_objects;
  if (n > 0) {
    /* constructor.rs:9-36 construct_tree: every geometry is bounded, so all objects are leaves */
    aabb_t* boxes = (aabb_t*)malloc(sizeof(aabb_t) * (size_t)n);
    for (int32_t i = 0; i < n; ++i) object_bbox(&s->objects[i], &boxes[i]);
    build_t b;
    b.leaf_box = boxes;
    b.n = n;
    for (int a = 0; a < 3; ++a) {
      b.order[a] = (iv_t*)malloc(sizeof(iv_t) * (size_t)n);
      for (int32_t i = 0; i < n; ++i) { b.order[a][i].idx = i; b.order[a][i].v = vget(boxes[i].mn, a); }
      qsort(b.order[a], (size_t)n, sizeof(iv_t), iv_cmp);
    }
    b.tree = (node_t*)malloc(sizeof(node_t) * (size_t)(2 * n));
    b.n_tree = 0;
    b.mark = (uint8_t*)calloc((size_t)n, 1);
    int32_t* all = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    for (int32_t i = 0; i < n; ++i) all[i] = i;
    node_t root = partition_nodes(&b, all, n);
    s->root = b.n_tree;
    b.tree[b.n_tree++] = root;
    s->tree = b.tree;
    s->n_tree = b.n_tree;
    free(all);
    free(b.mark);
    for (int a = 0; a < 3; ++a) free(b.order[a]);
    free(boxes);
  }
  return s;
}

void or_scene_free(or_scene* s) {
  if (!s) return;
  for (int32_t i = 0; i < s->desc.n_images; ++i) free(s->image_pixels[i]);
  free(s->image_pixels);
  free(s->objects); free(s->materials); free(s->textures); free(s->perlin); free(s->images);
  free(s->tree);
  free(s);
}

int32_t or_tree_size(const or_scene* s) { return s->n_tree; }
int32_t or_tree_root(const or_scene* s) { return s->root; }
void or_tree_node(const or_scene* s, int32_t idx, double bbox[6], int32_t* leaf, int32_t* lhs, int32_t* rhs) {
  box_to(s->tree[idx].bbox, bbox);
  *leaf = s->tree[idx].leaf;
  *lhs = s->tree[idx].lhs;
  *rhs = s->tree[idx].rhs;
}

typedef struct work_t {
  int32_t* stack; /* BboxTreeWorkspace (bbox_tree.rs:38-41) */
  or_counters cnt;
  hctx_t ctx;     /* key of the path being traced (book-2 extensions only) */
} work_t;

/* bbox_tree.rs:56-91 hit_workspace */
static int tree_hit(const or_scene* s, work_t* w, const ray_t* r, double t_min, double t_max, hit_t* out,
                    int32_t* obj) {
  if (s->root < 0) return 0;
  int32_t sp = 0;
  w->stack[sp++] = s->root;
  int have = 0;
  hit_t closest;
  while (sp > 0) {
    int32_t ni = w->stack[--sp];
    double t_closest = have ? closest.t : t_max;
    const node_t* node = &s->tree[ni];
    w->cnt.node_visits++;
    if (!aabb_hit2(node->bbox, r, t_min, t_closest)) continue;
    if (node->leaf < 0) {
      w->stack[sp++] = node->lhs;
      w->stack[sp++] = node->rhs;
    } else {
      hit_t h;
      w->cnt.prim_tests++;
      const rt_object* o = &s->objects[node->leaf];
      int ok = is_extended(o) ? ext_object_hit(o, node->leaf, r, t_min, t_closest, &w->ctx, &h)
                              : object_hit(o, r, t_min, t_closest, &h);
      if (ok) { closest = h; have = 1; *obj = node->leaf; }
    }
  }
  if (have) *out = closest;
  return have;
}

/* scene/mod.rs:152-164: the unbounded HitList is always empty (every geometry is bounded) */
static int scene_hit(const or_scene* s, work_t* w, const ray_t* r, double t_min, double t_max, hit_t* out,
                     int32_t* obj) {
  return tree_hit(s, w, r, t_min, t_max, out, obj);
}

/* ------------------------------------------------------------------------------------------ */
/* textures                                                                                     */
/* ------------------------------------------------------------------------------------------ */
static int32_t sat_i32(double x) {
  if (isnan(x)) return 0;
  if (x >= 2147483647.0) return 2147483647;
  if (x <= -2147483648.0) return (int32_t)(-2147483647 - 1);
  return (int32_t)x;
}

/* perlin/mod.rs:87-109 noise + InterpolationKernel::interp 40-63 */
static double perlin_noise(const rt_perlin_table* T, v3 p) {
  double xf = floor(p.x), yf = floor(p.y), zf = floor(p.z);
  double u = p.x - xf, v = p.y - yf, w = p.z - zf;
  /* `xf as i32 as usize`: saturating cast, then sign-extension (so -1 -> ...FF -> & 0xFF = 255) */
  uint64_t i = (uint64_t)(int64_t)sat_i32(xf);
  uint64_t j = (uint64_t)(int64_t)sat_i32(yf);
  uint64_t k = (uint64_t)(int64_t)sat_i32(zf);
  v3 c[2][2][2];
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        int32_t idx = T->perm_x[(i + di) & 0xFF] ^ T->perm_y[(j + dj) & 0xFF] ^ T->perm_z[(k + dk) & 0xFF];
        c[di][dj][dk] = V(T->ranfloat[idx][0], T->ranfloat[idx][1], T->ranfloat[idx][2]);
      }
  double accum = 0.0;
  double uu = u * u * (3.0 - 2.0 * u);
  double vv = v * v * (3.0 - 2.0 * v);
  double ww = w * w * (3.0 - 2.0 * w);
  for (int di = 0; di < 2; ++di) {
    double fi = (double)di;
    for (int dj = 0; dj < 2; ++dj) {
      double fj = (double)dj;
      for (int dk = 0; dk < 2; ++dk) {
        double fk = (double)dk;
        v3 weight = V(u - fi, v - fj, w - fk);
        accum += (fi * uu + (1.0 - fi) * (1.0 - uu)) * (fj * vv + (1.0 - fj) * (1.0 - vv)) *
                 (fk * ww + (1.0 - fk) * (1.0 - ww)) * vdot(c[di][dj][dk], weight);
      }
    }
  }
  return accum;
}

/* perlin/mod.rs:111-124 */
static double perlin_turbulence(const rt_perlin_table* T, v3 p, int depth) {
  double accum = 0.0;
  v3 tp = p;
  double weight = 1.0;
  for (int i = 0; i < depth; ++i) {
    accum += weight * perlin_noise(T, tp);
    weight *= 0.5;
    tp = vscale(tp, 2.0);
  }
  return fabs(accum);
}

/* nalgebra::clamp(val, min, max) */
static double nclamp(double x, double mn, double mx) { return (x > mn) ? ((x < mx) ? x : mx) : mn; }
static uint32_t sat_u32(double x) {
  if (isnan(x) || x <= 0.0) return 0;
  if (x >= 4294967295.0) return 4294967295u;
  return (uint32_t)x;
}

static v3 texture_value(const or_scene* s, int32_t ti, double u, double v, v3 p) {
  for (;;) {
    const rt_texture* t = &s->textures[ti];
    switch (t->kind) {
      case RT_TEX_SOLID: /* solid.rs:17-21 */
        return V(t->color[0], t->color[1], t->color[2]);
      case RT_TEX_CHECKER: { /* checker.rs:27-37 */
        double sines = OR_SIN(t->scale * p.x) * OR_SIN(t->scale * p.y) * OR_SIN(t->scale * p.z);
        ti = (sines < 0.0) ? t->odd : t->even;
        continue;
      }
      case RT_TEX_PERLIN: { /* perlin/mod.rs:162-183 (marble) */
        const rt_perlin_table* T = &s->perlin[t->table];
        double turb = 10.0 * perlin_turbulence(T, p, 7);
        v3 dimm_scale = V(1.0 / 5.0, 1.0 / 10.0, 1.0);
        v3 dimm_weight = vunit(V(0.0, 0.0, 1.0));
        v3 vd = vmul(vscale(dimm_scale, t->scale), p);
        vd = V(OR_SIN(vd.x + turb), OR_SIN(vd.y + turb), OR_SIN(vd.z + turb));
        double total_noise = vdot(vd, dimm_weight);
        double noise = 0.5 * (1.0 + total_noise);
        return vscale(V(1.0, 1.0, 1.0), noise);
      }
      case RT_TEX_IMAGE: { /* image_texture.rs:34-56 */
        const rt_image* im = &s->images[t->table];
        double uu = nclamp(u, 0.0, 1.0);
        double vv = 1.0 - nclamp(v, 0.0, 1.0);
        uint32_t i = sat_u32(uu * (double)(im->width - 1));
        uint32_t j = sat_u32(vv * (double)(im->height - 1));
        double color_scale = 1.0 / 255.0;
        const uint8_t* px = im->rgb + ((size_t)j * (size_t)im->width + i) * 3;
        return V((double)px[0] * color_scale, (double)px[1] * color_scale, (double)px[2] * color_scale);
      }
    }
    return V(0, 0, 0);
  }
}

/* ------------------------------------------------------------------------------------------ */
/* materials (material_type.rs:51-79 dispatch)                                                  */
/* ------------------------------------------------------------------------------------------ */
/* dielectric.rs:15-19 */
static double reflectance(double cosine, double ref_idx) {
  double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * OR_POW5(1.0 - cosine);
}

/* emitted: lighting.rs:21-24 (DiffuseLight), 59-66 (FairyLight); default None (mod.rs:22-24) */
static int material_emitted(const or_scene* s, const rt_material* m, const ray_t* r, const hit_t* h, v3* e) {
  if (m->kind == RT_MAT_DIFFUSE_LIGHT) {
    *e = texture_value(s, m->texture, h->u, h->v, h->point);
    return 1;
  }
  if (m->kind == RT_MAT_FAIRY_LIGHT) {
    v3 src = texture_value(s, m->texture, h->u, h->v, h->point);
    double scale = vdot(h->normal, vscale(r->d, -1.0));
    *e = vscale(src, scale / vlen(r->d));
    return 1;
  }
  return 0;
}

static int material_scatter(const or_scene* s, const rt_material* m, rng_t* rng, const ray_t* r, const hit_t* h,
                            ray_t* out, v3* att) {
  switch (m->kind) {
    case RT_MAT_METAL: { /* metal.rs:26-40 */
      v3 reflected = reflect(vunit(r->d), h->normal);
      out->o = h->point;
      out->d = vadd(reflected, vscale(random_in_unit_sphere(rng), m->param));
      *att = V(m->albedo[0], m->albedo[1], m->albedo[2]);
      return 1;
    }
    case RT_MAT_DIELECTRIC: { /* dielectric.rs:21-49 */
      double ratio = h->front_face ? (1.0 / m->param) : m->param;
      v3 ud = vunit(r->d);
      double cos_theta = or_fmin(vdot(vscale(ud, -1.0), h->normal), 1.0);
      double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
      v3 dir;
      /* `||` short-circuits: the uniform is drawn only when not totally internally reflected */
      if (ratio * sin_theta > 1.0 || reflectance(cos_theta, ratio) > rng_gen(rng)) dir = reflect(ud, h->normal);
      else dir = refract(ud, h->normal, ratio);
      out->o = h->point;
      out->d = dir;
      *att = V(1.0, 1.0, 1.0);
      return 1;
    }
    case RT_MAT_LAMBERTIAN: { /* lambertian.rs:21-37 */
      v3 sc = vadd(h->normal, random_unit_vector(rng));
      if (near_zero(sc)) sc = h->normal;
      out->o = h->point;
      out->d = sc;
      *att = texture_value(s, m->texture, h->u, h->v, h->point);
      return 1;
    }
    case RT_MAT_DIFFUSE_LIGHT: /* lighting.rs:26-28 */
      return 0;
    case RT_MAT_ISOTROPIC: { /* book-2 isotropic (extension): ray(rec.p, random_in_unit_sphere()) */
      out->o = h->point;
      out->d = random_in_unit_sphere(rng);
      *att = texture_value(s, m->texture, h->u, h->v, h->point);
      return 1;
    }
    case RT_MAT_FAIRY_LIGHT: { /* lighting.rs:42-57 */
      v3 sc = vadd(h->normal, random_unit_vector(rng));
      if (near_zero(sc)) sc = h->normal;
      out->o = h->point;
      out->d = sc;
      v3 a = texture_value(s, m->texture, h->u, h->v, h->point);
      *att = vunit(a);
      return 1;
    }
  }
  return 0;
}

/* skybox/mod.rs:5-25 */
static v3 sky_background(const or_scene* s, const ray_t* r) {
  if (s->desc.sky == RT_SKY_ABOVE) {
    v3 unit = vunit(r->d);
    double t = 0.5 * (unit.y + 1.0);
    return vadd(vscale(V(1.0, 1.0, 1.0), 1.0 - t), vscale(V(0.5, 0.7, 1.0), t));
  }
  if (s->desc.sky == RT_SKY_FLAT) return V(s->desc.sky_color[0], s->desc.sky_color[1], s->desc.sky_color[2]);
  return V(0.0, 0.0, 0.0);
}

/* render.rs:17-48 */
static v3 ray_color(const or_scene* s, work_t* w, rng_t* rng, ray_t ray, int32_t max_depth) {
  v3 attenuation = V(1.0, 1.0, 1.0);
  v3 emitted = V(0.0, 0.0, 0.0);
  while (max_depth > 0) {
    hit_t h;
    int32_t obj = -1;
    w->cnt.segments++;
    w->ctx.draw = rng->draw; /* book-2 media key their free flight by the segment's first draw index */
    if (scene_hit(s, w, &ray, 0.001, INFINITY, &h, &obj)) {
      const rt_material* m = &s->materials[s->objects[obj].material];
      v3 e;
      if (material_emitted(s, m, &ray, &h, &e)) emitted = vadd(emitted, vmul(attenuation, e));
      ray_t sc;
      v3 att;
      if (material_scatter(s, m, rng, &ray, &h, &sc, &att)) {
        attenuation = vmul(attenuation, att);
        ray = sc;
      } else {
        break;
      }
    } else {
      emitted = vadd(emitted, vmul(attenuation, sky_background(s, &ray)));
      break;
    }
    max_depth -= 1;
  }
  return emitted;
}

/* camera/mod.rs:97-132 */
static ray_t pixel_ray(const rt_camera* cam, rng_t* rng, double x, double y) {
  double x_percent = x / (double)cam->image_width;
  double y_percent = y / (double)cam->image_height;
  v3 u = V(cam->u[0], cam->u[1], cam->u[2]);
  v3 v = V(cam->v[0], cam->v[1], cam->v[2]);
  v3 w = V(cam->w[0], cam->w[1], cam->w[2]);
  v3 origin = V(cam->origin[0], cam->origin[1], cam->origin[2]);
  v3 horizontal = vscale(u, cam->width * cam->focus_length);
  v3 vertical = vscale(v, cam->height * cam->focus_length);
  v3 lower_left = vsub(vsub(vsub(origin, vscale(horizontal, 0.5)), vscale(vertical, 0.5)),
                       vscale(w, cam->focal_length * cam->focus_length));
  v3 offset = V(0.0, 0.0, 0.0);
  if (cam->has_lens) {
    v3 rd = vscale(random_in_unit_disk(rng), cam->lens_radius);
    offset = vadd(vscale(u, rd.x), vscale(v, rd.y));
  }
  v3 direction = vsub(vsub(vadd(vadd(lower_left, vscale(horizontal, x_percent)), vscale(vertical, y_percent)), origin),
                      offset);
  ray_t r;
  r.o = vadd(origin, offset);
  r.d = direction;
  return r;
}

/* one sample of render_scanline's inner loop (render.rs:60-66) */
static v3 sample_color(const or_scene* s, work_t* w, const rt_camera* cam, const rt_render_params* p, int32_t px,
                       int32_t py, uint32_t sample) {
  rng_t rng;
  rng.seed = p->seed;
  rng.pixel = (uint32_t)py * (uint32_t)cam->image_width + (uint32_t)px;
  rng.sample = sample;
  rng.draw = 0;
  double jx = (double)px + rng_gen(&rng);
  double jy = (double)py + rng_gen(&rng);
  ray_t r = pixel_ray(cam, &rng, jx, jy);
  w->cnt.samples++;
  w->ctx.seed = rng.seed;
  w->ctx.pixel = rng.pixel;
  w->ctx.sample = rng.sample;
  w->ctx.time0 = cam->time0;
  w->ctx.time1 = cam->time1;
  return ray_color(s, w, &rng, r, p->max_depth);
}

static int32_t eff_samples(const rt_render_params* p) { return p->samples == 0 ? 1 : p->samples; }

static void work_init(const or_scene* s, work_t* w) {
  w->stack = (int32_t*)malloc(sizeof(int32_t) * (size_t)(s->n_tree + 2));
  memset(&w->cnt, 0, sizeof(w->cnt));
  memset(&w->ctx, 0, sizeof(w->ctx));
}
static void cnt_add(or_counters* a, const or_counters* b) {
  if (!a) return;
  a->samples += b->samples;
  a->segments += b->segments;
  a->node_visits += b->node_visits;
  a->prim_tests += b->prim_tests;
}

/* render.rs:49-70; samples [sample_begin, sample_begin + sample_count) of the frame's eff_samples (ABI 6
 * sample range, 0 = to the end): render.rs:58-69's loop over that sub-range, summed in order */
static void scanline(const or_scene* s, work_t* w, const rt_camera* cam, const rt_render_params* p, int32_t line,
                     double* buf) {
  int32_t S = eff_samples(p);
  int32_t k0 = p->sample_begin, k1 = p->sample_count ? p->sample_begin + p->sample_count : S;
  if (k0 < 0) k0 = 0;
  if (k1 > S) k1 = S;
  for (int32_t idx = 0; idx < cam->image_width; ++idx) {
    v3 c = V(0.0, 0.0, 0.0);
    for (int32_t k = k0; k < k1; ++k) c = vadd(c, sample_color(s, w, cam, p, idx, line, (uint32_t)k));
    buf[3 * idx + 0] = c.x;
    buf[3 * idx + 1] = c.y;
    buf[3 * idx + 2] = c.z;
  }
}

void or_render_scanline(const or_scene* s, const rt_camera* cam, const rt_render_params* p, int32_t line_idx,
                        double* buf, or_counters* cnt) {
  work_t w;
  work_init(s, &w);
  scanline(s, &w, cam, p, line_idx, buf);
  cnt_add(cnt, &w.cnt);
  free(w.stack);
}

typedef struct pool_t {
  const or_scene* s;
  const rt_camera* cam;
  const rt_render_params* p;
  int32_t line_begin, line_end;
  double* out;
  atomic_int next;
  pthread_mutex_t mu;
  or_counters total;
} pool_t;

static void* pool_worker(void* arg) {
  pool_t* P = (pool_t*)arg;
  work_t w;
  work_init(P->s, &w);
  for (;;) {
    int32_t line = P->line_begin + atomic_fetch_add(&P->next, 1);
    if (line >= P->line_end) break;
    scanline(P->s, &w, P->cam, P->p, line, P->out + (size_t)(line - P->line_begin) * (size_t)P->cam->image_width * 3);
  }
  pthread_mutex_lock(&P->mu);
  cnt_add(&P->total, &w.cnt);
  pthread_mutex_unlock(&P->mu);
  free(w.stack);
  return NULL;
}

int32_t or_render_rows(const or_scene* s, const rt_camera* cam, const rt_render_params* p, int32_t line_begin,
                       int32_t line_end, int32_t nthreads, double* out, or_counters* cnt) {
  if (!s || !cam || !p || !out || line_begin < 0 || line_end > cam->image_height || line_begin > line_end) return 1;
  if (nthreads < 1) nthreads = 1;
  pool_t P;
  P.s = s; P.cam = cam; P.p = p; P.line_begin = line_begin; P.line_end = line_end; P.out = out;
  atomic_init(&P.next, 0);
  pthread_mutex_init(&P.mu, NULL);
  memset(&P.total, 0, sizeof(P.total));
  if (nthreads == 1) {
    pool_worker(&P);
  } else {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int32_t i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, pool_worker, &P);
    for (int32_t i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    free(th);
  }
  pthread_mutex_destroy(&P.mu);
  if (cnt) { memset(cnt, 0, sizeof(*cnt)); cnt_add(cnt, &P.total); }
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* test-facing wrappers                                                                         */
/* ------------------------------------------------------------------------------------------ */
static ray_t ray_from(const double r[6]) { ray_t q = {V(r[0], r[1], r[2]), V(r[3], r[4], r[5])}; return q; }

int32_t or_aabb_hit(const double box[6], const double ray[6], double t_min, double t_max) {
  ray_t r = ray_from(ray);
  return aabb_hit(box_from(box), &r, t_min, t_max);
}
int32_t or_aabb_hit2(const double box[6], const double ray[6], double t_min, double t_max) {
  ray_t r = ray_from(ray);
  return aabb_hit2(box_from(box), &r, t_min, t_max);
}
void or_surrounding_box(const double a[6], const double b[6], double out[6]) {
  box_to(surrounding(box_from(a), box_from(b)), out);
}
double or_aabb_area(const double box[6]) { return aabb_area(box_from(box)); }
int32_t or_object_bbox(const rt_object* obj, double out[6]) {
  aabb_t b;
  if (!object_bbox(obj, &b)) return 0;
  box_to(b, out);
  return 1;
}
static void hit_out(const hit_t* h, int32_t obj, or_hit* out) {
  out->hit = 1; out->object = obj; out->t = h->t;
  out->point[0] = h->point.x; out->point[1] = h->point.y; out->point[2] = h->point.z;
  out->normal[0] = h->normal.x; out->normal[1] = h->normal.y; out->normal[2] = h->normal.z;
  out->front_face = h->front_face; out->u = h->u; out->v = h->v;
}
int32_t or_object_hit(const rt_object* obj, const double ray[6], double t_min, double t_max, or_hit* out) {
  ray_t r = ray_from(ray);
  hit_t h;
  hctx_t cx;
  memset(&cx, 0, sizeof(cx));
  memset(out, 0, sizeof(*out));
  out->object = -1;
  if (!(is_extended(obj) ? ext_object_hit(obj, 0, &r, t_min, t_max, &cx, &h) : object_hit(obj, &r, t_min, t_max, &h)))
    return 0;
  hit_out(&h, -1, out);
  return 1;
}
void or_scene_hit_at(const or_scene* s, const double ray[6], double t_min, double t_max, uint32_t ray_index,
                     or_hit* out) {
  ray_t r = ray_from(ray);
  work_t w;
  work_init(s, &w);
  w.ctx.pixel = ray_index; /* rt_scene_hit's key: (seed 0, pixel = ray index, sample 0, draw 0), time 0 */
  hit_t h;
  int32_t obj = -1;
  memset(out, 0, sizeof(*out));
  out->object = -1;
  if (scene_hit(s, &w, &r, t_min, t_max, &h, &obj)) {
    const rt_object* o = &s->objects[obj];
    if (o->geometry == RT_GEOM_SPHERE && !o->transform && o->rotate_y_deg != 0.0) {
      /* a flattened rotated instance: u, v on its object-frame outward normal (sphere.rs:17-26) */
      double cs, sn;
      rotate_y_cs(o, &cs, &sn);
      v3 n = h.front_face ? h.normal : vscale(h.normal, -1.0);
      v3 on = V(cs * n.x - sn * n.z, n.y, sn * n.x + cs * n.z);
      h.u = (OR_ATAN2(-on.z, on.x) + PI_) / (2.0 * PI_);
      h.v = OR_ACOS(-on.y) / PI_;
    }
    hit_out(&h, obj, out);
  }
  free(w.stack);
}
void or_scene_hit(const or_scene* s, const double ray[6], double t_min, double t_max, or_hit* out) {
  or_scene_hit_at(s, ray, t_min, t_max, 0u, out);
}
void or_texture_value(const or_scene* s, int32_t tex, double u, double v, const double p[3], double out[3]) {
  v3 c = texture_value(s, tex, u, v, V(p[0], p[1], p[2]));
  out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
double or_perlin_noise(const or_scene* s, int32_t table, const double p[3]) {
  return perlin_noise(&s->perlin[table], V(p[0], p[1], p[2]));
}
double or_perlin_turbulence(const or_scene* s, int32_t table, const double p[3], int32_t depth) {
  return perlin_turbulence(&s->perlin[table], V(p[0], p[1], p[2]), depth);
}
void or_pixel_ray(const rt_camera* cam, uint64_t seed, int32_t px, int32_t py, uint32_t sample, double ray[6]) {
  rng_t rng;
  rng.seed = seed;
  rng.pixel = (uint32_t)py * (uint32_t)cam->image_width + (uint32_t)px;
  rng.sample = sample;
  rng.draw = 0;
  double jx = (double)px + rng_gen(&rng);
  double jy = (double)py + rng_gen(&rng);
  ray_t r = pixel_ray(cam, &rng, jx, jy);
  ray[0] = r.o.x; ray[1] = r.o.y; ray[2] = r.o.z; ray[3] = r.d.x; ray[4] = r.d.y; ray[5] = r.d.z;
}
void or_sample_color(const or_scene* s, const rt_camera* cam, const rt_render_params* p, int32_t px, int32_t py,
                     uint32_t sample, double out[3], or_counters* cnt) {
  work_t w;
  work_init(s, &w);
  v3 c = sample_color(s, &w, cam, p, px, py, sample);
  out[0] = c.x; out[1] = c.y; out[2] = c.z;
  cnt_add(cnt, &w.cnt);
  free(w.stack);
}

/* one iteration of ray_color's loop (render.rs:30-46) for a given ray and path key: the closest hit
 * (t in [0.001, inf)), material_type.rs:51-79's emitted and scatter, or the sky on a miss */
void or_probe_segment(const or_scene* s, const double ray[6], uint64_t seed, uint32_t pixel, uint32_t sample,
                      uint32_t draw, or_probe* out) {
  ray_t r = ray_from(ray);
  work_t w;
  work_init(s, &w);
  rng_t rng;
  rng.seed = seed;
  rng.pixel = pixel;
  rng.sample = sample;
  rng.draw = draw;
  w.ctx.seed = seed;
  w.ctx.pixel = pixel;
  w.ctx.sample = sample;
  w.ctx.draw = draw;
  w.ctx.time0 = w.ctx.time1 = 0.0;
  memset(out, 0, sizeof(*out));
  out->object = -1;
  hit_t h;
  int32_t obj = -1;
  if (scene_hit(s, &w, &r, 0.001, INFINITY, &h, &obj)) {
    const rt_material* m = &s->materials[s->objects[obj].material];
    out->object = obj;
    out->front_face = h.front_face;
    out->t = h.t;
    out->point[0] = h.point.x; out->point[1] = h.point.y; out->point[2] = h.point.z;
    out->normal[0] = h.normal.x; out->normal[1] = h.normal.y; out->normal[2] = h.normal.z;
    v3 e;
    if (material_emitted(s, m, &r, &h, &e)) {
      out->emits = 1;
      out->emitted[0] = e.x; out->emitted[1] = e.y; out->emitted[2] = e.z;
    }
    ray_t sc;
    v3 att;
    if (material_scatter(s, m, &rng, &r, &h, &sc, &att)) {
      out->scattered = 1;
      out->attenuation[0] = att.x; out->attenuation[1] = att.y; out->attenuation[2] = att.z;
      out->origin[0] = sc.o.x; out->origin[1] = sc.o.y; out->origin[2] = sc.o.z;
      out->direction[0] = sc.d.x; out->direction[1] = sc.d.y; out->direction[2] = sc.d.z;
    }
  } else {
    v3 e = sky_background(s, &r);
    out->emits = 1;
    out->emitted[0] = e.x; out->emitted[1] = e.y; out->emitted[2] = e.z;
  }
  out->draw = rng.draw;
  free(w.stack);
}
double or_reflectance(double cosine, double ref_idx) { return reflectance(cosine, ref_idx); }

/* image.rs:31-44 + color.rs:31-38: (x * 255.999) as u8 saturates, NaN -> 0 */
static uint8_t to_u8(double x) {
  double y = x * 255.999;
  if (isnan(y) || y <= 0.0) return 0;
  if (y >= 255.0) return 255;
  return (uint8_t)y;
}
void or_tonemap(const double* accum, int32_t width, int32_t height, int32_t samples, uint8_t* rgb8) {
  double inv = 1.0 / (double)samples;
  for (int32_t j = 0; j < height; ++j)
    for (int32_t i = 0; i < width; ++i) {
      const double* c = accum + ((size_t)j * width + i) * 3;
      uint8_t* o = rgb8 + ((size_t)(height - j - 1) * width + i) * 3;
      for (int k = 0; k < 3; ++k) o[k] = to_u8(sqrt(c[k] * inv));
    }
}
