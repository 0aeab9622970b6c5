/* Adversarial CPU check of the megakernel's sure-pass rule for sphere leaves (rt_device.h leaf_tests4,
 * RT_SPHERE_SURE): whenever
 *   t_min < t < t_best, max|o_i| <= L, every |d_i| in [2^-300, 2^300], and
 *   |fma(t, d_i, o_i - c_i)| < p5 on every axis, p5 = r - eta rounded down, eta = 2^-48 (B + L),
 * for the sphere root t (sphere.rs:28-46), the reference's box test of the sphere (aabb.rs:62-79 hit2 on
 * c -+ r, with the per-call 1.0 / d) must pass.  Spheres inside the scene bound B (|c_i| + r <= B), rays
 * from inside L, many of them built to graze the box faces, hit the sphere near its poles, start on or
 * near the sphere, or run nearly parallel to an axis.  Prints the counts; exit 1 on any violation.
 * Test infrastructure (tests/test_divisions.py builds and runs it); compile with -ffp-contract=off. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64(void) {
  uint64_t x = s_state;
  x ^= x << 13; x ^= x >> 7; x ^= x << 17;
  return s_state = x;
}
static double unif(void) { return (double)(next_u64() >> 11) * 0x1p-53; }
static double range(double a, double b) { return a + (b - a) * unif(); }

/* sphere.rs:28-46 (t only), the reference's operation order */
static int sphere_t(const double c[3], double r, const double o[3], const double d[3], double t_min, double t_max,
                    double* t) {
  const double oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]};
  const double a = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
  const double hb = (oc[0] * d[0] + oc[1] * d[1]) + oc[2] * d[2];
  const double cc = ((oc[0] * oc[0] + oc[1] * oc[1]) + oc[2] * oc[2]) - r * r;
  const double disc = hb * hb - a * cc;
  if (disc < 0.0) return 0;
  const double sq = sqrt(disc);
  double root = (-hb - sq) / a;
  if (root < t_min || t_max < root) {
    root = (-hb + sq) / a;
    if (root < t_min || t_max < root) return 0;
  }
  *t = root;
  return 1;
}

/* aabb.rs:62-79 hit2 on (c - r, c + r) */
static int hit2(const double c[3], double r, const double o[3], const double d[3], double t_min, double t_max) {
  for (int a = 0; a < 3; ++a) {
    const double inv = 1.0 / d[a];
    double t0 = ((c[a] - r) - o[a]) * inv, t1 = ((c[a] + r) - o[a]) * inv;
    if (inv < 0.0) { const double x = t0; t0 = t1; t1 = x; }
    t_min = t0 > t_min ? t0 : t_min;
    t_max = t1 < t_max ? t1 : t_max;
    if (t_max <= t_min) return 0;
  }
  return 1;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 2000000;
  const double B = 100.0, L = 4.0 * B, t_min = 0.001;
  const double eta = ldexp(B + L, -48);
  long tested = 0, hits = 0, sure = 0, sure_but_reject = 0, pass_not_sure = 0, rejects = 0;
  for (long i = 0; i < n; ++i) {
    const int mode = (int)(next_u64() % 7);
    double r = mode == 5 ? range(1e-6, 1e-3) : range(0.01, 20.0);
    double c[3], o[3], d[3];
    for (int k = 0; k < 3; ++k) c[k] = range(-(B - r), B - r);
    /* a target point: on the sphere near a pole (the box-face tangent points), anywhere on it, or beside it */
    double q[3];
    const int ax = (int)(next_u64() % 3);
    for (int k = 0; k < 3; ++k) q[k] = range(-1.0, 1.0);
    if (mode <= 1) {  /* near a pole: the hit point touches (almost) the box face */
      const double eps = mode == 0 ? ldexp(1.0, -(int)(next_u64() % 50)) : 0.0;
      for (int k = 0; k < 3; ++k) q[k] *= eps;
      q[ax] = (next_u64() & 1) ? 1.0 : -1.0;
    }
    const double qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    double tgt[3];
    for (int k = 0; k < 3; ++k) tgt[k] = c[k] + r * q[k] / qn * range(0.999, 1.001);
    /* origin: anywhere in L, near the target (surface starts), or on an axis-parallel line to it */
    for (int k = 0; k < 3; ++k) o[k] = range(-L, L);
    if (mode == 2) for (int k = 0; k < 3; ++k) o[k] = tgt[k] + range(-1e-3, 1e-3) * r;
    if (mode == 3) { for (int k = 0; k < 3; ++k) o[k] = tgt[k]; o[ax] = tgt[ax] + range(-50.0, 50.0); }
    for (int k = 0; k < 3; ++k) d[k] = tgt[k] - o[k];
    if (mode == 3 || mode == 4) {  /* nearly axis-parallel directions: tiny other components */
      for (int k = 0; k < 3; ++k)
        if (k != ax) d[k] = ldexp(range(-1.0, 1.0), -(int)(next_u64() % 200));
    }
    if (mode == 6) {  /* tangent at a pole, in (or next to) the box face's plane: the box test degenerates */
      double pole[3] = {c[0], c[1], c[2]};
      const double sg = (next_u64() & 1) ? 1.0 : -1.0;
      pole[ax] = c[ax] + sg * r;
      const double back = range(0.5, 30.0);
      for (int k = 0; k < 3; ++k) d[k] = range(-1.0, 1.0);
      d[ax] = (next_u64() & 1) ? 0x1p-290 * range(1.0, 2.0) : ldexp(range(-1.0, 1.0), -(int)(next_u64() % 60));
      for (int k = 0; k < 3; ++k) o[k] = pole[k] - back * d[k];
    }
    int ok = 1;
    for (int k = 0; k < 3; ++k) {
      if (fabs(o[k]) > L) ok = 0;
      if (!(fabs(d[k]) >= 0x1p-300 && fabs(d[k]) <= 0x1p300)) ok = 0;
    }
    if (!ok) continue;
    ++tested;
    const double t_best = (next_u64() & 3) ? INFINITY : range(t_min, 1e3);
    double t;
    if (!sphere_t(c, r, o, d, t_min, t_best, &t)) continue;
    ++hits;
    double p5 = r - eta;
    p5 = p5 > 0.0 ? nextafter(p5, 0.0) : 0.0;
    const int s = t > t_min && t < t_best && fabs(fma(t, d[0], o[0] - c[0])) < p5 &&
                  fabs(fma(t, d[1], o[1] - c[1])) < p5 && fabs(fma(t, d[2], o[2] - c[2])) < p5;
    const int h = hit2(c, r, o, d, t_min, t_best);
    sure += s;
    rejects += !h;
    if (s && !h) ++sure_but_reject;
    if (!s && h) ++pass_not_sure;
  }
  printf("sphere_sure_check: %ld rays in range, %ld sphere hits, %ld box rejects among them, %ld sure, "
         "%ld box passes not sure, %ld sure but box rejects\n", tested, hits, rejects, sure, pass_not_sure,
         sure_but_reject);
  return sure_but_reject ? 1 : 0;
}
