/* CPU check of the megakernel's sphere-box fast accept (rt_device.h leaf_tests4, RT_SPHERE_FAST_ACCEPT):
 * whenever the rule clears a sphere hit, the reference's exact box test on that sphere's bounding box
 * (bvh/aabb.rs:62-79 hit2 via the oracle, on sphere.rs:54-60's box c -+ r) must pass.  The rule:
 *     ray fast (max|o| <= L) && t_min < t < t_best && |fma(t, d_a, fl(o_a - c_a))| < r - 2 m  (every axis)
 * with m = 2^-46 (B + L), B = the largest box plane, L = the origin bound — the values rt_api.cpp uses.
 * Rays: random ones through random spheres, and adversarial ones aimed at the sphere's silhouette, its
 * six tangent points, its box edges, axis-parallel and nearly axis-parallel directions, with t_best
 * placed at, just above and just below the root.  Test infrastructure (tests/test_fast_accept.py).
 *
 * usage: fast_accept_check <n_cases> <seed>  ->  prints "cases N cleared C slab_needed S violations V"
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../oracle/oracle.h"

static uint64_t g_s;
static uint64_t nxt(void) {
  g_s ^= g_s << 13;
  g_s ^= g_s >> 7;
  g_s ^= g_s << 17;
  return g_s;
}
static double uni(void) { return (double)(nxt() >> 11) * (1.0 / 9007199254740992.0); }
static double rng(double a, double b) { return a + (b - a) * uni(); }

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 1000000;
  g_s = argc > 2 ? strtoull(argv[2], NULL, 0) : 0x5EEDull;
  const double B = 30.0;                      /* random_scene: the ground's 30-unit planes */
  const double L = 4.0 * B > 16.0 ? 4.0 * B : 16.0;
  const double m2 = 2.0 * ldexp(B + (double)(float)L, -46);
  long cleared = 0, needed = 0, bad = 0, hits = 0;
  for (long i = 0; i < n; ++i) {
    rt_object sp;
    memset(&sp, 0, sizeof sp);
    sp.geometry = RT_GEOM_SPHERE;
    const double r = (nxt() & 7) == 0 ? rng(1e-3, 2.0) : rng(0.05, 0.25);
    double c[3] = {rng(-11.0, 11.0), rng(0.0, 2.0), rng(-11.0, 11.0)};
    for (int k = 0; k < 3; ++k) sp.p[k] = c[k];
    sp.p[3] = r;
    /* origin: anywhere within L / 4, or right on the sphere (a scattered ray's start) */
    double o[3], d[3];
    const int kind = (int)(nxt() % 8);
    if (kind == 0) {
      double u[3] = {rng(-1, 1), rng(-1, 1), rng(-1, 1)};
      double len = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
      for (int k = 0; k < 3; ++k) o[k] = c[k] + r * u[k] / len;
    } else {
      for (int k = 0; k < 3; ++k) o[k] = rng(-L / 4, L / 4);
    }
    /* target: a point on / near the silhouette, a tangent point, a box corner or edge, or the centre */
    double tg[3];
    const int aim = (int)(nxt() % 6);
    for (int k = 0; k < 3; ++k) tg[k] = c[k];
    if (aim == 1) {
      const int ax = (int)(nxt() % 3);
      tg[ax] += (nxt() & 1 ? r : -r) * (1.0 + rng(-1e-12, 1e-12));
    } else if (aim == 2) {
      for (int k = 0; k < 3; ++k) tg[k] += (nxt() & 1 ? r : -r) * (1.0 + rng(-1e-9, 1e-9));
    } else if (aim == 3) {
      const int ax = (int)(nxt() % 3);
      for (int k = 0; k < 3; ++k)
        if (k != ax) tg[k] += (nxt() & 1 ? r : -r);
    } else if (aim >= 4) {
      double u[3] = {rng(-1, 1), rng(-1, 1), rng(-1, 1)};
      double len = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
      const double s = aim == 4 ? 1.0 + rng(-1e-7, 1e-7) : rng(0.0, 1.0);
      for (int k = 0; k < 3; ++k) tg[k] += r * s * u[k] / len;
    }
    for (int k = 0; k < 3; ++k) d[k] = (tg[k] - o[k]) * rng(0.2, 3.0);
    if ((nxt() & 15) == 0) d[nxt() % 3] = 0.0;                   /* axis-parallel */
    if ((nxt() & 15) == 0) d[nxt() % 3] *= 1e-12;                /* nearly */
    const double ray[6] = {o[0], o[1], o[2], d[0], d[1], d[2]};
    const double t_min = 0.001;
    /* the sphere test at t_best = inf, then again with t_best at / around the root */
    or_hit h;
    if (!or_object_hit(&sp, ray, t_min, INFINITY, &h)) continue;
    ++hits;
    double tb_cand[4] = {INFINITY, h.t, nextafter(h.t, INFINITY), h.t * (1.0 + rng(0.0, 1e-9))};
    for (int q = 0; q < 4; ++q) {
      const double t_best = tb_cand[q];
      or_hit h2;
      if (!or_object_hit(&sp, ray, t_min, t_best, &h2)) continue;
      const double t = h2.t;
      const double mo = fmax(fmax(fabs(o[0]), fabs(o[1])), fabs(o[2]));
      const int fast = mo <= (double)(float)L;
      int sure = fast && t > t_min && t < t_best;
      const double r_in = r - m2;
      for (int k = 0; k < 3 && sure; ++k) sure = fabs(fma(t, d[k], o[k] - c[k])) < r_in;
      double box[6];
      or_object_bbox(&sp, box);
      const int slab = or_aabb_hit2(box, ray, t_min, t_best) != 0;
      if (sure) {
        ++cleared;
        if (!slab) {
          ++bad;
          if (bad < 10)
            fprintf(stderr, "violation: o %.17g %.17g %.17g d %.17g %.17g %.17g c %.17g %.17g %.17g r %.17g t %.17g tb %.17g\n",
                    o[0], o[1], o[2], d[0], d[1], d[2], c[0], c[1], c[2], r, t, t_best);
        }
      } else {
        ++needed;
      }
    }
  }
  printf("cases %ld sphere_hits %ld cleared %ld slab_needed %ld violations %ld\n", n, hits, cleared, needed, bad);
  return bad ? 1 : 0;
}
