/* Sphere-leaf outcome statistics (a study tool, not a test and not the product): the oracle built with
 * its OR_SPHERE_STAT hook counting, for every sphere test the reference's traversal makes (a leaf whose
 * box passed), whether the discriminant is negative (k = 0), no root lies in [t_min, t_max] (k = 1) or
 * the sphere is hit (k = 2), and how many k = 0 cases an f32 evaluation of the discriminant could
 * reject with a relative margin of 2^-16 (the size of a conservative f32 error bound).
 * Build: gcc -O2 -std=c11 -fPIC -ffp-contract=off -shared -o tools/libsphere_stats.so tools/sphere_stats.c -lm -lpthread
 * Driver: tools/sphere_stats.py. */
#include <math.h>
#include <stdatomic.h>
#include <stdint.h>

static _Atomic uint64_t g_outcome[3];
static _Atomic uint64_t g_f32_reject;

static void sphere_stat(int k, double ocx, double ocy, double ocz, double dx, double dy, double dz, double radius) {
  atomic_fetch_add_explicit(&g_outcome[k], 1, memory_order_relaxed);
  if (k != 0) return;
  const float ox = (float)ocx, oy = (float)ocy, oz = (float)ocz, fx = (float)dx, fy = (float)dy, fz = (float)dz;
  const float r = (float)radius;
  const float a = fx * fx + fy * fy + fz * fz;
  const float hb = ox * fx + oy * fy + oz * fz;
  const float l2 = ox * ox + oy * oy + oz * oz;
  const float cc = l2 - r * r;
  const float disc = hb * hb - a * cc;
  const float mag = hb * hb + a * (l2 + r * r);
  if (disc < -0x1p-16f * mag) atomic_fetch_add_explicit(&g_f32_reject, 1, memory_order_relaxed);
}

#define OR_SPHERE_STAT(k, oc, d, half_b, cc, radius, disc) sphere_stat(k, oc.x, oc.y, oc.z, d.x, d.y, d.z, radius)
#include "../oracle/oracle.c"

void ss_get(uint64_t out[4]) {
  for (int i = 0; i < 3; ++i) out[i] = atomic_load(&g_outcome[i]);
  out[3] = atomic_load(&g_f32_reject);
}
void ss_reset(void) {
  for (int i = 0; i < 3; ++i) atomic_store(&g_outcome[i], 0);
  atomic_store(&g_f32_reject, 0);
}
