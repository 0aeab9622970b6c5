/* CPU check of the megakernel's two-pass RectBox tests (rt_device.h box_t2, box_t1f) against the sequential six-face
 * test (box_t, rect.rs:132-156): the same IEEE binary64 operations (gcc -ffp-contract=off; the device's
 * face_div is the correctly rounded quotient, as `/` here; the slab test multiplies by RN(1/d)).
 * Adversarial draws: boxes from unit cubes to slabs 1e-9 thin and far from the origin, rays aimed at face
 * interiors, edges and corners (where faces of two axes tie and entry meets exit), grazing a face plane,
 * starting inside the box or on a face, and direction components down to 1e-250 (face_div's range starts
 * at 2^-300).  Only rays whose slab test passes are compared (leaf_tests4 calls the face test after it).
 * Prints "<mismatches> mismatches: <n> compared, <p> one pass, <t> ties, <e> second pass" and exits 1 on a
 * mismatch.  -DNO_MARGIN drops the 2^-50 margins (the check then finds mismatches: it has teeth).
 * usage: box_pass_check <draws> */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#ifdef NO_MARGIN
#define MARGIN 0.0
#else
#define MARGIN 0x1p-50
#endif

typedef struct { double x, y, z; } v3;
static double comp(v3 v, int i) { return i == 0 ? v.x : i == 1 ? v.y : v.z; }

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t nxt(void) {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return rs;
}
static double uni(void) { return (nxt() >> 11) * 0x1p-53; }
static double rng(double a, double b) { return a + (b - a) * uni(); }

static int rect_t(int D1, int D2, const double* q, v3 o, v3 d, double t_min, double t_max, double* t_out) {
  const int n = 3 - D1 - D2;
  double t = (q[4] - comp(o, n)) / comp(d, n);
  if (t < t_min || t > t_max) return 0;
  double d1v = comp(o, D1) + t * comp(d, D1);
  double d2v = comp(o, D2) + t * comp(d, D2);
  if (d1v < q[0] || d1v > q[1] || d2v < q[2] || d2v > q[3]) return 0;
  *t_out = t;
  return 1;
}

static int box_t(const double* b, v3 o, v3 d, double t_min, double t_max, double* t_out) {
  double q[5], tc = t_max, t;
  int face = -1;
  q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4];
  q[4] = b[5]; if (rect_t(0, 1, q, o, d, t_min, tc, &t)) { tc = t; face = 0; }
  q[4] = b[2]; if (rect_t(0, 1, q, o, d, t_min, tc, &t)) { tc = t; face = 1; }
  q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5];
  q[4] = b[3]; if (rect_t(1, 2, q, o, d, t_min, tc, &t)) { tc = t; face = 2; }
  q[4] = b[0]; if (rect_t(1, 2, q, o, d, t_min, tc, &t)) { tc = t; face = 3; }
  q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5];
  q[4] = b[4]; if (rect_t(0, 2, q, o, d, t_min, tc, &t)) { tc = t; face = 4; }
  q[4] = b[1]; if (rect_t(0, 2, q, o, d, t_min, tc, &t)) { tc = t; face = 5; }
  *t_out = tc;
  return face;
}

static void slab_axis(double lo, double hi, int neg, double o, double iv, double* t_min, double* t_max) {
  const double pn = neg ? hi : lo, pf = neg ? lo : hi;
  const double t0 = (pn - o) * iv, t1 = (pf - o) * iv;
  *t_min = fmax(t0, *t_min);
  *t_max = fmin(t1, *t_max);
}
static int slab_s(const double* b, v3 o, v3 inv, double t_min, double t_max, double* te, double* tx) {
  slab_axis(b[0], b[3], inv.x < 0.0, o.x, inv.x, &t_min, &t_max);
  slab_axis(b[1], b[4], inv.y < 0.0, o.y, inv.y, &t_min, &t_max);
  slab_axis(b[2], b[5], inv.z < 0.0, o.z, inv.z, &t_min, &t_max);
  *te = t_min;
  *tx = t_max;
  return !(t_max <= t_min);
}

static long n_second;
static int box_t2(const double* b, v3 o, v3 d, v3 inv, double t_min, double t_max, double t_enter, double t_exit,
                  double* t_out) {
  const int nz = inv.z < 0.0, nx = inv.x < 0.0, ny = inv.y < 0.0;
  const int far_first = !(t_enter > t_min);
  double tc = t_max, t1 = t_max;
  int f1 = -1;
  for (int pass = 0; pass < 2; ++pass) {
    const int flip = far_first != (pass == 1);
    double q[5], t;
    int f = -1, hi = nz != flip;
    q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4];
    q[4] = hi ? b[5] : b[2];
    if (rect_t(0, 1, q, o, d, t_min, tc, &t)) { tc = t; f = hi ? 0 : 1; }
    hi = nx != flip;
    q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5];
    q[4] = hi ? b[3] : b[0];
    if (rect_t(1, 2, q, o, d, t_min, tc, &t)) { tc = t; f = hi ? 2 : 3; }
    hi = ny != flip;
    q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5];
    q[4] = hi ? b[4] : b[1];
    if (rect_t(0, 2, q, o, d, t_min, tc, &t)) { tc = t; f = hi ? 4 : 5; }
    if (pass == 0) {
      t1 = tc; f1 = f;
      if (f >= 0 && (far_first ? tc > t_min * (1.0 + MARGIN) : tc < t_exit * (1.0 - MARGIN))) break;
      ++n_second;
    } else if (f >= 0 && (f1 < 0 || tc < t1 || f > f1)) {
      t1 = tc; f1 = f;
    }
  }
  *t_out = t1;
  return f1;
}

/* rt_device.h box_t1f: box_t2's first pass, else the six-face sequence */
static int box_t1f(const double* b, v3 o, v3 d, v3 inv, double t_min, double t_max, double t_enter, double t_exit,
                   double* t_out) {
  const int nz = inv.z < 0.0, nx = inv.x < 0.0, ny = inv.y < 0.0;
  const int far_first = !(t_enter > t_min);
  double q[5], t, tc = t_max;
  int f = -1, hi = nz != far_first;
  q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4];
  q[4] = hi ? b[5] : b[2];
  if (rect_t(0, 1, q, o, d, t_min, tc, &t)) { tc = t; f = hi ? 0 : 1; }
  hi = nx != far_first;
  q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5];
  q[4] = hi ? b[3] : b[0];
  if (rect_t(1, 2, q, o, d, t_min, tc, &t)) { tc = t; f = hi ? 2 : 3; }
  hi = ny != far_first;
  q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5];
  q[4] = hi ? b[4] : b[1];
  if (rect_t(0, 2, q, o, d, t_min, tc, &t)) { tc = t; f = hi ? 4 : 5; }
  if (!(f >= 0 && (far_first ? tc > t_min * (1.0 + MARGIN) : tc < t_exit * (1.0 - MARGIN))))
    f = box_t(b, o, d, t_min, t_max, &tc);
  *t_out = tc;
  return f;
}

/* a point on the box: interior of a face, an edge, or a corner */
static v3 box_point(const double* b, int kind) {
  double p[3];
  for (int a = 0; a < 3; ++a) p[a] = rng(b[a], b[a + 3]);
  const int a0 = nxt() % 3, a1 = (a0 + 1 + nxt() % 2) % 3;
  p[a0] = (nxt() & 1) ? b[a0 + 3] : b[a0];
  if (kind >= 1) p[a1] = (nxt() & 1) ? b[a1 + 3] : b[a1];
  if (kind >= 2) { const int a2 = 3 - a0 - a1; p[a2] = (nxt() & 1) ? b[a2 + 3] : b[a2]; }
  v3 r = {p[0], p[1], p[2]};
  return r;
}

int main(int argc, char** argv) {
  const long draws = argc > 1 ? atol(argv[1]) : 1000000;
  long compared = 0, one_pass = 0, ties = 0, bad = 0;
  for (long i = 0; i < draws; ++i) {
    double b[6];
    const double scale = pow(10.0, rng(-2, 2)), off = (nxt() & 3) ? rng(-30, 30) : rng(-1e6, 1e6);
    for (int a = 0; a < 3; ++a) {
      const double lo = off * uni() + scale * rng(-1, 1);
      const int thin = nxt() % 8;
      const double w = thin == 0 ? 1e-9 * scale : thin == 1 ? 0.01 : thin == 2 ? 0.0 : scale * rng(0.01, 2);
      b[a] = lo; b[a + 3] = lo + w;
    }
    /* target on the box (face / edge / corner) or inside it; origin outside, inside, or on a face */
    const int tk = nxt() % 4;
    v3 tg;
    if (tk < 3) tg = box_point(b, tk);
    else { tg.x = rng(b[0], b[3]); tg.y = rng(b[1], b[4]); tg.z = rng(b[2], b[5]); }
    const int ok = nxt() % 4;
    v3 o;
    if (ok == 0) { o.x = rng(b[0], b[3]); o.y = rng(b[1], b[4]); o.z = rng(b[2], b[5]); }
    else if (ok == 1) o = box_point(b, 0);
    else {
      const double R = scale * pow(10.0, rng(-1, 2));
      o.x = tg.x + rng(-R, R); o.y = tg.y + rng(-R, R); o.z = tg.z + rng(-R, R);
    }
    v3 d = {tg.x - o.x, tg.y - o.y, tg.z - o.z};
    /* grazing: one component tiny (the ray runs (nearly) in a face plane) */
    const int gz = nxt() % 6;
    if (gz < 3) {
      const double tiny = pow(10.0, -rng(20, 250)) * ((nxt() & 1) ? 1 : -1);
      if (gz == 0) d.x = tiny; else if (gz == 1) d.y = tiny; else d.z = tiny;
    }
    if ((nxt() & 7) == 0) { d.x *= 1e-3; d.y *= 1e-3; d.z *= 1e-3; }
    const double m[3] = {fabs(d.x), fabs(d.y), fabs(d.z)};
    int in_range = 1;
    for (int a = 0; a < 3; ++a) in_range &= m[a] >= 0x1p-300 && m[a] <= 0x1p300;
    if (!in_range) continue;
    const v3 inv = {1.0 / d.x, 1.0 / d.y, 1.0 / d.z};
    const double t_min = (nxt() & 1) ? 0.001 : rng(0.001, 0.5);
    const double t_max = (nxt() & 1) ? INFINITY : rng(0.01, 3.0);
    double te, tx, ta, tb;
    if (!slab_s(b, o, inv, t_min, t_max, &te, &tx)) continue;
    const long before = n_second;
    const int fa = box_t(b, o, d, t_min, t_max, &ta);
    const int fb = box_t2(b, o, d, inv, t_min, t_max, te, tx, &tb);
    ++compared;
    one_pass += n_second == before;
    if (fa >= 0) {
      /* a tie: another face passes at exactly the winning t */
      double tt;
      for (int k = 0; k < 6; ++k) {
        if (k == fa) continue;
        const int D1 = k < 2 ? 0 : k < 4 ? 1 : 0, D2 = k < 2 ? 1 : 2;
        double q[5] = {b[D1], b[D1 + 3], b[D2], b[D2 + 3], b[(3 - D1 - D2) + ((k & 1) ? 0 : 3)]};
        if (rect_t(D1, D2, q, o, d, t_min, t_max, &tt) && tt == ta) { ++ties; break; }
      }
    }
    double tf;
    const int ff = box_t1f(b, o, d, inv, t_min, t_max, te, tx, &tf);
    if (ff != fa || (fa >= 0 && tf != ta)) {
      if (bad < 5) printf("box_t1f mismatch: face %d/%d t %a/%a\n", fa, ff, ta, tf);
      ++bad;
    }
    if (fa != fb || (fa >= 0 && ta != tb)) {
      if (bad < 5)
        printf("mismatch: box (%a %a %a)-(%a %a %a) o (%a %a %a) d (%a %a %a) face %d/%d t %a/%a\n", b[0], b[1], b[2],
               b[3], b[4], b[5], o.x, o.y, o.z, d.x, d.y, d.z, fa, fb, ta, tb);
      ++bad;
    }
  }
  printf("%ld mismatches: %ld compared, %ld one pass, %ld ties, %ld second pass\n", bad, compared, one_pass, ties,
         n_second);
  return bad != 0;
}
