// trace.hip — MI355X (gfx950) path-tracing kernels for the reference's ray_color() hot path.
//
// Semantics follow the reference line by line (citations below); arithmetic is binary64 like the
// reference (core/math.rs:5) and the file is compiled with -ffp-contract=off (Rust never fuses).
//
// Execution model (MI355X-first):
//   * persistent waves: every lane owns one work unit = (pixel, chunk of samples) and runs the
//     reference's bounce loop one segment per iteration; a lane whose path ends starts its next
//     sample at once (path regeneration), a lane whose unit ends takes a new unit from the wave's
//     64-unit window (ballot + popcount rank, one global atomic per 64 units);
//   * units are enumerated tile-major (8x8 pixel tile x sample chunk x lane), so a fresh window
//     hands a wave 64 neighbouring pixels: coherent primary rays;
//   * BVH2 with both child boxes inline (112-B nodes), near-child-first traversal, per-lane
//     stack in LDS laid out [depth][lane] (bank = lane % 32: conflict-free at any depth);
//   * per-unit partial sums go to HBM once; a reduce kernel sums chunks in order (deterministic).
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
__device__ __forceinline__ double len(v3 a) { return sqrt(len2(a)); }
__device__ __forceinline__ v3 unit(v3 a) {
  double n = len(a);
  return V(a.x / n, a.y / n, a.z / n);
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
  double r_out_parallel_mag = sqrt(fabs(1.0 - len2(r_out_perp))) * -1.0;
  return r_out_perp + scale(n, r_out_parallel_mag);
}

// ------------------------------------------------------------------------------------------
// counter-based RNG: Philox4x32-10 keyed by seed, counter (draw/2, sample, pixel, 0).
// A draw is converted like rand 0.8's Standard f64: (u64 >> 11) * 2^-53.
// ------------------------------------------------------------------------------------------
struct Rng {
  uint32_t pixel, sample, draw, c2, c3;
};
__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                         uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
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

// ------------------------------------------------------------------------------------------
// intersection (t only during traversal; the full hit record is rebuilt for the winner)
// ------------------------------------------------------------------------------------------
// aabb.rs:62-79 hit2; axes evaluated without early exit (t_min only grows, t_max only shrinks,
// so the final `t_max <= t_min` test equals the reference's per-axis early return).
__device__ __forceinline__ bool slab(const double* b, v3 o, v3 inv, double t_min, double t_max, double& t_enter) {
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    double iv = comp(inv, a);
    double t0 = (b[a] - comp(o, a)) * iv;
    double t1 = (b[a + 3] - comp(o, a)) * iv;
    if (iv < 0.0) {
      double tmp = t0;
      t0 = t1;
      t1 = tmp;
    }
    t_min = (t0 > t_min) ? t0 : t_min;
    t_max = (t1 < t_max) ? t1 : t_max;
  }
  t_enter = t_min;
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
  double sqrt_d = sqrt(disc);
  double root = (-half_b - sqrt_d) / a;
  if (root < t_min || t_max < root) {
    root = (-half_b + sqrt_d) / a;
    if (root < t_min || t_max < root) return false;
  }
  t = root;
  return true;
}

// rect.rs:54-65 (t only): axes (D1, D2), normal axis n = 3-D1-D2; q = d1_min d1_max d2_min d2_max offset
template <int D1, int D2>
__device__ __forceinline__ bool rect_t(const double* q, v3 o, v3 d, double t_min, double t_max, double& t_out) {
  constexpr int n = 3 - D1 - D2;
  double t = (q[4] - comp(o, n)) / comp(d, n);
  if (t < t_min || t > t_max) return false;
  double d1v = comp(o, D1) + t * comp(d, D1);
  double d2v = comp(o, D2) + t * comp(d, D2);
  if (d1v < q[0] || d1v > q[1] || d2v < q[2] || d2v > q[3]) return false;
  t_out = t;
  return true;
}

// rect.rs:132-156 RectBox::hit — six faces in order, each against the running closest.
// Returns the face index (0..5) that won, or -1.
__device__ __forceinline__ int box_t(const double* b, v3 o, v3 d, double t_min, double t_max, double& t_out) {
  double q[5];
  int face = -1;
  double tc = t_max, t;
  // xy_sides: (p0.x, p1.x, p0.y, p1.y, p1.z), (..., p0.z)
  q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4];
  q[4] = b[5];
  if (rect_t<0, 1>(q, o, d, t_min, tc, t)) { tc = t; face = 0; }
  q[4] = b[2];
  if (rect_t<0, 1>(q, o, d, t_min, tc, t)) { tc = t; face = 1; }
  // yz_sides: (p0.y, p1.y, p0.z, p1.z, p1.x), (..., p0.x)
  q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5];
  q[4] = b[3];
  if (rect_t<1, 2>(q, o, d, t_min, tc, t)) { tc = t; face = 2; }
  q[4] = b[0];
  if (rect_t<1, 2>(q, o, d, t_min, tc, t)) { tc = t; face = 3; }
  // xz_sides: (p0.x, p1.x, p0.z, p1.z, p1.y), (..., p0.y)
  q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5];
  q[4] = b[4];
  if (rect_t<0, 2>(q, o, d, t_min, tc, t)) { tc = t; face = 4; }
  q[4] = b[1];
  if (rect_t<0, 2>(q, o, d, t_min, tc, t)) { tc = t; face = 5; }
  t_out = tc;
  return face;
}

__device__ __forceinline__ bool prim_t(const DPrim& pr, v3 o, v3 d, double a, double t_min, double t_max, double& t,
                                       int& face) {
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
  double theta = acos(-ny);
  double phi = atan2(-nz, nx) + 3.14159265358979323846;
  return UV{phi / (2.0 * 3.14159265358979323846), theta / 3.14159265358979323846};
}

// Rebuild the winner's HitRecord with the exact reference formulas (same t => same record).
__device__ __forceinline__ void prim_record(const DPrim& pr, int face, v3 o, v3 d, double t, Hit& h) {
  h.t = t;
  if (pr.kind == kPrimSphere) {
    // sphere.rs:46-51 + get_uv 17-26
    v3 c = V(pr.p[0], pr.p[1], pr.p[2]);
    h.point = o + scale(d, t);
    v3 normal = scale(h.point - c, 1.0 / pr.p[3]);
    UV uv = sphere_uv(normal.x, normal.y, normal.z);
    h.u = uv.u;
    h.v = uv.v;
    finish_hit(h, d, normal);
    return;
  }
  // rect.rs:66-79 ; a RectBox face is a rect with the face's parameters
  double q[5];
  int kind = pr.kind;
  if (kind == kPrimBox) {
    const double* b = pr.p;
    if (face < 2) { q[0] = b[0]; q[1] = b[3]; q[2] = b[1]; q[3] = b[4]; q[4] = face == 0 ? b[5] : b[2]; kind = kPrimRectXY; }
    else if (face < 4) { q[0] = b[1]; q[1] = b[4]; q[2] = b[2]; q[3] = b[5]; q[4] = face == 2 ? b[3] : b[0]; kind = kPrimRectYZ; }
    else { q[0] = b[0]; q[1] = b[3]; q[2] = b[2]; q[3] = b[5]; q[4] = face == 4 ? b[4] : b[1]; kind = kPrimRectXZ; }
  } else {
    for (int i = 0; i < 5; ++i) q[i] = pr.p[i];
  }
  int D1 = (kind == kPrimRectYZ) ? 1 : 0;
  int D2 = (kind == kPrimRectXY) ? 1 : 2;
  int n = 3 - D1 - D2;
  double d1v = comp(o, D1) + t * comp(d, D1);
  double d2v = comp(o, D2) + t * comp(d, D2);
  h.u = (d1v - q[0]) / (q[1] - q[0]);
  h.v = (d2v - q[2]) / (q[3] - q[2]);
  v3 normal = V(n == 0 ? 1.0 : 0.0, n == 1 ? 1.0 : 0.0, n == 2 ? 1.0 : 0.0);
  h.point = o + scale(d, t);
  finish_hit(h, d, normal);
}

// ------------------------------------------------------------------------------------------
// BVH traversal: closest hit in [t_min, t_max] (bbox_tree.rs:56-91 semantics, near-first order)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int traverse(const DScene& S, v3 o, v3 d, double t_min, double& t_best, int& face_best,
                                        int* stk_node, float* stk_t, unsigned& visits, unsigned& ptests) {
  v3 inv = V(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
  double a = len2(d);
  int best = -1;
  int sp = 0;
  int node = 0;  // top node: child[0] = root
  for (;;) {
    const DNode& nd = S.nodes[node];
    int c0 = nd.child[0], c1 = nd.child[1];
    double te0 = 0.0, te1 = 0.0;
    bool h0 = (c0 != kEmptyChild) && slab(nd.box[0], o, inv, t_min, t_best, te0);
    bool h1 = (c1 != kEmptyChild) && slab(nd.box[1], o, inv, t_min, t_best, te1);
    visits += (c0 != kEmptyChild ? 1u : 0u) + (c1 != kEmptyChild ? 1u : 0u);
    // leaves first (one primitive each): test now, they can shrink t_best for the siblings
    if (h0 && c0 < 0) {
      const DPrim& pr = S.prims[~c0];
      double t;
      int f = -1;
      ++ptests;
      if (prim_t(pr, o, d, a, t_min, t_best, t, f)) { t_best = t; best = ~c0; face_best = f; }
      h0 = false;
    }
    if (h1 && c1 < 0) {
      const DPrim& pr = S.prims[~c1];
      double t;
      int f = -1;
      ++ptests;
      if (prim_t(pr, o, d, a, t_min, t_best, t, f)) { t_best = t; best = ~c1; face_best = f; }
      h1 = false;
    }
    int next;
    if (h0 && h1) {
      bool first0 = te0 <= te1;
      next = first0 ? c0 : c1;
      int far = first0 ? c1 : c0;
      double tfar = first0 ? te1 : te0;
      stk_node[sp * kBlockThreads] = far;
      stk_t[sp * kBlockThreads] = __double2float_rd(tfar);
      ++sp;
    } else if (h0) {
      next = c0;
    } else if (h1) {
      next = c1;
    } else {
      next = -1;
      while (sp > 0) {
        --sp;
        // a pushed subtree whose entry lies beyond the current closest hit cannot hold it
        if ((double)stk_t[sp * kBlockThreads] <= t_best) {
          next = stk_node[sp * kBlockThreads];
          break;
        }
      }
      if (next < 0) break;
    }
    node = next;
  }
  return best;
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

// perlin/mod.rs:87-109 + interp 40-63
__device__ __noinline__ double perlin_noise(const DPerlin* T, v3 p) {
  double xf = floor(p.x), yf = floor(p.y), zf = floor(p.z);
  double u = p.x - xf, v = p.y - yf, w = p.z - zf;
  uint32_t i = (uint32_t)sat_i32(xf), j = (uint32_t)sat_i32(yf), k = (uint32_t)sat_i32(zf);
  double uu = u * u * (3.0 - 2.0 * u);
  double vv = v * v * (3.0 - 2.0 * v);
  double ww = w * w * (3.0 - 2.0 * w);
  double accum = 0.0;
#pragma unroll 1
  for (int di = 0; di < 2; ++di) {
    double fi = (double)di;
    int px = T->perm_x[(i + di) & 0xFF];
#pragma unroll 1
    for (int dj = 0; dj < 2; ++dj) {
      double fj = (double)dj;
      int pxy = px ^ T->perm_y[(j + dj) & 0xFF];
#pragma unroll 1
      for (int dk = 0; dk < 2; ++dk) {
        double fk = (double)dk;
        int idx = pxy ^ T->perm_z[(k + dk) & 0xFF];
        v3 c = V(T->ranfloat[idx][0], T->ranfloat[idx][1], T->ranfloat[idx][2]);
        v3 weight = V(u - fi, v - fj, w - fk);
        accum += (fi * uu + (1.0 - fi) * (1.0 - uu)) * (fj * vv + (1.0 - fj) * (1.0 - vv)) *
                 (fk * ww + (1.0 - fk) * (1.0 - ww)) * dot(c, weight);
      }
    }
  }
  return accum;
}

// perlin/mod.rs:162-183 NoiseTexture::value ("marble"): 0.5 (1 + sin(scale p.z + 10 turb(p, 7)));
// the x/y terms of the reference's dot with (0,0,1) contribute exactly 0.
__device__ __noinline__ double marble(const DPerlin* T, double sc, v3 p) {
  double accum = 0.0;
  v3 tp = p;
  double weight = 1.0;
  for (int i = 0; i < 7; ++i) {  // turbulence, perlin/mod.rs:111-124
    accum += weight * perlin_noise(T, tp);
    weight *= 0.5;
    tp = scale(tp, 2.0);
  }
  double turb = 10.0 * fabs(accum);
  double total_noise = sin(sc * p.z + turb);
  return 0.5 * (1.0 + total_noise);
}

// checker.rs:28-30
__device__ __noinline__ double checker_sines(double s, double x, double y, double z) {
  return sin(s * x) * sin(s * y) * sin(s * z);
}

__device__ __forceinline__ v3 texture_value(const DScene& S, int ti, double u, double v, v3 p) {
  for (;;) {
    const DTex& t = S.texs[ti];
    if (t.kind == RT_TEX_SOLID) return V(t.color[0], t.color[1], t.color[2]);  // solid.rs:17-21
    if (t.kind == RT_TEX_CHECKER) {                                             // checker.rs:27-37
      double sines = checker_sines(t.scale, p.x, p.y, p.z);
      ti = (sines < 0.0) ? t.odd : t.even;
      continue;
    }
    if (t.kind == RT_TEX_PERLIN) {
      double n = marble(S.perlin + t.table, t.scale, p);
      return V(n, n, n);
    }
    // image_texture.rs:34-56: clamp, flip v, truncate, /255
    const DImage im = S.images[t.table];
    double uu = (u > 0.0) ? ((u < 1.0) ? u : 1.0) : 0.0;
    double vv = 1.0 - ((v > 0.0) ? ((v < 1.0) ? v : 1.0) : 0.0);
    uint32_t ix = (uint32_t)(uu * (double)(im.width - 1));
    uint32_t iy = (uint32_t)(vv * (double)(im.height - 1));
    const uint8_t* px = S.texels + im.offset + ((size_t)iy * (size_t)im.width + ix) * 3;
    const double cs = 1.0 / 255.0;
    return V((double)px[0] * cs, (double)px[1] * cs, (double)px[2] * cs);
  }
}

// dielectric.rs:15-19
__device__ __noinline__ double reflectance(double cosine, double ref_idx) {
  double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * pow(1.0 - cosine, 5.0);
}

// skybox/mod.rs:5-25
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
__device__ __forceinline__ bool shade(const DScene& S, const DMat& m, Rng& rng, uint64_t seed, v3& o, v3& d,
                                      const Hit& h, v3& att, v3& em) {
  if (m.kind == RT_MAT_DIFFUSE_LIGHT) {  // lighting.rs:21-29: emits, never scatters
    v3 e = texture_value(S, m.tex, h.u, h.v, h.point);
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
  // RT_MAT_LAMBERTIAN (lambertian.rs:21-37) / RT_MAT_FAIRY_LIGHT (lighting.rs:42-66)
  v3 a = texture_value(S, m.tex, h.u, h.v, h.point);
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

// camera/mod.rs:97-132 (horizontal / vertical / lower_left precomputed on the host, same ops)
__device__ __forceinline__ void camera_ray(const DCamera& C, Rng& rng, uint64_t seed, double x, double y, v3& o,
                                           v3& d) {
  double xp = x / (double)C.width;
  double yp = y / (double)C.height;
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

// ------------------------------------------------------------------------------------------
// persistent trace kernel
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long lanemask_lt() {
  unsigned lane = __lane_id();
  return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

__global__ __launch_bounds__(kBlockThreads, 3) void trace_kernel(KParams P) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  int* stk_node = reinterpret_cast<int*>(lds_raw) + tid;
  float* stk_t = reinterpret_cast<float*>(lds_raw + (size_t)P.scene.stack_depth * kBlockThreads * 4) + tid;

  const DScene& S = P.scene;
  const DCamera& C = P.cam;
  const DWork& W = P.work;
  const uint64_t seed = W.seed;
  const int lane = __lane_id();

  // wave-uniform window of unit indices
  unsigned long long w_next = 0, w_end = 0;
  bool exhausted = false;

  // lane state
  bool has_unit = false, active = false;
  int px = 0, py = 0, s_cur = 0, s_end = 0;
  unsigned long long part_index = 0;  // partial-buffer slot of the unit
  v3 sum = V(0, 0, 0), o = V(0, 0, 0), d = V(0, 0, 0), att = V(0, 0, 0), em = V(0, 0, 0);
  int depth_left = 0;
  Rng rng{0, 0, 0, 0, 0};
  unsigned long long n_seg = 0, n_samp = 0;
  unsigned visits = 0, ptests = 0;
  unsigned long long n_vis = 0, n_pt = 0;
  const unsigned long long pix_per_chunk = (unsigned long long)W.n_tiles_rank * kTilePixels;

  for (;;) {
    // 1. a finished unit publishes its in-order sample sum (render.rs:58-69: *buf_c = c)
    if (has_unit && !active && s_cur >= s_end) {
      double* dst = P.partial + part_index * 3;
      dst[0] = sum.x;
      dst[1] = sum.y;
      dst[2] = sum.z;
      has_unit = false;
    }
    // 2. idle lanes take units from the wave's window
    bool need = !has_unit;
    unsigned long long mask = __ballot(need);
    if (mask != 0ull && !exhausted) {
      unsigned long long k = __popcll(mask);
      unsigned long long rank = __popcll(mask & lanemask_lt());
      unsigned long long avail = w_end - w_next;
      unsigned long long idx;
      if (avail >= k) {
        idx = w_next + rank;
        w_next += k;
      } else {
        unsigned long long nb = 0;
        if (lane == 0) nb = atomicAdd(P.unit_counter, (unsigned long long)kWave);
        nb = __shfl(nb, 0);
        idx = (rank < avail) ? (w_next + rank) : (nb + (rank - avail));
        w_next = nb + (k - avail);
        w_end = nb + kWave;
        if (nb >= W.n_units) exhausted = true;
      }
      if (need && idx < W.n_units) {
        // unit -> (local tile, chunk, lane-in-tile); tile-major so a window = 64 neighbours
        unsigned long long per_tile = (unsigned long long)W.n_chunks * kTilePixels;
        unsigned long long lt = idx / per_tile;
        unsigned long long rem = idx - lt * per_tile;
        int chunk = (int)(rem / kTilePixels);
        int lp = (int)(rem % kTilePixels);
        unsigned long long gt = lt * (unsigned long long)W.tile_world + (unsigned long long)W.tile_rank;
        int tx = (int)(gt % (unsigned long long)W.tiles_x), ty = W.ty0 + (int)(gt / (unsigned long long)W.tiles_x);
        px = tx * kTile + (lp % kTile);
        py = ty * kTile + (lp / kTile);
        if (px < C.width && py < C.height) {
          has_unit = true;
          s_cur = chunk * W.chunk;
          s_end = min(W.samples, s_cur + W.chunk);
          part_index = (unsigned long long)chunk * pix_per_chunk + lt * kTilePixels + (unsigned long long)lp;
          sum = V(0.0, 0.0, 0.0);
        }
      }
    }
    // 3. lanes between paths start the next sample (render.rs:60-65)
    if (has_unit && !active && s_cur < s_end) {
      rng.pixel = (uint32_t)py * (uint32_t)C.width + (uint32_t)px;
      rng.sample = (uint32_t)s_cur;
      rng.draw = 0;
      double jx = (double)px + rng_next(rng, seed);
      double jy = (double)py + rng_next(rng, seed);
      camera_ray(C, rng, seed, jx, jy, o, d);
      att = V(1.0, 1.0, 1.0);
      em = V(0.0, 0.0, 0.0);
      depth_left = W.max_depth;
      active = depth_left > 0;
      ++s_cur;
      ++n_samp;
      if (!active) sum = sum + em;  // max_depth == 0: ray_color returns black
    }
    if (!__any(active)) {
      if (exhausted || __ballot(has_unit) == 0ull) {
        if (exhausted) break;
      }
      continue;
    }
    // 4. one ray_color iteration (render.rs:30-46)
    if (active) {
      ++n_seg;
      double t_best = __builtin_inf();
      int face = -1;
      int prim = traverse(S, o, d, 0.001, t_best, face, stk_node, stk_t, visits, ptests);
      bool alive;
      if (prim >= 0) {
        const DPrim pr = S.prims[prim];
        Hit h;
        prim_record(pr, face, o, d, t_best, h);
        const DMat m = S.mats[pr.material];
        alive = shade(S, m, rng, seed, o, d, h, att, em);
      } else {
        em = em + hmul(att, sky(S, d));
        alive = false;
      }
      if (alive) alive = --depth_left > 0;
      if (!alive) {
        sum = sum + em;
        active = false;
      }
    }
    if (visits > (1u << 30)) { n_vis += visits; visits = 0; }
    if (ptests > (1u << 30)) { n_pt += ptests; ptests = 0; }
  }
  n_vis += visits;
  n_pt += ptests;
  // wave-reduce the counters, one atomic per wave
  for (int off = 32; off > 0; off >>= 1) {
    n_seg += __shfl_down(n_seg, off);
    n_samp += __shfl_down(n_samp, off);
    n_vis += __shfl_down(n_vis, off);
    n_pt += __shfl_down(n_pt, off);
  }
  if (lane == 0) {
    atomicAdd(&P.counters->segments, n_seg);
    atomicAdd(&P.counters->samples, n_samp);
    atomicAdd(&P.counters->node_visits, n_vis);
    atomicAdd(&P.counters->prim_tests, n_pt);
  }
}

// Sum the per-chunk partials of each pixel in chunk order and write the Image.data layout
// (row 0 = bottom, image.rs:10-14) or the packed tile layout used by the multi-GPU gather.
__global__ __launch_bounds__(256) void reduce_kernel(const double* __restrict__ partial, int n_chunks,
                                                     int n_tiles_rank, int tiles_x, int ty0, int tile_rank,
                                                     int tile_world, int width, int row0, int row1, int packed,
                                                     double* __restrict__ out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long n_pix = (long long)n_tiles_rank * kTilePixels;
  if (i >= n_pix) return;
  long long lt = i / kTilePixels;
  int lp = (int)(i % kTilePixels);
  long long gt = lt * tile_world + tile_rank;
  int px = (int)(gt % tiles_x) * kTile + lp % kTile;
  int py = (ty0 + (int)(gt / tiles_x)) * kTile + lp / kTile;
  bool inside = px < width && py >= row0 && py < row1;
  double r = 0.0, g = 0.0, b = 0.0;
  if (inside) {
    for (int c = 0; c < n_chunks; ++c) {
      const double* p = partial + ((long long)c * n_pix + i) * 3;
      r += p[0];
      g += p[1];
      b += p[2];
    }
  }
  if (packed) {
    out[i * 3 + 0] = r;
    out[i * 3 + 1] = g;
    out[i * 3 + 2] = b;
  } else if (inside) {
    long long o = ((long long)(py - row0) * width + px) * 3;
    out[o + 0] = r;
    out[o + 1] = g;
    out[o + 2] = b;
  }
}

// Scatter a gathered [world][max_tiles][64][3] buffer into the [H][W][3] image.
__global__ __launch_bounds__(256) void unpack_kernel(const double* __restrict__ gathered, int world, int max_tiles,
                                                     int n_tiles_total, int tiles_x, int width, int height,
                                                     double* __restrict__ out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)world * max_tiles * kTilePixels;
  if (i >= total) return;
  int lp = (int)(i % kTilePixels);
  long long t = i / kTilePixels;
  int lt = (int)(t % max_tiles);
  int r = (int)(t / max_tiles);
  long long gt = (long long)lt * world + r;
  if (gt >= n_tiles_total) return;
  int px = (int)(gt % tiles_x) * kTile + lp % kTile;
  int py = (int)(gt / tiles_x) * kTile + lp / kTile;
  if (px >= width || py >= height) return;
  long long o = ((long long)py * width + px) * 3;
  out[o + 0] = gathered[i * 3 + 0];
  out[o + 1] = gathered[i * 3 + 1];
  out[o + 2] = gathered[i * 3 + 2];
}

// Closest hit for a batch of rays (rt_scene_hit): one lane per ray, same traversal + record code.
struct HitOut {
  int32_t object, front_face;
  double t, point[3], normal[3], u, v;
};
__global__ __launch_bounds__(kBlockThreads) void hit_kernel(DScene S, const double* __restrict__ rays, int n,
                                                            double t_min, double t_max, HitOut* __restrict__ out) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  int* stk_node = reinterpret_cast<int*>(lds_raw) + tid;
  float* stk_t = reinterpret_cast<float*>(lds_raw + (size_t)S.stack_depth * kBlockThreads * 4) + tid;
  int i = blockIdx.x * kBlockThreads + tid;
  if (i >= n) return;
  v3 o = V(rays[i * 6 + 0], rays[i * 6 + 1], rays[i * 6 + 2]);
  v3 d = V(rays[i * 6 + 3], rays[i * 6 + 4], rays[i * 6 + 5]);
  double t_best = t_max;
  int face = -1;
  unsigned visits = 0, ptests = 0;
  int prim = traverse(S, o, d, t_min, t_best, face, stk_node, stk_t, visits, ptests);
  HitOut r{};
  r.object = prim;
  if (prim >= 0) {
    const DPrim pr = S.prims[prim];
    Hit h;
    prim_record(pr, face, o, d, t_best, h);
    r.front_face = h.front_face ? 1 : 0;
    r.t = h.t;
    r.point[0] = h.point.x; r.point[1] = h.point.y; r.point[2] = h.point.z;
    r.normal[0] = h.normal.x; r.normal[1] = h.normal.y; r.normal[2] = h.normal.z;
    r.u = h.u;
    r.v = h.v;
  }
  out[i] = r;
}

// ------------------------------------------------------------------------------------------
// launch wrappers (called from rt_api.cpp)
// ------------------------------------------------------------------------------------------
size_t trace_lds_bytes(int stack_depth) { return (size_t)stack_depth * kBlockThreads * 8; }

hipError_t trace_occupancy(int stack_depth, int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, trace_kernel, kBlockThreads,
                                                       trace_lds_bytes(stack_depth));
}

hipError_t launch_trace(const KParams& p, int blocks, hipStream_t stream) {
  size_t lds = trace_lds_bytes(p.scene.stack_depth);
  hipLaunchKernelGGL(trace_kernel, dim3(blocks), dim3(kBlockThreads), lds, stream, p);
  return hipGetLastError();
}

hipError_t launch_hit(const DScene& S, const double* rays, int n, double t_min, double t_max, void* out,
                      hipStream_t stream) {
  int blocks = (n + kBlockThreads - 1) / kBlockThreads;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(hit_kernel, dim3(blocks), dim3(kBlockThreads), trace_lds_bytes(S.stack_depth), stream, S, rays,
                     n, t_min, t_max, static_cast<HitOut*>(out));
  return hipGetLastError();
}

hipError_t launch_reduce(const double* partial, int n_chunks, int n_tiles_rank, int tiles_x, int ty0, int tile_rank,
                         int tile_world, int width, int row0, int row1, int packed, double* out, hipStream_t stream) {
  long long n = (long long)n_tiles_rank * kTilePixels;
  int blocks = (int)((n + 255) / 256);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(reduce_kernel, dim3(blocks), dim3(256), 0, stream, partial, n_chunks, n_tiles_rank, tiles_x,
                     ty0, tile_rank, tile_world, width, row0, row1, packed, out);
  return hipGetLastError();
}

hipError_t launch_unpack(const double* gathered, int world, int max_tiles, int n_tiles_total, int tiles_x, int width,
                         int height, double* out, hipStream_t stream) {
  long long n = (long long)world * max_tiles * kTilePixels;
  int blocks = (int)((n + 255) / 256);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(unpack_kernel, dim3(blocks), dim3(256), 0, stream, gathered, world, max_tiles, n_tiles_total,
                     tiles_x, width, height, out);
  return hipGetLastError();
}

}  // namespace rt
