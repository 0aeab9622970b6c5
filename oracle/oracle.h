/*
 * oracle.h — CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity checker.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product path (shirley-raytracing-rs_amd/) never links or calls it.
 *
 * Every function follows a reference file:line (paths relative to the reference repo root).
 * Pinning: the reference is Rust and cannot be built here (no cargo/rustc, no crates offline,
 * SURVEY.md §8c).  The oracle is pinned by the reference's own known-answer unit tests
 * (core/fp.rs:30-113, bvh/aabb.rs:89-179, bvh/bbox_tree.rs:94-234; restated in tests/test_oracle_kat.py)
 * plus analytic known-answer tests.  Image-level parity against a reference run is UNPINNED:
 * the reference has no image fixtures and no seedable RNG.
 */
#ifndef SHIRLEY_ORACLE_H
#define SHIRLEY_ORACLE_H

#include <stdint.h>
#include "../include/shirley_rt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_scene or_scene;

typedef struct or_counters {
  uint64_t samples;
  uint64_t segments;
  uint64_t node_visits;
  uint64_t prim_tests;
} or_counters;

/* hit record (geometry/hittable.rs:6-14) + the object index that was hit */
typedef struct or_hit {
  int32_t hit;
  int32_t object;
  double t;
  double point[3];
  double normal[3];
  int32_t front_face;
  double u, v;
} or_hit;

/* RNG: Philox4x32-10 (Salmon et al., SC'11) — the build's counter-based RNG. */
void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint64_t or_rng_u64(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t draw);
double or_rng_f64(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t draw);

/* core/fp.rs */
double or_fmin(double a, double b);
double or_fmax(double a, double b);
double or_non_nan(double a, double b);

/* bvh/aabb.rs ; box = {min.x,min.y,min.z,max.x,max.y,max.z}, ray = {ox,oy,oz,dx,dy,dz} */
int32_t or_aabb_hit(const double box[6], const double ray[6], double t_min, double t_max);
int32_t or_aabb_hit2(const double box[6], const double ray[6], double t_min, double t_max);
void or_surrounding_box(const double a[6], const double b[6], double out[6]);
double or_aabb_area(const double box[6]);
int32_t or_object_bbox(const rt_object* obj, double out[6]);
int32_t or_object_hit(const rt_object* obj, const double ray[6], double t_min, double t_max, or_hit* out);

/* scene/mod.rs:111-137 finalize (BVH via bvh/bbox_tree/constructor.rs); NULL on error */
or_scene* or_scene_new(const rt_scene_desc* desc);
void or_scene_free(or_scene* s);
/* BBox tree inspection: n nodes; root index; per node: bbox[6], leaf index (-1 for branch), lhs, rhs */
int32_t or_tree_size(const or_scene* s);
int32_t or_tree_root(const or_scene* s);
void or_tree_node(const or_scene* s, int32_t idx, double bbox[6], int32_t* leaf, int32_t* lhs, int32_t* rhs);
/* WorkspaceScene::hit_workspace (scene/mod.rs:152-164) */
void or_scene_hit(const or_scene* s, const double ray[6], double t_min, double t_max, or_hit* out);
/* the same with the key rt_scene_hit gives ray `ray_index` (book-2 media draw from it) */
void or_scene_hit_at(const or_scene* s, const double ray[6], double t_min, double t_max, uint32_t ray_index,
                     or_hit* out);

/* texture value (material/texture/{solid,checker,image_texture}.rs, perlin/mod.rs:162-183) */
void or_texture_value(const or_scene* s, int32_t tex, double u, double v, const double p[3], double out[3]);
double or_perlin_noise(const or_scene* s, int32_t table, const double p[3]);
double or_perlin_turbulence(const or_scene* s, int32_t table, const double p[3], int32_t depth);

/* camera/mod.rs:97-132 pixel_ray for (pixel, sample) of the counter RNG, draws starting at 2 */
void or_pixel_ray(const rt_camera* cam, uint64_t seed, int32_t px, int32_t py, uint32_t sample, double ray[6]);

/* render.rs:17-48 ray_color for one (pixel, sample) path (including the jitter + camera draws) */
void or_sample_color(const or_scene* s, const rt_camera* cam, const rt_render_params* p, int32_t px, int32_t py,
                     uint32_t sample, double out[3], or_counters* cnt);

/* render.rs:49-70 render_scanline: buf = [image_width][3] per-pixel sums for row line_idx */
void or_render_scanline(const or_scene* s, const rt_camera* cam, const rt_render_params* p, int32_t line_idx,
                        double* buf, or_counters* cnt);

/* main.rs:65-130 render_scene's loop: rows [line_begin, line_end) on nthreads workers with
 * row-granular dynamic scheduling (rayon analogue); out = [(line_end-line_begin)][W][3] sums. */
int32_t or_render_rows(const or_scene* s, const rt_camera* cam, const rt_render_params* p, int32_t line_begin,
                       int32_t line_end, int32_t nthreads, double* out, or_counters* cnt);

/* one iteration of render.rs:30-46 (ray_color's loop body) for `ray` with the path key (seed, pixel,
 * sample, draw): closest hit, emitted, scatter (material_type.rs:51-79) — or the sky on a miss; the
 * layout of rt_probe (include/shirley_rt.h, the device's rt_probe_segment).  Book-2 ray time 0. */
typedef rt_probe or_probe;
void or_probe_segment(const or_scene* s, const double ray[6], uint64_t seed, uint32_t pixel, uint32_t sample,
                      uint32_t draw, or_probe* out);
/* dielectric.rs:15-19 */
double or_reflectance(double cosine, double ref_idx);

/* image.rs:31-44 + color.rs:31-38 */
void or_tonemap(const double* accum, int32_t width, int32_t height, int32_t samples, uint8_t* rgb8);

#ifdef __cplusplus
}
#endif
#endif
