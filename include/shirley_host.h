/*
 * shirley_host.h — C API of the C++ host layer above the boundary (libshirley_host.so).
 *
 * The reference's host side is Rust (src/scenes.rs, src/main.rs, src/argparse.rs); with no Rust
 * toolchain in this image the host is C++ and this API exposes it to Python (tests, bench) and the
 * ray-cli binary.  It produces the rt_scene_desc / rt_camera values that cross the render ABI
 * (shirley_rt.h).  Errors: non-zero status + sh_last_error() (thread-local message).
 */
#ifndef SHIRLEY_HOST_H
#define SHIRLEY_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "shirley_rt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sh_scene sh_scene; /* SceneBuilder (scene/mod.rs:79-110) */
typedef struct sh_desc sh_desc;   /* finalized scene: owns the arrays behind an rt_scene_desc */

const char* sh_last_error(void);

/* SceneBuilder */
sh_scene* sh_scene_new(void);
void sh_scene_free(sh_scene* s);
int sh_scene_set_skybox(sh_scene* s, int32_t sky, const double color[3]);
/* add one SceneLoadObject given as serde JSON: {"geometry": {...}, "material": {...}} */
int sh_scene_add_json(sh_scene* s, const char* object_json);
int32_t sh_scene_len(const sh_scene* s);
/* serde JSON of the whole builder (scenes.rs:140-143 --scene-output); *needed includes the NUL */
int sh_scene_to_json(const sh_scene* s, int32_t pretty, char* buf, size_t cap, size_t* needed);
int sh_scene_from_json(const char* json, sh_scene** out); /* render saved (scenes.rs:128-134) */
/* scenes.rs entry points by name: random, random-night, demo, perlin, earth, box-light, cornell,
 * spheres[:side] (gen_spheres), final[:n_ground[:n_cluster]] (book-2 final_scene, BASELINE config 5;
 * uses the book-2 extensions the reference lacks) */
int sh_scene_builtin(const char* name, uint64_t seed, sh_scene** out);

/* SceneBuilder::finalize (scene/mod.rs:111-137): textures loaded + deduplicated, Perlin tables from
 * `seed` (or the scene's "perlin_seed"). */
int sh_scene_finalize(const sh_scene* s, uint64_t seed, sh_desc** out);
const rt_scene_desc* sh_desc_view(const sh_desc* d);
void sh_desc_free(sh_desc* d);

/* Camera: CameraBuilder::build + CameraPosition::look_at (camera/mod.rs:13-86) */
typedef struct sh_camera_spec {
  int32_t width;
  int32_t ratio_num, ratio_den;
  double vfov;
  double focal_length;
  int32_t has_aperture;
  double aperture;
  double look_from[3], look_at[3], up[3];
  int32_t override_focus; /* pos.focus_length = focus_length after look_at (scenes.rs:209,229) */
  double focus_length;
  double time0, time1;    /* shutter (book-2 extension, absent from the reference) */
} sh_camera_spec;
int sh_camera_build(const sh_camera_spec* spec, rt_camera* out);
/* scenes.rs:214-231 default_camera(CameraSettings) ; argparse.rs:125-170 defaults: 640, 20, 1.0, 0.001, std3x2 */
int sh_default_camera(int32_t width, const char* aspect_ratio, double vfov, double focal_length, double aperture,
                      rt_camera* out);
int sh_cornell_camera(int32_t width, rt_camera* out); /* scenes.rs:191-212 */
int sh_scene_camera(const char* scene_name, int32_t width, const char* aspect_ratio, double vfov,
                    double focal_length, double aperture, rt_camera* out); /* camera each entry point uses */

/* Perlin::new from a seeded stream (perlin/mod.rs:73-85) */
int sh_perlin_generate(uint64_t seed, uint32_t table_index, rt_perlin_table* out);

/* PNG writer for rt_tonemap output (image.rs:40-43 save_with_format Png) */
int sh_write_png(const char* path, const uint8_t* rgb8, int32_t width, int32_t height);
/* image loader used by ImagePath / EarthBuiltin (PNG or .rgb8.gz); caller frees *rgb with sh_free */
int sh_load_image(const char* path, int32_t* width, int32_t* height, uint8_t** rgb);
void sh_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
