// scenes.hpp — the reference's scene entry points (src/scenes.rs) and camera construction
// (src/raytracer/camera/mod.rs), on the C++ host side of the boundary.
#pragma once

#include <cstdint>
#include <string>

#include "../../../include/shirley_rt.h"
#include "scene.hpp"

namespace host {

// scenes.rs
SceneBuilder create_cornell_box();                    // :23-63
SceneBuilder create_perlin_demo();                    // :65-79
SceneBuilder create_earth_demo();                     // :81-93
SceneBuilder create_box_light();                      // :94-127
SceneBuilder create_scene();                          // :431-483 ("demo")
void create_ground_checker(SceneBuilder& scene);      // :233-249
void create_fancy_ground(SceneBuilder& scene);        // :251-279
SceneBuilder random_scene(uint64_t seed, bool night); // :281-429, thread_rng -> seeded stream
// benches/my_benchmark.rs:35-60 gen_spheres(side_len) with random_scene-style materials: the
// ~10k-primitive stand-in for BASELINE config 5 (no such scene exists in the reference).
SceneBuilder gen_spheres_scene(uint64_t seed, int32_t side_len);
// "The Next Week" final_scene (book 2 §10; BASELINE config 5): boxes ground, moving sphere, glass,
// metal, a glass ball filled with blue smoke, global mist, earth, marble, and a rotated + translated
// cluster of `n_cluster` white spheres.  Uses the book-2 extensions absent from the reference
// (parity unpinned).  n_ground: ground boxes per side (book: 20).
SceneBuilder final_scene(uint64_t seed, int32_t n_ground, int32_t n_cluster);

// camera/mod.rs:13-61 CameraBuilder + 63-86 CameraPosition::look_at
struct CameraSpec {
  int32_t width = 640;
  int32_t ratio_num = 3, ratio_den = 2;  // AspectRatio::Rational
  double vfov = 20.0;
  double focal_length = 1.0;
  bool has_aperture = true;
  double aperture = 0.001;
  Vec3 look_from{13.0, 2.0, 3.0}, look_at{0.0, 0.0, 0.0}, up{0.0, 1.0, 0.0};
  bool override_focus = true;  // `pos.focus_length = 10.0` (scenes.rs:209,229)
  double focus_length = 10.0;
  double time0 = 0.0, time1 = 0.0;  // shutter (book-2 extension)
};
rt_camera build_camera(const CameraSpec& s);
CameraSpec default_camera_spec(int32_t width, int32_t ratio_num, int32_t ratio_den, double vfov, double focal_length,
                               double aperture);  // scenes.rs:214-231
CameraSpec cornell_camera_spec(int32_t width);    // scenes.rs:191-212
CameraSpec spheres_camera_spec(int32_t width, int32_t ratio_num, int32_t ratio_den);
CameraSpec final_camera_spec(int32_t width, int32_t ratio_num, int32_t ratio_den);  // book 2 §10 camera

// argparse.rs:160-170 CameraAspectRatio
bool aspect_ratio_from_name(const std::string& name, int32_t* num, int32_t* den);

// scene by CLI name: random, random-night, demo, perlin, earth, box-light, cornell, spheres[:side]
bool builtin_scene(const std::string& name, uint64_t seed, SceneBuilder* out, std::string* err);

}  // namespace host
