// scene.hpp — host-side scene model mirroring the reference's SceneBuilder / TextureLoader /
// MaterialType / GeometricObject (scene/mod.rs:23-110, texture/loader.rs:17-61,
// material/material_type.rs:20-49, geometry/object.rs:9-16), its serde-JSON format
//  and SceneBuilder::finalize -> the C ABI's rt_scene_desc.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/shirley_rt.h"
#include "json.hpp"

namespace host {

// core/vec3.rs over nalgebra: same evaluation order as the kernels
struct Vec3 {
  double x = 0, y = 0, z = 0;
  Vec3() = default;
  Vec3(double a, double b, double c) : x(a), y(b), z(c) {}
  Vec3 operator+(const Vec3& o) const { return {x + o.x, y + o.y, z + o.z}; }
  Vec3 operator-(const Vec3& o) const { return {x - o.x, y - o.y, z - o.z}; }
  Vec3 operator*(const Vec3& o) const { return {x * o.x, y * o.y, z * o.z}; }
  Vec3 scale(double s) const { return {x * s, y * s, z * s}; }
  double dot(const Vec3& o) const { return (x * o.x + y * o.y) + z * o.z; }
  double length() const;
  Vec3 unit() const;
  Vec3 cross(const Vec3& b) const { return {y * b.z - z * b.y, z * b.x - x * b.z, x * b.y - y * b.x}; }
};

// texture/loader.rs:17-28
struct TextureLoader {
  enum Kind { Solid, ImagePath, Perlin, EarthBuiltin, Checker } kind = Solid;
  Vec3 color;         // Solid
  std::string path;   // ImagePath
  double scalar = 0;  // Perlin scale / Checker size
  std::shared_ptr<TextureLoader> odd, even;

  static TextureLoader solid(double r, double g, double b);
  static TextureLoader solid_from_vec(Vec3 v);
  static TextureLoader checker(double size, TextureLoader odd, TextureLoader even);
  static TextureLoader noise(double scale);
  static TextureLoader earth();
  static TextureLoader image(std::string path);
  std::string key() const;  // bitwise identity (ColorSetting / ScalarSetting Hash+Eq, loader.rs:172-210)
};

// material/material_type.rs:20-27 (MaterialType<TextureLoader>)
struct Material {
  enum Kind { Metal, Dielectric, Lambertian, DiffuseLight, FairyLight, Isotropic } kind = Lambertian;
  Vec3 albedo;  // Metal
  double fuzz = 0, ir = 1;
  TextureLoader tex;  // Lambertian / DiffuseLight / FairyLight
  static Material metal(Vec3 albedo, const double* fuzz);  // Metal::new (metal.rs:17-23), fuzz None -> 0, clamp <= 1
  static Material dielectric(double ir);
  static Material lambertian(TextureLoader t);
  static Material diffuse_light(TextureLoader t);
  static Material fairy_light(TextureLoader t);
  static Material isotropic(TextureLoader t);  // book-2 extension (absent from the reference)
};

// geometry/object.rs:9-16, plus the book-2 extensions (absent from the reference):
// MovingSphere, and the object wrappers ConstantMedium (this shape as the boundary) and
// Translate(RotateY(.)) — serde JSON: "MovingSphere" geometry, "medium" / "transform" object keys.
struct Geometry {
  int32_t kind = RT_GEOM_SPHERE;
  double p[6] = {0, 0, 0, 0, 0, 0};
  double q[5] = {0, 0, 0, 0, 0};  // MovingSphere: center1 xyz, time0, time1
  bool medium = false;            // ConstantMedium boundary
  double density = 0;
  bool transform = false;         // Translate(offset) . RotateY(rotate_y)
  double rotate_y = 0;
  Vec3 offset;
  static Geometry moving_sphere(Vec3 c0, Vec3 c1, double time0, double time1, double r);
  Geometry with_medium(double density) const;
  Geometry with_transform(double rotate_y_deg, Vec3 offset) const;
  static Geometry sphere(Vec3 c, double r);
  static Geometry xy_rect(double d1_min, double d1_max, double d2_min, double d2_max, double offset);
  static Geometry yz_rect(double d1_min, double d1_max, double d2_min, double d2_max, double offset);
  static Geometry xz_rect(double d1_min, double d1_max, double d2_min, double d2_max, double offset);
  static Geometry rect_box(Vec3 p0, Vec3 p1);  // RectBox::new (rect.rs:111-129)
};

// Owning storage behind an rt_scene_desc
struct SceneDesc {
  int32_t sky = RT_SKY_ABOVE;
  double sky_color[3] = {0, 0, 0};
  std::vector<rt_object> objects;
  std::vector<rt_material> materials;
  std::vector<rt_texture> textures;
  std::vector<rt_perlin_table> perlin;
  std::vector<std::vector<uint8_t>> image_pixels;
  std::vector<rt_image> images;
  rt_scene_desc view() const;
};

// scene/mod.rs:79-110
struct SceneBuilder {
  int32_t skybox = RT_SKY_ABOVE;
  Vec3 sky_color;
  std::vector<std::pair<Geometry, Material>> objects;
  bool has_perlin_seed = false;  // JSON extension "perlin_seed"
  uint64_t perlin_seed = 0;

  void set_skybox(int32_t kind, Vec3 color = Vec3());
  void add(const Geometry& g, const Material& m) { objects.emplace_back(g, m); }

  Json to_json() const;
  static SceneBuilder from_json(const Json& j);
  // SceneBuilder::finalize (scene/mod.rs:111-137): load + dedup textures (TextureManager,
  // loader.rs:113-131), generate Perlin tables (perlin/mod.rs:73-85) from `seed` (or perlin_seed).
  // Throws std::runtime_error on load failure.
  SceneDesc finalize(uint64_t seed) const;
};

// Perlin::new from a seeded stream (perlin/mod.rs:73-85, 126-139)
void perlin_generate(uint64_t seed, uint32_t table_index, rt_perlin_table* out);

// decoded image textures (image_texture.rs:11-31): ImagePath files (PNG / .rgb8.gz)
bool load_image_file(const std::string& path, int32_t* w, int32_t* h, std::vector<uint8_t>* rgb, std::string* err);
// EarthBuiltin: assets/earthmap.rgb8.gz linked into the library (earth_embed.S), like include_bytes!
bool load_earth_builtin(int32_t* w, int32_t* h, std::vector<uint8_t>* rgb, std::string* err);

}  // namespace host
