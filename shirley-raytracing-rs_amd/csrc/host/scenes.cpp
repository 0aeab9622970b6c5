// scenes.cpp — scene entry points of src/scenes.rs and the camera of src/raytracer/camera/mod.rs.
#include "scenes.hpp"

#include <cmath>
#include <cstring>
#include <vector>

#include "rng.hpp"

namespace host {

SceneBuilder create_cornell_box() {
  SceneBuilder scene;
  scene.set_skybox(RT_SKY_NONE);
  Material red = Material::lambertian(TextureLoader::solid(0.65, 0.05, 0.05));
  Material white = Material::lambertian(TextureLoader::solid(0.73, 0.73, 0.73));
  Material green = Material::lambertian(TextureLoader::solid(0.12, 0.45, 0.15));
  Material light = Material::fairy_light(TextureLoader::solid(15.0, 15.0, 15.0));
  const double box_size = 555.0;
  scene.add(Geometry::yz_rect(0.0, box_size, 0.0, box_size, box_size), green);
  scene.add(Geometry::yz_rect(0.0, box_size, 0.0, box_size, 0.0), red);
  scene.add(Geometry::xz_rect(213.0, 343.0, 227.0, 332.0, 554.0), light);
  scene.add(Geometry::xz_rect(0.0, box_size, 0.0, box_size, 0.0), white);
  scene.add(Geometry::xz_rect(0.0, box_size, 0.0, box_size, box_size), white);
  scene.add(Geometry::xy_rect(0.0, box_size, 0.0, box_size, box_size), white);
  scene.add(Geometry::rect_box(Vec3(130.0, 0.0, 65.0), Vec3(295.0, 165.0, 230.0)), white);
  scene.add(Geometry::rect_box(Vec3(265.0, 0.0, 295.0), Vec3(430.0, 330.0, 460.0)), white);
  return scene;
}

SceneBuilder create_perlin_demo() {
  SceneBuilder scene;
  create_ground_checker(scene);
  scene.add(Geometry::sphere(Vec3(0.0, 2.0, -0.0), 2.0), Material::lambertian(TextureLoader::noise(4.0)));
  return scene;
}

SceneBuilder create_earth_demo() {
  SceneBuilder scene;
  create_ground_checker(scene);
  scene.add(Geometry::sphere(Vec3(4.0, 1.0, 1.0), 1.0), Material::lambertian(TextureLoader::earth()));
  return scene;
}

SceneBuilder create_box_light() {
  SceneBuilder scene;
  scene.set_skybox(RT_SKY_NONE);
  create_ground_checker(scene);
  scene.add(Geometry::sphere(Vec3(0.0, 2.0, -0.0), 2.0), Material::lambertian(TextureLoader::noise(4.0)));
  scene.add(Geometry::xz_rect(3.0, 5.0, 1.0, 3.0, 3.5), Material::diffuse_light(TextureLoader::solid(4.0, 4.0, 4.0)));
  return scene;
}

void create_ground_checker(SceneBuilder& scene) {
  TextureLoader ground = TextureLoader::checker(10.0, TextureLoader::solid(0.2, 0.3, 0.1), TextureLoader::solid(0.9, 0.9, 0.9));
  const double rect = 30.0;
  scene.add(Geometry::xz_rect(-rect, rect, -rect, rect, -0.0001), Material::lambertian(ground));
}

void create_fancy_ground(SceneBuilder& scene) {
  const double RECT_SIZE = 30.0, TOP_COAT_DEPTH = 0.01, LAYER_SEP = 0.01;
  Material lower = Material::lambertian(
      TextureLoader::checker(3.0, TextureLoader::noise(1.0), TextureLoader::solid(0.1, 0.1, 0.1)));
  scene.add(Geometry::xz_rect(-RECT_SIZE, RECT_SIZE, -RECT_SIZE, RECT_SIZE, -TOP_COAT_DEPTH - LAYER_SEP), lower);
  scene.add(Geometry::rect_box(Vec3(-RECT_SIZE, -TOP_COAT_DEPTH, -RECT_SIZE), Vec3(RECT_SIZE, 0.0, RECT_SIZE)),
            Material::dielectric(1.0));
}

namespace {
int total_cmp(double a, double b) {
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  ia ^= (int64_t)(((uint64_t)(ia >> 63)) >> 1);
  ib ^= (int64_t)(((uint64_t)(ib >> 63)) >> 1);
  return (ia < ib) ? -1 : (ia > ib ? 1 : 0);
}

struct Ball {
  Vec3 c;
  double r;
};

// scenes.rs:295-306 check_fit_ball: shrink to touch every earlier ball, sink by the shrink
Ball check_fit_ball(std::vector<Ball>& balls, Ball s) {
  double orig = s.r;
  for (const Ball& other : balls) {
    double dist = (other.c - s.c).length();
    double rem = dist - other.r;
    s.r = (total_cmp(s.r, rem) > 0) ? rem : s.r;  // std::cmp::min_by(s.radius, rem, total_cmp)
  }
  double delta = orig - s.r;
  s.c = s.c - Vec3(0.0, delta, 0.0);
  balls.push_back(s);
  return s;
}

enum BallType { Color = 0, SphereLight, Glass, MetalT, CheckerT, Marble };

Vec3 gen_vec3(SceneRng& rng) {
  double x = rng.gen_f64();
  double y = rng.gen_f64();
  double z = rng.gen_f64();
  return Vec3(x, y, z);
}
Vec3 random_range_vec(SceneRng& rng, double mn, double mx) {
  double x = rng.random_real(mn, mx);
  double y = rng.random_real(mn, mx);
  double z = rng.random_real(mn, mx);
  return Vec3(x, y, z);
}

// scenes.rs:384-424: material draws per ball type
Material ball_material(SceneRng& rng, int item, double radius) {
  switch (item) {
    case Color: {
      Vec3 a = gen_vec3(rng);
      Vec3 b = gen_vec3(rng);
      return Material::lambertian(TextureLoader::solid_from_vec(a * b));
    }
    case SphereLight: {
      Vec3 a = gen_vec3(rng);
      Vec3 b = gen_vec3(rng);
      return Material::fairy_light(TextureLoader::solid_from_vec((a * b).scale(5.0)));
    }
    case Glass: return Material::dielectric(1.5);
    case MetalT: {
      Vec3 albedo = random_range_vec(rng, 0.5, 1.0);
      double fuzz = rng.random_real(0.0, 0.5);
      return Material::metal(albedo, &fuzz);
    }
    case CheckerT: {
      Vec3 a = gen_vec3(rng);
      Vec3 b = gen_vec3(rng);
      return Material::lambertian(
          TextureLoader::checker(8.0 / radius, TextureLoader::solid_from_vec(a * b), TextureLoader::solid(0.9, 0.9, 0.9)));
    }
    default: return Material::lambertian(TextureLoader::noise(16.0));
  }
}
}  // namespace

SceneBuilder random_scene(uint64_t seed, bool night) {
  SceneRng rng(seed, kStreamRandomScene);
  SceneBuilder scene;
  if (night) scene.set_skybox(RT_SKY_NONE);
  if (night) create_ground_checker(scene);
  else create_fancy_ground(scene);

  std::vector<Ball> balls;
  Ball b = check_fit_ball(balls, Ball{Vec3(0.0, 1.0, 0.0), 1.0});
  scene.add(Geometry::sphere(b.c, b.r), Material::dielectric(1.5));
  if (night) {
    b = check_fit_ball(balls, Ball{Vec3(-4.0, 1.0, 0.0), 1.0});
    scene.add(Geometry::sphere(b.c, b.r), Material::fairy_light(TextureLoader::solid_from_vec(Vec3(0.7, 0.6, 0.5).scale(1.3))));
  } else {
    b = check_fit_ball(balls, Ball{Vec3(-4.0, 1.0, 0.0), 1.0});
    scene.add(Geometry::sphere(b.c, b.r), Material::lambertian(TextureLoader::solid(0.4, 0.2, 0.1)));
  }
  b = check_fit_ball(balls, Ball{Vec3(4.0, 1.0, 0.0), 1.0});
  scene.add(Geometry::sphere(b.c, b.r), Material::metal(Vec3(0.7, 0.6, 0.5), nullptr));

  const double light_weight = night ? 4.0 : 0.0;
  const std::vector<double> weights = {4.0, light_weight, 1.0, 4.0, 0.3, 0.0};
  for (int a = -11; a < 11; ++a) {
    for (int bb = -11; bb < 11; ++bb) {
      int item = (int)rng.choose_weighted(weights);
      double radius = rng.random_real(0.05, 0.25);
      double cx = (double)a + 0.9 * rng.gen_f64();
      double cz = (double)bb + 0.9 * rng.gen_f64();
      Vec3 center(cx, radius, cz);
      Vec3 keepout(3.0, radius, 0.0);
      if ((center - keepout).length() <= 0.9) continue;
      Ball s = check_fit_ball(balls, Ball{center, radius});
      scene.add(Geometry::sphere(s.c, s.r), ball_material(rng, item, radius));  // 8.0 / radius uses the drawn radius
    }
  }
  return scene;
}

SceneBuilder gen_spheres_scene(uint64_t seed, int32_t side_len) {
  SceneRng rng(seed, kStreamGenSpheres);
  SceneBuilder scene;
  const std::vector<double> weights = {4.0, 0.0, 1.0, 4.0, 0.3, 0.0};
  for (int x = -side_len; x < side_len; ++x)
    for (int y = -side_len; y < side_len; ++y)
      for (int z = -side_len; z < side_len; ++z) {
        double ox = rng.random_real(-1.0, 1.0);
        double oy = rng.random_real(-1.0, 1.0);
        double oz = rng.random_real(-1.0, 1.0);
        double radius = std::exp(0.5 + 0.5 * rng.gen_normal());  // LogNormal(0.5, 0.5)
        Vec3 c = Vec3((double)x, (double)y, (double)z) + Vec3(ox, oy, oz);
        int item = (int)rng.choose_weighted(weights);
        scene.add(Geometry::sphere(c, radius), ball_material(rng, item, radius));
      }
  return scene;
}

// book 2 ("The Next Week") §10 final_scene, drawn from the scene stream in the book's order.
SceneBuilder final_scene(uint64_t seed, int32_t n_ground, int32_t n_cluster) {
  SceneRng rng(seed, kStreamFinalScene);
  SceneBuilder scene;
  scene.set_skybox(RT_SKY_NONE);  // background black
  const Material ground = Material::lambertian(TextureLoader::solid(0.48, 0.83, 0.53));
  for (int i = 0; i < n_ground; i++)
    for (int j = 0; j < n_ground; j++) {
      const double w = 100.0;
      const double x0 = -1000.0 + i * w, z0 = -1000.0 + j * w, y0 = 0.0;
      const double x1 = x0 + w, y1 = rng.random_real(1.0, 101.0), z1 = z0 + w;
      scene.add(Geometry::rect_box(Vec3(x0, y0, z0), Vec3(x1, y1, z1)), ground);
    }
  scene.add(Geometry::xz_rect(123.0, 423.0, 147.0, 412.0, 554.0), Material::diffuse_light(TextureLoader::solid(7.0, 7.0, 7.0)));
  const Vec3 center1(400.0, 400.0, 200.0);
  const Vec3 center2 = center1 + Vec3(30.0, 0.0, 0.0);
  scene.add(Geometry::moving_sphere(center1, center2, 0.0, 1.0, 50.0), Material::lambertian(TextureLoader::solid(0.7, 0.3, 0.1)));
  scene.add(Geometry::sphere(Vec3(260.0, 150.0, 45.0), 50.0), Material::dielectric(1.5));
  const double fuzz = 1.0;
  scene.add(Geometry::sphere(Vec3(0.0, 150.0, 145.0), 50.0), Material::metal(Vec3(0.8, 0.8, 0.9), &fuzz));
  const Geometry boundary = Geometry::sphere(Vec3(360.0, 150.0, 145.0), 70.0);
  scene.add(boundary, Material::dielectric(1.5));
  scene.add(boundary.with_medium(0.2), Material::isotropic(TextureLoader::solid(0.2, 0.4, 0.9)));
  const Geometry mist = Geometry::sphere(Vec3(0.0, 0.0, 0.0), 5000.0);
  scene.add(mist.with_medium(0.0001), Material::isotropic(TextureLoader::solid(1.0, 1.0, 1.0)));
  scene.add(Geometry::sphere(Vec3(400.0, 200.0, 400.0), 100.0), Material::lambertian(TextureLoader::earth()));
  scene.add(Geometry::sphere(Vec3(220.0, 280.0, 300.0), 80.0), Material::lambertian(TextureLoader::noise(0.1)));
  const Material white = Material::lambertian(TextureLoader::solid(0.73, 0.73, 0.73));
  for (int j = 0; j < n_cluster; j++) {
    const double x = rng.random_real(0.0, 165.0), y = rng.random_real(0.0, 165.0), z = rng.random_real(0.0, 165.0);
    scene.add(Geometry::sphere(Vec3(x, y, z), 10.0).with_transform(15.0, Vec3(-100.0, 270.0, 395.0)), white);
  }
  return scene;
}

// ---------------------------------------------------------------------------------------------
rt_camera build_camera(const CameraSpec& s) {
  rt_camera c{};
  // Dimmensions::from_two_of_three(None, Some(w), Some(r)) (camera/mod.rs:150-159)
  double ratio = (double)s.ratio_num / (double)s.ratio_den;
  c.image_width = s.width;
  c.image_height = (int32_t)((double)s.width / ratio);
  // CameraBuilder::build (camera/mod.rs:44-60)
  double theta = s.vfov * 3.14159265358979323846 / 180.0;
  double h = std::tan(theta / 2.0);
  c.height = 2.0 * h;
  c.width = ratio * c.height;
  c.focal_length = s.focal_length;
  c.has_lens = s.has_aperture ? 1 : 0;
  c.lens_radius = s.has_aperture ? s.aperture / 2.0 : 0.0;
  // CameraPosition::look_at (camera/mod.rs:72-86)
  Vec3 w = s.look_from - s.look_at;
  double fl = w.length();
  w = Vec3(w.x / fl, w.y / fl, w.z / fl);
  Vec3 u = s.up.cross(w).unit();
  Vec3 v = w.cross(u);
  c.origin[0] = s.look_from.x; c.origin[1] = s.look_from.y; c.origin[2] = s.look_from.z;
  c.w[0] = w.x; c.w[1] = w.y; c.w[2] = w.z;
  c.u[0] = u.x; c.u[1] = u.y; c.u[2] = u.z;
  c.v[0] = v.x; c.v[1] = v.y; c.v[2] = v.z;
  c.focus_length = s.override_focus ? s.focus_length : fl;
  c.time0 = s.time0;
  c.time1 = s.time1;
  return c;
}

CameraSpec default_camera_spec(int32_t width, int32_t rn, int32_t rd, double vfov, double focal_length, double aperture) {
  CameraSpec s;
  s.width = width;
  s.ratio_num = rn;
  s.ratio_den = rd;
  s.vfov = vfov;
  s.focal_length = focal_length;
  s.has_aperture = true;
  s.aperture = aperture;
  return s;
}

CameraSpec cornell_camera_spec(int32_t width) {
  CameraSpec s;
  s.width = width;
  s.ratio_num = 1;
  s.ratio_den = 1;
  s.vfov = 40.0;
  s.focal_length = 1.0;
  s.aperture = 0.00001;
  s.look_from = Vec3(278.0, 278.0, -800.0);
  s.look_at = Vec3(278.0, 278.0, 0.0);
  s.up = Vec3(0.0, 1.0, 0.0);
  return s;
}

CameraSpec spheres_camera_spec(int32_t width, int32_t rn, int32_t rd) {
  CameraSpec s = default_camera_spec(width, rn, rd, 35.0, 1.0, 0.001);
  s.look_from = Vec3(40.0, 25.0, 35.0);
  s.look_at = Vec3(0.0, 0.0, 0.0);
  return s;
}

// book 2 §10: lookfrom (478, 278, -600), lookat (278, 278, 0), vfov 40, aperture 0, focus 10,
// shutter [0, 1] (the book's camera has no lens at aperture 0: no disk draws)
CameraSpec final_camera_spec(int32_t width, int32_t rn, int32_t rd) {
  CameraSpec s = default_camera_spec(width, rn, rd, 40.0, 1.0, 0.0);
  s.has_aperture = false;
  s.look_from = Vec3(478.0, 278.0, -600.0);
  s.look_at = Vec3(278.0, 278.0, 0.0);
  s.time0 = 0.0;
  s.time1 = 1.0;
  return s;
}

bool aspect_ratio_from_name(const std::string& n, int32_t* num, int32_t* den) {
  struct R {
    const char* name;
    int32_t a, b;
  };
  static const R table[] = {{"std3x2", 3, 2}, {"std16x9", 16, 9}, {"std16x10", 16, 10}, {"square", 1, 1},
                            {"target-iphone", 1170, 2532}};
  for (const R& r : table)
    if (n == r.name) {
      *num = r.a;
      *den = r.b;
      return true;
    }
  return false;
}

bool builtin_scene(const std::string& name, uint64_t seed, SceneBuilder* out, std::string* err) {
  if (name == "random") *out = random_scene(seed, false);
  else if (name == "random-night") *out = random_scene(seed, true);
  else if (name == "demo") *out = create_scene();
  else if (name == "perlin") *out = create_perlin_demo();
  else if (name == "earth") *out = create_earth_demo();
  else if (name == "box-light" || name == "boxlight") *out = create_box_light();
  else if (name == "cornell") *out = create_cornell_box();
  else if (name.rfind("spheres", 0) == 0) {
    int side = 11;
    if (name.size() > 8 && name[7] == ':') side = std::atoi(name.c_str() + 8);
    if (side < 1 || side > 64) {
      *err = "spheres side length must be in [1, 64]";
      return false;
    }
    *out = gen_spheres_scene(seed, side);
  } else if (name.rfind("final", 0) == 0) {
    // final[:n_ground[:n_cluster]] (book: 20 and 1000)
    int g = 20, n = 1000;
    if (name.size() > 6 && name[5] == ':') {
      g = std::atoi(name.c_str() + 6);
      const size_t c2 = name.find(':', 6);
      if (c2 != std::string::npos) n = std::atoi(name.c_str() + c2 + 1);
    }
    if (g < 0 || g > 1000 || n < 0 || n > 1000000) {
      *err = "final scene: n_ground in [0, 1000], n_cluster in [0, 1e6]";
      return false;
    }
    *out = final_scene(seed, g, n);
  } else {
    *err = "unknown scene `" + name + "`";
    return false;
  }
  return true;
}

SceneBuilder create_scene() {
  SceneBuilder scene;
  Material mat_ground = Material::lambertian(TextureLoader::solid(0.8, 0.8, 0.0));
  Material mat_center = Material::lambertian(TextureLoader::solid(0.1, 0.2, 0.5));
  Material mat_left = Material::dielectric(1.5);
  double zero = 0.0;
  Material mat_right = Material::metal(Vec3(0.8, 0.6, 0.2), &zero);
  scene.add(Geometry::sphere(Vec3(0.0, -100.5, -1.0), 100.0), mat_ground);
  scene.add(Geometry::sphere(Vec3(0.0, 0.0, -1.0), 0.5), mat_center);
  scene.add(Geometry::sphere(Vec3(-1.0, 0.0, -1.0), 0.5), mat_left);
  scene.add(Geometry::sphere(Vec3(-1.0, 0.0, -1.0), -0.4), mat_left);  // invisible: inverted bbox (sphere.rs:54-60)
  scene.add(Geometry::sphere(Vec3(1.0, 0.0, -1.0), 0.5), mat_right);
  return scene;
}

}  // namespace host
