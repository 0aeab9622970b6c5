// host_api.cpp — C API over the C++ host layer (include/shirley_host.h).
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "../../../include/shirley_host.h"
#include "scene.hpp"
#include "scenes.hpp"

using namespace host;

struct sh_scene {
  SceneBuilder b;
};
struct sh_desc {
  SceneDesc d;
  rt_scene_desc view;
};

namespace {
thread_local std::string g_err;
int fail(const std::string& m) {
  g_err = m;
  return RT_E_INVALID;
}
}  // namespace

extern "C" {

const char* sh_last_error(void) { return g_err.c_str(); }

sh_scene* sh_scene_new(void) { return new sh_scene(); }
void sh_scene_free(sh_scene* s) { delete s; }

int sh_scene_set_skybox(sh_scene* s, int32_t sky, const double color[3]) {
  if (!s || sky < RT_SKY_ABOVE || sky > RT_SKY_NONE) return fail("bad skybox");
  Vec3 c = color ? Vec3(color[0], color[1], color[2]) : Vec3();
  s->b.set_skybox(sky, c);
  return RT_OK;
}

int sh_scene_add_json(sh_scene* s, const char* object_json) {
  if (!s || !object_json) return fail("NULL argument");
  try {
    Json j = JsonParser(object_json).parse();
    SceneBuilder tmp = SceneBuilder::from_json(Json::object().set("skybox", Json::string("Above")).set("objects", [&] {
      Json a = Json::array();
      a.push(j);
      return a;
    }()));
    s->b.add(tmp.objects[0].first, tmp.objects[0].second);
  } catch (const std::exception& e) {
    return fail(e.what());
  }
  return RT_OK;
}

int32_t sh_scene_len(const sh_scene* s) { return s ? (int32_t)s->b.objects.size() : 0; }

int sh_scene_to_json(const sh_scene* s, int32_t pretty, char* buf, size_t cap, size_t* needed) {
  if (!s) return fail("NULL scene");
  std::string out;
  json_write(s->b.to_json(), out, 0, pretty != 0);
  if (needed) *needed = out.size() + 1;
  if (buf) {
    if (cap < out.size() + 1) return fail("buffer too small");
    std::memcpy(buf, out.c_str(), out.size() + 1);
  }
  return RT_OK;
}

int sh_scene_from_json(const char* json, sh_scene** out) {
  if (!json || !out) return fail("NULL argument");
  try {
    Json j = JsonParser(json).parse();
    std::unique_ptr<sh_scene> s(new sh_scene());  // freed if from_json throws (found by tools/sanitize)
    s->b = SceneBuilder::from_json(j);
    *out = s.release();
  } catch (const std::exception& e) {
    return fail(e.what());
  }
  return RT_OK;
}

int sh_scene_builtin(const char* name, uint64_t seed, sh_scene** out) {
  if (!name || !out) return fail("NULL argument");
  sh_scene* s = new sh_scene();
  std::string err;
  if (!builtin_scene(name, seed, &s->b, &err)) {
    delete s;
    return fail(err);
  }
  *out = s;
  return RT_OK;
}

int sh_scene_finalize(const sh_scene* s, uint64_t seed, sh_desc** out) {
  if (!s || !out) return fail("NULL argument");
  try {
    std::unique_ptr<sh_desc> d(new sh_desc());  // freed if finalize throws
    d->d = s->b.finalize(seed);
    for (size_t i = 0; i < d->d.images.size(); ++i) d->d.images[i].rgb = d->d.image_pixels[i].data();
    d->view = d->d.view();
    *out = d.release();
  } catch (const std::exception& e) {
    return fail(e.what());
  }
  return RT_OK;
}

const rt_scene_desc* sh_desc_view(const sh_desc* d) { return d ? &d->view : nullptr; }
void sh_desc_free(sh_desc* d) { delete d; }

static CameraSpec spec_from(const sh_camera_spec* s) {
  CameraSpec c;
  c.width = s->width;
  c.ratio_num = s->ratio_num;
  c.ratio_den = s->ratio_den;
  c.vfov = s->vfov;
  c.focal_length = s->focal_length;
  c.has_aperture = s->has_aperture != 0;
  c.aperture = s->aperture;
  c.look_from = Vec3(s->look_from[0], s->look_from[1], s->look_from[2]);
  c.look_at = Vec3(s->look_at[0], s->look_at[1], s->look_at[2]);
  c.up = Vec3(s->up[0], s->up[1], s->up[2]);
  c.override_focus = s->override_focus != 0;
  c.focus_length = s->focus_length;
  c.time0 = s->time0;
  c.time1 = s->time1;
  return c;
}

static int check_spec(const CameraSpec& c) {
  if (c.width < 1 || c.ratio_num < 1 || c.ratio_den < 1) return fail("bad camera width / aspect ratio");
  double h = (double)c.width / ((double)c.ratio_num / (double)c.ratio_den);
  if (h < 1.0) return fail("camera height would be 0");
  return RT_OK;
}

int sh_camera_build(const sh_camera_spec* s, rt_camera* out) {
  if (!s || !out) return fail("NULL argument");
  CameraSpec c = spec_from(s);
  if (int st = check_spec(c)) return st;
  *out = build_camera(c);
  return RT_OK;
}

int sh_default_camera(int32_t width, const char* aspect, double vfov, double focal_length, double aperture,
                      rt_camera* out) {
  if (!out) return fail("NULL argument");
  int32_t n = 3, d = 2;
  if (aspect && !aspect_ratio_from_name(aspect, &n, &d)) return fail(std::string("unknown aspect ratio ") + aspect);
  CameraSpec c = default_camera_spec(width, n, d, vfov, focal_length, aperture);
  if (int st = check_spec(c)) return st;
  *out = build_camera(c);
  return RT_OK;
}

int sh_cornell_camera(int32_t width, rt_camera* out) {
  if (!out) return fail("NULL argument");
  CameraSpec c = cornell_camera_spec(width);
  if (int st = check_spec(c)) return st;
  *out = build_camera(c);
  return RT_OK;
}

int sh_scene_camera(const char* name, int32_t width, const char* aspect, double vfov, double focal_length,
                    double aperture, rt_camera* out) {
  if (!name || !out) return fail("NULL argument");
  std::string n = name;
  if (n == "cornell") return sh_cornell_camera(width, out);
  int32_t rn = 3, rd = 2;
  if (aspect && !aspect_ratio_from_name(aspect, &rn, &rd)) return fail(std::string("unknown aspect ratio ") + aspect);
  CameraSpec c = (n.rfind("spheres", 0) == 0) ? spheres_camera_spec(width, rn, rd)
                 : (n.rfind("final", 0) == 0)  ? final_camera_spec(width, rn, rd)
                                               : default_camera_spec(width, rn, rd, vfov, focal_length, aperture);
  if (int st = check_spec(c)) return st;
  *out = build_camera(c);
  return RT_OK;
}

int sh_perlin_generate(uint64_t seed, uint32_t table_index, rt_perlin_table* out) {
  if (!out) return fail("NULL argument");
  perlin_generate(seed, table_index, out);
  return RT_OK;
}

static void put32(std::string& s, uint32_t v) {
  s += (char)(v >> 24);
  s += (char)(v >> 16);
  s += (char)(v >> 8);
  s += (char)v;
}
static void chunk(std::string& png, const char* type, const std::string& data) {
  put32(png, (uint32_t)data.size());
  std::string td = std::string(type, 4) + data;
  png += td;
  put32(png, (uint32_t)crc32(0L, (const Bytef*)td.data(), (uInt)td.size()));
}

int sh_write_png(const char* path, const uint8_t* rgb, int32_t w, int32_t h) {
  if (!path || !rgb || w < 1 || h < 1) return fail("bad PNG arguments");
  std::string raw;
  raw.reserve((size_t)h * ((size_t)w * 3 + 1));
  for (int32_t y = 0; y < h; ++y) {
    raw += '\0';
    raw.append((const char*)rgb + (size_t)y * w * 3, (size_t)w * 3);
  }
  uLongf zl = compressBound((uLong)raw.size());
  std::string z(zl, '\0');
  if (compress2((Bytef*)&z[0], &zl, (const Bytef*)raw.data(), (uLong)raw.size(), 6) != Z_OK) return fail("deflate failed");
  z.resize(zl);
  std::string png("\x89PNG\r\n\x1a\n", 8), ihdr;
  put32(ihdr, (uint32_t)w);
  put32(ihdr, (uint32_t)h);
  ihdr += (char)8;  // bit depth
  ihdr += (char)2;  // RGB
  ihdr += (char)0;
  ihdr += (char)0;
  ihdr += (char)0;
  chunk(png, "IHDR", ihdr);
  chunk(png, "IDAT", z);
  chunk(png, "IEND", "");
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(std::string("cannot write ") + path);
  size_t n = std::fwrite(png.data(), 1, png.size(), f);
  std::fclose(f);
  return n == png.size() ? RT_OK : fail("short write");
}

int sh_load_image(const char* path, int32_t* w, int32_t* h, uint8_t** rgb) {
  if (!path || !w || !h || !rgb) return fail("NULL argument");
  std::vector<uint8_t> px;
  std::string err;
  if (!load_image_file(path, w, h, &px, &err)) return fail(err);
  *rgb = (uint8_t*)std::malloc(px.size());
  std::memcpy(*rgb, px.data(), px.size());
  return RT_OK;
}

void sh_free(void* p) { std::free(p); }

}  // extern "C"
