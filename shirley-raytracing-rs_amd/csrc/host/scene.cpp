// scene.cpp — SceneBuilder model, serde-JSON interchange, finalize (texture load + Perlin tables).
#include "scene.hpp"

#include <zlib.h>

#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

#include "rng.hpp"

namespace host {

double Vec3::length() const { return std::sqrt(dot(*this)); }
Vec3 Vec3::unit() const {
  double n = length();
  return {x / n, y / n, z / n};
}

// ---------------------------------------------------------------------------------------------
TextureLoader TextureLoader::solid(double r, double g, double b) { return solid_from_vec(Vec3(r, g, b)); }
TextureLoader TextureLoader::solid_from_vec(Vec3 v) {
  TextureLoader t;
  t.kind = Solid;
  t.color = v;
  return t;
}
TextureLoader TextureLoader::checker(double size, TextureLoader odd, TextureLoader even) {
  TextureLoader t;
  t.kind = Checker;
  t.scalar = size;
  t.odd = std::make_shared<TextureLoader>(std::move(odd));
  t.even = std::make_shared<TextureLoader>(std::move(even));
  return t;
}
TextureLoader TextureLoader::noise(double scale) {
  TextureLoader t;
  t.kind = Perlin;
  t.scalar = scale;
  return t;
}
TextureLoader TextureLoader::earth() {
  TextureLoader t;
  t.kind = EarthBuiltin;
  return t;
}
TextureLoader TextureLoader::image(std::string path) {
  TextureLoader t;
  t.kind = ImagePath;
  t.path = std::move(path);
  return t;
}

static std::string bits(double v) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  char b[24];
  std::snprintf(b, sizeof b, "%016" PRIx64, u);
  return b;
}

std::string TextureLoader::key() const {
  switch (kind) {
    case Solid: return "S(" + bits(color.x) + "," + bits(color.y) + "," + bits(color.z) + ")";
    case ImagePath: return "I(" + path + ")";
    case Perlin: return "P(" + bits(scalar) + ")";
    case EarthBuiltin: return "E";
    case Checker: return "C(" + bits(scalar) + "," + odd->key() + "," + even->key() + ")";
  }
  return "?";
}

Material Material::metal(Vec3 albedo, const double* fuzz) {
  Material m;
  m.kind = Metal;
  m.albedo = albedo;
  double f = fuzz ? *fuzz : 0.0;  // fuzz.unwrap_or(0.0)
  if (f > 1.0) f = 1.0;
  m.fuzz = f;
  return m;
}
Material Material::dielectric(double ir) {
  Material m;
  m.kind = Dielectric;
  m.ir = ir;
  return m;
}
Material Material::lambertian(TextureLoader t) {
  Material m;
  m.kind = Lambertian;
  m.tex = std::move(t);
  return m;
}
Material Material::diffuse_light(TextureLoader t) {
  Material m;
  m.kind = DiffuseLight;
  m.tex = std::move(t);
  return m;
}
Material Material::fairy_light(TextureLoader t) {
  Material m;
  m.kind = FairyLight;
  m.tex = std::move(t);
  return m;
}

Material Material::isotropic(TextureLoader t) {
  Material m;
  m.kind = Isotropic;
  m.tex = std::move(t);
  return m;
}

Geometry Geometry::moving_sphere(Vec3 c0, Vec3 c1, double time0, double time1, double r) {
  Geometry g;
  g.kind = RT_GEOM_MOVING_SPHERE;
  g.p[0] = c0.x; g.p[1] = c0.y; g.p[2] = c0.z; g.p[3] = r;
  g.q[0] = c1.x; g.q[1] = c1.y; g.q[2] = c1.z; g.q[3] = time0; g.q[4] = time1;
  return g;
}
Geometry Geometry::with_medium(double d) const {
  Geometry g = *this;
  g.medium = true;
  g.density = d;
  return g;
}
Geometry Geometry::with_transform(double deg, Vec3 off) const {
  Geometry g = *this;
  g.transform = true;
  g.rotate_y = deg;
  g.offset = off;
  return g;
}
Geometry Geometry::sphere(Vec3 c, double r) {
  Geometry g;
  g.kind = RT_GEOM_SPHERE;
  g.p[0] = c.x; g.p[1] = c.y; g.p[2] = c.z; g.p[3] = r;
  return g;
}
static Geometry rect(int32_t kind, double a, double b, double c, double d, double k) {
  Geometry g;
  g.kind = kind;
  g.p[0] = a; g.p[1] = b; g.p[2] = c; g.p[3] = d; g.p[4] = k;
  return g;
}
Geometry Geometry::xy_rect(double a, double b, double c, double d, double k) { return rect(RT_GEOM_RECT_XY, a, b, c, d, k); }
Geometry Geometry::yz_rect(double a, double b, double c, double d, double k) { return rect(RT_GEOM_RECT_YZ, a, b, c, d, k); }
Geometry Geometry::xz_rect(double a, double b, double c, double d, double k) { return rect(RT_GEOM_RECT_XZ, a, b, c, d, k); }
Geometry Geometry::rect_box(Vec3 p0, Vec3 p1) {
  Geometry g;
  g.kind = RT_GEOM_RECT_BOX;
  g.p[0] = p0.x; g.p[1] = p0.y; g.p[2] = p0.z; g.p[3] = p1.x; g.p[4] = p1.y; g.p[5] = p1.z;
  return g;
}

void SceneBuilder::set_skybox(int32_t kind, Vec3 color) {
  skybox = kind;
  sky_color = color;
}

// ---------------------------------------------------------------------------------------------
// JSON (serde externally-tagged enums; Vec3 = {"vec":[x,y,z]}, newtypes transparent)
// ---------------------------------------------------------------------------------------------
static Json jvec(const Vec3& v) {
  Json a = Json::array();
  a.push(Json::number(v.x));
  a.push(Json::number(v.y));
  a.push(Json::number(v.z));
  return Json::object().set("vec", a);
}
static Vec3 pvec(const Json& j) {
  const Json* a = (j.kind == Json::Object) ? j.find("vec") : &j;
  if (!a || a->kind != Json::Array || a->arr.size() != 3) throw std::runtime_error("expected Vec3 {\"vec\":[x,y,z]}");
  return Vec3(a->arr[0].as_number(), a->arr[1].as_number(), a->arr[2].as_number());
}
static Json tagged(const char* tag, Json v) { return Json::object().set(tag, std::move(v)); }
static const char* variant(const Json& j, const Json** payload) {
  if (j.kind == Json::String) {
    *payload = nullptr;
    return j.str.c_str();
  }
  if (j.kind != Json::Object || j.obj.size() != 1) throw std::runtime_error("expected an externally tagged enum");
  *payload = &j.obj[0].second;
  return j.obj[0].first.c_str();
}

static Json tex_json(const TextureLoader& t) {
  switch (t.kind) {
    case TextureLoader::Solid: return tagged("Solid", jvec(t.color));
    case TextureLoader::ImagePath: return tagged("ImagePath", Json::string(t.path));
    case TextureLoader::Perlin: return tagged("Perlin", Json::number(t.scalar));
    case TextureLoader::EarthBuiltin: return Json::string("EarthBuiltin");
    case TextureLoader::Checker: {
      Json c = Json::object();
      c.set("size", Json::number(t.scalar)).set("odd", tex_json(*t.odd)).set("even", tex_json(*t.even));
      return tagged("Checker", c);
    }
  }
  return Json();
}
static TextureLoader tex_parse(const Json& j) {
  const Json* p;
  std::string tag = variant(j, &p);
  if (tag == "EarthBuiltin") return TextureLoader::earth();
  if (!p) throw std::runtime_error("texture variant `" + tag + "` needs a payload");
  if (tag == "Solid") return TextureLoader::solid_from_vec(pvec(*p));
  if (tag == "ImagePath") return TextureLoader::image(p->as_string());
  if (tag == "Perlin") return TextureLoader::noise(p->as_number());
  if (tag == "Checker")
    return TextureLoader::checker(p->at("size").as_number(), tex_parse(p->at("odd")), tex_parse(p->at("even")));
  throw std::runtime_error("unknown texture variant `" + tag + "`");
}

static Json rect_json(double a, double b, double c, double d, double k) {
  Json r = Json::object();
  r.set("d1_min", Json::number(a)).set("d1_max", Json::number(b)).set("d2_min", Json::number(c));
  r.set("d2_max", Json::number(d)).set("offset", Json::number(k));
  return r;
}
static Json geom_json(const Geometry& g) {
  const double* p = g.p;
  switch (g.kind) {
    case RT_GEOM_SPHERE:
      return tagged("Sphere", Json::object().set("center", jvec(Vec3(p[0], p[1], p[2]))).set("radius", Json::number(p[3])));
    case RT_GEOM_RECT_XY: return tagged("RectXY", rect_json(p[0], p[1], p[2], p[3], p[4]));
    case RT_GEOM_RECT_YZ: return tagged("RectYZ", rect_json(p[0], p[1], p[2], p[3], p[4]));
    case RT_GEOM_RECT_XZ: return tagged("RectXZ", rect_json(p[0], p[1], p[2], p[3], p[4]));
    case RT_GEOM_RECT_BOX: {
      // RectBox::new sides (rect.rs:111-129)
      Json o = Json::object();
      o.set("min", jvec(Vec3(p[0], p[1], p[2]))).set("max", jvec(Vec3(p[3], p[4], p[5])));
      Json xy = Json::array(), yz = Json::array(), xz = Json::array();
      xy.push(rect_json(p[0], p[3], p[1], p[4], p[5]));
      xy.push(rect_json(p[0], p[3], p[1], p[4], p[2]));
      yz.push(rect_json(p[1], p[4], p[2], p[5], p[3]));
      yz.push(rect_json(p[1], p[4], p[2], p[5], p[0]));
      xz.push(rect_json(p[0], p[3], p[2], p[5], p[4]));
      xz.push(rect_json(p[0], p[3], p[2], p[5], p[1]));
      o.set("xy_sides", xy).set("yz_sides", yz).set("xz_sides", xz);
      return tagged("RectBox", o);
    }
    case RT_GEOM_MOVING_SPHERE: {
      Json o = Json::object();
      o.set("center0", jvec(Vec3(p[0], p[1], p[2]))).set("center1", jvec(Vec3(g.q[0], g.q[1], g.q[2])));
      o.set("time0", Json::number(g.q[3])).set("time1", Json::number(g.q[4])).set("radius", Json::number(p[3]));
      return tagged("MovingSphere", o);
    }
  }
  return Json();
}
static Geometry geom_parse(const Json& j) {
  const Json* p;
  std::string tag = variant(j, &p);
  if (!p) throw std::runtime_error("geometry variant `" + tag + "` needs a payload");
  if (tag == "Sphere") return Geometry::sphere(pvec(p->at("center")), p->at("radius").as_number());
  auto rf = [&](const char* k) { return p->at(k).as_number(); };
  if (tag == "RectXY") return Geometry::xy_rect(rf("d1_min"), rf("d1_max"), rf("d2_min"), rf("d2_max"), rf("offset"));
  if (tag == "RectYZ") return Geometry::yz_rect(rf("d1_min"), rf("d1_max"), rf("d2_min"), rf("d2_max"), rf("offset"));
  if (tag == "RectXZ") return Geometry::xz_rect(rf("d1_min"), rf("d1_max"), rf("d2_min"), rf("d2_max"), rf("offset"));
  if (tag == "RectBox") return Geometry::rect_box(pvec(p->at("min")), pvec(p->at("max")));
  if (tag == "MovingSphere")
    return Geometry::moving_sphere(pvec(p->at("center0")), pvec(p->at("center1")), rf("time0"), rf("time1"),
                                   rf("radius"));
  throw std::runtime_error("unknown geometry variant `" + tag + "`");
}

static Json mat_json(const Material& m) {
  switch (m.kind) {
    case Material::Metal: return tagged("Metal", Json::object().set("albedo", jvec(m.albedo)).set("fuzz", Json::number(m.fuzz)));
    case Material::Dielectric: return tagged("Dielectric", Json::object().set("ir", Json::number(m.ir)));
    case Material::Lambertian: return tagged("Lambertian", Json::object().set("albedo", tex_json(m.tex)));
    case Material::DiffuseLight: return tagged("DiffuseLight", Json::object().set("albedo", tex_json(m.tex)));
    case Material::FairyLight: return tagged("FairyLight", Json::object().set("albedo", tex_json(m.tex)));
    case Material::Isotropic: return tagged("Isotropic", Json::object().set("albedo", tex_json(m.tex)));
  }
  return Json();
}
static Material mat_parse(const Json& j) {
  const Json* p;
  std::string tag = variant(j, &p);
  if (!p) throw std::runtime_error("material variant `" + tag + "` needs a payload");
  if (tag == "Metal") {
    // deserialised directly (serde), so the stored fuzz is taken as is
    Material m;
    m.kind = Material::Metal;
    m.albedo = pvec(p->at("albedo"));
    m.fuzz = p->at("fuzz").as_number();
    return m;
  }
  if (tag == "Dielectric") return Material::dielectric(p->at("ir").as_number());
  if (tag == "Lambertian") return Material::lambertian(tex_parse(p->at("albedo")));
  if (tag == "DiffuseLight") return Material::diffuse_light(tex_parse(p->at("albedo")));
  if (tag == "FairyLight") return Material::fairy_light(tex_parse(p->at("albedo")));
  if (tag == "Isotropic") return Material::isotropic(tex_parse(p->at("albedo")));
  throw std::runtime_error("unknown material variant `" + tag + "`");
}

Json SceneBuilder::to_json() const {
  Json root = Json::object();
  if (skybox == RT_SKY_ABOVE) root.set("skybox", Json::string("Above"));
  else if (skybox == RT_SKY_NONE) root.set("skybox", Json::string("None"));
  else root.set("skybox", tagged("Flat", jvec(sky_color)));
  Json objs = Json::array();
  for (const auto& gm : objects) {
    Json o = Json::object();
    o.set("geometry", geom_json(gm.first)).set("material", mat_json(gm.second));
    if (gm.first.medium) o.set("medium", Json::object().set("density", Json::number(gm.first.density)));
    if (gm.first.transform)
      o.set("transform", Json::object().set("rotate_y", Json::number(gm.first.rotate_y)).set("offset", jvec(gm.first.offset)));
    objs.push(o);
  }
  root.set("objects", objs);
  if (has_perlin_seed) root.set("perlin_seed", Json::number((double)perlin_seed));
  return root;
}

SceneBuilder SceneBuilder::from_json(const Json& j) {
  SceneBuilder b;
  const Json* p;
  std::string sky = variant(j.at("skybox"), &p);
  if (sky == "Above") b.skybox = RT_SKY_ABOVE;
  else if (sky == "None") b.skybox = RT_SKY_NONE;
  else if (sky == "Flat" && p) { b.skybox = RT_SKY_FLAT; b.sky_color = pvec(*p); }
  else throw std::runtime_error("unknown skybox `" + sky + "`");
  const Json& objs = j.at("objects");
  if (objs.kind != Json::Array) throw std::runtime_error("`objects` must be an array");
  for (const Json& o : objs.arr) {
    Geometry g = geom_parse(o.at("geometry"));
    if (const Json* m = o.find("medium")) g = g.with_medium(m->at("density").as_number());
    if (const Json* t = o.find("transform")) g = g.with_transform(t->at("rotate_y").as_number(), pvec(t->at("offset")));
    b.add(g, mat_parse(o.at("material")));
  }
  if (const Json* ps = j.find("perlin_seed")) {
    b.has_perlin_seed = true;
    b.perlin_seed = (uint64_t)ps->as_number();
  }
  return b;
}

// ---------------------------------------------------------------------------------------------
// finalize
// ---------------------------------------------------------------------------------------------
void perlin_generate(uint64_t seed, uint32_t table_index, rt_perlin_table* out) {
  SceneRng rng(seed, kStreamPerlinBase + table_index);
  for (int i = 0; i < 256; ++i) {  // Vec3::random_range_with_rng(-1, 1): x, y, z
    out->ranfloat[i][0] = rng.random_real(-1.0, 1.0);
    out->ranfloat[i][1] = rng.random_real(-1.0, 1.0);
    out->ranfloat[i][2] = rng.random_real(-1.0, 1.0);
  }
  int32_t* perms[3] = {out->perm_x, out->perm_y, out->perm_z};
  for (int32_t* p : perms) {  // perlin_generate_perm + permute (perlin/mod.rs:126-139)
    for (int i = 0; i < 256; ++i) p[i] = i;
    for (int idx = 255; idx >= 1; --idx) {
      int target = (int)rng.gen_range((uint64_t)idx + 1);
      std::swap(p[idx], p[target]);
    }
  }
}

static bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

// "RGB8 <w> <h>\n" + w*h*3 bytes, gzip-wrapped (tools/decode_earthmap.py)
static bool parse_rgb8_gz(const unsigned char* gz, size_t gz_len, const std::string& what, int32_t* w, int32_t* h,
                          std::vector<uint8_t>* rgb, std::string* err) {
  z_stream zs{};
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) { *err = "inflateInit failed for " + what; return false; }
  zs.next_in = const_cast<Bytef*>(gz);
  zs.avail_in = (uInt)gz_len;
  std::string data;
  unsigned char buf[1 << 16];
  int zr;
  do {
    zs.next_out = buf;
    zs.avail_out = sizeof buf;
    zr = inflate(&zs, Z_NO_FLUSH);
    data.append((const char*)buf, sizeof buf - zs.avail_out);
  } while (zr == Z_OK);
  inflateEnd(&zs);
  if (zr != Z_STREAM_END) { *err = "corrupt gzip stream in " + what; return false; }
  size_t nl = data.find('\n');
  int ww = 0, hh = 0;
  if (nl == std::string::npos || std::sscanf(data.c_str(), "RGB8 %d %d", &ww, &hh) != 2 || ww < 1 || hh < 1) {
    *err = "bad RGB8 header in " + what;
    return false;
  }
  size_t need = (size_t)ww * hh * 3;
  if (data.size() - nl - 1 != need) { *err = "truncated RGB8 data in " + what; return false; }
  rgb->assign(data.begin() + (long)nl + 1, data.end());
  *w = ww;
  *h = hh;
  return true;
}

static bool load_rgb8_gz(const std::string& path, int32_t* w, int32_t* h, std::vector<uint8_t>* rgb, std::string* err) {
  std::string gz;
  if (!read_file(path, &gz)) { *err = "cannot open " + path; return false; }
  return parse_rgb8_gz((const unsigned char*)gz.data(), gz.size(), path, w, h, rgb, err);
}

// linked in by earth_embed.S (the reference's include_bytes!, image_texture.rs:11,18-20)
extern "C" const unsigned char shirley_earth_rgb8_gz[];
extern "C" const unsigned char shirley_earth_rgb8_gz_end[];

bool load_earth_builtin(int32_t* w, int32_t* h, std::vector<uint8_t>* rgb, std::string* err) {
  return parse_rgb8_gz(shirley_earth_rgb8_gz, (size_t)(shirley_earth_rgb8_gz_end - shirley_earth_rgb8_gz),
                       "EarthBuiltin (embedded)", w, h, rgb, err);
}

static uint32_t be32(const unsigned char* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// 8-bit non-interlaced PNG (grey, RGB, grey+alpha, RGBA) -> RGB8
static bool load_png(const std::string& data, int32_t* w, int32_t* h, std::vector<uint8_t>* rgb, std::string* err) {
  const unsigned char* d = (const unsigned char*)data.data();
  size_t n = data.size(), pos = 8;
  uint32_t W = 0, H = 0;
  int depth = 0, ctype = 0, interlace = 0;
  std::string idat;
  while (pos + 12 <= n) {
    uint32_t len = be32(d + pos);
    std::string type((const char*)d + pos + 4, 4);
    if (pos + 12 + len > n) break;
    const unsigned char* c = d + pos + 8;
    if (type == "IHDR") { W = be32(c); H = be32(c + 4); depth = c[8]; ctype = c[9]; interlace = c[12]; }
    else if (type == "IDAT") idat.append((const char*)c, len);
    else if (type == "IEND") break;
    pos += 12 + len;
  }
  int ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
  if (!W || !H || depth != 8 || ch == 0 || interlace) { *err = "unsupported PNG (need 8-bit, non-interlaced, grey/RGB[A])"; return false; }
  size_t stride = (size_t)W * ch;
  std::vector<unsigned char> raw((stride + 1) * H);
  uLongf rl = (uLongf)raw.size();
  if (uncompress(raw.data(), &rl, (const Bytef*)idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size()) {
    *err = "PNG inflate failed";
    return false;
  }
  std::vector<unsigned char> img(stride * H), prev(stride, 0);
  for (uint32_t y = 0; y < H; ++y) {
    unsigned char f = raw[y * (stride + 1)];
    const unsigned char* s = &raw[y * (stride + 1) + 1];
    unsigned char* o = &img[y * stride];
    for (size_t x = 0; x < stride; ++x) {
      int a = x >= (size_t)ch ? o[x - ch] : 0, b = prev[x], c = x >= (size_t)ch ? prev[x - ch] : 0;
      int v = s[x];
      switch (f) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: {
          int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
          v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
          break;
        }
        default: *err = "bad PNG filter"; return false;
      }
      o[x] = (unsigned char)v;
    }
    std::memcpy(prev.data(), o, stride);
  }
  rgb->resize((size_t)W * H * 3);
  for (size_t i = 0; i < (size_t)W * H; ++i)
    for (int k = 0; k < 3; ++k) (*rgb)[i * 3 + k] = img[i * ch + (ch >= 3 ? k : 0)];
  *w = (int32_t)W;
  *h = (int32_t)H;
  return true;
}

bool load_image_file(const std::string& path, int32_t* w, int32_t* h, std::vector<uint8_t>* rgb, std::string* err) {
  if (path.size() > 8 && path.compare(path.size() - 8, 8, ".rgb8.gz") == 0) return load_rgb8_gz(path, w, h, rgb, err);
  std::string data;
  if (!read_file(path, &data)) { *err = "cannot open " + path; return false; }
  if (data.size() > 8 && std::memcmp(data.data(), "\x89PNG\r\n\x1a\n", 8) == 0) return load_png(data, w, h, rgb, err);
  *err = "unsupported image format: " + path + " (PNG or .rgb8.gz; decode JPEGs with tools/decode_earthmap.py)";
  return false;
}

rt_scene_desc SceneDesc::view() const {
  rt_scene_desc d{};
  d.sky = sky;
  for (int k = 0; k < 3; ++k) d.sky_color[k] = sky_color[k];
  d.n_objects = (int32_t)objects.size();
  d.objects = objects.data();
  d.n_materials = (int32_t)materials.size();
  d.materials = materials.data();
  d.n_textures = (int32_t)textures.size();
  d.textures = textures.data();
  d.n_perlin = (int32_t)perlin.size();
  d.perlin = perlin.data();
  d.n_images = (int32_t)images.size();
  d.images = images.data();
  return d;
}

namespace {
struct Loader {
  SceneDesc& d;
  uint64_t seed;
  std::map<std::string, int32_t> image_cache;  // identical files share texels (no semantic change)

  int32_t earth_image = -1;  // EarthBuiltin's image, once loaded (the embedded texels, earth_embed.S)

  // builtin: EarthBuiltin; else `path` names a user file (ImagePath)
  int32_t image(const std::string& path, bool builtin = false) {
    if (builtin && earth_image >= 0) return earth_image;
    if (!builtin) {
      auto it = image_cache.find(path);
      if (it != image_cache.end()) return it->second;
    }
    int32_t w = 0, h = 0;
    std::vector<uint8_t> px;
    std::string err;
    bool ok = builtin ? load_earth_builtin(&w, &h, &px, &err) : load_image_file(path, &w, &h, &px, &err);
    if (!ok) throw std::runtime_error(err);
    d.image_pixels.push_back(std::move(px));
    rt_image im{w, h, nullptr};
    d.images.push_back(im);
    int32_t idx = (int32_t)d.images.size() - 1;
    if (builtin) earth_image = idx;
    else image_cache[path] = idx;
    return idx;
  }

  // TextureLoader::load (loader.rs:47-60): a fresh instance per call; Checker loads odd then even
  int32_t load(const TextureLoader& t) {
    rt_texture x{};
    x.odd = x.even = x.table = -1;
    switch (t.kind) {
      case TextureLoader::Solid:
        x.kind = RT_TEX_SOLID;
        x.color[0] = t.color.x; x.color[1] = t.color.y; x.color[2] = t.color.z;
        break;
      case TextureLoader::Perlin: {
        x.kind = RT_TEX_PERLIN;
        x.scale = t.scalar;
        rt_perlin_table T;
        perlin_generate(seed, (uint32_t)d.perlin.size(), &T);
        d.perlin.push_back(T);
        x.table = (int32_t)d.perlin.size() - 1;
        break;
      }
      case TextureLoader::EarthBuiltin:
        x.kind = RT_TEX_IMAGE;
        x.table = image(std::string(), true);
        break;
      case TextureLoader::ImagePath:
        x.kind = RT_TEX_IMAGE;
        x.table = image(t.path);
        break;
      case TextureLoader::Checker: {
        int32_t odd = load(*t.odd);
        int32_t even = load(*t.even);
        x.kind = RT_TEX_CHECKER;
        x.odd = odd;
        x.even = even;
        x.scale = t.scalar;
        break;
      }
    }
    d.textures.push_back(x);
    return (int32_t)d.textures.size() - 1;
  }
};
}  // namespace

SceneDesc SceneBuilder::finalize(uint64_t seed) const {
  SceneDesc d;
  d.sky = skybox;
  d.sky_color[0] = sky_color.x;
  d.sky_color[1] = sky_color.y;
  d.sky_color[2] = sky_color.z;
  Loader L{d, has_perlin_seed ? perlin_seed : seed, {}};
  std::map<std::string, int32_t> manager;  // TextureManager (loader.rs:113-131)
  for (const auto& gm : objects) {
    const Material& m = gm.second;
    rt_material rm{};
    rm.texture = -1;
    switch (m.kind) {
      case Material::Metal:
        rm.kind = RT_MAT_METAL;
        rm.albedo[0] = m.albedo.x; rm.albedo[1] = m.albedo.y; rm.albedo[2] = m.albedo.z;
        rm.param = m.fuzz;
        break;
      case Material::Dielectric:
        rm.kind = RT_MAT_DIELECTRIC;
        rm.param = m.ir;
        break;
      default: {
        rm.kind = m.kind == Material::Lambertian     ? RT_MAT_LAMBERTIAN
                  : m.kind == Material::DiffuseLight ? RT_MAT_DIFFUSE_LIGHT
                  : m.kind == Material::Isotropic    ? RT_MAT_ISOTROPIC
                                                     : RT_MAT_FAIRY_LIGHT;
        std::string key = m.tex.key();
        auto it = manager.find(key);
        if (it != manager.end()) {
          rm.texture = it->second;
        } else {
          rm.texture = L.load(m.tex);
          manager[key] = rm.texture;
        }
      }
    }
    d.materials.push_back(rm);
    rt_object o{};
    o.geometry = gm.first.kind;
    o.material = (int32_t)d.materials.size() - 1;
    const Geometry& g = gm.first;
    for (int k = 0; k < 6; ++k) o.p[k] = g.p[k];
    for (int k = 0; k < 5; ++k) o.q[k] = g.q[k];
    o.medium = g.medium ? 1 : 0;
    o.density = g.density;
    o.transform = g.transform ? 1 : 0;
    o.rotate_y_deg = g.rotate_y;
    o.offset[0] = g.offset.x; o.offset[1] = g.offset.y; o.offset[2] = g.offset.z;
    d.objects.push_back(o);
  }
  for (size_t i = 0; i < d.images.size(); ++i) d.images[i].rgb = d.image_pixels[i].data();
  return d;
}

}  // namespace host
