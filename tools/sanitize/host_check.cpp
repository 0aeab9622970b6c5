// host_check.cpp — ASan/UBSan driver for the CPU side of the boundary: the C++ host
// layer (serde-JSON SceneBuilder loader/saver, scenes, finalize, camera, PNG), the BVH builders of
// libshirley_rt (bvh_build.cpp) and the C oracle, compiled from their sources with
// -fsanitize=address,undefined (tools/sanitize/Makefile).  No GPU code is involved.
//
//   1. every builtin scene: build -> to_json -> from_json -> to_json (byte-equal round trip) ->
//      finalize -> both BVH builders over the objects' bounding boxes -> oracle scene -> a tiny
//      render + tonemap -> PNG;
//   2. a mutation fuzzer over the scenes' JSON (the input `ray-cli render saved` parses, reference
//      scenes.rs:128-134): byte flips, JSON-significant insertions, deletions, duplications,
//      truncations, extreme numbers, deep nesting, escapes.  Each mutant goes through from_json and,
//      when it parses, finalize + the builders + a 4x3 oracle render.  Errors are expected; crashes,
//      leaks and undefined behaviour are not (the sanitizers abort the run).
//
// usage: host_check <asset_dir> <n_mutants> [seed]
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/shirley_host.h"
#include "../../oracle/oracle.h"
#include "../../shirley-raytracing-rs_amd/csrc/rt/bvh_build.h"

namespace {

struct XorShift {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  size_t below(size_t n) { return n ? (size_t)(next() % n) : 0; }
};

int g_failures = 0;
#define CHECK(c, ...)                   \
  do {                                  \
    if (!(c)) {                         \
      std::fprintf(stderr, __VA_ARGS__); \
      std::fprintf(stderr, "\n");       \
      ++g_failures;                     \
    }                                   \
  } while (0)

std::string to_json(const sh_scene* s, int pretty) {
  size_t need = 0;
  if (sh_scene_to_json(s, pretty, nullptr, 0, &need) != 0 && need == 0) return {};
  std::string out(need, '\0');
  if (sh_scene_to_json(s, pretty, out.data(), out.size(), &need) != 0) return {};
  out.resize(need ? need - 1 : 0);
  return out;
}

// finalize + both builders + a tiny oracle render; returns 0 when every step succeeded
int exercise(const sh_scene* s, uint64_t seed, int w, int spp, bool big_ok) {
  sh_desc* d = nullptr;
  if (sh_scene_finalize(s, seed, &d) != 0) return 1;
  const rt_scene_desc* v = sh_desc_view(d);
  std::vector<rt::Box> boxes;
  for (int i = 0; i < v->n_objects; ++i) {
    double b[6];
    if (or_object_bbox(&v->objects[i], b)) {
      rt::Box bx;
      for (int k = 0; k < 3; ++k) {
        bx.mn[k] = b[k];
        bx.mx[k] = b[3 + k];
      }
      boxes.push_back(bx);
    }
  }
  rt::BuiltTree ref = rt::build_reference_tree(boxes);
  rt::BuiltTree sah = rt::build_sah_tree(boxes, false);  // 32-bin SAH
  rt::BuiltTree sweep = rt::build_sah_tree(boxes, true);  // exact-sweep SAH (the RT_BVH_SAH default)
  (void)rt::tree_branch_depth(ref);
  (void)rt::tree_branch_depth(sah);
  (void)rt::tree_branch_depth(sweep);
  int rc = 0;
  if (big_ok || v->n_objects <= 4000) {
    or_scene* os = or_scene_new(v);
    if (!os) {
      rc = 2;
    } else {
      rt_camera cam;
      if (sh_default_camera(w, "std16x9", 20.0, 1.0, 0.001, &cam) == 0) {
        rt_render_params p{};
        p.samples = spp;
        p.max_depth = 8;
        p.seed = seed;
        p.tile_world = 1;
        std::vector<double> acc((size_t)cam.image_width * cam.image_height * 3);
        or_counters cnt{};
        or_render_rows(os, &cam, &p, 0, cam.image_height, 1, acc.data(), &cnt);
        std::vector<uint8_t> rgb(acc.size());
        or_tonemap(acc.data(), cam.image_width, cam.image_height, spp, rgb.data());
      }
      or_scene_free(os);
    }
  }
  sh_desc_free(d);
  return rc;
}

std::string mutate(const std::string& in, XorShift& r) {
  static const char* tokens[] = {"{", "}", "[", "]", ",", ":", "\"", "\\", "\\u", "\\ud800", "\\udc00\\ud800",
                                 "null", "true", "-", "e", "E+", ".", "0", "-0", "1e308", "1e309", "-1e999",
                                 "4.9e-324", "1e-400", "nan", "inf", "0x1p3", "+1", "\"Sphere\"", "\"RectBox\"",
                                 "\"Checker\"", "\"Perlin\"", "\"ImagePath\"", "\"EarthBuiltin\"", "\"vec\"",
                                 "\"objects\"", "\"skybox\"", "\x01", "\xff", "\xc3\xa9", "1e5", "123456789012345678901234567890"};
  std::string s = in;
  // half of the mutants only replace numbers (they still parse, so they reach finalize, the BVH
  // builders and the oracle with extreme values); the rest mutate the syntax
  const bool numbers_only = r.below(2) == 0;
  const int n_ops = 1 + (int)r.below(numbers_only ? 8 : 4);
  for (int op = 0; op < n_ops; ++op) {
    const size_t pos = r.below(s.size() + 1);
    switch (numbers_only ? 5 : r.below(8)) {
      case 0:  // flip a byte
        if (!s.empty()) s[r.below(s.size())] ^= (char)(1u << r.below(8));
        break;
      case 1:  // insert a JSON-significant token
        s.insert(pos, tokens[r.below(sizeof tokens / sizeof *tokens)]);
        break;
      case 2: {  // delete a range
        const size_t len = 1 + r.below(32);
        if (pos < s.size()) s.erase(pos, len);
        break;
      }
      case 3: {  // duplicate a range
        const size_t len = 1 + r.below(256);
        if (pos < s.size()) s.insert(r.below(s.size() + 1), s.substr(pos, len));
        break;
      }
      case 4:  // truncate
        s.resize(pos);
        break;
      case 5: {  // replace a number by an extreme one
        const size_t k = s.find_first_of("0123456789", pos);
        if (k != std::string::npos) {
          size_t e = k;
          while (e < s.size() && std::strchr("0123456789.eE+-", s[e])) ++e;
          static const char* ext[] = {"0", "-0.0", "1e308", "-1e308", "1e-320", "5e-324", "1e300", "-7", "0.5e-10",
                                      "340282366920938463463374607431768211456", "1e19", "-2147483649", "1e10",
                                      "0.0001", "3"};
          s.replace(k, e - k, ext[r.below(sizeof ext / sizeof *ext)]);
        }
        break;
      }
      case 6: {  // deep nesting
        const size_t depth = 100 + r.below(400);
        s.insert(pos, std::string(depth, r.below(2) ? '[' : '{'));
        break;
      }
      default: {  // swap two bytes
        if (s.size() > 1) std::swap(s[r.below(s.size())], s[r.below(s.size())]);
      }
    }
  }
  return s;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <asset_dir> <n_mutants> [seed]\n", argv[0]);
    return 2;
  }
  (void)argv[1];  // asset dir: unused since EarthBuiltin is linked in (earth_embed.S)
  const long n_mut = std::atol(argv[2]);
  XorShift rng{argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 0x5EEDull};

  static const char* scenes[] = {"random", "random-night", "demo", "perlin", "earth", "box-light", "cornell",
                                 "spheres:5", "final:4:30"};
  std::vector<std::string> corpus;
  for (const char* name : scenes) {
    sh_scene* s = nullptr;
    CHECK(sh_scene_builtin(name, 0x5EED, &s) == 0, "%s: builtin failed: %s", name, sh_last_error());
    if (!s) continue;
    const std::string j1 = to_json(s, 1);
    sh_scene* s2 = nullptr;
    CHECK(sh_scene_from_json(j1.c_str(), &s2) == 0, "%s: from_json of its own JSON failed: %s", name, sh_last_error());
    if (s2) {
      CHECK(to_json(s2, 1) == j1, "%s: JSON round trip differs", name);
      sh_scene_free(s2);
    }
    CHECK(exercise(s, 0x5EED, 16, 2, true) == 0, "%s: finalize/build/render failed: %s", name, sh_last_error());
    corpus.push_back(to_json(s, 0));
    corpus.push_back(j1);
    sh_scene_free(s);
  }
  // hand-written edge cases
  static const char* edge[] = {"", "{", "}", "[]", "null", "{\"skybox\":\"Above\"}", "{\"objects\":[]}",
                               "{\"skybox\":\"Above\",\"objects\":[]}", "{\"skybox\":{\"Flat\":{\"vec\":[1,2]}},\"objects\":[]}",
                               "{\"skybox\":\"None\",\"objects\":[{\"geometry\":{\"Sphere\":{\"center\":{\"vec\":[0,0,0]},"
                               "\"radius\":-1e308}},\"material\":{\"Metal\":{\"albedo\":{\"vec\":[1,1,1]},\"fuzz\":1e308}}}]}",
                               "\"\\ud800\"", "\"\\u00e9\\ud83d\\ude00\"", "[1e309]", "[-]", "[01]", "[1.]", "[.5]", "[1e]",
                               "\"\x01\""};
  for (const char* e : edge) {
    sh_scene* s = nullptr;
    if (sh_scene_from_json(e, &s) == 0 && s) {
      exercise(s, 1, 4, 1, false);
      sh_scene_free(s);
    }
  }
  {  // boxes whose centroids are NaN (opposite infinite planes, NaN planes) or infinite, mixed with
     // ordinary ones: every builder must terminate and place each object in exactly one leaf (the
     // sweep builder's sort needs a strict weak ordering for that)
    const double inf = INFINITY, nan = NAN;
    std::vector<rt::Box> boxes;
    for (int i = 0; i < 64; ++i) {
      rt::Box b;
      for (int k = 0; k < 3; ++k) {
        const double c = (double)((i * 37 + k * 11) % 17);
        b.mn[k] = c;
        b.mx[k] = c + 1.0;
      }
      switch (i % 5) {
        case 1: b.mn[i % 3] = -inf; b.mx[i % 3] = inf; break;  // centroid NaN
        case 2: b.mn[(i + 1) % 3] = nan; break;               // NaN plane
        case 3: b.mn[i % 3] = inf; b.mx[i % 3] = inf; break;   // centroid +inf
        default: break;
      }
      boxes.push_back(b);
    }
    for (int which = 0; which < 3; ++which) {
      const rt::BuiltTree t = which == 0 ? rt::build_reference_tree(boxes) : rt::build_sah_tree(boxes, which == 2);
      std::vector<int> seen(boxes.size(), 0);
      for (const rt::BuildNode& n : t.nodes)
        if (n.leaf >= 0 && n.leaf < (int)boxes.size()) seen[n.leaf]++;
      for (size_t i = 0; i < seen.size(); ++i) CHECK(seen[i] == 1, "builder %d: object %zu in %d leaves", which, i, seen[i]);
    }
  }
  {  // nesting far beyond the recursion limit must be an error, not a stack overflow
    std::string deep(200000, '[');
    sh_scene* s = nullptr;
    CHECK(sh_scene_from_json(deep.c_str(), &s) != 0, "200000-deep nesting accepted");
    if (s) sh_scene_free(s);
  }
  long parsed = 0, rendered = 0;
  for (long i = 0; i < n_mut; ++i) {
    const std::string m = mutate(corpus[rng.below(corpus.size())], rng);
    sh_scene* s = nullptr;
    if (sh_scene_from_json(m.c_str(), &s) == 0 && s) {
      ++parsed;
      if (exercise(s, rng.next(), 4, 1, false) == 0) ++rendered;
      sh_scene_free(s);
    }
  }
  std::printf("host_check: %zu scenes round-tripped, %ld mutants: %ld parsed, %ld finalized+built+rendered, "
              "%d failures\n",
              sizeof scenes / sizeof *scenes, n_mut, parsed, rendered, g_failures);
  return g_failures ? 1 : 0;
}
