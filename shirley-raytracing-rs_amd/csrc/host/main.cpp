// main.cpp — ray-cli: the reference's CLI (src/main.rs, src/argparse.rs) on the C++ host, with
// render_scene (main.rs:65-130) calling the MI355X render ABI instead of the rayon scanline loop.
//
//   ray-cli [-v...] render <random|saved|demo|perlin|earth|box-light|cornell|spheres|final> [options]
//   ray-cli test
//
// Reference flags (argparse.rs:106-167): -o/--output out.png, -s/--samples 100, -m/--max-reflect 50,
// --single-threaded (accepted; the GPU path has no CPU thread count), -w/--width 640, --camera-fov 20,
// --camera-focal-length 1.0, --camera-aperture 0.001, --camera-aspect-ratio std3x2;
// random: --night, --scene-output FILE; saved: <scene_input>.
// Added: --seed N (the reference is unseeded), --device N, --bvh reference|sah, --sample-chunk N,
// --dump-accum FILE (raw f64 [H][W][3] sums, row 0 = bottom), --side-len N (spheres),
// --gpus N (devices [device, device + N): the frame's tiles sharded over N GPUs with an RCCL gather,
// rt_render_multi — the counterpart of the reference's whole-machine rayon loop, main.rs:117-125),
// --partition tiles|samples (how --gpus splits the frame, RT_PARTITION_*; default: the library's),
// --progressive K (the frame's samples in K consecutive ranges, rt_render_params.sample_begin / count;
// after each range the running sums go to --dump-accum FILE + FILE.json and the PNG shows the samples so
// far: a checkpoint), --resume FILE (continue from such a checkpoint: its sums cover samples [0, N)).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../../include/shirley_host.h"
#include "../../../include/shirley_rt.h"

namespace {

int verbose = 0;

struct Args {
  std::string scene, output = "out.png", scene_output, scene_input, dump_accum, aspect = "std3x2", bvh = "reference";
  int samples = 100, max_reflect = 50, width = 640, device = 0, sample_chunk = 0, side_len = 11, gpus = 1;
  int partition = RT_PARTITION_AUTO;
  int progressive = 1;
  std::string resume;
  double fov = 20.0, focal = 1.0, aperture = 0.001;
  bool night = false, single_threaded = false;
  unsigned long long seed = 0x5EED;
};

[[noreturn]] void usage(const char* msg) {
  if (msg && *msg) std::fprintf(stderr, "error: %s\n", msg);
  std::fprintf(stderr,
               "usage: ray-cli [-v] render <random|saved|demo|perlin|earth|box-light|cornell|spheres|final> [options]\n"
               "       ray-cli test\n"
               "options: -o FILE -s N -m N -w N --single-threaded --camera-fov F --camera-focal-length F\n"
               "         --camera-aperture F --camera-aspect-ratio std3x2|std16x9|std16x10|square|target-iphone\n"
               "         --night --scene-output FILE (random)  <scene_input> (saved)  --side-len N (spheres)\n"
               "         --seed N --device N --gpus N --partition tiles|samples --bvh reference|sah --sample-chunk N\n"
               "         --dump-accum FILE --progressive K --resume FILE\n");
  std::exit(2);
}

// A checkpoint's identity (--dump-accum FILE + FILE.json, --resume FILE): its sums are the per-pixel sums
// of samples [0, samples_done) of one frame, so a resume must render that same frame — the same scene
// (rt_scene_digest_host of the description and BVH builder), camera (FNV-1a over its fields), seed,
// max_depth and sample_chunk (the unit length decides the sums' bits) — and may only add samples.
struct Checkpoint {
  long long samples_done = -1, samples = -1, width = -1, height = -1, max_depth = -1, sample_chunk = -1;
  unsigned long long seed = 0, scene = 0, camera = 0;
};

unsigned long long camera_digest(const rt_camera& c) {
  unsigned long long h = 14695981039346656037ull;
  auto bytes = [&](const void* p, size_t n) {
    for (size_t i = 0; i < n; ++i) h = (h ^ static_cast<const unsigned char*>(p)[i]) * 1099511628211ull;
  };
  bytes(&c.image_width, sizeof c.image_width); bytes(&c.image_height, sizeof c.image_height);
  bytes(&c.height, sizeof c.height); bytes(&c.width, sizeof c.width); bytes(&c.focal_length, sizeof c.focal_length);
  bytes(&c.has_lens, sizeof c.has_lens); bytes(&c.lens_radius, sizeof c.lens_radius);
  bytes(c.origin, sizeof c.origin); bytes(c.w, sizeof c.w); bytes(c.u, sizeof c.u); bytes(c.v, sizeof c.v);
  bytes(&c.focus_length, sizeof c.focus_length); bytes(&c.time0, sizeof c.time0); bytes(&c.time1, sizeof c.time1);
  return h;
}

Checkpoint checkpoint_of(const Args& a, const rt_scene_desc* desc, const rt_camera& cam, int samples, int done) {
  Checkpoint k;
  k.samples_done = done;
  k.samples = samples;
  k.width = cam.image_width;
  k.height = cam.image_height;
  k.max_depth = a.max_reflect;
  k.sample_chunk = a.sample_chunk;
  k.seed = a.seed;
  uint64_t d = 0;
  if (rt_scene_digest_host(desc, a.bvh == "sah" ? RT_BVH_SAH : RT_BVH_REFERENCE, &d) == RT_OK) k.scene = d;
  k.camera = camera_digest(cam);
  return k;
}

void write_checkpoint(const std::string& path, const std::vector<double>& accum, const Checkpoint& k) {
  std::ofstream f(path, std::ios::binary);
  f.write((const char*)accum.data(), (std::streamsize)(accum.size() * sizeof(double)));
  char digests[80];
  std::snprintf(digests, sizeof digests, "\"scene_digest\": \"%016llx\", \"camera_digest\": \"%016llx\"", k.scene,
                k.camera);
  std::ofstream fj(path + ".json");
  fj << "{\"samples_done\": " << k.samples_done << ", \"samples\": " << k.samples << ", \"width\": " << k.width
     << ", \"height\": " << k.height << ", \"seed\": " << k.seed << ", \"max_depth\": " << k.max_depth
     << ", \"sample_chunk\": " << k.sample_chunk << ", " << digests << "}\n";
}

// FILE.json's fields (the writer's own flat format); false when one is missing
bool read_checkpoint(const std::string& path, Checkpoint* k) {
  std::ifstream fj(path + ".json");
  const std::string js((std::istreambuf_iterator<char>(fj)), std::istreambuf_iterator<char>());
  auto field = [&](const char* name, bool hex, unsigned long long* out) {
    const std::string key = std::string("\"") + name + "\":";
    const size_t at = js.find(key);
    if (at == std::string::npos) return false;
    const char* s = js.c_str() + at + key.size();
    while (*s == ' ' || *s == '"') ++s;
    char* end = nullptr;
    *out = std::strtoull(s, &end, hex ? 16 : 10);
    return end != s;
  };
  unsigned long long v[9];
  const char* names[9] = {"samples_done", "samples", "width", "height", "max_depth", "sample_chunk", "seed",
                          "scene_digest", "camera_digest"};
  for (int i = 0; i < 9; ++i)
    if (!field(names[i], i >= 7, &v[i])) return false;
  k->samples_done = (long long)v[0]; k->samples = (long long)v[1]; k->width = (long long)v[2];
  k->height = (long long)v[3]; k->max_depth = (long long)v[4]; k->sample_chunk = (long long)v[5];
  k->seed = v[6]; k->scene = v[7]; k->camera = v[8];
  return true;
}

// Why checkpoint `c` cannot be continued as frame `want` (empty: it can)
std::string checkpoint_mismatch(const Checkpoint& c, const Checkpoint& want) {
  char m[160] = "";
  if (c.scene != want.scene) std::snprintf(m, sizeof m, "scene %016llx, this run %016llx", c.scene, want.scene);
  else if (c.width != want.width || c.height != want.height)
    std::snprintf(m, sizeof m, "%lldx%lld, this run %lldx%lld", c.width, c.height, want.width, want.height);
  else if (c.camera != want.camera) std::snprintf(m, sizeof m, "another camera");
  else if (c.seed != want.seed) std::snprintf(m, sizeof m, "seed %llu, this run %llu", c.seed, want.seed);
  else if (c.max_depth != want.max_depth)
    std::snprintf(m, sizeof m, "max_depth %lld, this run %lld", c.max_depth, want.max_depth);
  else if (c.sample_chunk != want.sample_chunk)
    std::snprintf(m, sizeof m, "sample_chunk %lld, this run %lld", c.sample_chunk, want.sample_chunk);
  else if (c.samples_done < 0 || c.samples_done > want.samples)
    std::snprintf(m, sizeof m, "it covers %lld samples, this run renders %lld", c.samples_done, want.samples);
  return m;
}

// --gpus N > 1: one ctx per device, the scene uploaded to each, rt_render_multi (tiles + RCCL gather
// to the first device), to_image on the host.
int render_scene_multi(const Args& a, const rt_scene_desc* desc, const rt_camera& cam, int samples) {
  std::vector<rt_ctx*> ctxs(a.gpus, nullptr);
  int st = 0;
  auto done = [&](int rc) {
    for (rt_ctx* c : ctxs)
      if (c) rt_destroy(c);
    return rc;
  };
  const int builder = a.bvh == "sah" ? RT_BVH_SAH : RT_BVH_REFERENCE;
  for (int i = 0; i < a.gpus; ++i) {
    if ((st = rt_create(a.device + i, &ctxs[i]))) {
      std::fprintf(stderr, "error: rt_create(device %d) failed (%d)\n", a.device + i, st);
      return done(1);
    }
    if ((st = rt_scene_upload(ctxs[i], desc, builder))) {
      std::fprintf(stderr, "error: %s\n", rt_last_error(ctxs[i]));
      return done(1);
    }
  }
  rt_render_params p{};
  p.samples = samples;
  p.max_depth = a.max_reflect;
  p.seed = a.seed;
  p.tile_world = 1;
  p.sample_chunk = a.sample_chunk;
  p.partition = a.partition;
  const size_t n = (size_t)cam.image_width * cam.image_height * 3;
  std::vector<double> accum(n);
  std::vector<uint8_t> rgb(n);
  auto t1 = std::chrono::steady_clock::now();
  if ((st = rt_render_multi(ctxs.data(), a.gpus, &cam, &p, accum.data()))) {
    std::fprintf(stderr, "error: %s\n", rt_last_error(ctxs[0]));
    return done(1);
  }
  auto t2 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
  if (verbose >= 1)
    std::fprintf(stderr, "INFO %d GPUs: render %.1f ms (incl. gather and copy-back): %.1f Msamples/s\n", a.gpus, ms,
                 (double)cam.image_width * cam.image_height * samples / (ms * 1e3));
  rt_tonemap(accum.data(), cam.image_width, cam.image_height, samples, rgb.data());  // image.rs:31-44
  if (!a.dump_accum.empty()) write_checkpoint(a.dump_accum, accum, checkpoint_of(a, desc, cam, samples, samples));
  if (sh_write_png(a.output.c_str(), rgb.data(), cam.image_width, cam.image_height)) {
    std::fprintf(stderr, "error: %s\n", sh_last_error());
    return done(1);
  }
  return done(0);
}

int render_scene(const Args& a, const rt_scene_desc* desc, const rt_camera& cam) {
  int samples = a.samples;
  if (samples == 0) {  // main.rs:75-80
    std::fprintf(stderr, "WARN samples set to 0, using 1\n");
    samples = 1;
  }
  if (a.gpus > 1) return render_scene_multi(a, desc, cam, samples);
  rt_ctx* ctx = nullptr;
  int st = rt_create(a.device, &ctx);
  if (st) {
    std::fprintf(stderr, "error: rt_create(device %d) failed (%d): no usable MI355X device?\n", a.device, st);
    return 1;
  }
  int builder = a.bvh == "sah" ? RT_BVH_SAH : RT_BVH_REFERENCE;
  auto t0 = std::chrono::steady_clock::now();
  if ((st = rt_scene_upload(ctx, desc, builder))) {
    std::fprintf(stderr, "error: %s\n", rt_last_error(ctx));
    rt_destroy(ctx);
    return 1;
  }
  rt_render_params p{};
  p.samples = samples;
  p.max_depth = a.max_reflect;
  p.seed = a.seed;
  p.tile_rank = 0;
  p.tile_world = 1;
  p.sample_chunk = a.sample_chunk;
  const size_t n = (size_t)cam.image_width * cam.image_height * 3;
  std::vector<double> accum;
  std::vector<uint8_t> rgb(n);
  auto t1 = std::chrono::steady_clock::now();
  if (a.progressive > 1 || !a.resume.empty()) {
    // progressive rendering with checkpoints: sample ranges [b_k, b_k+1) of the frame; the host adds each
    // range's sums to the running sums in range order (so a resumed run adds exactly what an
    // uninterrupted one does) and writes the checkpoint after every range
    accum.assign(n, 0.0);
    int done = 0;
    if (!a.resume.empty()) {
      Checkpoint ck;
      if (!read_checkpoint(a.resume, &ck)) {
        std::fprintf(stderr, "error: %s.json is not a checkpoint record\n", a.resume.c_str());
        rt_destroy(ctx);
        return 1;
      }
      const std::string why = checkpoint_mismatch(ck, checkpoint_of(a, desc, cam, samples, 0));
      if (!why.empty()) {
        std::fprintf(stderr, "error: %s is a checkpoint of another frame: %s\n", a.resume.c_str(), why.c_str());
        rt_destroy(ctx);
        return 1;
      }
      std::ifstream f(a.resume, std::ios::binary);
      f.read((char*)accum.data(), (std::streamsize)(n * sizeof(double)));
      if (!f || f.gcount() != (std::streamsize)(n * sizeof(double)) || f.peek() != std::char_traits<char>::eof()) {
        std::fprintf(stderr, "error: %s does not hold the %zu sums of a %dx%d frame\n", a.resume.c_str(), n,
                     cam.image_width, cam.image_height);
        rt_destroy(ctx);
        return 1;
      }
      done = (int)ck.samples_done;
    }
    std::vector<double> part(n);
    const int ranges = std::max(1, a.progressive);
    const int left = samples - done;
    for (int k = 0; k < ranges && left > 0; ++k) {
      const int b = done + (int)((long long)left * k / ranges), e = done + (int)((long long)left * (k + 1) / ranges);
      if (e <= b) continue;
      p.sample_begin = b;
      p.sample_count = e - b;
      if ((st = rt_render(ctx, &cam, &p, part.data()))) {
        std::fprintf(stderr, "error: %s\n", rt_last_error(ctx));
        rt_destroy(ctx);
        return 1;
      }
      for (size_t i = 0; i < n; ++i) accum[i] += part[i];
      rt_tonemap(accum.data(), cam.image_width, cam.image_height, e, rgb.data());
      if (!a.dump_accum.empty()) write_checkpoint(a.dump_accum, accum, checkpoint_of(a, desc, cam, samples, e));
      if (sh_write_png(a.output.c_str(), rgb.data(), cam.image_width, cam.image_height)) {
        std::fprintf(stderr, "error: %s\n", sh_last_error());
        rt_destroy(ctx);
        return 1;
      }
      if (verbose >= 1) std::fprintf(stderr, "INFO checkpoint: samples [0, %d) of %d\n", e, samples);
    }
    rt_destroy(ctx);
    if (left == 0) {  // a complete checkpoint: just its picture
      rt_tonemap(accum.data(), cam.image_width, cam.image_height, samples, rgb.data());
      if (sh_write_png(a.output.c_str(), rgb.data(), cam.image_width, cam.image_height)) {
        std::fprintf(stderr, "error: %s\n", sh_last_error());
        return 1;
      }
    }
    return 0;
  } else if (!a.dump_accum.empty()) {  // the raw sums are wanted on the host: render + host tonemap
    accum.resize(n);
    if ((st = rt_render(ctx, &cam, &p, accum.data()))) {
      std::fprintf(stderr, "error: %s\n", rt_last_error(ctx));
      rt_destroy(ctx);
      return 1;
    }
    rt_tonemap(accum.data(), cam.image_width, cam.image_height, samples, rgb.data());  // image.rs:31-44
  } else {  // sums stay in HBM; to_image runs on the device and only RGB8 crosses PCIe
    double* acc_dev = nullptr;
    uint8_t* rgb_dev = nullptr;
    if (hipMalloc((void**)&acc_dev, n * sizeof(double)) != hipSuccess || hipMalloc((void**)&rgb_dev, n) != hipSuccess) {
      std::fprintf(stderr, "error: device allocation of the image failed\n");
      rt_destroy(ctx);
      return 1;
    }
    st = rt_render_device(ctx, &cam, &p, acc_dev, nullptr);
    if (!st) st = rt_tonemap_device(ctx, acc_dev, cam.image_width, cam.image_height, samples, rgb_dev, nullptr);
    if (!st) st = rt_synchronize(ctx);
    if (!st && hipMemcpy(rgb.data(), rgb_dev, n, hipMemcpyDeviceToHost) != hipSuccess) st = RT_E_HIP;
    (void)hipFree(acc_dev);
    (void)hipFree(rgb_dev);
    if (st) {
      std::fprintf(stderr, "error: %s\n", rt_last_error(ctx));
      rt_destroy(ctx);
      return 1;
    }
  }
  auto t2 = std::chrono::steady_clock::now();
  rt_counters cnt{};
  rt_counters_get(ctx, &cnt);
  double ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
  double msamp = (double)cam.image_width * cam.image_height * samples / (cnt.kernel_ms * 1e3);
  if (verbose >= 1)
    std::fprintf(stderr,
                 "INFO upload %.1f ms, render %.1f ms (kernel %.2f ms, reduce %.3f ms): %.1f Msamples/s, %.3f segments/sample\n",
                 std::chrono::duration<double, std::milli>(t1 - t0).count(), ms, cnt.kernel_ms, cnt.reduce_ms, msamp,
                 (double)cnt.segments / (double)(cnt.samples ? cnt.samples : 1));
  rt_destroy(ctx);
  if (!a.dump_accum.empty())  // a complete checkpoint
    write_checkpoint(a.dump_accum, accum, checkpoint_of(a, desc, cam, samples, samples));
  if (sh_write_png(a.output.c_str(), rgb.data(), cam.image_width, cam.image_height)) {
    std::fprintf(stderr, "error: %s\n", sh_last_error());
    return 1;
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) usage(("missing value for " + s).c_str());
      return argv[++i];
    };
    if (s == "-v" || s == "--verbose") ++verbose;
    else if (s.size() > 2 && s[0] == '-' && s[1] == 'v' && s.find_first_not_of('v', 1) == std::string::npos) verbose += (int)s.size() - 1;
    else if (s == "-o" || s == "--output") a.output = next();
    else if (s == "-s" || s == "--samples") a.samples = std::atoi(next().c_str());
    else if (s == "-m" || s == "--max-reflect") a.max_reflect = std::atoi(next().c_str());
    else if (s == "--single-threaded") a.single_threaded = true;
    else if (s == "-w" || s == "--width") a.width = std::atoi(next().c_str());
    else if (s == "--camera-fov") a.fov = std::atof(next().c_str());
    else if (s == "--camera-focal-length") a.focal = std::atof(next().c_str());
    else if (s == "--camera-aperture") a.aperture = std::atof(next().c_str());
    else if (s == "--camera-aspect-ratio") a.aspect = next();
    else if (s == "--night") a.night = true;
    else if (s == "--scene-output") a.scene_output = next();
    else if (s == "--seed") a.seed = std::strtoull(next().c_str(), nullptr, 0);
    else if (s == "--device") a.device = std::atoi(next().c_str());
    else if (s == "--gpus") a.gpus = std::atoi(next().c_str());
    else if (s == "--bvh") a.bvh = next();
    else if (s == "--sample-chunk") a.sample_chunk = std::atoi(next().c_str());
    else if (s == "--progressive") a.progressive = std::atoi(next().c_str());
    else if (s == "--resume") a.resume = next();
    else if (s == "--partition") {
      const std::string v = next();
      if (v == "tiles") a.partition = RT_PARTITION_TILES;
      else if (v == "samples") a.partition = RT_PARTITION_SAMPLES;
      else usage("--partition must be tiles or samples");
    }
    else if (s == "--dump-accum") a.dump_accum = next();
    else if (s == "--side-len") a.side_len = std::atoi(next().c_str());
    else if (s == "-h" || s == "--help") usage("");
    else if (!s.empty() && s[0] == '-') usage(("unknown option " + s).c_str());
    else pos.push_back(s);
  }
  if (pos.empty()) usage("missing subcommand");
  if (pos[0] == "test") {  // main.rs:60-63
    std::fprintf(stderr, "ERROR there is nothing to test!\n");
    return 0;
  }
  if (pos[0] != "render" || pos.size() < 2) usage("expected `render <scene>`");
  a.scene = pos[1];
  if (a.samples < 0 || a.max_reflect < 0 || a.width < 1) usage("samples / max-reflect / width out of range");
  if (a.gpus < 1 || a.gpus > 64) usage("--gpus must be in [1, 64]");
  if (a.progressive < 1) usage("--progressive must be >= 1");
  if (a.gpus > 1 && (a.progressive > 1 || !a.resume.empty())) usage("--progressive / --resume render on one GPU");

  sh_scene* scene = nullptr;
  std::string cam_scene = a.scene;
  if (a.scene == "saved") {
    if (pos.size() < 3) usage("render saved needs <scene_input>");
    std::ifstream f(pos[2]);
    if (!f) usage(("cannot open " + pos[2]).c_str());
    std::stringstream ss;
    ss << f.rdbuf();
    if (sh_scene_from_json(ss.str().c_str(), &scene)) {
      std::fprintf(stderr, "error: %s\n", sh_last_error());
      return 1;
    }
  } else {
    std::string name = a.scene;
    if (name == "random" && a.night) name = "random-night";
    if (name == "spheres") name = "spheres:" + std::to_string(a.side_len);
    if (sh_scene_builtin(name.c_str(), a.seed, &scene)) {
      std::fprintf(stderr, "error: %s\n", sh_last_error());
      return 1;
    }
  }
  if (!a.scene_output.empty()) {  // scenes.rs:140-143
    size_t need = 0;
    sh_scene_to_json(scene, 1, nullptr, 0, &need);
    std::string buf(need, '\0');
    sh_scene_to_json(scene, 1, &buf[0], need, &need);
    std::ofstream f(a.scene_output);
    f << buf.c_str();
  }
  sh_desc* desc = nullptr;
  if (sh_scene_finalize(scene, a.seed, &desc)) {
    std::fprintf(stderr, "error: %s\n", sh_last_error());
    return 1;
  }
  rt_camera cam{};
  if (sh_scene_camera(cam_scene.c_str(), a.width, a.aspect.c_str(), a.fov, a.focal, a.aperture, &cam)) {
    std::fprintf(stderr, "error: %s\n", sh_last_error());
    return 1;
  }
  int rc = render_scene(a, sh_desc_view(desc), cam);
  sh_desc_free(desc);
  sh_scene_free(scene);
  return rc;
}
