// rt_api.cpp — implementation of the C ABI in include/shirley_rt.h.
//
// Host side of the boundary: validates the flattened scene, builds the BBox tree, lays the scene
// out in HBM (rt_layout.h), sizes the persistent launch and runs trace -> reduce on a HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "../../../include/shirley_rt.h"
#include "bvh_build.h"
#include "keycheck.h"
#include "plan.h"
#include "rccl_loader.h"
#include "rt_layout.h"

namespace rt {
size_t trace_lds_bytes(int n_lds_nodes4, int node4_size, int n_lds_prims, int n_lds_perlin, int stack_depth4,
                       int threads, int n_lds_mats, int n_lds_texs);
hipError_t trace_occupancy(const DScene& S, int threads, int* blocks_per_cu);
hipError_t launch_trace(const KParams& p, int blocks, int threads, hipStream_t stream);
bool split_supported_nt(int nt);
hipError_t split_prepare(const DScene& S, int nt, int* blocks_per_cu);
hipError_t launch_split(const KParams& p, int nt, int blocks, hipStream_t stream);
#ifdef RT_PHASE_TIMING
void phase_counters_dump();
#endif
#ifdef RT_TIMELINE
void timeline_dump();
#endif
hipError_t launch_reduce(const double* partial, int n_chunks, int n_tiles_rank, int tiles_x, int ty0, int tile_rank,
                         int tile_world, int width, int row0, int row1, int packed, int accumulate, double* out,
                         hipStream_t stream);
hipError_t launch_tonemap(const double* accum, int width, int height, double inv, uint8_t* rgb8, hipStream_t stream);
hipError_t launch_unpack(const double* gathered, int world, int max_tiles, int n_tiles_total, int tiles_x, int width,
                         int height, double* out, hipStream_t stream);
hipError_t launch_sum_parts(const double* parts, int n_parts, long long n, double* out, hipStream_t stream);
hipError_t launch_hit(const DScene& S, const double* rays, int n, double t_min, double t_max, void* out,
                      hipStream_t stream);
hipError_t launch_hit4(const DScene& S, bool wide, const double* rays, int n, double t_min, double t_max, void* out,
                       hipStream_t stream);
hipError_t launch_probe(const DScene& S, bool wide, const double* rays, int n, uint64_t seed, uint32_t sample,
                        uint32_t draw, void* out, hipStream_t stream);
// wavefront.hip
size_t wf_extend_lds(int n_lds_nodes, int stack_depth);
int wf_extend_threads();
int wf_grid_threads();
hipError_t wf_prepare(const DScene& S, int* extend_blocks_per_cu);
hipError_t wf_prepare4(const DScene& S, int* extend_blocks_per_cu);
hipError_t wf_launch_extend4(const WfParams& P, int extend_blocks, hipStream_t s);
hipError_t wf_start(const WfParams& P, int grid_blocks, hipStream_t s);
hipError_t wf_launch_extend(const WfParams& P, int extend_blocks, hipStream_t s);
hipError_t wf_launch_shade(const WfParams& P, int grid_blocks, hipStream_t s);
hipError_t wf_launch_texture(const WfParams& P, int grid_blocks, hipStream_t s);
}  // namespace rt

using namespace rt;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// A rank of an RCCL communicator (multi-GPU frame sharding).
struct rt_comm {
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0, device = 0;
  // rt_render_sharded's cross-rank check (keycheck.h): the key the ranks last agreed on, and the gathered
  // (digest, key) words of the last two calls in pinned host memory ([2 slots][world + 1][2]: the gathered
  // words, then this rank's own), each slot's copy marked by an event
  KeyState ks;
  uint64_t* key_words = nullptr;
  hipEvent_t key_ev[2] = {nullptr, nullptr};
  int key_slot = 0;       // slot of the next call
  int key_pending = 0;    // slot of the pending (deferred) check
};

struct rt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int cu_count = 0;
  // scene
  bool have_scene = false;
  DScene scene{};
  DevBuf nodes, nodes4, prims, mats, texs, perlin, texels, exts;
  rt_scene_stats stats{};
  int blocks_per_cu = 0;
  int mk_threads = kTraceThreads;  // megakernel block size (kTraceThreadsWide: whole BVH in LDS)
  int split_nt = 0;                // RT_ENGINE_SPLIT: traversal waves per block (0: scene not eligible)
  int split_refill = 8;            // idle traversal lanes before a traversal wave claims rays
  // wavefront engine: the scene with its LDS node count sized for the extend block
  DScene wf_scene{};
  int wf_blocks_per_cu = 0;
  bool wf_wide = false;      // wavefront extend runs the 4-wide scene-in-LDS kernel (wf_extend4)
  int wf4_blocks_per_cu = 0;
  bool has_perlin = false;
  int n_perlin = 0;
  // per-render scratch
  DevBuf partial, accum, counters, unit_counter, kcam;
  DevBuf shutter0;  // {0, 0}: the shutter of rt_scene_hit / rt_probe_segment queries (DScene.shutter)
  DevBuf wf_pool, wf_iters;          // path slots (SoA) + texture queue; per-iteration counters ring
  uint32_t* wf_host = nullptr;       // pinned readback of the retired-slot count, one word per batch
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  hipEvent_t wf_ev[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> lap_ev;    // RT_ENGINE_TIMING: one event after every launch
  bool have_timing = false;
  int last_engine = 0, last_iters = 0, last_timing = 0, last_chunk = 0, last_n_chunks = 0, last_passes = 0;
  uint64_t last_slots = 0, last_scratch = 0;
  std::vector<hipEvent_t> pass_ev;   // before / after the trace launch of each sample pass
  std::vector<KBlock> host_blocks;    // host sources of the device KBlocks (KParams.kconst)
  uint64_t digest = 0;               // rt_scene_digest of the uploaded scene
  // device primitive number -> object index (primitives are numbered in the reference tree's leaf order)
  std::vector<int32_t> prim_object;
  // flattened rotated spheres (flat_object): object index -> RotateY's cos, sin, for rt_scene_hit's u, v
  std::vector<std::pair<int32_t, std::pair<double, double>>> uv_fixups;
  uint64_t host_samples = 0;  // samples of a frame served without a trace kernel (max_depth == 0)
  double lap_ms[3] = {0, 0, 0};
  // multi-GPU: this rank's packed tiles, the root's gathered buffer, and (root of rt_render_multi)
  // the communicators of the device set last used, kept for the next call
  DevBuf packed, gathered, parts, band, digests;
  std::vector<int> group_devices;
  std::vector<rt_comm> group_comms;
};

namespace {

int fail(rt_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIP_TRY(ctx, expr)                                                                      \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return fail(ctx, e_ == hipErrorOutOfMemory ? RT_E_OOM : RT_E_HIP, "%s: %s (%s:%d)", #expr, \
                  hipGetErrorString(e_), __FILE__, __LINE__);                                   \
  } while (0)

int ensure(rt_ctx* c, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return RT_OK;
  if (c) HIP_TRY(c, hipSetDevice(c->device));  // (rt_render_multi drives several devices from one thread)
  if (b.p) {
    (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  if (bytes == 0) return RT_OK;
  HIP_TRY(c, hipMalloc(&b.p, bytes));
  b.bytes = bytes;
  return RT_OK;
}

void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

int upload(rt_ctx* c, DevBuf& b, const void* src, size_t bytes) {
  int st = ensure(c, b, std::max<size_t>(bytes, 16));
  if (st) return st;
  if (bytes) HIP_TRY(c, hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
  return RT_OK;
}

// Book-2 extension parameters of an object, shared by the bounding box and the
// device record: RotateY's cos / sin (rotate_y.h: radians = degrees * pi / 180).
bool is_extended(const rt_object& o) {
  return o.geometry == RT_GEOM_MOVING_SPHERE || o.medium != 0 || o.transform != 0;
}
void rotate_y_cs(const rt_object& o, double& cs, double& sn) {
  const double rad = o.rotate_y_deg * 3.14159265358979323846 / 180.0;
  cs = std::cos(rad);
  sn = std::sin(rad);
}
// Does texture `ti` (a tree: children are earlier textures, validate()) read the hit's u, v?  Only an
// image leaf does (image_texture.rs:34-56); checker and marble read the point, solid nothing.
bool texture_uses_uv(const rt_scene_desc* d, int32_t ti) {
  if (ti < 0 || ti >= d->n_textures) return false;
  const rt_texture& t = d->textures[ti];
  if (t.kind == RT_TEX_IMAGE) return true;
  if (t.kind == RT_TEX_CHECKER) return texture_uses_uv(d, t.odd) || texture_uses_uv(d, t.even);
  return false;
}
// Book-2: Translate(RotateY(sphere)) of a plain sphere is the sphere about the moved centre — flattened
// into a world-space sphere before the tree is built, by the formula that maps an instance's hit point
// back to the world, so the instances take the reference sphere path (sphere leaf loop, no per-leaf ray
// transform).  t, point and normal agree with per-ray instancing in real arithmetic; u, v do not under a
// rotation (the instance's u is taken in its own frame, shifted by angle / 360), so a rotated sphere is
// flattened only when its material never reads u, v; rt_scene_hit then derives the instance's u, v from
// the record (uv_fixups).  The oracle flattens by the same rule (oracle.c flatten_instanced_sphere).
// DESIGN.md §10.
bool flattens(const rt_scene_desc* d, const rt_object& o) {
  if (o.geometry != RT_GEOM_SPHERE || !o.transform || o.medium) return false;
  if (o.rotate_y_deg == 0.0) return true;
  return o.material >= 0 && o.material < d->n_materials && !texture_uses_uv(d, d->materials[o.material].texture);
}
rt_object flat_object(const rt_scene_desc* d, const rt_object& o) {
  rt_object f = o;
  if (!flattens(d, o)) return f;
  double cs, sn;
  rotate_y_cs(o, cs, sn);
  const double cx = o.p[0], cy = o.p[1], cz = o.p[2];
  f.p[0] = (cs * cx + sn * cz) + o.offset[0];
  f.p[1] = cy + o.offset[1];
  f.p[2] = (-sn * cx + cs * cz) + o.offset[2];
  f.transform = 0;
  f.rotate_y_deg = 0.0;
  f.offset[0] = f.offset[1] = f.offset[2] = 0.0;
  return f;
}
// A scene description whose objects are flat_object's (the objects live in `store`).
rt_scene_desc flat_scene(const rt_scene_desc* d, std::vector<rt_object>& store) {
  store.resize((size_t)std::max(0, d->n_objects));
  for (int i = 0; i < d->n_objects; ++i) store[i] = flat_object(d, d->objects[i]);
  rt_scene_desc f = *d;
  f.objects = store.data();
  return f;
}
// A flattened rotated sphere's u, v as its instance reports them (sphere.rs:17-26 on the object-frame
// outward normal): the world normal rotated back by RotateY's inverse (rotate_y.h).
void instance_sphere_uv(double cs, double sn, rt_hit& h) {
  const double s = h.front_face ? 1.0 : -1.0;
  const double nx = s * h.normal[0], ny = s * h.normal[1], nz = s * h.normal[2];
  const double ox = cs * nx - sn * nz, oz = sn * nx + cs * nz;
  const double pi = 3.14159265358979323846;
  h.u = (std::atan2(-oz, ox) + pi) / (2.0 * pi);
  h.v = std::acos(-ny) / pi;
}
// moving_sphere.h center(time), the device's formula (the bounding box uses it at time0 and time1)
void moving_center(const rt_object& o, double tm, double* c) {
  const double s = (tm - o.q[3]) / (o.q[4] - o.q[3]);
  for (int k = 0; k < 3; ++k) c[k] = o.p[k] + (o.q[k] - o.p[k]) * s;
}

Box reference_box(const rt_object& o);
// object -> leaf box: the reference's bounding_box for reference objects; for book-2 objects the
// book's: moving_sphere.h (union of the boxes at time0 and time1), rotate_y.h (the 8 rotated
// corners), translate (box + offset), constant_medium.h (the boundary's box).
Box object_box(const rt_object& o) {
  if (!is_extended(o)) return reference_box(o);
  Box b{};
  if (o.geometry == RT_GEOM_MOVING_SPHERE) {
    double c0[3], c1[3];
    moving_center(o, o.q[3], c0);
    moving_center(o, o.q[4], c1);
    Box b0{}, b1{};
    for (int k = 0; k < 3; ++k) {
      b0.mn[k] = c0[k] - o.p[3];
      b0.mx[k] = c0[k] + o.p[3];
      b1.mn[k] = c1[k] - o.p[3];
      b1.mx[k] = c1[k] + o.p[3];
    }
    b = surrounding(b0, b1);
  } else {
    b = reference_box(o);
  }
  if (o.transform) {
    double cs, sn;
    rotate_y_cs(o, cs, sn);
    Box r{};
    for (int k = 0; k < 3; ++k) {
      r.mn[k] = std::numeric_limits<double>::infinity();
      r.mx[k] = -std::numeric_limits<double>::infinity();
    }
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int k = 0; k < 2; ++k) {
          const double x = i * b.mx[0] + (1 - i) * b.mn[0];
          const double y = j * b.mx[1] + (1 - j) * b.mn[1];
          const double z = k * b.mx[2] + (1 - k) * b.mn[2];
          const double nx = cs * x + sn * z, nz = -sn * x + cs * z;
          const double t[3] = {nx, y, nz};
          for (int c = 0; c < 3; ++c) {
            r.mn[c] = std::fmin(r.mn[c], t[c]);
            r.mx[c] = std::fmax(r.mx[c], t[c]);
          }
        }
    for (int k = 0; k < 3; ++k) {
      r.mn[k] += o.offset[k];
      r.mx[k] += o.offset[k];
    }
    b = r;
  }
  return b;
}

// exactly the reference's bounding_box (sphere.rs:54-60, rect.rs:82-99, rect.rs:158-163)
Box reference_box(const rt_object& o) {
  Box b{};
  if (o.geometry == RT_GEOM_SPHERE) {
    for (int k = 0; k < 3; ++k) {
      b.mn[k] = o.p[k] - o.p[3];
      b.mx[k] = o.p[k] + o.p[3];
    }
  } else if (o.geometry == RT_GEOM_RECT_BOX) {
    for (int k = 0; k < 3; ++k) {
      b.mn[k] = o.p[k];
      b.mx[k] = o.p[k + 3];
    }
  } else {
    int D1 = (o.geometry == RT_GEOM_RECT_YZ) ? 1 : 0;
    int D2 = (o.geometry == RT_GEOM_RECT_XY) ? 1 : 2;
    int n = 3 - D1 - D2;
    b.mn[D1] = o.p[0];
    b.mx[D1] = o.p[1];
    b.mn[D2] = o.p[2];
    b.mx[D2] = o.p[3];
    b.mn[n] = o.p[4] - 0.0001;  // BBOX_WIDTH, rect.rs:9
    b.mx[n] = o.p[4] + 0.0001;
  }
  return b;
}

int validate(rt_ctx* c, const rt_scene_desc* d) {
  if (!d) return fail(c, RT_E_INVALID, "scene is NULL");
  if (d->n_objects < 0 || d->n_materials < 0 || d->n_textures < 0 || d->n_perlin < 0 || d->n_images < 0)
    return fail(c, RT_E_INVALID, "negative count in scene");
  if ((d->n_objects && !d->objects) || (d->n_materials && !d->materials) || (d->n_textures && !d->textures) ||
      (d->n_perlin && !d->perlin) || (d->n_images && !d->images))
    return fail(c, RT_E_INVALID, "NULL array with non-zero count");
  if (d->sky < RT_SKY_ABOVE || d->sky > RT_SKY_NONE) return fail(c, RT_E_INVALID, "bad skybox %d", d->sky);
  for (int i = 0; i < d->n_objects; ++i) {
    const rt_object& o = d->objects[i];
    if (o.geometry < RT_GEOM_SPHERE || o.geometry > RT_GEOM_MOVING_SPHERE)
      return fail(c, RT_E_INVALID, "object %d: bad geometry %d", i, o.geometry);
    if ((o.medium != 0 && o.medium != 1) || (o.transform != 0 && o.transform != 1))
      return fail(c, RT_E_INVALID, "object %d: medium / transform flags must be 0 or 1", i);
    if (o.geometry == RT_GEOM_MOVING_SPHERE && !(o.q[4] != o.q[3]))
      return fail(c, RT_E_INVALID, "object %d: moving sphere needs time0 != time1", i);
    if (o.medium && (o.material < 0 || o.material >= d->n_materials || d->materials[o.material].kind != RT_MAT_ISOTROPIC))
      return fail(c, RT_E_INVALID, "object %d: a constant medium takes an isotropic material", i);
    if (o.material < 0 || o.material >= d->n_materials)
      return fail(c, RT_E_INVALID, "object %d: material %d out of range", i, o.material);
  }
  for (int i = 0; i < d->n_materials; ++i) {
    const rt_material& m = d->materials[i];
    if (m.kind < RT_MAT_METAL || m.kind > RT_MAT_ISOTROPIC)
      return fail(c, RT_E_INVALID, "material %d: bad kind %d", i, m.kind);
    bool textured = m.kind == RT_MAT_LAMBERTIAN || m.kind == RT_MAT_DIFFUSE_LIGHT || m.kind == RT_MAT_FAIRY_LIGHT ||
                    m.kind == RT_MAT_ISOTROPIC;
    if (textured && (m.texture < 0 || m.texture >= d->n_textures))
      return fail(c, RT_E_INVALID, "material %d: texture %d out of range", i, m.texture);
  }
  for (int i = 0; i < d->n_textures; ++i) {
    const rt_texture& t = d->textures[i];
    switch (t.kind) {
      case RT_TEX_SOLID: break;
      case RT_TEX_CHECKER:
        if (t.odd < 0 || t.odd >= d->n_textures || t.even < 0 || t.even >= d->n_textures)
          return fail(c, RT_E_INVALID, "texture %d: checker child out of range", i);
        // children must be earlier textures: guarantees the lookup terminates (no cycles)
        if (t.odd >= i || t.even >= i) return fail(c, RT_E_INVALID, "texture %d: checker children must precede it", i);
        break;
      case RT_TEX_PERLIN:
        if (t.table < 0 || t.table >= d->n_perlin) return fail(c, RT_E_INVALID, "texture %d: perlin table", i);
        break;
      case RT_TEX_IMAGE:
        if (t.table < 0 || t.table >= d->n_images) return fail(c, RT_E_INVALID, "texture %d: image index", i);
        break;
      default: return fail(c, RT_E_INVALID, "texture %d: bad kind %d", i, t.kind);
    }
  }
  for (int i = 0; i < d->n_perlin; ++i)
    for (int k = 0; k < 256; ++k) {
      const rt_perlin_table& T = d->perlin[i];
      if (T.perm_x[k] < 0 || T.perm_x[k] > 255 || T.perm_y[k] < 0 || T.perm_y[k] > 255 || T.perm_z[k] < 0 ||
          T.perm_z[k] > 255)
        return fail(c, RT_E_INVALID, "perlin table %d: permutation entry out of [0,255]", i);
    }
  for (int i = 0; i < d->n_images; ++i)
    if (d->images[i].width < 1 || d->images[i].height < 1 || !d->images[i].rgb)
      return fail(c, RT_E_INVALID, "image %d: empty", i);
  return RT_OK;
}

// 64-bit FNV-1a digest of a scene description and its BVH builder, field by field (no struct padding
// hashed): rt_scene_digest / the multi-GPU scene check.
struct Fnv1a {
  uint64_t h = 14695981039346656037ull;
  void bytes(const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  }
  template <class T>
  void val(const T& v) { bytes(&v, sizeof v); }
};
uint64_t scene_digest(const rt_scene_desc* d, int32_t builder) {
  Fnv1a f;
  f.val(builder);
  f.val(d->sky);
  f.bytes(d->sky_color, sizeof d->sky_color);
  f.val(d->n_objects);
  for (int i = 0; i < d->n_objects; ++i) {
    const rt_object& o = d->objects[i];
    f.val(o.geometry); f.val(o.material); f.bytes(o.p, sizeof o.p); f.val(o.medium); f.val(o.transform);
    f.bytes(o.q, sizeof o.q); f.val(o.density); f.val(o.rotate_y_deg); f.bytes(o.offset, sizeof o.offset);
  }
  f.val(d->n_materials);
  for (int i = 0; i < d->n_materials; ++i) {
    const rt_material& m = d->materials[i];
    f.val(m.kind); f.val(m.texture); f.bytes(m.albedo, sizeof m.albedo); f.val(m.param);
  }
  f.val(d->n_textures);
  for (int i = 0; i < d->n_textures; ++i) {
    const rt_texture& t = d->textures[i];
    f.val(t.kind); f.val(t.odd); f.val(t.even); f.val(t.table); f.bytes(t.color, sizeof t.color); f.val(t.scale);
  }
  f.val(d->n_perlin);
  for (int i = 0; i < d->n_perlin; ++i) {
    const rt_perlin_table& t = d->perlin[i];
    f.bytes(t.ranfloat, sizeof t.ranfloat); f.bytes(t.perm_x, sizeof t.perm_x); f.bytes(t.perm_y, sizeof t.perm_y);
    f.bytes(t.perm_z, sizeof t.perm_z);
  }
  f.val(d->n_images);
  for (int i = 0; i < d->n_images; ++i) {
    const rt_image& m = d->images[i];
    f.val(m.width); f.val(m.height);
    f.bytes(m.rgb, (size_t)m.width * m.height * 3);
  }
  return f.h;
}

// Leaf order of a tree, lhs before rhs (in-order): rank[object]; objects outside it (a SAH tree leaves out
// the never-hit inverted boxes) follow in index order.
std::vector<int32_t> reference_ranks(const BuiltTree& t, int32_t n) {
  std::vector<int32_t> rank((size_t)std::max(0, n), -1);
  int32_t next = 0;
  if (t.root >= 0) {
    std::vector<int32_t> stack{t.root};
    while (!stack.empty()) {
      const BuildNode& nd = t.nodes[stack.back()];
      stack.pop_back();
      if (nd.leaf >= 0) {
        if (rank[nd.leaf] < 0) rank[nd.leaf] = next++;
        continue;
      }
      stack.push_back(nd.rhs);  // (popped after the whole lhs subtree)
      stack.push_back(nd.lhs);
    }
  }
  for (int32_t i = 0; i < n; ++i)
    if (rank[i] < 0) rank[i] = next++;
  return rank;
}

BuiltTree build_tree(const rt_scene_desc* d, int32_t builder) {
  std::vector<Box> boxes(d->n_objects);
  for (int i = 0; i < d->n_objects; ++i) boxes[i] = object_box(d->objects[i]);
  // The sweep's split cost weighs a RectBox leaf (six faces, the costliest exact test) 4, every other
  // object 1: Cornell +5.4 %, headline ±0.  SHIRLEY_SAH_BOXW=<c>: the weight (tuning; 1 = the
  // plain count).  Scenes without a RectBox build the unweighted tree.
  std::vector<double> w;
  const char* bw = getenv("SHIRLEY_SAH_BOXW");
  const double box_weight = bw ? atof(bw) : 4.0;
  bool any_box = false;
  for (int i = 0; i < d->n_objects; ++i) any_box = any_box || d->objects[i].geometry == RT_GEOM_RECT_BOX;
  if (any_box && box_weight != 1.0) {
    w.assign(d->n_objects, 1.0);
    for (int i = 0; i < d->n_objects; ++i)
      if (d->objects[i].geometry == RT_GEOM_RECT_BOX) w[i] = box_weight;
  }
  return builder == RT_BVH_SAH ? build_sah_tree(boxes, getenv("SHIRLEY_SAH_BINNED") == nullptr, w.empty() ? nullptr : &w)
                               : build_reference_tree(boxes);
}

void box_to6(const Box& b, double* o) {
  for (int k = 0; k < 3; ++k) {
    o[k] = b.mn[k];
    o[k + 3] = b.mx[k];
  }
}

// f64 -> f32 rounded toward -inf / +inf
void box_to_node(const Box& b, double* o) {
  for (int k = 0; k < 3; ++k) {
    o[k] = b.mn[k];
    o[k + 3] = b.mx[k];
  }
}

// BuiltTree -> DNode array in breadth-first order (node 0 = top node whose child 0 is the root), so
// that a prefix of the array = the top levels of the tree, which the kernels keep in LDS.
void flatten(const BuiltTree& t, std::vector<DNode>& out) {
  out.clear();
  DNode top{};
  top.child[0] = kEmptyChild;
  top.child[1] = kEmptyChild;
  out.push_back(top);
  if (t.root < 0) return;
  struct Item {
    int32_t built;
    int32_t parent;
    int slot;
  };
  std::vector<Item> q{{t.root, 0, 0}};
  for (size_t head = 0; head < q.size(); ++head) {
    Item it = q[head];
    const BuildNode& bn = t.nodes[it.built];
    box_to_node(bn.box, out[it.parent].box[it.slot]);
    if (bn.leaf >= 0) {
      out[it.parent].child[it.slot] = ~bn.leaf;
      continue;
    }
    int32_t idx = (int32_t)out.size();
    out[it.parent].child[it.slot] = idx;
    out.push_back(DNode{});
    q.push_back({bn.lhs, idx, 0});
    q.push_back({bn.rhs, idx, 1});
  }
}

// Collapse heuristic: half the surface area of a box (0 for an inverted or NaN box).
double half_area(const Box& b) {
  const double x = b.mx[0] - b.mn[0], y = b.mx[1] - b.mn[1], z = b.mx[2] - b.mn[2];
  if (!(x >= 0.0 && y >= 0.0 && z >= 0.0)) return 0.0;
  return x * y + y * z + z * x;
}

// BuiltTree -> 4-wide nodes for the megakernel: each node takes its two children and then, while
// it has fewer than four, replaces its largest-area internal child by that child's two children
// (order kept).  Boxes stay the reference's exact boxes.  `stack_bound` = the worst-case traversal
// stack: the sum over a root path of (internal children - 1) per node (at most that many pushes).
// f32 bounds rounded outward (f32 cast rounds to nearest; step once more if it landed inside).
float round_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -INFINITY);
  return f;
}
float round_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, INFINITY);
  return f;
}

// Node-box inflation and the ray-origin range it covers.  The f32 node test computes
// t = fma(plane, 1/d, -o*(1/d)) from o and 1/d rounded to f32: in space units its error is at most
// ~2^-22 (|o| + |plane|); inflating every stored box by delta = 2^-20 (L + B) (B = largest finite
// |plane|) and rounding outward keeps the test a superset of the exact one for every ray with
// max|o| <= L, with a 4x margin.
struct Inflation {
  double delta;
  float origin_limit;
  double box_bound;  // B: the largest finite |plane| of any box
};
Inflation inflation_for(const BuiltTree& t) {
  double B = 0.0;
  for (const BuildNode& n : t.nodes)
    for (int k = 0; k < 3; ++k) {
      if (std::isfinite(n.box.mn[k])) B = std::max(B, std::fabs(n.box.mn[k]));
      if (std::isfinite(n.box.mx[k])) B = std::max(B, std::fabs(n.box.mx[k]));
    }
  const double L = std::max(16.0, 4.0 * B);
  return Inflation{std::ldexp(L + B, -20), (float)L, B};
}

// child slot of a 4-wide node: an empty slot never passes (lo = +inf > hi = -inf); a box with a
// NaN plane always passes (its leaf is tested exactly anyway)
void set_child_box(DNode4F& n, int slot, const Box* b, double delta) {
  for (int a = 0; a < 3; ++a) {
    float lo, hi;
    if (!b) {
      lo = INFINITY;
      hi = -INFINITY;
    } else if (std::isnan(b->mn[a]) || std::isnan(b->mx[a])) {
      lo = -INFINITY;
      hi = INFINITY;
    } else {
      lo = round_down(b->mn[a] - delta);
      hi = round_up(b->mx[a] + delta);
    }
    n.row[a][0][slot] = lo;
    n.row[a][1][slot] = hi;
    n.row[a][2][slot] = lo;
  }
}

// Optimal collapse of the binary tree into 4-wide nodes: minimises the sum of the surface areas of
// the 4-wide internal nodes (expected node visits of a ray, SAH), by dynamic programming over the
// binary tree.  H(n, j) = least cost of covering subtree n with at most j child slots of its
// parent: one slot holds n itself (a leaf: cost 0; an internal node: its own 4-wide node,
// F(n) = area(n) + G(n, 4)), more slots may open n into its two children, G(n, k) = min over the
// split j of H(lhs, j) + H(rhs, k - j).  Leaf costs do not depend on the collapse (every object is
// one child slot) and are left out.
struct Collapse4 {
  const BuiltTree* t = nullptr;
  std::vector<double> H, G;    // [n * 5 + j], j = 1..4
  std::vector<int8_t> split;   // argmin j of G(n, k), [n * 5 + k]
  bool ready() const { return t != nullptr; }
  void build(const BuiltTree& tree) {
    t = &tree;
    const size_t nn = tree.nodes.size();
    H.assign(nn * 5, 0.0);
    G.assign(nn * 5, INFINITY);
    split.assign(nn * 5, 1);
    // children come before parents in neither builder's order for sure: iterative post-order
    std::vector<std::pair<int32_t, bool>> st{{tree.root, false}};
    while (!st.empty()) {
      auto [n, done] = st.back();
      st.pop_back();
      const BuildNode& b = tree.nodes[n];
      if (b.leaf >= 0) continue;  // H = 0
      if (!done) {
        st.push_back({n, true});
        st.push_back({b.lhs, false});
        st.push_back({b.rhs, false});
        continue;
      }
      for (int k = 2; k <= 4; ++k)
        for (int j = 1; j < k; ++j) {
          const double c = H[b.lhs * 5 + j] + H[b.rhs * 5 + (k - j)];
          if (c < G[n * 5 + k]) { G[n * 5 + k] = c; split[n * 5 + k] = (int8_t)j; }
        }
      const double f = half_area(b.box) + G[n * 5 + 4];
      H[n * 5 + 1] = f;
      for (int j = 2; j <= 4; ++j) H[n * 5 + j] = std::min(f, G[n * 5 + j]);
    }
  }
  // the child slots of the 4-wide node made from internal binary node n
  void children(int32_t n, std::vector<int32_t>& out) const {
    out.clear();
    collect(t->nodes[n].lhs, split[n * 5 + 4], out);
    collect(t->nodes[n].rhs, 4 - split[n * 5 + 4], out);
  }
  void collect(int32_t c, int j, std::vector<int32_t>& out) const {
    const BuildNode& b = t->nodes[c];
    if (b.leaf >= 0 || j == 1 || !(G[c * 5 + j] < H[c * 5 + 1])) {
      out.push_back(c);
      return;
    }
    collect(b.lhs, split[c * 5 + j], out);
    collect(b.rhs, j - split[c * 5 + j], out);
  }
};

// use_dp: the optimal collapse (Collapse4) instead of the greedy one (open the largest-area internal
// child until four slots are filled).  rt_scene_upload picks it for the scenes the megakernel runs with
// the whole scene in LDS, greedy for the rest.
void flatten4(const BuiltTree& t, const rt_scene_desc* d, double delta, std::vector<DNode4F>& out,
              int32_t& stack_bound, bool use_dp) {
  Collapse4 dp;
  if (t.root >= 0 && use_dp) dp.build(t);
  out.clear();
  DNode4F top{};
  for (int k = 0; k < 4; ++k) {
    top.child[k] = kEmptyChild;
    set_child_box(top, k, nullptr, delta);
  }
  out.push_back(top);
  stack_bound = 1;
  if (t.root < 0) return;
  auto internal = [&](int32_t n) { return t.nodes[n].leaf < 0; };
  struct Item {
    int32_t built;
    int32_t parent;
    int slot;
    int32_t level;  // stack entries that can be live when this node is visited
  };
  std::vector<Item> q{{t.root, 0, 0, 0}};
  for (size_t head = 0; head < q.size(); ++head) {
    const Item it = q[head];
    const BuildNode& bn = t.nodes[it.built];
    set_child_box(out[it.parent], it.slot, &bn.box, delta);
    if (bn.leaf >= 0) {
      const int32_t g = d->objects[bn.leaf].geometry;
      // book-2 objects take the "box" (slow) leaf loop, which dispatches on the primitive
      const int32_t flags = is_extended(d->objects[bn.leaf]) ? kLeafGeneric | kLeafBox
                            : g == RT_GEOM_SPHERE            ? 0
                            : (g == RT_GEOM_RECT_BOX ? kLeafGeneric | kLeafBox : kLeafGeneric);
      out[it.parent].child[it.slot] = ~(bn.leaf | flags);
      continue;
    }
    const int32_t idx = (int32_t)out.size();
    out[it.parent].child[it.slot] = idx;
    DNode4F nd{};
    for (int k = 0; k < 4; ++k) {
      nd.child[k] = kEmptyChild;
      set_child_box(nd, k, nullptr, delta);
    }
    out.push_back(nd);
    std::vector<int32_t> ch;
    if (dp.ready()) {
      dp.children(it.built, ch);
    } else {
      ch = {bn.lhs, bn.rhs};
      while (ch.size() < 4) {
        int pick = -1;
        double best = -1.0;
        for (size_t i = 0; i < ch.size(); ++i)
          if (internal(ch[i]) && half_area(t.nodes[ch[i]].box) > best) {
            best = half_area(t.nodes[ch[i]].box);
            pick = (int)i;
          }
        if (pick < 0) break;
        const int32_t x = ch[pick];
        ch[pick] = t.nodes[x].lhs;
        ch.insert(ch.begin() + pick + 1, t.nodes[x].rhs);
      }
    }
    int n_int = 0;
    for (int32_t c : ch) n_int += internal(c) ? 1 : 0;
    const int32_t level = it.level + std::max(0, n_int - 1);
    stack_bound = std::max(stack_bound, level + 1);
    for (size_t i = 0; i < ch.size(); ++i) q.push_back({ch[i], idx, (int)i, level});
  }
}

int resolve_stream(rt_ctx* c, void* stream, hipStream_t* out) {
  *out = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
  return RT_OK;
}

struct Layout {
  int tiles_x, tiles_y, n_tiles, n_tiles_rank;
};

Layout layout(const rt_camera* cam, int ty0, int ty1, int rank, int world) {
  Layout L;
  L.tiles_x = (cam->image_width + kTile - 1) / kTile;
  L.tiles_y = ty1 - ty0;
  L.n_tiles = L.tiles_x * L.tiles_y;
  L.n_tiles_rank = (L.n_tiles > rank) ? (L.n_tiles - rank + world - 1) / world : 0;
  return L;
}

DCamera device_camera(const rt_camera* c) {
  // camera/mod.rs:99-108, evaluated once with the reference's operation order (-ffp-contract=off)
  DCamera d{};
  d.width = c->image_width;
  d.height = c->image_height;
  d.has_lens = c->has_lens;
  d.lens_radius = c->lens_radius;
  d.wd = (double)c->image_width;
  d.hd = (double)c->image_height;
  d.inv_w = 1.0 / d.wd;  // correctly rounded (IEEE division)
  d.inv_h = 1.0 / d.hd;
  for (int k = 0; k < 3; ++k) {
    d.origin[k] = c->origin[k];
    d.u[k] = c->u[k];
    d.v[k] = c->v[k];
    d.horizontal[k] = c->u[k] * (c->width * c->focus_length);
    d.vertical[k] = c->v[k] * (c->height * c->focus_length);
  }
  for (int k = 0; k < 3; ++k)
    d.lower_left[k] = ((c->origin[k] - d.horizontal[k] * 0.5) - d.vertical[k] * 0.5) -
                      c->w[k] * (c->focal_length * c->focus_length);
  return d;
}

int check_render_args(rt_ctx* c, const rt_camera* cam, const rt_render_params* p) {
  if (!c) return RT_E_INVALID;
  if (!c->have_scene) return fail(c, RT_E_INVALID, "no scene uploaded (call rt_scene_upload first)");
  if (!cam || !p) return fail(c, RT_E_INVALID, "camera/params is NULL");
  if (cam->image_width < 1 || cam->image_height < 1 || cam->image_width > (1 << 16) || cam->image_height > (1 << 16))
    return fail(c, RT_E_INVALID, "bad image size %dx%d", cam->image_width, cam->image_height);
  if (p->samples < 0 || p->max_depth < 0) return fail(c, RT_E_INVALID, "negative samples/max_depth");
  if (p->tile_world < 1 || p->tile_rank < 0 || p->tile_rank >= p->tile_world)
    return fail(c, RT_E_INVALID, "bad tile rank/world %d/%d", p->tile_rank, p->tile_world);
  if (p->sample_chunk < 0) return fail(c, RT_E_INVALID, "negative sample_chunk");
  return RT_OK;
}

constexpr long long kWfDefaultSlots = 1LL << 21;
constexpr int kWfBatch = 32;  // iterations launched between two host checks of the termination flag

int default_engine() {
  const char* e = getenv("SHIRLEY_ENGINE");
  if (e && !strcmp(e, "megakernel")) return RT_ENGINE_MEGAKERNEL;
  if (e && !strcmp(e, "wavefront")) return RT_ENGINE_WAVEFRONT;
  if (e && !strcmp(e, "split")) return RT_ENGINE_SPLIT;
  return RT_ENGINE_MEGAKERNEL;  // measured faster on MI355X
}

// Carve the slot arrays out of one allocation (each array 256-B aligned).
struct Carver {
  char* base;
  size_t off = 0;
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base + off);
    off += n * sizeof(T);
    return p;
  }
};

size_t wf_pool_bytes(size_t n) {
  Carver cv{nullptr};
  for (int i = 0; i < 17; ++i) cv.take<double>(n);  // 15 path doubles + ht + tq.px/py/pz/scale below
  cv.take<uint64_t>(n);
  for (int i = 0; i < 11; ++i) cv.take<uint32_t>(n);
  cv.take<uint8_t>(n);
  for (int i = 0; i < 3; ++i) cv.take<double>(n);
  for (int i = 0; i < 3; ++i) cv.take<int32_t>(n);
  cv.take<unsigned long long>(2 * (n / kWave));  // unit windows
  cv.take<uint32_t>(n / kWave);                  // texture queue counts
  cv.take<unsigned>(64);                         // retired counter
  return cv.off + 256;
}

void wf_carve(void* base, size_t n, WfParams& P) {
  WfState& st = P.st;
  WfTexQ& tq = P.tq;
  Carver cv{static_cast<char*>(base)};
  double** dp[] = {&st.ox, &st.oy, &st.oz, &st.dx, &st.dy, &st.dz, &st.ax, &st.ay, &st.az,
                   &st.ex, &st.ey, &st.ez, &st.sx, &st.sy, &st.sz, &st.ht, &tq.px};
  for (double** q : dp) *q = cv.take<double>(n);
  st.part = cv.take<uint64_t>(n);
  st.pixel = cv.take<uint32_t>(n);
  st.sample = cv.take<uint32_t>(n);
  st.draw = cv.take<uint32_t>(n);
  st.c2 = cv.take<uint32_t>(n);
  st.c3 = cv.take<uint32_t>(n);
  st.s_next = cv.take<int32_t>(n);
  st.s_end = cv.take<int32_t>(n);
  st.depth = cv.take<int32_t>(n);
  st.hprim = cv.take<int32_t>(n);
  st.hface = cv.take<int32_t>(n);
  (void)cv.take<uint32_t>(n);  // spare
  st.state = cv.take<uint8_t>(n);
  tq.py = cv.take<double>(n);
  tq.pz = cv.take<double>(n);
  tq.scale = cv.take<double>(n);
  tq.slot = cv.take<int32_t>(n);
  tq.tex = cv.take<int32_t>(n);
  tq.kind = cv.take<int32_t>(n);
  P.win = cv.take<unsigned long long>(2 * (n / kWave));
  tq.count = cv.take<uint32_t>(n / kWave);
  P.retired = cv.take<unsigned>(64);
}

// The wavefront engine: start (every slot takes a unit and a camera ray), then rounds of
// extend -> shade -> texture until no slot holds work.  Rounds are launched in batches; the host
// reads the retired-slot count after the previous batch while the next batch runs, so the GPU
// never waits on the host.
int run_wavefront(rt_ctx* c, const KParams& kp, bool timing, hipStream_t s) {
  const uint64_t n_units = kp.work.n_units;
  long long slots = kWfDefaultSlots;
  if (const char* e = getenv("SHIRLEY_WF_SLOTS")) slots = std::max(64LL, atoll(e));
  slots = std::min<long long>(slots, std::max<long long>(64, (long long)n_units));
  slots = (slots + 63) / 64 * 64;
  const size_t n = (size_t)slots;
  int st = ensure(c, c->wf_pool, wf_pool_bytes(n));
  if (st) return st;
  st = ensure(c, c->wf_iters, sizeof(WfIter));  // extend cursors (wf_shade re-zeroes them each round)
  if (st) return st;

  WfParams P{};
  P.scene = c->wf_scene;
  P.scene.time0 = kp.scene.time0;
  P.scene.time1 = kp.scene.time1;
  P.scene.shutter = kp.scene.shutter;  // (the call's shutter, in the pass's KBlock)
  P.cam = kp.cam;
  P.work = kp.work;
  wf_carve(c->wf_pool.p, n, P);
  P.n_slots = (uint32_t)n;
  P.n_perlin = c->n_perlin;
  P.ext_window = 256;
  if (const char* e = getenv("SHIRLEY_WF_WINDOW")) P.ext_window = (uint32_t)std::max(1, atoi(e) / 64) * 64;
  P.partial = kp.partial;
  P.unit_counter = kp.unit_counter;
  P.counters = kp.counters;
  P.it = static_cast<WfIter*>(c->wf_iters.p);

  HIP_TRY(c, hipMemsetAsync(P.st.state, 0, n, s));           // kSlotIdle
  HIP_TRY(c, hipMemsetAsync(P.st.pixel, 0xff, n * 4, s));    // no unit
  HIP_TRY(c, hipMemsetAsync(P.it, 0, sizeof(WfIter), s));
  HIP_TRY(c, hipMemsetAsync(P.retired, 0, sizeof(unsigned), s));
  const int gt = wf_grid_threads();
  const int grid = (int)((n + gt - 1) / gt);
  const bool texture_pass = c->has_perlin;  // deferred entries exist only for Perlin leaves
  const int tex_grid = std::min(grid, 4 * c->cu_count);  // strided over slot groups, tables staged once per block
  const int ext_blocks = std::max(1, c->cu_count * std::max(1, c->wf_blocks_per_cu));

  // timing: an event before and after each launch of a round, elapsed times summed per kernel
  std::vector<hipEvent_t>& lap = c->lap_ev;
  std::vector<int> lap_tag;  // kernel the interval starting at this mark belongs to (3: none)
  auto lap_mark = [&](int tag) -> int {
    if (!timing) return RT_OK;
    if (lap_tag.size() == lap.size()) {
      hipEvent_t e;
      HIP_TRY(c, hipEventCreate(&e));
      lap.push_back(e);
    }
    HIP_TRY(c, hipEventRecord(lap[lap_tag.size()], s));
    lap_tag.push_back(tag);
    return RT_OK;
  };

  HIP_TRY(c, wf_start(P, grid, s));
  long long iter = 1;
  // safety bound: every round advances each working slot by one segment or one regeneration
  const long long max_iters = 64 + 2LL * ((long long)((n_units + n - 1) / n) + 1) *
                                       (long long)(kp.work.chunk) * (long long)(kp.work.max_depth + 2);
  int batch = 0;
  for (;;) {
    for (int k = 0; k < kWfBatch; ++k, ++iter) {
      if ((st = lap_mark(0))) return st;
      if (c->wf_wide)
        HIP_TRY(c, wf_launch_extend4(P, c->cu_count * c->wf4_blocks_per_cu, s));
      else
        HIP_TRY(c, wf_launch_extend(P, ext_blocks, s));
      if ((st = lap_mark(1))) return st;
      HIP_TRY(c, wf_launch_shade(P, grid, s));
      if ((st = lap_mark(2))) return st;
      if (texture_pass) HIP_TRY(c, wf_launch_texture(P, tex_grid, s));
      if ((st = lap_mark(3))) return st;
    }
    HIP_TRY(c, hipMemcpyAsync(&c->wf_host[batch & 1], P.retired, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipEventRecord(c->wf_ev[batch & 1], s));
    if (batch > 0) {
      HIP_TRY(c, hipEventSynchronize(c->wf_ev[(batch - 1) & 1]));
      if (c->wf_host[(batch - 1) & 1] >= (uint32_t)n) break;  // every slot retired
    }
    ++batch;
    if (iter > max_iters) return fail(c, RT_E_HIP, "wavefront engine did not terminate after %lld rounds", iter);
  }
  c->last_iters += (int)iter;
  c->last_slots = n;
  c->last_timing = timing;
  if (timing && !lap_tag.empty()) {
    HIP_TRY(c, hipEventSynchronize(lap[lap_tag.size() - 1]));
    double acc[3] = {0, 0, 0};
    for (size_t i = 0; i + 1 < lap_tag.size(); ++i) {
      if (lap_tag[i] > 2) continue;
      float ms = 0.f;
      HIP_TRY(c, hipEventElapsedTime(&ms, lap[i], lap[i + 1]));
      acc[lap_tag[i]] += ms;
    }
    for (int k = 0; k < 3; ++k) c->lap_ms[k] += acc[k];  // (summed over the call's sample passes)
  }
  return RT_OK;
}

// The sample range [begin, end) of a call (rt_render_params.sample_begin / sample_count, ABI 6).
struct SampleRange {
  int begin = 0, end = 0;
};

int resolve_range(rt_ctx* c, const rt_render_params* p, SampleRange* r) {
  const int S = p->samples == 0 ? 1 : p->samples;  // main.rs:75-80
  if (p->sample_begin < 0 || p->sample_count < 0 || p->sample_begin > S ||
      (long long)p->sample_begin + p->sample_count > S)
    return fail(c, RT_E_INVALID, "sample range [%d, +%d) outside [0, %d)", p->sample_begin, p->sample_count, S);
  r->begin = p->sample_begin;
  r->end = p->sample_count ? p->sample_begin + p->sample_count : S;
  return RT_OK;
}

// trace + reduce of samples [R.begin, R.end) for tile rows [ty0, ty1); out layout: packed tiles
// (packed=1) or rows [row0, row1).  The call's work units (pixel x chunk of samples) are traced in
// sample passes of at most `scratch` bytes of partial sums each; every pass's reduce continues the
// per-pixel chunk-order sums of the passes before it (reduce_kernel `accumulate`), so the frame is the
// same for any number of passes.
int render_window(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, const SampleRange& R, int ty0, int ty1,
                  int row0, int row1, int packed, double* out_dev, hipStream_t s) {
  int st = check_render_args(c, cam, p);
  if (st) return st;
  HIP_TRY(c, hipSetDevice(c->device));
  const int count = R.end - R.begin;
  Layout L = layout(cam, ty0, ty1, p->tile_rank, p->tile_world);
  const long long n_pix = (long long)L.n_tiles_rank * kTilePixels;

  int engine = p->engine & 0xf;
  const bool timing = (p->engine & RT_ENGINE_TIMING) != 0;
  if (engine == RT_ENGINE_AUTO) engine = default_engine();
  if (engine != RT_ENGINE_MEGAKERNEL && engine != RT_ENGINE_WAVEFRONT && engine != RT_ENGINE_SPLIT)
    return fail(c, RT_E_INVALID, "bad engine %d", p->engine);
  if (engine == RT_ENGINE_SPLIT && c->split_nt == 0) engine = RT_ENGINE_MEGAKERNEL;  // scene not eligible

  const long long lanes = (long long)c->cu_count * std::max(1, c->blocks_per_cu) * c->mk_threads;
  long long budget = (long long)(p->scratch_mb > 0 ? p->scratch_mb : kDefaultScratchMiB) << 20;
  if (p->scratch_mb == 0)
    if (const char* e = getenv("SHIRLEY_SCRATCH_MB")) budget = std::max(1LL, atoll(e)) << 20;  // tuning
  SamplePlan plan = plan_samples(n_pix, count, engine, lanes, p->sample_chunk, budget);
  if (const char* e = getenv("SHIRLEY_SEGMENTS"))  // (tuning: per-block unit segments forced on / off)
    plan.segments = engine == RT_ENGINE_MEGAKERNEL && atoi(e) != 0;
  if (!plan.ok) return fail(c, RT_E_UNSUPPORTED, "frame too large (%lld pixels)", (long long)n_pix);
  // a device short of memory gets more, smaller passes instead of a failed call (the frame is the same
  // for any number of passes)
  // (SHIRLEY_SIMULATE_OOM_MB, tests only: a partial buffer above that many MiB fails like hipMalloc would)
  long long oom_limit = 0;
  if (const char* e = getenv("SHIRLEY_SIMULATE_OOM_MB")) oom_limit = atoll(e) << 20;
  auto alloc_partial = [&](size_t bytes) {
    if (oom_limit > 0 && (long long)bytes > oom_limit)
      return fail(c, RT_E_OOM, "simulated out-of-memory: %zu bytes of partial sums", bytes);
    return ensure(c, c->partial, bytes);
  };
  bool fell_back = false;
  const std::string err_before = c->err;
  while ((st = alloc_partial((size_t)plan.partial_bytes)) == RT_E_OOM && plan.per_pass > 1) {
    (void)hipGetLastError();
    fell_back = true;
    plan = plan_samples(n_pix, count, engine, lanes, p->sample_chunk, plan.partial_bytes / 2);
  }
  if (st) return st;
  if (fell_back) c->err = err_before;  // the call succeeds: the refused allocation leaves no message behind
  const int chunk = plan.chunk, n_chunks = plan.n_chunks, passes = plan.passes, per_pass = plan.per_pass;
  const size_t partial_bytes = (size_t)plan.partial_bytes;

  KParams kp{};
  kp.scene = c->scene;
  kp.scene.time0 = cam->time0;  // book-2 shutter (ray time side stream)
  kp.scene.time1 = cam->time1;
  kp.cam = device_camera(cam);
  kp.work.tiles_x = L.tiles_x;
  kp.work.tiles_y = L.tiles_y;
  kp.work.ty0 = ty0;
  kp.work.tile_rank = p->tile_rank;
  kp.work.tile_world = p->tile_world;
  kp.work.n_tiles_rank = L.n_tiles_rank;
  kp.work.chunk = chunk;
  kp.work.max_depth = p->max_depth;
  kp.work.seed = p->seed;
  kp.work.div_tiles_x = make_udiv((uint32_t)L.tiles_x);
  kp.partial = static_cast<double*>(c->partial.p);
  kp.counters = static_cast<DCounters*>(c->counters.p);

  // the megakernel's per-pass KBlock (KParams.kconst): device copies of the camera, the scene record, the
  // pass's work descriptor and the output / queue / statistics pointers; their host sources stay alive in
  // the ctx until the next call
  st = ensure(c, c->kcam, (size_t)passes * sizeof(KBlock));
  if (st) return st;
  // every kernel of the call reads the shutter from pass 0's device copy of the scene record
  kp.scene.shutter = &static_cast<KBlock*>(c->kcam.p)->scene.time0;
  c->host_blocks.assign(passes, KBlock{});
  const uint64_t nseg = (uint64_t)std::max(1, c->cu_count * std::max(1, c->blocks_per_cu));
  {
    const size_t bytes = std::max<size_t>(64, (size_t)nseg * sizeof(uint32_t));
    st = ensure(c, c->unit_counter, bytes);
    if (st) return st;
    kp.unit_counter = static_cast<unsigned long long*>(c->unit_counter.p);
  }
  if ((int)c->pass_ev.size() < 2 * passes) {
    const size_t have = c->pass_ev.size();
    c->pass_ev.resize(2 * passes, nullptr);
    for (size_t i = have; i < c->pass_ev.size(); ++i) HIP_TRY(c, hipEventCreate(&c->pass_ev[i]));
  }
  HIP_TRY(c, hipMemsetAsync(c->counters.p, 0, kCounterSlots * sizeof(DCounters), s));
  c->last_engine = engine;
  c->host_samples = 0;
  c->last_chunk = chunk;
  c->last_n_chunks = n_chunks;
  c->last_passes = 0;
  c->last_scratch = partial_bytes;
  c->last_iters = 0;
  c->last_slots = 0;
  c->last_timing = 0;
  for (double& x : c->lap_ms) x = 0.0;
  HIP_TRY(c, hipEventRecord(c->ev[0], s));
  const bool trace = n_pix > 0 && count > 0 && p->max_depth > 0;
  if (!trace) {
    // nothing to trace: ray_color's loop never runs with max_depth == 0 (render.rs:30: every sample is
    // black), or the range is empty.  The window is written by a reduce over no chunks (zeros); the
    // samples counter counts the window's in-image pixels of this rank's tiles, as the kernel would.
    uint64_t inside = 0;
    for (long long lt = 0; lt < L.n_tiles_rank; ++lt) {
      const long long gt = lt * p->tile_world + p->tile_rank;
      const int tx = (int)(gt % L.tiles_x), ty = ty0 + (int)(gt / L.tiles_x);
      const int w = std::min(kTile, cam->image_width - tx * kTile), h = std::min(kTile, cam->image_height - ty * kTile);
      if (w > 0 && h > 0) inside += (uint64_t)w * (uint64_t)h;
    }
    c->host_samples = inside * (uint64_t)count;
    HIP_TRY(c, hipEventRecord(c->ev[1], s));
    if (n_pix > 0)
      HIP_TRY(c, launch_reduce(kp.partial, 0, L.n_tiles_rank, L.tiles_x, ty0, p->tile_rank, p->tile_world,
                               cam->image_width, row0, row1, packed, 0, out_dev, s));
    HIP_TRY(c, hipEventRecord(c->ev[2], s));
    c->have_timing = true;
    return RT_OK;
  }
  for (int k = 0; k < passes; ++k) {
    const int c0 = k * per_pass, c1 = std::min(n_chunks, c0 + per_pass);
    DWork& w = kp.work;
    w.sample_base = R.begin + c0 * chunk;
    w.samples = (int)std::min<long long>(R.end, (long long)R.begin + (long long)c1 * chunk);
    w.n_chunks = c1 - c0;
    w.n_units = (uint64_t)n_pix * (uint64_t)w.n_chunks;
    w.div_unit_tile = make_udiv((uint32_t)w.n_chunks * (uint32_t)kTilePixels);
    // per-block unit segments (trace.hip; plan.h): one counter per megakernel block
    const uint64_t per = (w.n_units + nseg - 1) / nseg;
    w.n_segs = plan.segments ? (uint32_t)nseg : 0u;
    w.seg_len = (uint32_t)std::max<uint64_t>(kSegmentWindow, (per + kSegmentWindow - 1) / kSegmentWindow * kSegmentWindow);
    w.q_window = plan.queue_window;
    if (const char* e = getenv("SHIRLEY_WINDOW"))  // (tuning: the shared queue's window, units)
      w.q_window = (uint32_t)std::max(1, atoi(e) / kWave) * (uint32_t)kWave;
    // the device copy is taken after every field is set (the kernel may read any of them)
    KBlock& kb = c->host_blocks[k];
    kb.cam = kp.cam;
    kb.scene = kp.scene;
    kb.work = w;
    kb.partial = kp.partial;
    kb.unit_counter = kp.unit_counter;
    kb.counters = kp.counters;
    void* kdev = static_cast<KBlock*>(c->kcam.p) + k;
    HIP_TRY(c, hipMemcpyAsync(kdev, &kb, sizeof(KBlock), hipMemcpyHostToDevice, s));
    kp.kconst = (uint64_t)(uintptr_t)kdev;
    HIP_TRY(c, hipMemsetAsync(c->unit_counter.p, 0, std::max<size_t>(64, (size_t)nseg * sizeof(uint32_t)), s));
    HIP_TRY(c, hipEventRecord(c->pass_ev[2 * k], s));
    if (engine == RT_ENGINE_WAVEFRONT) {
      st = run_wavefront(c, kp, timing, s);
      if (st) return st;
    } else if (engine == RT_ENGINE_SPLIT) {
      kp.split_refill = c->split_refill;
      KParams ks = kp;  // (the split engine's LDS layout holds no material tables)
      ks.scene.n_lds_mats = ks.scene.n_lds_texs = 0;
      HIP_TRY(c, launch_split(ks, c->split_nt, c->cu_count, s));
    } else {
      HIP_TRY(c, launch_trace(kp, (int)nseg, c->mk_threads, s));
    }
    HIP_TRY(c, hipEventRecord(c->pass_ev[2 * k + 1], s));
    if (k == passes - 1) HIP_TRY(c, hipEventRecord(c->ev[1], s));
    HIP_TRY(c, launch_reduce(kp.partial, w.n_chunks, L.n_tiles_rank, L.tiles_x, ty0, p->tile_rank, p->tile_world,
                             cam->image_width, row0, row1, packed, k > 0 ? 1 : 0, out_dev, s));
    c->last_passes = k + 1;
  }
  HIP_TRY(c, hipEventRecord(c->ev[2], s));
  c->have_timing = true;
  return RT_OK;
}

}  // namespace

extern "C" {

const char* rt_version(void) { return "shirley-rt 0.2 (gfx950, f64 wavefront + persistent megakernel)"; }

int rt_device_count(int32_t* out) {
  if (!out) return RT_E_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *out = (e == hipSuccess) ? n : 0;
  return e == hipSuccess ? RT_OK : RT_E_HIP;
}

const char* rt_last_error(const rt_ctx* ctx) { return ctx ? ctx->err.c_str() : "NULL context"; }

int rt_create(int32_t device, rt_ctx** out) {
  if (!out) return RT_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return RT_E_HIP;
  if (device < 0 || device >= n) return RT_E_INVALID;
  rt_ctx* c = new rt_ctx();
  c->device = device;
  auto bail = [&](int code) {
    rt_destroy(c);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(RT_E_HIP);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail(RT_E_HIP);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return bail(RT_E_HIP);
  c->cu_count = prop.multiProcessorCount;
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return bail(RT_E_HIP);
  for (auto& e : c->wf_ev)
    if (hipEventCreate(&e) != hipSuccess) return bail(RT_E_HIP);
  if (hipHostMalloc((void**)&c->wf_host, 64, hipHostMallocDefault) != hipSuccess) return bail(RT_E_OOM);
  if (ensure(c, c->counters, kCounterSlots * sizeof(DCounters)) || ensure(c, c->unit_counter, 64)) return bail(RT_E_OOM);
  *out = c;
  return RT_OK;
}

int rt_destroy(rt_ctx* c) {
  if (!c) return RT_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&c->nodes, &c->nodes4, &c->prims, &c->mats, &c->texs, &c->perlin, &c->texels, &c->exts, &c->partial, &c->kcam, &c->shutter0,
                    &c->accum, &c->counters, &c->unit_counter, &c->wf_pool, &c->wf_iters, &c->packed, &c->gathered,
                    &c->parts, &c->band, &c->digests})
    release(*b);
  for (rt_comm& m : c->group_comms)
    if (m.comm) (void)rccl().CommDestroy(m.comm);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->wf_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->lap_ev) (void)hipEventDestroy(e);
  if (c->wf_host) (void)hipHostFree(c->wf_host);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return RT_OK;
}

int rt_scene_upload(rt_ctx* c, const rt_scene_desc* d, int32_t builder) {
  if (!c) return RT_E_INVALID;
  int st = validate(c, d);
  if (st) return st;
  const int32_t placement_mask = RT_BVH_NODES_GLOBAL | RT_BVH_NODES_HALF_LDS | RT_BVH_NODES_LDS;
  const int32_t placement = builder & placement_mask;
  builder &= ~placement_mask;
  if (builder != RT_BVH_REFERENCE && builder != RT_BVH_SAH) return fail(c, RT_E_INVALID, "bad bvh builder %d", builder);
  if (d->n_objects > kLeafPrimMask) return fail(c, RT_E_UNSUPPORTED, "too many objects (%d)", d->n_objects);
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->have_scene = false;
  const uint64_t digest = scene_digest(d, builder);  // (of the description as given)
  std::vector<rt_object> flat;
  const rt_scene_desc fd = flat_scene(d, flat);
  c->uv_fixups.clear();
  for (int i = 0; i < d->n_objects; ++i)
    if (d->objects[i].rotate_y_deg != 0.0 && flattens(d, d->objects[i])) {
      double cs, sn;
      rotate_y_cs(d->objects[i], cs, sn);
      c->uv_fixups.push_back({i, {cs, sn}});
    }
  d = &fd;

  BuiltTree tree = build_tree(d, builder);
  // Exact ties (rt_device.h tie_takes): the device numbers the primitives in the reference
  // tree's leaf order, lhs before rhs (constructor.rs:9-36 via build_reference_tree), so that the lower
  // number is the leaf the reference's rhs-first walk tests last; prim_object maps a number back.
  std::vector<rt_object> ranked;
  rt_scene_desc rd = *d;
  {
    const BuiltTree ref = builder == RT_BVH_REFERENCE ? tree : build_tree(d, RT_BVH_REFERENCE);
    std::vector<int32_t> rank = reference_ranks(ref, d->n_objects);
    ranked.resize((size_t)std::max(0, d->n_objects));
    c->prim_object.assign((size_t)std::max(0, d->n_objects), 0);
    for (int i = 0; i < d->n_objects; ++i) {
      ranked[rank[i]] = d->objects[i];
      c->prim_object[rank[i]] = i;
    }
    for (BuildNode& nd : tree.nodes)
      if (nd.leaf >= 0) nd.leaf = rank[nd.leaf];
    rd.objects = ranked.data();
    d = &rd;
  }
  std::vector<DNode> nodes;
  flatten(tree, nodes);
  std::vector<DNode4F> nodes4;
  int32_t stack4 = 1;
  const Inflation infl = inflation_for(tree);
  flatten4(tree, d, infl.delta, nodes4, stack4, false);
  std::vector<DPrim> prims(std::max(1, d->n_objects));
  std::vector<DExt> exts;
  for (int i = 0; i < d->n_objects; ++i) {
    const rt_object& o = d->objects[i];
    DPrim& q = prims[i];
    std::memset(&q, 0, sizeof q);
    for (int k = 0; k < 6; ++k) q.p[k] = o.p[k];
    q.kind = o.geometry == RT_GEOM_SPHERE     ? kPrimSphere
             : o.geometry == RT_GEOM_RECT_XY  ? kPrimRectXY
             : o.geometry == RT_GEOM_RECT_YZ  ? kPrimRectYZ
             : o.geometry == RT_GEOM_RECT_XZ  ? kPrimRectXZ
             : o.geometry == RT_GEOM_RECT_BOX ? kPrimBox
                                              : kPrimMovingSphere;
    // a sphere's 1 / radius (sphere.rs:48 `scale(1.0 / self.radius)`), the same IEEE quotient the device
    // would compute per hit record; p[4] is otherwise unused by spheres
    if (q.kind == kPrimSphere || q.kind == kPrimMovingSphere) q.p[4] = 1.0 / q.p[3];
    if (q.kind == kPrimSphere) {
      // the sure-pass bound of the sphere's box test (rt_device.h leaf_tests4): r - eta rounded down, eta =
      // 2^-48 (B + L) (B the largest box plane, L the fast-ray origin bound), or 0 (never sure)
      const double eta = std::ldexp(infl.box_bound + (double)infl.origin_limit, -48);
      const double rs = q.p[3] - eta;
      q.p[5] = (std::isfinite(rs) && rs > 0.0) ? std::nextafter(rs, 0.0) : 0.0;
    }
    q.material = o.material;
    if (is_extended(o)) {
      if (exts.size() >= (1u << (31 - kPrimExtShift)))
        return fail(c, RT_E_UNSUPPORTED, "too many extended objects");
      DExt e{};
      box_to6(object_box(o), e.box);
      for (int k = 0; k < 3; ++k) e.c1[k] = o.q[k];
      e.t0 = o.q[3];
      e.t1 = o.q[4];
      e.cos_t = 1.0;
      if (o.transform) {
        rotate_y_cs(o, e.cos_t, e.sin_t);
        for (int k = 0; k < 3; ++k) e.off[k] = o.offset[k];
      }
      e.neg_inv_density = -1.0 / o.density;
      e.object = c->prim_object[i];
      e.prim = i;
      q.kind |= kPrimExt | (o.medium ? kPrimMedium : 0) | (o.transform ? kPrimXform : 0) |
                ((int32_t)exts.size() << kPrimExtShift);
      exts.push_back(e);
    }
  }
  std::vector<DMat> mats(std::max(1, d->n_materials));
  for (int i = 0; i < d->n_materials; ++i) {
    const rt_material& m = d->materials[i];
    DMat& q = mats[i];
    std::memset(&q, 0, sizeof q);
    q.kind = m.kind;
    q.tex = m.texture;
    for (int k = 0; k < 3; ++k) q.albedo[k] = m.albedo[k];
    q.param = m.param;
    q.inv_param = 1.0 / m.param;  // IEEE division: the bits dielectric.rs:27 computes per hit
    if (m.kind == RT_MAT_DIELECTRIC) {
      // Schlick's r0^2 (dielectric.rs:15-19) for the two ratios a hit can have — front face 1 / ir, back face
      // ir — with the reference's operations (host and device are both IEEE binary64 without contraction), so
      // the megakernel's reflectance skips a division per hit; a dielectric has no albedo (its attenuation is 1)
      const double ratios[2] = {q.inv_param, m.param};
      for (int k = 0; k < 2; ++k) {
        double r0 = (1.0 - ratios[k]) / (1.0 + ratios[k]);
        q.albedo[k] = r0 * r0;
      }
      q.albedo[2] = 0.0;
    }
  }
  std::vector<DTex> texs(std::max(1, d->n_textures));
  for (int i = 0; i < d->n_textures; ++i) {
    const rt_texture& t = d->textures[i];
    DTex& q = texs[i];
    std::memset(&q, 0, sizeof q);
    q.kind = t.kind;
    q.odd = t.odd;
    q.even = t.even;
    q.table = t.table;
    if (t.kind != RT_TEX_IMAGE)
      for (int k = 0; k < 3; ++k) q.color[k] = t.color[k];
    q.scale = t.scale;
  }
  std::vector<DPerlin> perl(std::max(1, d->n_perlin));
  for (int i = 0; i < d->n_perlin; ++i) {
    std::memcpy(perl[i].ranfloat, d->perlin[i].ranfloat, sizeof perl[i].ranfloat);
    std::memcpy(perl[i].perm_x, d->perlin[i].perm_x, sizeof perl[i].perm_x);
    std::memcpy(perl[i].perm_y, d->perlin[i].perm_y, sizeof perl[i].perm_y);
    std::memcpy(perl[i].perm_z, d->perlin[i].perm_z, sizeof perl[i].perm_z);
  }
  // every image's RGB8 texels in one pool; an image texture's DTex points at its image (below, once the
  // pool is on the device)
  std::vector<size_t> img_off(std::max(1, d->n_images));
  std::vector<uint8_t> texels;
  for (int i = 0; i < d->n_images; ++i) {
    img_off[i] = texels.size();
    size_t nb = (size_t)d->images[i].width * d->images[i].height * 3;
    texels.insert(texels.end(), d->images[i].rgb, d->images[i].rgb + nb);
  }
  if (texels.empty()) texels.resize(16);

  // The 4-wide collapse: the optimal one (fewest expected node visits by area) for a reference scene that
  // will run in the scene-in-LDS instance — Cornell +15 %, headline +0.3 % — and the greedy one for the
  // scenes read through L1/L2 (gen_spheres −1.4 %, final_scene −1.6 % with the optimal one).
  // The same test as the placement below (tree, stacks, primitives and tables within the wide block's
  // LDS), on either tree.  SHIRLEY_COLLAPSE_DP=1 / =0: always / never (tuning).
  {
    const size_t mt = mats.size() * sizeof(DMat) + texs.size() * sizeof(DTex);
    auto scene_in_lds = [&](const std::vector<DNode4F>& n4, int32_t s4) {
      return (long long)s4 * kTraceThreadsWide * kStack4EntryBytes + (long long)n4.size() * (long long)sizeof(DNode4F) +
                 (long long)d->n_objects * (long long)sizeof(DPrim) + (long long)mt <=
             kLdsBytes;
    };
    const char* e = getenv("SHIRLEY_COLLAPSE_DP");
    const bool want = e ? atoi(e) != 0
                        : (exts.empty() && (placement == 0 || placement == RT_BVH_NODES_LDS) && scene_in_lds(nodes4, stack4));
    if (want) {
      std::vector<DNode4F> dp4;
      int32_t dp_stack = 1;
      flatten4(tree, d, infl.delta, dp4, dp_stack, true);
      if (e || scene_in_lds(dp4, dp_stack)) {
        nodes4.swap(dp4);
        stack4 = dp_stack;
      }
    }
  }
  if ((st = upload(c, c->nodes, nodes.data(), nodes.size() * sizeof(DNode)))) return st;
  // book-2 scenes run the EXT kernel instances, which read the compact node layout (rt_layout.h)
  const int n4_bytes = node4_bytes(!exts.empty());
  if (exts.empty()) {
    if ((st = upload(c, c->nodes4, nodes4.data(), nodes4.size() * sizeof(DNode4F)))) return st;
  } else {
    std::vector<DNode4C> compact(nodes4.size());
    for (size_t i = 0; i < nodes4.size(); ++i) {
      for (int a = 0; a < 3; ++a)
        for (int k = 0; k < 4; ++k) {
          compact[i].lo[a][k] = nodes4[i].row[a][0][k];
          compact[i].hi[a][k] = nodes4[i].row[a][1][k];
        }
      for (int k = 0; k < 4; ++k) compact[i].child[k] = nodes4[i].child[k];
    }
    if ((st = upload(c, c->nodes4, compact.data(), compact.size() * sizeof(DNode4C)))) return st;
  }
  if ((st = upload(c, c->prims, prims.data(), prims.size() * sizeof(DPrim)))) return st;
  if ((st = upload(c, c->mats, mats.data(), mats.size() * sizeof(DMat)))) return st;
  if ((st = upload(c, c->texels, texels.data(), texels.size()))) return st;
  for (int i = 0; i < d->n_textures; ++i)
    if (d->textures[i].kind == RT_TEX_IMAGE) {
      const int im = d->textures[i].table;  // (validated: a texture's image index is in range)
      texs[i].img.texels = static_cast<const uint8_t*>(c->texels.p) + img_off[im];
      texs[i].img.width = d->images[im].width;
      texs[i].img.height = d->images[im].height;
    }
  if ((st = upload(c, c->texs, texs.data(), texs.size() * sizeof(DTex)))) return st;
  if ((st = upload(c, c->perlin, perl.data(), perl.size() * sizeof(DPerlin)))) return st;
  if (!exts.empty()) {
    if ((st = upload(c, c->exts, exts.data(), exts.size() * sizeof(DExt)))) return st;
  } else {
    release(c->exts);
  }

  DScene& S = c->scene;
  S.nodes = static_cast<const DNode*>(c->nodes.p);
  S.nodes4 = c->nodes4.p;
  S.n_nodes4 = (int32_t)nodes4.size();
  S.stack_depth4 = stack4;
  S.root4 = (nodes4[0].child[0] >= 0 && nodes4[0].child[0] != kEmptyChild) ? nodes4[0].child[0] : 0;
  {
    int kbits = 1;
    while ((size_t)1 << kbits < nodes4.size()) ++kbits;
    if (kbits > kMaxKeyBits) return fail(c, RT_E_UNSUPPORTED, "BVH too large (%zu 4-wide nodes)", nodes4.size());
    S.key_mask = (1u << kbits) - 1u;
  }
  S.origin_limit = infl.origin_limit;
  S.prims = static_cast<const DPrim*>(c->prims.p);
  S.mats = static_cast<const DMat*>(c->mats.p);
  S.texs = static_cast<const DTex*>(c->texs.p);
  S.perlin = static_cast<const DPerlin*>(c->perlin.p);
  S.exts = exts.empty() ? nullptr : static_cast<const DExt*>(c->exts.p);
  S.time0 = S.time1 = 0.0;  // the shutter comes with each render call's camera
  if ((st = ensure(c, c->shutter0, 2 * sizeof(double)))) return st;
  HIP_TRY(c, hipMemset(c->shutter0.p, 0, 2 * sizeof(double)));
  S.shutter = static_cast<const double*>(c->shutter0.p);
  S.n_nodes = (int32_t)nodes.size();
  S.n_prims = d->n_objects;
  int32_t depth = tree_branch_depth(tree);
  S.stack_depth = depth + 2;  // ordered traversal holds at most one deferred child per branch level
  S.sky = d->sky;
  for (int k = 0; k < 3; ++k) S.sky_color[k] = d->sky_color[k];
  // LDS of one block: the traversal stacks, then a copy of (the top levels of) the BVH.
  // Megakernel (4-wide tree): the whole tree in LDS with one kTraceThreadsWide block per CU when it
  // fits beside the stacks (MI355X: 160 KiB per CU), else kTraceThreads blocks reading nodes
  // through L1/L2.  rt_scene_hit (2-wide tree): placement flags only.
  auto lds_count = [&](long long stack, size_t node_bytes, size_t n) -> int32_t {
    long long room = std::min<long long>((kLdsBytes - stack) / (long long)node_bytes, (long long)n);
    if (placement & RT_BVH_NODES_LDS) return (int32_t)room;
    if (placement & RT_BVH_NODES_HALF_LDS) return (int32_t)std::min<long long>(room, (long long)n / 2);
    if (const char* e = getenv("SHIRLEY_LDS_NODES")) return (int32_t)std::min<long long>(room, atoll(e));  // tuning
    return 0;  // nodes read through L1/L2
  };
  auto lds_nodes_for = [&](long long stack) { return lds_count(stack, sizeof(DNode), nodes.size()); };
  const long long stack_bytes = (long long)S.stack_depth * kTraceThreads * 8;
  const long long stack4_bytes = (long long)S.stack_depth4 * kTraceThreads * kStack4EntryBytes;
  // book-2 scenes: the EXT instance spills ~80 VGPRs at 4 waves per SIMD (1024 threads) and none at 3
  // (768 threads, 165 VGPRs): final_scene +3.3 % (profiles/r02/wide3.txt), so no 1024-thread EXT instance
  // is built.  The wide block's LDS holds the tree plus one stack per thread of the block actually launched.
  const int wide_threads = !exts.empty() ? kTraceThreadsWide3 : kTraceThreadsWide;
  const long long wide_bytes =
      (long long)S.stack_depth4 * wide_threads * kStack4EntryBytes + (long long)nodes4.size() * n4_bytes;
  if (stack_bytes > kLdsBytes || stack4_bytes > kLdsBytes)
    return fail(c, RT_E_UNSUPPORTED, "BVH too deep for the LDS traversal stack (depth %d)", depth);
  const bool wide = wide_bytes <= kLdsBytes && (placement == 0 || placement == RT_BVH_NODES_LDS) &&
                    !getenv("SHIRLEY_NO_WIDE");  // tuning
  c->mk_threads = wide ? wide_threads : kTraceThreads;
  S.n_lds_nodes = lds_nodes_for(kHitThreads * 8LL * S.stack_depth);
  S.n_lds_nodes4 = wide ? (int32_t)nodes4.size() : lds_count(stack4_bytes, n4_bytes, nodes4.size());
  // primitives too, with the material and texture tables (the megakernel's scene-in-LDS instance reads all
  // three from LDS), when they fit beside the wide block's tree and stacks
  const long long mt_bytes = (long long)mats.size() * (long long)sizeof(DMat) + (long long)texs.size() * (long long)sizeof(DTex);
  const bool prims_lds = wide && wide_bytes + (long long)d->n_objects * (long long)sizeof(DPrim) + mt_bytes <= kLdsBytes &&
                         !getenv("SHIRLEY_NO_LDS_PRIMS") && !getenv("SHIRLEY_NO_LDS_MATS");
  S.n_lds_prims = prims_lds ? d->n_objects : 0;
  // and the Perlin tables (marble's ~210 gathers per evaluation from LDS)
  const bool perlin_lds = prims_lds && d->n_perlin > 0 &&
                          wide_bytes + (long long)d->n_objects * (long long)sizeof(DPrim) + mt_bytes +
                                  (long long)d->n_perlin * (long long)sizeof(DPerlin) <= kLdsBytes &&
                          !getenv("SHIRLEY_NO_LDS_PERLIN");
  S.n_lds_perlin = perlin_lds ? d->n_perlin : 0;
  // the material and texture tables ride with the primitives (the record / shading reads: headline +1.0 %,
  // Cornell +0.7 %; SHIRLEY_NO_LDS_MATS keeps all three in global memory).  The wavefront and
  // split engines keep their own LDS layouts and read them from global memory (their scene copies carry
  // n_lds_mats = 0).
  S.n_lds_mats = prims_lds ? (int32_t)mats.size() : 0;
  S.n_lds_texs = prims_lds ? (int32_t)texs.size() : 0;

  int bpc = 0;
  HIP_TRY(c, trace_occupancy(S, c->mk_threads, &bpc));
  if (bpc < 1) return fail(c, RT_E_UNSUPPORTED, "trace kernel does not fit on a CU (LDS %lld B)", stack_bytes);
  c->blocks_per_cu = bpc;

  // wavefront extend block: its own (larger) stack area, the rest of LDS for nodes
  DScene W = S;
  W.n_lds_mats = W.n_lds_texs = 0;
  long long wf_stack = (long long)S.stack_depth * wf_extend_threads() * 8;
  if (wf_stack > kLdsBytes)
    return fail(c, RT_E_UNSUPPORTED, "BVH too deep for the LDS traversal stack (depth %d)", depth);
  W.n_lds_nodes = lds_nodes_for(wf_stack);
  int wbpc = 0;
  HIP_TRY(c, wf_prepare(W, &wbpc));
  if (wbpc < 1) return fail(c, RT_E_UNSUPPORTED, "wavefront extend kernel does not fit on a CU");
  c->wf_scene = W;
  c->wf_wide = false;
  if (c->mk_threads >= kTraceThreadsWide3 && S.n_lds_prims > 0 && !getenv("SHIRLEY_WF_EXTEND2")) {
    int b4 = 0;
    HIP_TRY(c, wf_prepare4(S, &b4));
    if (b4 >= 1) {
      c->wf_wide = true;
      c->wf4_blocks_per_cu = b4;
      c->wf_scene = S;  // wf_extend4 reads the megakernel's LDS layout (without the material tables)
      c->wf_scene.n_lds_mats = c->wf_scene.n_lds_texs = 0;
    }
  }
  c->n_perlin = d->n_perlin;
  c->has_perlin = false;
  for (int i = 0; i < d->n_textures; ++i) c->has_perlin |= d->textures[i].kind == RT_TEX_PERLIN;
  c->wf_blocks_per_cu = wbpc;
  // RT_ENGINE_SPLIT: the wide block's scene plus traversal stacks and ray slots in LDS
  c->split_nt = 0;
  if (c->mk_threads == kTraceThreadsWide && S.n_lds_prims == d->n_objects && !S.exts) {
    int nt = 8;
    if (const char* e = getenv("SHIRLEY_SPLIT_NT")) nt = atoi(e);  // tuning
    if (const char* e = getenv("SHIRLEY_SPLIT_REFILL")) c->split_refill = std::max(1, atoi(e));  // tuning
    int sb = 0;
    if (split_supported_nt(nt)) HIP_TRY(c, split_prepare(S, nt, &sb));
    if (sb >= 1) c->split_nt = nt;
  }

  c->stats.n_objects = d->n_objects;
  c->stats.n_nodes = (int32_t)tree.nodes.size();
  int32_t leaves = 0;
  for (const auto& n : tree.nodes) leaves += n.leaf >= 0;
  c->stats.n_leaves = leaves;
  c->stats.depth = depth;
  c->stats.n_nodes4 = S.n_nodes4;
  c->stats.wide_block = c->mk_threads >= kTraceThreadsWide3 ? 1 : 0;
  c->stats.origin_limit = S.origin_limit;
  c->stats.device_bytes = (int64_t)(nodes.size() * sizeof(DNode) + prims.size() * sizeof(DPrim) +
                                    mats.size() * sizeof(DMat) + texs.size() * sizeof(DTex) +
                                    perl.size() * sizeof(DPerlin) + texels.size());
  c->digest = digest;
  c->have_scene = true;
  return RT_OK;
}

int rt_scene_digest(rt_ctx* c, uint64_t* out) {
  if (!c || !out) return RT_E_INVALID;
  if (!c->have_scene) return fail(c, RT_E_INVALID, "no scene uploaded");
  *out = c->digest;
  return RT_OK;
}

int rt_scene_digest_host(const rt_scene_desc* d, int32_t builder, uint64_t* out) {
  if (!d || !out) return RT_E_INVALID;
  if (validate(nullptr, d)) return RT_E_INVALID;
  const int32_t placement_mask = RT_BVH_NODES_GLOBAL | RT_BVH_NODES_HALF_LDS | RT_BVH_NODES_LDS;
  *out = scene_digest(d, builder & ~placement_mask);
  return RT_OK;
}

int rt_scene_stats_get(rt_ctx* c, rt_scene_stats* out) {
  if (!c || !out) return RT_E_INVALID;
  if (!c->have_scene) return fail(c, RT_E_INVALID, "no scene uploaded");
  *out = c->stats;
  return RT_OK;
}

int rt_tile_layout(const rt_camera* cam, int32_t world, int32_t* n_tiles_total, int32_t* max_tiles_per_rank) {
  if (!cam || world < 1 || cam->image_width < 1 || cam->image_height < 1) return RT_E_INVALID;
  int tiles_y = (cam->image_height + kTile - 1) / kTile;
  Layout L = layout(cam, 0, tiles_y, 0, world);
  if (n_tiles_total) *n_tiles_total = L.n_tiles;
  if (max_tiles_per_rank) *max_tiles_per_rank = (L.n_tiles + world - 1) / world;
  return RT_OK;
}

int rt_render_device(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, double* accum_dev, void* stream) {
  if (!accum_dev) return fail(c, RT_E_INVALID, "accum_dev is NULL");
  hipStream_t s;
  resolve_stream(c, stream, &s);
  int tiles_y = cam ? (cam->image_height + kTile - 1) / kTile : 0;
  SampleRange R;
  if (p && resolve_range(c, p, &R)) return RT_E_INVALID;
  return render_window(c, cam, p, R, 0, tiles_y, 0, cam ? cam->image_height : 0, 0, accum_dev, s);
}

int rt_render_tiles_device(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, double* packed_dev,
                           void* stream) {
  if (!packed_dev) return fail(c, RT_E_INVALID, "packed_dev is NULL");
  hipStream_t s;
  resolve_stream(c, stream, &s);
  int tiles_y = cam ? (cam->image_height + kTile - 1) / kTile : 0;
  SampleRange R;
  if (p && resolve_range(c, p, &R)) return RT_E_INVALID;
  return render_window(c, cam, p, R, 0, tiles_y, 0, cam ? cam->image_height : 0, 1, packed_dev, s);
}

int rt_unpack_tiles_device(rt_ctx* c, const rt_camera* cam, int32_t world, const double* gathered_dev,
                           double* accum_dev, void* stream) {
  if (!c || !cam || !gathered_dev || !accum_dev || world < 1) return fail(c, RT_E_INVALID, "bad unpack args");
  hipStream_t s;
  resolve_stream(c, stream, &s);
  int32_t n_total = 0, max_tiles = 0;
  rt_tile_layout(cam, world, &n_total, &max_tiles);
  int tiles_x = (cam->image_width + kTile - 1) / kTile;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, launch_unpack(gathered_dev, world, max_tiles, n_total, tiles_x, cam->image_width, cam->image_height,
                           accum_dev, s));
  return RT_OK;
}

int rt_render(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, double* accum_host) {
  if (!c) return RT_E_INVALID;
  if (!accum_host || !cam) return fail(c, RT_E_INVALID, "NULL argument");
  return rt_render_scanlines(c, cam, p, 0, cam->image_height, accum_host);
}

int rt_render_scanlines(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, int32_t line_begin,
                        int32_t line_end, double* rows_host) {
  if (!c) return RT_E_INVALID;
  if (!cam || !rows_host) return fail(c, RT_E_INVALID, "NULL argument");
  if (line_begin < 0 || line_end > cam->image_height || line_begin > line_end)
    return fail(c, RT_E_INVALID, "bad line range [%d, %d)", line_begin, line_end);
  if (line_begin == line_end) return RT_OK;
  if (p && p->tile_world != 1) return fail(c, RT_E_INVALID, "host-buffer render needs tile_world == 1");
  size_t bytes = (size_t)(line_end - line_begin) * cam->image_width * 3 * sizeof(double);
  int st = ensure(c, c->accum, bytes);
  if (st) return st;
  int ty0 = line_begin / kTile, ty1 = (line_end + kTile - 1) / kTile;
  SampleRange R;
  if (p && resolve_range(c, p, &R)) return RT_E_INVALID;
  st = render_window(c, cam, p, R, ty0, ty1, line_begin, line_end, 0, static_cast<double*>(c->accum.p), c->stream);
  if (st) return st;
  HIP_TRY(c, hipMemcpyAsync(rows_host, c->accum.p, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return RT_OK;
}

int rt_scene_hit(rt_ctx* c, const double* rays, int32_t n, double t_min, double t_max, rt_hit* out) {
  return rt_scene_hit_ex(c, rays, n, t_min, t_max, RT_TRAVERSAL_BINARY, out);
}

int rt_scene_hit_ex(rt_ctx* c, const double* rays, int32_t n, double t_min, double t_max, int32_t traversal,
                    rt_hit* out) {
  if (!c) return RT_E_INVALID;
  if (!c->have_scene) return fail(c, RT_E_INVALID, "no scene uploaded");
  if (n < 0 || (n > 0 && (!rays || !out))) return fail(c, RT_E_INVALID, "bad ray batch");
  if (traversal != RT_TRAVERSAL_BINARY && traversal != RT_TRAVERSAL_RENDER)
    return fail(c, RT_E_INVALID, "bad traversal %d", traversal);
  if (n == 0) return RT_OK;
  static_assert(sizeof(rt_hit) == 80, "rt_hit layout");
  HIP_TRY(c, hipSetDevice(c->device));
  DevBuf r, h;
  int st = upload(c, r, rays, (size_t)n * 6 * sizeof(double));
  if (!st) st = ensure(c, h, (size_t)n * sizeof(rt_hit));
  if (!st) {
    const double* rd = static_cast<const double*>(r.p);
    hipError_t e = traversal == RT_TRAVERSAL_RENDER
                       ? launch_hit4(c->scene, c->mk_threads >= kTraceThreadsWide3, rd, n, t_min, t_max, h.p, c->stream)
                       : launch_hit(c->scene, rd, n, t_min, t_max, h.p, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, h.p, (size_t)n * sizeof(rt_hit), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) st = fail(c, RT_E_HIP, "rt_scene_hit: %s", hipGetErrorString(e));
  }
  if (!st)
    for (int32_t i = 0; i < n; ++i)
      if (out[i].object >= 0) out[i].object = c->prim_object[out[i].object];
  if (!st && !c->uv_fixups.empty())  // (sorted by object index)
    for (int32_t i = 0; i < n; ++i) {
      auto it = std::lower_bound(c->uv_fixups.begin(), c->uv_fixups.end(), out[i].object,
                                 [](const auto& f, int32_t o) { return f.first < o; });
      if (it != c->uv_fixups.end() && it->first == out[i].object) instance_sphere_uv(it->second.first, it->second.second, out[i]);
    }
  release(r);
  release(h);
  return st;
}

int rt_probe_segment(rt_ctx* c, const double* rays, int32_t n, uint64_t seed, uint32_t sample, uint32_t draw,
                     rt_probe* out) {
  if (!c) return RT_E_INVALID;
  if (!c->have_scene) return fail(c, RT_E_INVALID, "no scene uploaded");
  if (n < 0 || (n > 0 && (!rays || !out))) return fail(c, RT_E_INVALID, "bad ray batch");
  if (n == 0) return RT_OK;
  static_assert(sizeof(rt_probe) == 176, "rt_probe layout (trace.hip ProbeOut)");
  HIP_TRY(c, hipSetDevice(c->device));
  DevBuf r, h;
  int st = upload(c, r, rays, (size_t)n * 6 * sizeof(double));
  if (!st) st = ensure(c, h, (size_t)n * sizeof(rt_probe));
  if (!st) {
    DScene S = c->scene;
    S.time0 = S.time1 = 0.0;  // (book-2 ray time 0, like the oracle's or_probe_segment)
    hipError_t e = launch_probe(S, c->mk_threads >= kTraceThreadsWide3, static_cast<const double*>(r.p), n, seed,
                                sample, draw, h.p, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, h.p, (size_t)n * sizeof(rt_probe), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) st = fail(c, RT_E_HIP, "rt_probe_segment: %s", hipGetErrorString(e));
  }
  if (!st)
    for (int32_t i = 0; i < n; ++i)
      if (out[i].object >= 0) out[i].object = c->prim_object[out[i].object];
  release(r);
  release(h);
  return st;
}

int rt_synchronize(rt_ctx* c) {
  if (!c) return RT_E_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipDeviceSynchronize());
  return RT_OK;
}

int rt_counters_get(rt_ctx* c, rt_counters* out) {
  if (!c || !out) return RT_E_INVALID;
  std::memset(out, 0, sizeof *out);
  if (!c->have_timing) return fail(c, RT_E_INVALID, "no render has run on this context");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipEventSynchronize(c->ev[2]));
  std::vector<DCounters> dc(kCounterSlots);
  HIP_TRY(c, hipMemcpy(dc.data(), c->counters.p, kCounterSlots * sizeof(DCounters), hipMemcpyDeviceToHost));
  out->samples = c->host_samples;
  for (const DCounters& k : dc) {
    out->samples += k.samples;
    out->segments += k.segments;
    out->node_visits += k.node_visits;
    out->prim_tests += k.prim_tests;
  }
#ifdef RT_PHASE_TIMING
  {
    double ph[kPhBuckets] = {};
    for (const DCounters& k : dc)
      for (int i = 0; i < kPhBuckets; ++i) ph[i] += (double)k.pad[i];
    const int order[] = {kPhTrav, kPhRecord, kPhRegen, kPhMarble, kPhDraws, kPhCamera, kPhShade, kPhTail};
    const char* names[] = {"trav", "record", "regen", "marble", "draws", "camera", "shade", "tail"};
    double tot = 0;
    for (int b : order) tot += ph[b];
    fprintf(stderr, "[phase] wave-time fractions:");
    for (int i = 0; i < 8; ++i) fprintf(stderr, " %s %.4f", names[i], ph[order[i]] / tot);
    fprintf(stderr, " (wave-cycles %.4g)\n", tot);
    const double lane = ph[kPhLaneSteps], wave = ph[kPhWaveSteps];
    fprintf(stderr, "[phase] traversal lane steps %.4g, wave steps %.4g, SIMD utilisation %.3f\n", lane, wave,
            lane / (64.0 * wave));
    phase_counters_dump();
  }
#endif
#ifdef RT_TIMELINE
  timeline_dump();
#endif
  // kernel_ms: the trace launches of the call (one per sample pass); reduce_ms: the rest of the call's
  // device time (the reduces)
  float all = 0.f;
  HIP_TRY(c, hipEventElapsedTime(&all, c->ev[0], c->ev[2]));
  double trace = 0.0;
  for (int k = 0; k < c->last_passes; ++k) {
    float t = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&t, c->pass_ev[2 * k], c->pass_ev[2 * k + 1]));
    trace += t;
  }
  out->kernel_ms = trace;
  out->reduce_ms = std::max(0.0, (double)all - trace);
  out->passes = c->last_passes;
  out->trace_launches = c->last_passes;
  out->scratch_bytes = c->last_scratch;
  out->engine = c->last_engine;
  out->sample_chunk = c->last_chunk;
  out->n_chunks = c->last_n_chunks;
  out->iterations = c->last_iters;
  out->slots = c->last_slots;
  if (c->last_timing) {
    out->extend_ms = c->lap_ms[0];
    out->shade_ms = c->lap_ms[1];
    out->texture_ms = c->lap_ms[2];
  }
  return RT_OK;
}

int rt_bvh_build_host(const rt_scene_desc* d, int32_t builder, int32_t* n_nodes, rt_bvh_node* nodes, int32_t* root) {
  if (!d || !n_nodes) return RT_E_INVALID;
  if (validate(nullptr, d)) return RT_E_INVALID;
  std::vector<rt_object> flat;
  const rt_scene_desc fd = flat_scene(d, flat);
  BuiltTree t = build_tree(&fd, builder);
  if (nodes) {
    if (*n_nodes < (int32_t)t.nodes.size()) return RT_E_INVALID;
    for (size_t i = 0; i < t.nodes.size(); ++i) {
      box_to6(t.nodes[i].box, nodes[i].box);
      nodes[i].leaf = t.nodes[i].leaf;
      nodes[i].lhs = t.nodes[i].lhs;
      nodes[i].rhs = t.nodes[i].rhs;
      nodes[i].pad = 0;
    }
  }
  *n_nodes = (int32_t)t.nodes.size();
  if (root) *root = t.root;
  return RT_OK;
}

int rt_tonemap(const double* accum, int32_t width, int32_t height, int32_t samples, uint8_t* rgb8) {
  if (!accum || !rgb8 || width < 1 || height < 1) return RT_E_INVALID;
  const double inv = 1.0 / (double)(samples == 0 ? 1 : samples);
  for (int32_t j = 0; j < height; ++j)
    for (int32_t i = 0; i < width; ++i) {
      const double* c = accum + ((size_t)j * width + i) * 3;
      uint8_t* o = rgb8 + ((size_t)(height - j - 1) * width + i) * 3;
      for (int k = 0; k < 3; ++k) {
        double y = std::sqrt(c[k] * inv) * 255.999;  // (x * COLOR_SCALE) as u8, color.rs:31-38
        o[k] = (std::isnan(y) || y <= 0.0) ? 0 : (y >= 255.0 ? 255 : (uint8_t)y);
      }
    }
  return RT_OK;
}

int rt_tonemap_device(rt_ctx* c, const double* accum_dev, int32_t width, int32_t height, int32_t samples,
                      uint8_t* rgb8_dev, void* stream) {
  if (!c || !accum_dev || !rgb8_dev || width < 1 || height < 1) return RT_E_INVALID;
  hipStream_t s;
  resolve_stream(c, stream, &s);
  HIP_TRY(c, hipSetDevice(c->device));
  const double inv = 1.0 / (double)(samples == 0 ? 1 : samples);
  HIP_TRY(c, launch_tonemap(accum_dev, width, height, inv, rgb8_dev, s));
  return RT_OK;
}


// ---- multi-GPU ---------------------------------------------------------------------------------
}  // extern "C"

namespace {

#define RCCL_TRY(ctx, expr)                                                                       \
  do {                                                                                            \
    ncclResult_t r_ = (expr);                                                                     \
    if (r_ != ncclSuccess) return fail(ctx, RT_E_RCCL, "%s: %s (%s:%d)", #expr, rccl().GetErrorString(r_), \
                                       __FILE__, __LINE__);                                       \
  } while (0)

int need_rccl(rt_ctx* c) {
  if (!rccl().ok()) return fail(c, RT_E_RCCL, "%s", rccl().error.c_str());
  return RT_OK;
}

// Partition of a multi-GPU frame (rt_render_params.partition): RT_PARTITION_AUTO picks the measured
// default; SHIRLEY_PARTITION=tiles|samples overrides it (tuning).
int frame_partition(rt_ctx* c, const rt_render_params* p, int world, int* out) {
  int part = p->partition;
  if (part < RT_PARTITION_AUTO || part > RT_PARTITION_SAMPLES) return fail(c, RT_E_INVALID, "bad partition %d", part);
  if (part == RT_PARTITION_AUTO) {
    part = RT_PARTITION_TILES;
    if (const char* e = getenv("SHIRLEY_PARTITION")) part = !strcmp(e, "samples") ? RT_PARTITION_SAMPLES : RT_PARTITION_TILES;
  }
  (void)world;
  *out = part;
  return RT_OK;
}

// Row bands of a sample-partitioned frame: rank b owns rows [b * band_rows, (b + 1) * band_rows).
int band_rows(const rt_camera* cam, int world) { return (cam->image_height + world - 1) / world; }

// One rank's share before the exchange.
//   tiles: its tiles rendered into c->packed ([max_tiles][64][3]); *count = doubles per rank of the gather
//     (rank 0 also sizes the gathered buffer).
//   samples: all pixels for its part of the frame's sample range, rendered into c->packed as
//     [world * band_rows][W][3] (rows >= H zero); *count = doubles of one row band.
int shard_render(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, int part, int world, int rank,
                 hipStream_t s, size_t* count) {
  int st = check_render_args(c, cam, p);
  if (st) return st;
  HIP_TRY(c, hipSetDevice(c->device));
  SampleRange R;
  if ((st = resolve_range(c, p, &R))) return st;
  rt_render_params q = *p;
  q.tile_rank = 0;
  q.tile_world = 1;
  const int tiles_y = (cam->image_height + kTile - 1) / kTile;
  if (part == RT_PARTITION_SAMPLES) {
    const int rows = band_rows(cam, world);
    *count = (size_t)rows * cam->image_width * 3;
    const size_t total = *count * world;
    if ((st = ensure(c, c->packed, total * sizeof(double)))) return st;
    if ((st = ensure(c, c->parts, total * sizeof(double)))) return st;
    if ((st = ensure(c, c->band, *count * sizeof(double)))) return st;
    if (rank == 0 && (st = ensure(c, c->gathered, total * sizeof(double)))) return st;
    const size_t image = (size_t)cam->image_height * cam->image_width * 3;
    double* local = static_cast<double*>(c->packed.p);
    HIP_TRY(c, hipSetDevice(c->device));
    if (total > image) HIP_TRY(c, hipMemsetAsync(local + image, 0, (total - image) * sizeof(double), s));
    const long long n = R.end - R.begin;
    SampleRange mine;
    mine.begin = R.begin + (int)(n * rank / world);
    mine.end = R.begin + (int)(n * (rank + 1) / world);
    return render_window(c, cam, &q, mine, 0, tiles_y, 0, cam->image_height, 0, local, s);
  }
  int32_t n_total = 0, max_tiles = 0;
  if (rt_tile_layout(cam, world, &n_total, &max_tiles)) return fail(c, RT_E_INVALID, "bad tile layout");
  *count = (size_t)max_tiles * kTilePixels * 3;
  if ((st = ensure(c, c->packed, std::max<size_t>(*count, 1) * sizeof(double)))) return st;
  if (rank == 0 && (st = ensure(c, c->gathered, std::max<size_t>(*count * world, 1) * sizeof(double)))) return st;
  q.tile_rank = rank;
  q.tile_world = world;
  return render_window(c, cam, &q, R, 0, tiles_y, 0, cam->image_height, 1, static_cast<double*>(c->packed.p), s);
}

// samples partition, after the all-to-all (c->parts = [world][band] partial bands of this rank's rows):
// the rank-order sum of its band
int shard_band_sum(rt_ctx* c, int world, size_t count, hipStream_t s) {
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, launch_sum_parts(static_cast<const double*>(c->parts.p), world, (long long)count,
                              static_cast<double*>(c->band.p), s));
  return RT_OK;
}

// Root: the gathered buffer -> accum_dev [H][W][3] (tiles: scatter the packed tiles; samples: the
// gathered row bands are the image's rows in order, padding rows dropped).
int shard_unpack(rt_ctx* c, const rt_camera* cam, int part, int world, double* accum_dev, hipStream_t s) {
  HIP_TRY(c, hipSetDevice(c->device));
  if (part == RT_PARTITION_SAMPLES) {
    const size_t bytes = (size_t)cam->image_height * cam->image_width * 3 * sizeof(double);
    HIP_TRY(c, hipMemcpyAsync(accum_dev, c->gathered.p, bytes, hipMemcpyDeviceToDevice, s));
    return RT_OK;
  }
  int32_t n_total = 0, max_tiles = 0;
  rt_tile_layout(cam, world, &n_total, &max_tiles);
  const int tiles_x = (cam->image_width + kTile - 1) / kTile;
  HIP_TRY(c, launch_unpack(static_cast<const double*>(c->gathered.p), world, max_tiles, n_total, tiles_x,
                           cam->image_width, cam->image_height, accum_dev, s));
  return RT_OK;
}

// What every rank of a sharded frame must agree on: the scene (its digest) and the arguments that decide
// the collectives' shapes and the frame's bits — the resolved partition, the resolved sample range, samples,
// seed, max_depth, sample_chunk and the camera (field by field, no padding hashed).  FNV-1a, 64 bits.
uint64_t call_key(const rt_ctx* c, const rt_camera* cam, const rt_render_params* p, int part, const SampleRange& R) {
  Fnv1a f;
  f.val(c->digest);
  f.val(part);
  f.val(R.begin);
  f.val(R.end);
  f.val(p->samples);
  f.val(p->seed);
  f.val(p->max_depth);
  f.val(p->sample_chunk);
  f.val(cam->image_width);
  f.val(cam->image_height);
  f.val(cam->height);
  f.val(cam->width);
  f.val(cam->focal_length);
  f.val(cam->has_lens);
  f.val(cam->lens_radius);
  f.bytes(cam->origin, sizeof cam->origin);
  f.bytes(cam->w, sizeof cam->w);
  f.bytes(cam->u, sizeof cam->u);
  f.bytes(cam->v, sizeof cam->v);
  f.val(cam->focus_length);
  f.val(cam->time0);
  f.val(cam->time1);
  return f.h;
}

// The gathered words of one call: RT_OK, or RT_E_INVALID naming the first rank that differs from rank 0.
int key_verdict(rt_ctx* c, const uint64_t* words, int world) {
  int what = 0;
  const int r = key_mismatch(words, world, &what);
  if (r < 0) return RT_OK;
  if (what == 0)
    return fail(c, RT_E_INVALID, "scene mismatch across ranks: rank %d holds scene %016llx, rank 0 %016llx", r,
                (unsigned long long)words[2 * r], (unsigned long long)words[0]);
  return fail(c, RT_E_INVALID,
              "render arguments differ across ranks (partition, sample range, samples, seed, max_depth, "
              "sample_chunk or camera): rank %d key %016llx, rank 0 %016llx",
              r, (unsigned long long)words[2 * r + 1], (unsigned long long)words[1]);
}

// Every rank must render the same scene with the same call key (keycheck.h states the rule).  Every call
// all-gathers each rank's 16-byte (scene digest, key) on every rank — one collective sequence on all ranks
// whatever their arguments — copies the gathered words into pinned host memory and checks them: at once
// when this rank's key is new (or SHIRLEY_KEY_CHECK=sync), else at the next call (no host round trip in a
// steady loop of frames).  A failed check leaves no frame collective issued by this rank.
int check_call_key(rt_ctx* c, rt_comm* m, uint64_t key, hipStream_t s) {
  const int W = m->world;
  const size_t slot_words = 2 * (size_t)(W + 1);
  int st;
  if (!m->key_words) {
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&m->key_words), 2 * slot_words * sizeof(uint64_t), 0));
    for (hipEvent_t& e : m->key_ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // the previous call's words: the deferred half of its check
  if (m->ks.pending) {
    m->ks.pending = false;
    HIP_TRY(c, hipEventSynchronize(m->key_ev[m->key_pending]));
    if ((st = key_verdict(c, m->key_words + m->key_pending * slot_words, W))) {
      m->ks.verified = false;
      m->ks.poisoned = true;
      return st;
    }
  }
  if ((st = ensure(c, c->digests, 2 * slot_words * sizeof(uint64_t)))) return st;
  const int slot = m->key_slot;
  m->key_slot ^= 1;
  uint64_t* hw = m->key_words + slot * slot_words;  // (this slot's last check was done: at most one pending)
  uint64_t* dw = static_cast<uint64_t*>(c->digests.p) + slot * slot_words;
  hw[2 * W] = c->digest;
  hw[2 * W + 1] = key;
  HIP_TRY(c, hipMemcpyAsync(dw + 2 * W, hw + 2 * W, 2 * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  RCCL_TRY(c, rccl().AllGather(dw + 2 * W, dw, 2, ncclUint64, m->comm, s));
  HIP_TRY(c, hipMemcpyAsync(hw, dw, 2 * (size_t)W * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipEventRecord(m->key_ev[slot], s));
  const char* e = getenv("SHIRLEY_KEY_CHECK");
  if (key_check_now(m->ks, key, e && !strcmp(e, "sync"))) {
    HIP_TRY(c, hipEventSynchronize(m->key_ev[slot]));
    if ((st = key_verdict(c, hw, W))) {
      m->ks.verified = false;
      m->ks.poisoned = true;
      return st;
    }
    m->ks.verified = true;
    m->ks.verified_key = key;
  } else {
    m->ks.pending = true;
    m->key_pending = slot;
  }
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]) {
  if (!id) return RT_E_INVALID;
  if (!rccl().ok()) return RT_E_RCCL;
  ncclUniqueId u;
  static_assert(sizeof u == RT_COMM_ID_BYTES, "ncclUniqueId size");
  if (rccl().GetUniqueId(&u) != ncclSuccess) return RT_E_RCCL;
  std::memcpy(id, &u, sizeof u);
  return RT_OK;
}

int rt_comm_init_rank(rt_ctx* c, const uint8_t id[RT_COMM_ID_BYTES], int32_t world, int32_t rank, rt_comm** out) {
  if (!c) return RT_E_INVALID;
  if (!id || !out || world < 1 || rank < 0 || rank >= world)
    return fail(c, RT_E_INVALID, "bad communicator arguments (world %d, rank %d)", world, rank);
  *out = nullptr;
  int st = need_rccl(c);
  if (st) return st;
  HIP_TRY(c, hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  rt_comm* m = new rt_comm();
  m->world = world;
  m->rank = rank;
  m->device = c->device;
  const ncclResult_t r = rccl().CommInitRank(&m->comm, world, u, rank);
  if (r != ncclSuccess) {
    delete m;
    return fail(c, RT_E_RCCL, "ncclCommInitRank(world %d, rank %d): %s", world, rank, rccl().GetErrorString(r));
  }
  *out = m;
  return RT_OK;
}

int rt_comm_destroy(rt_comm* m) {
  if (!m) return RT_OK;
  (void)hipSetDevice(m->device);
  if (m->comm && rccl().ok()) (void)rccl().CommDestroy(m->comm);
  for (hipEvent_t e : m->key_ev)
    if (e) (void)hipEventDestroy(e);
  if (m->key_words) (void)hipHostFree(m->key_words);
  delete m;
  return RT_OK;
}

int rt_render_sharded(rt_ctx* c, rt_comm* m, const rt_camera* cam, const rt_render_params* p, double* accum_dev,
                      void* stream) {
  if (!c) return RT_E_INVALID;
  if (!m || !m->comm) return fail(c, RT_E_INVALID, "no communicator");
  if (m->device != c->device) return fail(c, RT_E_INVALID, "communicator of device %d used with device %d", m->device, c->device);
  if (m->ks.poisoned)  // (keycheck.h: its peers may still hold the failed call's frame collectives)
    return fail(c, RT_E_INVALID, "communicator poisoned by a failed cross-rank check: destroy and re-create it");
  if (m->rank == 0 && !accum_dev) return fail(c, RT_E_INVALID, "accum_dev is NULL on the root");
  if (!c->have_scene) return fail(c, RT_E_INVALID, "no scene uploaded (call rt_scene_upload first)");
  if (!p || !cam) return fail(c, RT_E_INVALID, "camera/params is NULL");
  int part = 0;
  int st = frame_partition(c, p, m->world, &part);
  if (st) return st;
  if ((st = check_render_args(c, cam, p))) return st;
  SampleRange R;
  if ((st = resolve_range(c, p, &R))) return st;
  hipStream_t s;
  resolve_stream(c, stream, &s);
  HIP_TRY(c, hipSetDevice(c->device));
  if ((st = check_call_key(c, m, call_key(c, cam, p, part, R), s))) return st;
  size_t count = 0;
  if ((st = shard_render(c, cam, p, part, m->world, m->rank, s, &count))) return st;
  if (part == RT_PARTITION_SAMPLES) {
    RCCL_TRY(c, rccl().AllToAll(c->packed.p, c->parts.p, count, ncclFloat64, m->comm, s));
    if ((st = shard_band_sum(c, m->world, count, s))) return st;
    RCCL_TRY(c, rccl().Gather(c->band.p, m->rank == 0 ? c->gathered.p : nullptr, count, ncclFloat64, 0, m->comm, s));
  } else {
    RCCL_TRY(c, rccl().Gather(c->packed.p, m->rank == 0 ? c->gathered.p : nullptr, count, ncclFloat64, 0, m->comm, s));
  }
  if (m->rank == 0) return shard_unpack(c, cam, part, m->world, accum_dev, s);
  return RT_OK;
}

int rt_render_multi(rt_ctx* const* ctxs, int32_t n, const rt_camera* cam, const rt_render_params* p,
                    double* accum_host) {
  if (!ctxs || n < 1 || !ctxs[0]) return RT_E_INVALID;
  rt_ctx* root = ctxs[0];
  if (!cam || !p || !accum_host) return fail(root, RT_E_INVALID, "NULL argument");
  if (p->tile_world != 1) return fail(root, RT_E_INVALID, "rt_render_multi shards the frame itself (tile_world must be 1)");
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) return fail(root, RT_E_INVALID, "ctxs[%d] is NULL", i);
    devs[i] = ctxs[i]->device;
    for (int j = 0; j < i; ++j)
      if (devs[j] == devs[i]) return fail(root, RT_E_INVALID, "device %d appears twice", devs[i]);
  }
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]->have_scene) return fail(root, RT_E_INVALID, "device %d: no scene uploaded", devs[i]);
    if (ctxs[i]->digest != root->digest)
      return fail(root, RT_E_INVALID, "scene mismatch: device %d holds scene %016llx, device %d %016llx", devs[i],
                  (unsigned long long)ctxs[i]->digest, devs[0], (unsigned long long)root->digest);
  }
  int part = 0;
  int st = frame_partition(root, p, n, &part);
  if (st) return st;
  if ((st = need_rccl(root))) return st;
  if (root->group_devices != devs) {  // (re)build the communicators of this device set
    for (rt_comm& m : root->group_comms)
      if (m.comm) (void)rccl().CommDestroy(m.comm);
    root->group_comms.clear();
    root->group_devices.clear();
    std::vector<ncclComm_t> comms(n, nullptr);
    RCCL_TRY(root, rccl().CommInitAll(comms.data(), n, devs.data()));
    for (int i = 0; i < n; ++i) root->group_comms.push_back(rt_comm{comms[i], n, i, devs[i]});
    root->group_devices = devs;
  }
  // every device renders its share (asynchronous, all devices at once), then grouped collectives
  std::vector<size_t> count(n);
  for (int i = 0; i < n; ++i) {
    if ((st = shard_render(ctxs[i], cam, p, part, n, i, ctxs[i]->stream, &count[i])))
      return i ? fail(root, st, "device %d: %s", devs[i], ctxs[i]->err.c_str()) : st;
  }
  auto grouped = [&](auto&& one) -> int {
    RCCL_TRY(root, rccl().GroupStart());
    for (int i = 0; i < n; ++i) {
      const ncclResult_t r = one(i);
      if (r != ncclSuccess) {
        (void)rccl().GroupEnd();
        return fail(root, RT_E_RCCL, "collective (rank %d): %s", i, rccl().GetErrorString(r));
      }
    }
    RCCL_TRY(root, rccl().GroupEnd());
    return RT_OK;
  };
  if (part == RT_PARTITION_SAMPLES) {
    if ((st = grouped([&](int i) {
           return rccl().AllToAll(ctxs[i]->packed.p, ctxs[i]->parts.p, count[i], ncclFloat64, root->group_comms[i].comm,
                                  ctxs[i]->stream);
         })))
      return st;
    for (int i = 0; i < n; ++i)
      if ((st = shard_band_sum(ctxs[i], n, count[i], ctxs[i]->stream))) return i ? fail(root, st, "device %d: %s", devs[i], ctxs[i]->err.c_str()) : st;
    if ((st = grouped([&](int i) {
           return rccl().Gather(ctxs[i]->band.p, i == 0 ? root->gathered.p : nullptr, count[i], ncclFloat64, 0,
                                root->group_comms[i].comm, ctxs[i]->stream);
         })))
      return st;
  } else {
    if ((st = grouped([&](int i) {
           return rccl().Gather(ctxs[i]->packed.p, i == 0 ? root->gathered.p : nullptr, count[i], ncclFloat64, 0,
                                root->group_comms[i].comm, ctxs[i]->stream);
         })))
      return st;
  }
  const size_t bytes = (size_t)cam->image_width * cam->image_height * 3 * sizeof(double);
  HIP_TRY(root, hipSetDevice(root->device));
  if ((st = ensure(root, root->accum, bytes))) return st;
  if ((st = shard_unpack(root, cam, part, n, static_cast<double*>(root->accum.p), root->stream))) return st;
  HIP_TRY(root, hipMemcpyAsync(accum_host, root->accum.p, bytes, hipMemcpyDeviceToHost, root->stream));
  for (int i = n - 1; i >= 0; --i) {
    HIP_TRY(root, hipSetDevice(ctxs[i]->device));
    HIP_TRY(root, hipStreamSynchronize(ctxs[i]->stream));
  }
  return RT_OK;
}

}  // extern "C"
