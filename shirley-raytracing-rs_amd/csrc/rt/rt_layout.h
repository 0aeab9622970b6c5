// rt_layout.h — HBM layout of a flattened scene and the trace-kernel parameter block.
//
// Shared by the host side of the C ABI (rt_api.cpp, bvh_build.cpp) and the HIP kernels
// (trace.hip).  Plain structs only; sizes are checked with static_assert so host and device
// agree byte for byte.
#pragma once

#include <stdint.h>

namespace rt {

// Tile geometry: a wave (64 lanes) owns an 8x8 pixel tile of one sample chunk.
constexpr int kTile = 8;
constexpr int kTilePixels = kTile * kTile;  // == wavefront size
constexpr int kBlockThreads = 256;          // 4 waves per workgroup
constexpr int kWave = 64;

// BVH2 node with both child boxes inline (one 112-B record per internal node).
// child >= 0: internal node index; child < 0: leaf, primitive index = ~child; kEmptyChild: none.
constexpr int32_t kEmptyChild = 0x7fffffff;
struct alignas(16) DNode {
  // child c: lo = {box[c][0..2]}, hi = {box[c][3..5]}
  double box[2][6];
  int32_t child[2];
  int32_t pad[2];
};
static_assert(sizeof(DNode) == 112, "DNode layout");

// Primitive kinds (device-side, rect axis folded into the kind).
enum : int32_t { kPrimSphere = 0, kPrimRectXY = 1, kPrimRectYZ = 2, kPrimRectXZ = 3, kPrimBox = 4 };

// One primitive = one reference leaf object (a RectBox stays ONE leaf of 6 faces, rect.rs:146-156).
struct alignas(16) DPrim {
  double p[6];       // sphere: cx cy cz r ; rect: d1_min d1_max d2_min d2_max offset ; box: min xyz max xyz
  int32_t kind;
  int32_t material;
};
static_assert(sizeof(DPrim) == 64, "DPrim layout");

struct alignas(16) DMat {
  int32_t kind;   // RT_MAT_*
  int32_t tex;
  double albedo[3];
  double param;
  double pad;
};
static_assert(sizeof(DMat) == 48, "DMat layout");

struct alignas(16) DTex {
  int32_t kind;   // RT_TEX_*
  int32_t odd, even, table;
  double color[3];
  double scale;
};
static_assert(sizeof(DTex) == 48, "DTex layout");

struct DPerlin {
  double ranfloat[256][3];
  int32_t perm_x[256], perm_y[256], perm_z[256];
};

struct DImage {
  int32_t width, height;
  int64_t offset;  // byte offset of the RGB8 texels in the image pool
};

struct DScene {
  const DNode* nodes;      // node 0 = top node (child[0] = root, child[1] = empty)
  const DPrim* prims;
  const DMat* mats;
  const DTex* texs;
  const DPerlin* perlin;
  const DImage* images;
  const uint8_t* texels;
  int32_t n_nodes, n_prims;
  int32_t stack_depth;     // max stack entries a traversal can need
  int32_t sky;
  double sky_color[3];
};

struct DCamera {
  int32_t width, height;   // image dims
  int32_t has_lens;
  int32_t pad;
  double lens_radius;
  double origin[3], u[3], v[3];
  double horizontal[3], vertical[3], lower_left[3];  // precomputed exactly as camera/mod.rs:99-108
};

// Work decomposition: unit = (local tile, sample chunk, lane) ; see trace.hip.
struct DWork {
  int32_t tiles_x, tiles_y;      // tile grid of the rendered window (tiles_y rows from ty0)
  int32_t tile_rank, tile_world;
  int32_t n_tiles_rank;          // tiles owned by this rank
  int32_t samples;               // spp
  int32_t chunk;                 // samples per unit
  int32_t n_chunks;
  int32_t max_depth;
  int32_t ty0;                   // first tile row of the window (rt_render_scanlines)
  uint64_t seed;
  uint64_t n_units;              // n_tiles_rank * n_chunks * 64
};

struct DCounters {
  unsigned long long samples, segments, node_visits, prim_tests;
};

struct KParams {
  DScene scene;
  DCamera cam;
  DWork work;
  double* partial;               // [n_chunks][n_tiles_rank*64][3]
  unsigned long long* unit_counter;  // work-queue head (one 64-unit batch per fetch)
  DCounters* counters;
};

}  // namespace rt
