// rt_layout.h — HBM layout of a flattened scene and the trace-kernel parameter block.
//
// Shared by the host side of the C ABI (rt_api.cpp, bvh_build.cpp) and the HIP kernels
// (trace.hip).  Plain structs only; sizes are checked with static_assert so host and device
// agree byte for byte.
#pragma once

#include <stdint.h>

#include "plan.h"  // (unit window sizes)

namespace rt {

// Tile geometry: a wave (64 lanes) owns an 8x8 pixel tile of one sample chunk.
constexpr int kTile = 8;
constexpr int kTilePixels = kTile * kTile;  // == wavefront size
constexpr int kTraceThreads = 256;      // megakernel block, BVH in L1/L2: 4 waves, several blocks per CU
constexpr int kTraceThreadsWide = 1024; // megakernel block holding the whole BVH in LDS: 16 waves (4 per SIMD), one per CU
#ifndef RT_EXT_WIDE_THREADS
#define RT_EXT_WIDE_THREADS 768
#endif
constexpr int kTraceThreadsWide3 = RT_EXT_WIDE_THREADS;  // book-2 (EXT) scenes' wide block: 768 = 3 waves per SIMD (168 VGPRs)
constexpr int kHitThreads = 256;    // rt_scene_hit kernel
constexpr int kWave = 64;
constexpr int kLdsBytes = 160 * 1024;  // LDS per CU (gfx950)

// BVH2 node with both child boxes inline (one 112-B record per internal node).  The boxes are the
// reference's exact f64 bounding boxes, so testing a child box with the f64 slab test IS the
// reference's Aabb::hit2 on that child (bbox_tree.rs:60-71): for a leaf child that is the test of
// the object's own bounding_box() before the object itself.
// child >= 0: internal node index; child < 0: leaf, primitive index = ~child; kEmptyChild: none.
constexpr int32_t kEmptyChild = 0x7fffffff;
struct alignas(16) DNode {
  double box[2][6];  // child c: lo = box[c][0..2], hi = box[c][3..5]
  int32_t child[2];
  int32_t pad[2];
};
static_assert(sizeof(DNode) == 112, "DNode layout");

// 4-wide node of the collapsed tree (megakernel, wf_extend4): child boxes in f32, SoA [axis][child],
// inflated by the scene's inflation distance and rounded outward, so an f32 slab test on them accepts
// a superset of what the reference's f64 Aabb::hit2 accepts on the exact box.  That is all an
// internal level needs: the reference's test is monotone in the box planes and a parent's planes
// are its children's, so whenever the reference passes a leaf's box it passes every enclosing box
// too — internal tests never decide which primitives are tested; leaf tests do, and those run
// exactly (f64 hit2 on the leaf's own bounding box, recomputed from the primitive).
// child >= 0: node index; child < 0: leaf ~(prim | kind flags): kLeafGeneric when not a sphere, plus
// kLeafBox for a RectBox, so traversal tests sphere, rect and box leaves in three tight loops (a wave
// runs each leaf kind's code once per round, not the union of all kinds); kEmptyChild: none.
constexpr int32_t kLeafGeneric = 1 << 29;
constexpr int32_t kLeafBox = 1 << 28;
constexpr int32_t kLeafPrimMask = kLeafBox - 1;  // primitive index bits
constexpr int kMaxKeyBits = 20;      // node-index bits of a traversal entry (so <= 2^20 4-wide nodes)
constexpr int kStack4EntryBytes = 4; // one packed (entry t | node) word per 4-wide stack entry
// Two layouts of the same node.  DNode4F (reference scenes): per axis three rows lo, hi, lo
// (row[axis][r][child]); a ray whose 1/d is negative on the axis starts one row later (16 B), so its
// near plane row is at 48 axis + s and its far row 16 B after it — one address add per axis and
// visit, the reads' immediate offsets do the rest.  DNode4C (book-2 scenes, EXT kernel instances):
// rows lo x y z, hi x y z, 112 B, so final_scene's tree still fits the wide block's LDS beside its
// stacks; near / far rows at 16 axis + s and 16 axis + 48 - s (s = 48 when 1/d < 0), two adds per axis.
struct alignas(16) DNode4F {
  float row[3][3][4];
  int32_t child[4];
  static constexpr bool kRows3 = true;
  static constexpr int kNegRow = 16;  // the ray's row offset on an axis where 1/d < 0
};
static_assert(sizeof(DNode4F) == 160, "DNode4F layout");
struct alignas(16) DNode4C {
  float lo[3][4];  // lo[axis][child]
  float hi[3][4];
  int32_t child[4];
  static constexpr bool kRows3 = false;
  static constexpr int kNegRow = 48;
};
static_assert(sizeof(DNode4C) == 112, "DNode4C layout");
template <bool EXT> struct Node4Sel { typedef DNode4F T; };
template <> struct Node4Sel<true> { typedef DNode4C T; };
inline constexpr int node4_bytes(bool ext) { return ext ? (int)sizeof(DNode4C) : (int)sizeof(DNode4F); }

// Where a kernel instance reads BVH nodes from (template parameter of the traversal):
enum : int { kNodesGlobal = 0, kNodesLds = 1, kNodesMixed = 2,
             kSceneLds = 3 };  // kSceneLds: all nodes AND all primitives in LDS (megakernel, small scenes)

// Primitive kinds (device-side, rect axis folded into the kind).
enum : int32_t { kPrimSphere = 0, kPrimRectXY = 1, kPrimRectYZ = 2, kPrimRectXZ = 3, kPrimBox = 4,
                 kPrimMovingSphere = 5 };
// Book-2 extensions (absent from the reference): DPrim.kind = base kind | flags |
// (ext record index << kPrimExtShift).  Any extended primitive is a "slow" leaf (kLeafBox path).
constexpr int32_t kPrimBaseMask = 0xff;
constexpr int32_t kPrimMedium = 1 << 8;     // ConstantMedium with this shape as its boundary
constexpr int32_t kPrimXform = 1 << 9;      // instance transform (RotateY then Translate)
constexpr int32_t kPrimExt = 1 << 10;       // has a DExt record
constexpr int kPrimExtShift = 11;
// The extra parameters of an extended primitive (DScene.exts[kind >> kPrimExtShift]).
struct alignas(16) DExt {
  double box[6];            // the exact world bounding box (leaf box test), computed on the host
  double c1[3], t0, t1;     // moving sphere: centre at t1 (centre at t0 = p[0..2]), motion interval
  double cos_t, sin_t;      // RotateY: cos / sin of the angle in radians
  double off[3];            // Translate offset
  double neg_inv_density;   // ConstantMedium: -1 / density
  int32_t object;           // the object's index in the scene description (its side-stream key; primitives
                            //   are numbered by the reference's leaf order, rt_api.cpp)
  int32_t prim;             // its primitive number (the deferred object tests, rt_device.h ext_deferred)
};
static_assert(sizeof(DExt) == 144, "DExt layout");

// One primitive = one reference leaf object (a RectBox stays ONE leaf of 6 faces, rect.rs:146-156).
struct alignas(16) DPrim {
  double p[6];       // sphere: cx cy cz r 1/r sure-pass bound (r - eta) ; rect: d1_min d1_max d2_min d2_max offset ; box: min xyz max xyz
  int32_t kind;
  int32_t material;  // material index
};
static_assert(sizeof(DPrim) == 64, "DPrim layout");

struct alignas(16) DMat {
  int32_t kind;   // RT_MAT_*
  int32_t tex;
  double albedo[3];  // Metal albedo; a Dielectric's Schlick r0^2 for its front / back face ratio (host-computed)
  double param;
  double inv_param;  // 1.0 / param, computed on the host (the dielectric's front-face ratio 1.0 / ir)
};
static_assert(sizeof(DMat) == 48, "DMat layout");

// An image texture's RGB8 texels (device) and size, held in its DTex record: the texel lookup needs
// no scene-wide table (whose pointers the megakernel would otherwise keep in SGPRs across its loop).
struct DTexImage {
  const uint8_t* texels;
  int32_t width, height;
};
struct alignas(16) DTex {
  int32_t kind;   // RT_TEX_*
  int32_t odd, even, table;
  union {
    double color[3];  // RT_TEX_SOLID
    DTexImage img;    // RT_TEX_IMAGE
  };
  double scale;
};
static_assert(sizeof(DTex) == 48, "DTex layout");

struct DPerlin {
  double ranfloat[256][3];
  int32_t perm_x[256], perm_y[256], perm_z[256];
};

struct DScene {
  const DNode* nodes;      // node 0 = top node (child[0] = root, child[1] = empty)
  const DPrim* prims;
  const DMat* mats;
  const DTex* texs;
  const DPerlin* perlin;
  int32_t n_nodes, n_prims;
  int32_t stack_depth;     // max stack entries a traversal can need
  int32_t n_lds_nodes;     // nodes [0, n_lds_nodes) are copied into LDS per block (BFS order: top levels)
  const void* nodes4;      // the same tree collapsed to 4-wide f32 nodes (node 0 = top node): DNode4F, or
                           // DNode4C when exts != null (Node4Sel<EXT>)
  int32_t n_nodes4;
  int32_t stack_depth4;    // exact worst-case stack of the 4-wide traversal
  int32_t n_lds_nodes4;    // 4-wide nodes [0, n_lds_nodes4) copied into LDS per megakernel block
  int32_t n_lds_prims;     // 0, or n_prims when the megakernel block also keeps the primitives in LDS
  int32_t n_lds_perlin;    // 0, or n_perlin when the megakernel block also keeps the Perlin tables in LDS
  float origin_limit;      // rays with max|o| <= origin_limit take the f32 node test (its error bound
                           // assumes it); others evaluate the same inflated boxes in f64
  int32_t root4;           // first 4-wide node a traversal visits: the root when it is internal (its
                           // own box test only culls, so it is skipped), else the top node 0
  uint32_t key_mask;       // 2^K - 1 >= n_nodes4 - 1: a 4-wide traversal entry is one 32-bit word,
                           // the f32 entry t with its low K bits replaced by the node index
  int32_t sky;
  double sky_color[3];
  const DExt* exts;        // book-2 extension records (null when the scene has none)
  double time0, time1;     // camera shutter (set per render call)
  const double* shutter;   // device copy of {time0, time1}: moving spheres read it at the use site (an
                           // opaque pointer: held in SGPRs across the megakernel's loop the two doubles spill)
  int32_t n_lds_mats;      // 0, or n_mats / n_texs when the scene-in-LDS block also keeps the materials and
  int32_t n_lds_texs;      // textures in LDS (after the Perlin tables)
};

struct DCamera {
  int32_t width, height;   // image dims
  int32_t has_lens;
  int32_t pad;
  double lens_radius;
  double origin[3], u[3], v[3];
  double horizontal[3], vertical[3], lower_left[3];  // precomputed exactly as camera/mod.rs:99-108
  // the image size as doubles and their correctly rounded reciprocals (host IEEE divisions): the
  // jittered pixel's x / width as one correction step on x * (1 / width) (pixel_coord_div)
  double wd, hd, inv_w, inv_h;
};

// Work decomposition: unit = (local tile, sample chunk, lane) ; see trace.hip.
// Unsigned 32-bit division by a divisor fixed for a launch (Granlund & Montgomery 1994, "Division by
// invariant integers using multiplication", Fig. 4.1): q = (t + ((n - t) >> s1)) >> s2 with
// t = mulhi(m, n), l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1, s1 = min(l, 1), s2 = max(l - 1, 0);
// exact for every 32-bit n.  Built on the host, applied per lane in a few instructions instead of a
// generic division sequence.
struct UDiv {
  uint32_t m, s1, s2;
};
inline UDiv make_udiv(uint32_t d) {
  uint32_t l = 0;
  while (l < 32 && (1ull << l) < d) ++l;
  const uint64_t m = (((1ull << l) - d) << 32) / d + 1;
  return UDiv{(uint32_t)m, l < 1 ? l : 1u, l > 0 ? l - 1 : 0u};
}

struct DWork {
  UDiv div_unit_tile;            // / (n_chunks * kTilePixels): unit index -> the rank's local tile
  UDiv div_tiles_x;              // / tiles_x
  int32_t tiles_x, tiles_y;      // tile grid of the rendered window (tiles_y rows from ty0)
  int32_t tile_rank, tile_world;
  int32_t n_tiles_rank;          // tiles owned by this rank
  int32_t samples;               // end of the launch's sample range (exclusive): a unit's samples stop here
  int32_t sample_base;           // first sample of the launch's range: chunk c = samples [base + c chunk, ..)
  int32_t chunk;                 // samples per unit
  int32_t n_chunks;
  int32_t max_depth;
  int32_t ty0;                   // first tile row of the window (rt_render_scanlines)
  uint64_t seed;
  uint64_t n_units;              // n_tiles_rank * n_chunks * 64
  // megakernel: the (tile-major) unit space cut into n_segs contiguous segments
  // of seg_len units (a multiple of 64), one per block (XCD-major: the blocks of one XCD own adjacent
  // segments), each with its own counter in unit_counter[]; a block's waves take windows from their
  // segment, then steal from the next segments that still hold units
  uint32_t seg_len, n_segs;
  // shared queue (n_segs == 0): units a wave takes per atomic (plan.h)
  uint32_t q_window, pad_q;
};

// Statistics counters, kCounterSlots copies one 128-B line apart: a block adds into slot
// blockIdx % kCounterSlots, so atomics from different blocks do not serialise on one address.
struct DCounters {
  unsigned long long samples, segments, node_visits, prim_tests;
  unsigned long long pad[12];
};
constexpr int kCounterSlots = 64;
// (work units a megakernel wave takes per queue atomic: kSegmentWindow / kQueueWindow, plan.h)
// instrumented build: DCounters.pad slots of the megakernel's phase clocks (PH_STAMP in trace.hip) and
// traversal step statistics
enum : int {
  kPhRegen = 0, kPhTrav = 1, kPhShade = 2, kPhLaneSteps = 3, kPhWaveSteps = 4, kPhRecord = 5, kPhMarble = 6,
  kPhDraws = 7, kPhCamera = 8, kPhTail = 9, kPhBuckets = 10
};

struct KParams {
  DScene scene;
  DCamera cam;
  DWork work;
  double* partial;               // [n_chunks][n_tiles_rank*64][3]
  unsigned long long* unit_counter;  // work-queue head (one 64-unit batch per fetch)
  DCounters* counters;
  int32_t split_refill;          // split_kernel: idle traversal lanes before a wave claims rays (>= 1)
  // the megakernel's KBlock of this pass (device memory): its rarely used uniforms are read there with
  // scalar loads at their use sites instead of being held in SGPRs across the whole loop, where they
  // spill to VGPR lanes and come back one v_readlane each
  uint64_t kconst;
};

// Device copy of a pass's launch parameters for the megakernel (KParams.kconst): the camera (read where
// a new sample's ray is formed), the scene record (the sky, where a missed ray is shaded), the work
// descriptor and the output / queue / statistics pointers (where a unit is taken or published).
struct alignas(16) KBlock {
  DCamera cam;
  DScene scene;
  DWork work;
  double* partial;
  unsigned long long* unit_counter;
  DCounters* counters;
};

// ---- wavefront engine (wavefront.hip): path state of P slots as structure-of-arrays in HBM ----
struct WfState {
  double *ox, *oy, *oz, *dx, *dy, *dz;  // ray to trace
  double *ax, *ay, *az;                 // throughput of the current sample
  double *ex, *ey, *ez;                 // radiance of the current sample
  double *sx, *sy, *sz;                 // in-order sum of the unit's finished samples
  double* ht;                           // closest hit t
  uint64_t* part;                       // partial-sum slot of the unit
  uint32_t* pixel;                      // rng pixel id (py * W + px), 0xffffffff: no unit
  uint32_t *sample, *draw, *c2, *c3;    // rng counter state of the current sample
  int32_t *s_next, *s_end;              // next sample to start / end of the unit
  int32_t* depth;                       // bounces left
  int32_t *hprim, *hface;               // closest primitive (-1: miss), RectBox face
  uint8_t* state;
};
constexpr size_t kWfSlotBytes = 16 * 8 + 8 + 11 * 4 + 1;  // bytes of one slot across the arrays

struct WfTexQ {  // deferred (Perlin) texture evaluations, compacted per 64-slot group
  double *px, *py, *pz, *scale;
  int32_t *slot, *tex, *kind;
  uint32_t* count;  // entries of each group this round
};
constexpr size_t kWfTexBytes = 4 * 8 + 3 * 4;

// wf_extend hands out slots from kWfQueues cursors (one 128-B line each, zeroed every round);
// queue q covers slots [q * qlen, (q + 1) * qlen).  A wave starts on queue (wave id % kWfQueues)
// and moves on when it is drained, so the fetch atomics spread over kWfQueues addresses.
constexpr int kWfQueues = 64;
struct WfIter {
  unsigned long long fetch[kWfQueues][16];
};

struct WfParams {
  DScene scene;
  DCamera cam;
  DWork work;
  WfState st;
  WfTexQ tq;
  uint32_t n_slots;     // multiple of 64: slot group g = slots [64 g, 64 g + 64) = one wave of wf_shade
  uint32_t first;       // wf_shade's first round: group g's unit window is [64 g, 64 g + 64)
  int32_t n_perlin;     // Perlin tables of the scene (wf_texture copies up to 2 into LDS)
  uint32_t ext_window;  // wf_extend4: slots a wave claims per cursor atomic (multiple of 64)
  double* partial;
  unsigned long long* unit_counter;  // dynamic units are n_slots + the counter (64 per fetch)
  unsigned long long* win;           // per group: [next, end) of its unit window
  unsigned* retired;                 // slots with no work left (== n_slots: frame done)
  DCounters* counters;               // [kCounterSlots]
  WfIter* it;
};

}  // namespace rt
