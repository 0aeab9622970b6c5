/*
 * shirley_rt.h — drop-in C ABI for the reference's render hot path on MI355X.
 *
 * What this replaces (all paths relative to scottschroeder/shirley-raytracing-rs):
 *   - src/main.rs:65-130        render_scene(): the rayon loop over scanlines (main.rs:92-126)
 *   - src/raytracer/render.rs:49-70  render_scanline(frame, rng, samples, max_depth, ws, line_idx, buf)
 *   - src/raytracer/render.rs:17-48  ray_color()  (the per-sample bounce loop)
 *   - src/raytracer/scene/mod.rs:111-137  SceneBuilder::finalize (texture load + BBox tree build)
 *
 * A host (the C++ host in this repo, or a Rust crate binding this header verbatim with
 * bindgen/#[repr(C)]) owns the scene description, the camera and the
 * image buffer.  The library owns device memory.  Everything here is plain C: fixed-width
 * integers, doubles, raw pointers and sizes.  No C++ types and no exceptions cross this ABI.
 *
 * Arithmetic is IEEE binary64 throughout, like the reference (core/math.rs:5 `type Real = f64`).
 *
 * Errors: every entry point returns an rt_status; rt_last_error(ctx) holds a message.
 * Threading: one rt_ctx per device; a ctx must not be used from two host threads at once.
 */
#ifndef SHIRLEY_RT_H
#define SHIRLEY_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 7

typedef enum rt_status {
  RT_OK = 0,
  RT_E_INVALID = 1,     /* bad argument / malformed scene */
  RT_E_HIP = 2,         /* HIP runtime error (no device, launch failure, ...) */
  RT_E_OOM = 3,         /* device allocation failed */
  RT_E_UNSUPPORTED = 4, /* feature not compiled in / not available */
  RT_E_RCCL = 5         /* RCCL (librccl) missing or a collective failed (multi-GPU entry points) */
} rt_status;

/* geometry/object.rs:9-16  GeometricObject */
enum { RT_GEOM_SPHERE = 0, RT_GEOM_RECT_XY = 1, RT_GEOM_RECT_YZ = 2, RT_GEOM_RECT_XZ = 3, RT_GEOM_RECT_BOX = 4,
       /* book-2 ("The Next Week") extension, absent from the reference:
        * a sphere whose centre moves linearly from p[0..2] at q[3] to q[0..2] at q[4] */
       RT_GEOM_MOVING_SPHERE = 5 };
/* material/material_type.rs:20-27  MaterialType */
enum { RT_MAT_METAL = 0, RT_MAT_DIELECTRIC = 1, RT_MAT_LAMBERTIAN = 2, RT_MAT_DIFFUSE_LIGHT = 3, RT_MAT_FAIRY_LIGHT = 4,
       /* book-2 extension (absent from the reference): the phase function of a ConstantMedium —
        * scatters to random_in_unit_sphere() with the texture's albedo */
       RT_MAT_ISOTROPIC = 5 };
/* material/texture/loader.rs:17-28  TextureLoader (after load: Solid / Checker / Noise / Image) */
enum { RT_TEX_SOLID = 0, RT_TEX_CHECKER = 1, RT_TEX_PERLIN = 2, RT_TEX_IMAGE = 3 };
/* skybox/mod.rs:11-16  SkyBox */
enum { RT_SKY_ABOVE = 0, RT_SKY_FLAT = 1, RT_SKY_NONE = 2 };
/* BVH builder selection for rt_scene_upload */
enum {
  RT_BVH_REFERENCE = 0, /* bvh/bbox_tree/constructor.rs split rules (median/midpoint on min-x/y/z, volume score) */
  RT_BVH_SAH = 1,       /* surface-area heuristic, exact sweep over every object boundary (performance option; the same hits:
                           exact ties in t go to the reference tree's winner whichever tree is walked) */
  /* node placement flags OR-ed into the builder argument (testing / tuning) */
  RT_BVH_NODES_GLOBAL = 0x100,   /* every node read through L1/L2 (the default) */
  RT_BVH_NODES_HALF_LDS = 0x200, /* top half of the nodes copied into LDS per block (mixed path) */
  RT_BVH_NODES_LDS = 0x400       /* as many nodes in LDS as fit next to the traversal stacks */
};
/* Trace engine for rt_render_params.engine.  Both compute the same ray_color() arithmetic and give
 * the same pixels; they differ only in how the bounce loop is scheduled on the GPU. */
enum {
  RT_ENGINE_AUTO = 0,       /* the faster engine on MI355X (today: the megakernel; env SHIRLEY_ENGINE overrides) */
  RT_ENGINE_MEGAKERNEL = 1, /* one persistent kernel runs whole paths, lane-level path regeneration */
  RT_ENGINE_WAVEFRONT = 2,  /* extend / shade / texture kernels over a pool of path slots in HBM;
                             * the host loop blocks until the frame is traced */
  RT_ENGINE_SPLIT = 3,      /* ABI 5: the megakernel with its traversal decoupled from its shading
                             * (one block per CU: shading waves post rays to traversal waves through
                             * LDS queues).  Scenes that fit it: reference primitives only, whole scene
                             * in LDS; otherwise the call falls back to RT_ENGINE_MEGAKERNEL and
                             * rt_counters.engine says so */
  RT_ENGINE_TIMING = 0x10   /* flag: time every kernel launch with HIP events (rt_counters *_ms) */
};

/* One scene object = SceneLoadObject{geometry, material} (scene/mod.rs:23-27).
 * The fields after p[] are book-2 ("The Next Week") extensions that the reference does not have
 * (SURVEY.md §0.1 config 5); all zero = a reference object.  Their semantics are DESIGN.md §10's
 * (parity unpinned: no reference implementation exists). */
typedef struct rt_object {
  int32_t geometry; /* RT_GEOM_* */
  int32_t material; /* index into rt_scene_desc.materials */
  /* Sphere  (geometry/sphere.rs:11-15): cx cy cz radius (radius may be negative: sphere.rs:48,54-60)
   * Rect    (geometry/rect.rs:45-52):   d1_min d1_max d2_min d2_max offset
   * RectBox (geometry/rect.rs:102-130): min.x min.y min.z max.x max.y max.z (sides derived as RectBox::new)
   * MovingSphere: center0 xyz, radius */
  double p[6];
  int32_t medium;     /* 1: a ConstantMedium whose boundary is this geometry (material: RT_MAT_ISOTROPIC) */
  int32_t transform;  /* 1: instance transform, world = Translate(offset) . RotateY(rotate_y_deg) . object */
  double q[5];        /* MovingSphere: center1 xyz, time0, time1 */
  double density;     /* ConstantMedium density (neg_inv_density = -1/density) */
  double rotate_y_deg;
  double offset[3];
} rt_object;

typedef struct rt_material {
  int32_t kind;      /* RT_MAT_* */
  int32_t texture;   /* albedo texture (Lambertian / DiffuseLight / FairyLight), -1 otherwise */
  double albedo[3];  /* Metal albedo (metal.rs:10-14) */
  double param;      /* Metal: fuzz, already clamped <= 1 (metal.rs:17-23); Dielectric: ir (dielectric.rs:10-13) */
} rt_material;

typedef struct rt_texture {
  int32_t kind;      /* RT_TEX_* */
  int32_t odd;       /* Checker: odd child texture index  (checker.rs:10-14) */
  int32_t even;      /* Checker: even child texture index */
  int32_t table;     /* Perlin: index into perlin tables; Image: index into images */
  double color[3];   /* Solid colour (solid.rs:5-21) */
  double scale;      /* Checker: size; Perlin: scale (perlin/mod.rs:143-153) */
} rt_texture;

/* Perlin tables (perlin/mod.rs:11-17): 256 non-normalised random vectors + 3 permutations. */
typedef struct rt_perlin_table {
  double ranfloat[256][3];
  int32_t perm_x[256];
  int32_t perm_y[256];
  int32_t perm_z[256];
} rt_perlin_table;

/* Decoded RGB8 image texture (image_texture.rs:15-17); row 0 = top, like image::DynamicImage. */
typedef struct rt_image {
  int32_t width;
  int32_t height;
  const uint8_t* rgb; /* width*height*3 bytes */
} rt_image;

/* Flattened SceneBuilder (scene/mod.rs:79-83) with textures already "loaded" and deduplicated
 * (TextureManager::load, texture/loader.rs:113-131).  Host-owned; borrowed for the call only. */
typedef struct rt_scene_desc {
  int32_t sky;            /* RT_SKY_* */
  double sky_color[3];    /* RT_SKY_FLAT colour */
  int32_t n_objects;
  const rt_object* objects;
  int32_t n_materials;
  const rt_material* materials;
  int32_t n_textures;
  const rt_texture* textures;
  int32_t n_perlin;
  const rt_perlin_table* perlin;
  int32_t n_images;
  const rt_image* images;
} rt_scene_desc;

/* Camera (camera/mod.rs:88-95) + CameraPosition (camera/mod.rs:63-70), as built by
 * CameraBuilder::build (camera/mod.rs:44-60) and CameraPosition::look_at (camera/mod.rs:72-86),
 * with the caller's `pos.focus_length = 10.0` override already applied (scenes.rs:209,229). */
typedef struct rt_camera {
  int32_t image_width;   /* Dimmensions.width */
  int32_t image_height;  /* Dimmensions.height */
  double height;         /* 2 tan(vfov/2) */
  double width;          /* aspect * height */
  double focal_length;
  int32_t has_lens;      /* lens_radius: Option<f64> */
  double lens_radius;
  double origin[3];
  double w[3], u[3], v[3];
  double focus_length;
  /* shutter interval (book-2 extension, absent from the reference): a path's ray time is
   * time0 + (time1 - time0) * U, U from its own counter-RNG stream; only moving spheres read it */
  double time0, time1;
} rt_camera;

/* Per-call render parameters (RenderSettings, argparse.rs:106-123, plus what the reference lacks). */
typedef struct rt_render_params {
  int32_t samples;      /* samples per pixel; 0 is treated as 1 (main.rs:75-80) */
  int32_t max_depth;    /* max_reflect: bounce limit of ray_color (render.rs:30) */
  uint64_t seed;        /* key of the counter-based RNG (the reference is unseeded: SURVEY.md §0) */
  int32_t tile_rank;    /* interleaved 8x8-tile sharding: this call renders tiles k with k % tile_world == tile_rank */
  int32_t tile_world;   /* 1 = whole frame */
  int32_t sample_chunk; /* samples per work unit (0 = automatic; >= samples gives in-order per-pixel sums).
                         * Automatic usually picks chunk < samples: each chunk is summed in order, then the
                         * chunk sums in chunk order — not render.rs:58-69's single running sum, so the
                         * frame differs from the in-order one by reassociation only (|d| <= 1e-12 |sum|,
                         * DESIGN.md §2).  The megakernel indexes a launch's work units (pixels x chunks) in 32 bits: a
                         * call with more runs in several sample passes (see scratch_mb).
                         * The automatic length depends on the pixels a call renders (its tiles) and on
                         * the device's CU count, so tile-sharded frames at different world sizes sum each
                         * pixel's chunks differently (bits differ within the reassociation bound); pass an
                         * explicit sample_chunk for frames that are bit-identical at every world size. */
  int32_t engine;       /* RT_ENGINE_* (0 = automatic), optionally | RT_ENGINE_TIMING */
  /* ABI 6: the call's sample range — SURVEY.md §8(b)'s "sample range" — and its scratch bound.
   * The call renders samples [sample_begin, sample_begin + sample_count) of every pixel (0 <= sample_begin,
   * range within [0, samples)); sample_count == 0 means "to samples".  The output holds the sums over the
   * range only.  The counter RNG is keyed by the global sample index, so ranges [0, k) and [k, S) render
   * exactly the samples of one [0, S) call (the pixel sums differ by reassociation only: the per-pixel
   * sum of two ranges is (sum of range 1) + (sum of range 2)).  Reference: render.rs:58-69's sample loop. */
  int32_t sample_begin;
  int32_t sample_count;
  /* multi-GPU entry points (rt_render_sharded / rt_render_multi): how the frame is split over the ranks,
   * RT_PARTITION_*; ignored by the single-device calls */
  int32_t partition;
  /* bound on the per-call partial-sum scratch in MiB (0 = default 8192).  A call whose [chunks][pixels][3]
   * f64 partial sums exceed it renders its chunks in consecutive sample passes, each reduced into the
   * output in chunk order — the same per-pixel additions in the same order as one pass, so the frame is
   * bit-identical for every bound. */
  int32_t scratch_mb;
} rt_render_params;

/* ABI 6: rt_render_params.partition (multi-GPU) */
enum {
  RT_PARTITION_AUTO = 0,    /* the measured default per world size */
  RT_PARTITION_TILES = 1,   /* interleaved 8x8 tiles (tile k -> rank k % world), gather of the packed tiles to
                             * rank 0: every pixel's sum is computed on one rank, so the frame equals the
                             * single-device frame whenever the unit length (sample_chunk) is the same */
  RT_PARTITION_SAMPLES = 2  /* every rank renders all pixels for its share of the sample range (rank r:
                             * [count*r/world, count*(r+1)/world) of it); the per-rank sums are exchanged by
                             * row bands (all-to-all), summed in rank order and gathered to rank 0:
                             * deterministic, equal to the single-device frame within reassociation */
};

typedef struct rt_scene_stats {
  int32_t n_objects;
  int32_t n_nodes;      /* BVH nodes (leaves included), like BboxTree.tree.len()+... */
  int32_t n_leaves;
  int32_t depth;        /* max root-to-leaf depth */
  int64_t device_bytes; /* scene bytes resident in HBM */
  /* ABI 4: the renderer's collapsed tree (the one rt_render* and RT_TRAVERSAL_RENDER walk) */
  int32_t n_nodes4;     /* 4-wide f32 nodes */
  int32_t wide_block;   /* 1: the trace kernel keeps the whole 4-wide tree in LDS (1024-thread blocks) */
  double origin_limit;  /* rays with max|origin| above this take the f64 re-test of the f32 node boxes */
} rt_scene_stats;

/* Counters of the last render call (deterministic for a given seed). */
typedef struct rt_counters {
  uint64_t samples;     /* paths started = pixels x spp */
  uint64_t segments;    /* ray_color loop iterations that traced a ray (hit + miss) */
  uint64_t node_visits; /* BVH child-box tests (4-wide trees: 4 per node visit); the 4-wide traversal of the
                         * megakernel / wavefront counts them only in the instrumented build (-DRT_PHASE_TIMING,
                         * DESIGN.md §5): 0 otherwise */
  uint64_t prim_tests;  /* primitive intersection calls (same condition) */
  double kernel_ms;     /* device time of the trace (all trace kernels of the frame, HIP events) */
  double reduce_ms;     /* device time of the partial-sum reduce kernel */
  int32_t engine;       /* RT_ENGINE_MEGAKERNEL, RT_ENGINE_WAVEFRONT or RT_ENGINE_SPLIT: the engine that ran */
  int32_t iterations;   /* wavefront: extend/shade/texture rounds (0 for the megakernel) */
  uint64_t slots;       /* wavefront: path slots in flight */
  double extend_ms;     /* wavefront + RT_ENGINE_TIMING: summed device time of wf_extend launches */
  double shade_ms;      /* ... wf_shade launches */
  double texture_ms;    /* ... wf_texture launches */
  int32_t sample_chunk; /* ABI 4: samples per work unit the call used (auto-sized when params.sample_chunk == 0;
                         * < samples means each pixel's sum is added up per chunk, then chunk sums in order) */
  int32_t n_chunks;     /* ceil(samples / sample_chunk) */
  /* ABI 6 */
  int32_t passes;        /* sample passes the call used (> 1 when the partial sums exceed scratch_mb) */
  int32_t trace_launches;/* trace-kernel launches of the call (one per pass; kernel_ms is their summed time) */
  uint64_t scratch_bytes;/* partial-sum scratch the call used */
} rt_counters;

typedef struct rt_ctx rt_ctx;

/* ---- library / device ---------------------------------------------------------------------- */
const char* rt_version(void);
int rt_device_count(int32_t* out);
int rt_create(int32_t device, rt_ctx** out);
int rt_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);

/* ---- scene (replaces SceneBuilder::finalize, scene/mod.rs:111-137) --------------------------- */
int rt_scene_upload(rt_ctx* ctx, const rt_scene_desc* scene, int32_t bvh_builder);
int rt_scene_stats_get(rt_ctx* ctx, rt_scene_stats* out);
/* ABI 6: 64-bit digest of the uploaded scene (its description and BVH builder; FNV-1a over every field),
 * and the same digest computed on the host from a description (no device needed).  Equal scenes give
 * equal digests; the multi-GPU calls compare them across ranks. */
int rt_scene_digest(rt_ctx* ctx, uint64_t* out);
int rt_scene_digest_host(const rt_scene_desc* scene, int32_t bvh_builder, uint64_t* out);

/* ---- rendering (replaces main.rs:92-126 + render.rs:17-70) ----------------------------------- */
/* Whole frame, blocking.  accum_host: [image_height][image_width][3] f64 per-pixel SUMS over the
 * samples (Image.data layout, image.rs:10-14), row 0 = bottom of the picture (image.rs:38). */
int rt_render(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* params, double* accum_host);

/* Rows [line_begin, line_end) only, blocking — the render_scanline (render.rs:49-57) granularity.
 * rows_host: [(line_end-line_begin)][image_width][3] sums; samples of row j identical to rt_render's. */
int rt_render_scanlines(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* params,
                        int32_t line_begin, int32_t line_end, double* rows_host);

/* Device-resident variants: asynchronous on `stream` (a hipStream_t, NULL = the ctx's own stream).
 * rt_render_device: accum_dev is [H][W][3] f64 in HBM; pixels of tiles not owned by this
 * (tile_rank, tile_world) are left untouched.
 * rt_render_tiles_device: packed output [n_tiles_rank][8][8][3] f64 (tile-local row 0 = lowest row),
 * for the multi-GPU gather; rt_unpack_tiles_device scatters a gathered [world][max_tiles][8][8][3]
 * buffer back into [H][W][3]. */
int rt_tile_layout(const rt_camera* cam, int32_t tile_world, int32_t* n_tiles_total, int32_t* max_tiles_per_rank);
int rt_render_device(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* params, double* accum_dev,
                     void* stream);
int rt_render_tiles_device(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* params,
                           double* packed_dev, void* stream);
int rt_unpack_tiles_device(rt_ctx* ctx, const rt_camera* cam, int32_t tile_world, const double* gathered_dev,
                           double* accum_dev, void* stream);
int rt_synchronize(rt_ctx* ctx);

/* Closest hit for a batch of rays, blocking — Hittable for Scene (scene/mod.rs:180-190) /
 * WorkspaceScene::hit_workspace (scene/mod.rs:152-164).  rays: [n][6] = origin xyz, direction xyz.
 * out[i].object = -1 on a miss; otherwise the HitRecord (geometry/hittable.rs:6-14) of object index. */
typedef struct rt_hit {
  int32_t object;
  int32_t front_face;
  double t;
  double point[3];
  double normal[3];
  double u, v;
} rt_hit;
int rt_scene_hit(rt_ctx* ctx, const double* rays, int32_t n, double t_min, double t_max, rt_hit* out);

/* ABI 4: the same query through a chosen traversal.
 *   RT_TRAVERSAL_BINARY: the 2-wide f64 tree (the reference's BboxTree as built; what rt_scene_hit walks);
 *   RT_TRAVERSAL_RENDER: the traversal the trace kernel runs — the 4-wide collapsed tree with conservative
 *     f32 (inflated) child boxes, exact f64 leaf re-tests and an f64 fallback for rays whose origin lies
 *     beyond rt_scene_stats.origin_limit, with nodes and primitives read from where the renderer reads them.
 * Both return the reference's closest hit (bbox_tree.rs:56-91 + hit2 + the object tests). */
enum { RT_TRAVERSAL_BINARY = 0, RT_TRAVERSAL_RENDER = 1 };
int rt_scene_hit_ex(rt_ctx* ctx, const double* rays, int32_t n, double t_min, double t_max, int32_t traversal,
                    rt_hit* out);

/* ABI 7: one iteration of ray_color's loop (render.rs:30-46) for each given ray, through the megakernel's
 * own device code — the render traversal (t in [0.001, inf)), the hit record, the material and its texture
 * (Perlin marble evaluated by the wave), the wave's sampler for the scatter's draws, and the shading —
 * with ray i on the path key (seed, pixel = i, sample, draw): emitted() and scatter() of the hit's material
 * (material_type.rs:51-79), or the sky on a miss (skybox/mod.rs:5-25), and the path's draw counter after
 * the segment.  A verification probe of the scatter semantics (tests/test_scatter_kat.py); book-2 ray time 0. */
typedef struct rt_probe {
  int32_t object;          /* closest object, -1: missed (the sky) */
  int32_t front_face;
  int32_t scattered;       /* scatter() returned Some: the path goes on along (origin, direction) */
  int32_t emits;           /* emitted() returned Some (or the sky): `emitted` holds it */
  uint32_t draw;           /* the path's draw counter after the segment */
  int32_t pad;
  double t, point[3], normal[3];
  double emitted[3];
  double attenuation[3];   /* scatter().attenuation */
  double origin[3], direction[3];  /* scatter().direction: the next ray */
} rt_probe;
int rt_probe_segment(rt_ctx* ctx, const double* rays, int32_t n, uint64_t seed, uint32_t sample, uint32_t draw,
                     rt_probe* out);

/* ---- multi-GPU (ABI 4) -------------------------------------------------------
 * The frame's 8x8 tiles are dealt round-robin over the ranks of a communicator (tile k -> rank
 * k % world); each rank renders its tiles into a packed buffer and RCCL gathers the packed buffers to
 * rank 0 over xGMI (ncclGather), which scatters them into the [H][W][3] image (RT_PARTITION_TILES), or
 * every rank renders all pixels for a share of the samples (RT_PARTITION_SAMPLES, see above).  The
 * counter RNG is keyed by the global pixel and sample, so a tile-sharded frame is bit-identical for every
 * world size given an explicit sample_chunk (the automatic chunk follows the rank's pixel count).  Every
 * ctx must hold the same scene and every rank must pass the same call arguments: every call of
 * rt_render_sharded all-gathers each rank's (scene digest, call key) — the key hashes the resolved partition
 * and sample range, samples, seed, max_depth, sample_chunk and the camera — so all ranks issue the same
 * collective sequence whatever their arguments, and checks the gathered words on the host: in the call,
 * before any collective of the frame, when this rank's key differs from the one the ranks last agreed on
 * (ranks changing scene or arguments together all fail there with RT_E_INVALID on a mismatch); otherwise
 * at the rank's next call, so a loop of frames needs no host round trip.  Misuse — one rank changing its
 * key alone — fails that rank in the call; its peers have already issued the frame's collectives, which it
 * never joins, so their stream waits (undefined from RCCL's side: do not rely on it).  A failed check poisons
 * the communicator: every later rt_render_sharded call on it returns RT_E_INVALID and issues no collective
 * (a new all-gather could otherwise be paired with a peer's pending frame collective); destroy it with
 * rt_comm_destroy and create a new one.  SHIRLEY_KEY_CHECK=sync
 * checks every call before the frame's collectives (every rank fails in the call itself, one host round
 * trip per call).  rt_render_multi compares the digests on the host.  Replaces the
 * reference's whole-machine rayon loop over scanlines (main.rs:92-126).  RCCL is loaded on first use
 * (dlopen "librccl.so.1": the copy already in the process if any); without it these calls return
 * RT_E_RCCL.
 *
 * One process per GPU: rank 0 calls rt_comm_unique_id, hands the id to every rank by any channel
 * (torch.distributed's store, MPI, a file), and each rank calls rt_comm_init_rank on its own ctx.
 * One process driving several GPUs: rt_render_multi (communicators created and cached per ctx set). */
#define RT_COMM_ID_BYTES 128
typedef struct rt_comm rt_comm;
int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
int rt_comm_init_rank(rt_ctx* ctx, const uint8_t id[RT_COMM_ID_BYTES], int32_t world, int32_t rank, rt_comm** out);
int rt_comm_destroy(rt_comm* comm);
/* One rank's share of a sharded frame, asynchronous on `stream` (NULL: the ctx's stream) after the
 * cross-rank check above: render the rank's share (params->partition: its tiles, or all pixels for its samples;
 * params->tile_rank / tile_world are ignored: the communicator's rank and size are used), exchange, and on
 * rank 0 write accum_dev ([H][W][3] f64 sums on its device; NULL on the other ranks).  The sample range of
 * params (sample_begin / sample_count) is the frame's; a sample partition splits it.  Every rank of the
 * communicator must make the call (a collective). */
int rt_render_sharded(rt_ctx* ctx, rt_comm* comm, const rt_camera* cam, const rt_render_params* params,
                      double* accum_dev, void* stream);
/* The whole frame on n devices from one process, blocking; accum_host as rt_render's ([H][W][3] sums, row
 * 0 = bottom).  ctxs[0] is the root; every ctx needs the same scene uploaded (the digests are compared
 * first: RT_E_INVALID on a mismatch).  params->partition as rt_render_sharded's.  n == 1 equals rt_render. */
int rt_render_multi(rt_ctx* const* ctxs, int32_t n, const rt_camera* cam, const rt_render_params* params,
                    double* accum_host);

/* Counters (segments etc.) of the most recent render call; blocks until it finished. */
int rt_counters_get(rt_ctx* ctx, rt_counters* out);

/* Host-only BVH inspection (no device needed): builds the tree rt_scene_upload would build.
 * Call with nodes = NULL to get *n_nodes, then again with room for that many.  Node layout follows
 * BboxTree.tree (bbox_tree.rs:10-26): leaf >= 0 is the object index, else lhs/rhs are node indices. */
typedef struct rt_bvh_node {
  double box[6]; /* min xyz, max xyz */
  int32_t leaf;
  int32_t lhs, rhs;
  int32_t pad;
} rt_bvh_node;
int rt_bvh_build_host(const rt_scene_desc* scene, int32_t bvh_builder, int32_t* n_nodes, rt_bvh_node* nodes,
                      int32_t* root);

/* Output stage on the host, exactly image::to_image (image.rs:31-44) + Color::to_pixel (color.rs:31-38):
 * c/samples -> sqrt -> (x*255.999) saturating to u8, row j -> output row H-1-j.  rgb8: [H][W][3], row 0 = top. */
int rt_tonemap(const double* accum, int32_t width, int32_t height, int32_t samples, uint8_t* rgb8);
/* The same on the device: accum_dev [H][W][3] sums -> rgb8_dev [H][W][3] with
 * row 0 = top, on `stream` (NULL: the context's stream), asynchronous.  Bit-identical to rt_tonemap. */
int rt_tonemap_device(rt_ctx* ctx, const double* accum_dev, int32_t width, int32_t height, int32_t samples,
                      uint8_t* rgb8_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SHIRLEY_RT_H */
