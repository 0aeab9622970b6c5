// trace.hip — MI355X (gfx950) path-tracing kernels for the reference's ray_color() hot path.
//
// Semantics follow the reference line by line (citations below); arithmetic is binary64 like the
// reference (core/math.rs:5) and the file is compiled with -ffp-contract=off (Rust never fuses).
//
// Execution model (MI355X-first):
//   * persistent waves: every lane owns one work unit = (pixel, chunk of samples) and runs the
//     reference's bounce loop one segment per iteration; a lane whose path ends starts its next
//     sample at once (path regeneration), a lane whose unit ends takes a new unit from the wave's
//     64-unit window (ballot + popcount rank, one global atomic per 64 units);
//   * units are enumerated tile-major (8x8 pixel tile x sample chunk x lane), so a fresh window
//     hands a wave 64 neighbouring pixels: coherent primary rays;
//   * 4-wide collapsed BVH with conservative f32 child boxes (160-B DNode4F) and exact f64 leaf
//     tests, nearest-first traversal, per-lane stack in LDS laid out [depth][lane] (conflict-free
//     at any depth); for scenes that fit, the nodes, primitives and Perlin tables live in LDS too
//     (one 1024-thread block per CU: 4 waves per SIMD at 128 VGPRs);
//   * Perlin marble octaves and rejection-sampling attempts of a segment are dealt across the whole
//     wave (marble_coop, random_in_unit_sphere_coop);
//   * per-unit partial sums go to HBM once; a reduce kernel sums chunks in order (deterministic).
#include "rt_device.h"

#include <algorithm>
#include <vector>

namespace rt {

// ------------------------------------------------------------------------------------------
// persistent trace kernel
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long lanemask_lt() {
  unsigned lane = __lane_id();
  return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

// LDS of a block: [n_lds_nodes x DNode][stack_depth x STRIDE int][stack_depth x STRIDE float]
__host__ __device__ inline size_t lds_bytes(int n_lds_nodes, int stack_depth, int stride) {
  return (size_t)n_lds_nodes * sizeof(DNode) + (size_t)stack_depth * stride * 8;
}

// THREADS = kTraceThreads (256-thread blocks, several per CU, at least 4 waves per SIMD: 128 VGPRs)
// or kTraceThreadsWide (one 1024-thread block per CU whose LDS holds the scene next to the stacks:
// 4 waves per SIMD, 128 VGPRs).  HIP's second launch-bounds argument is the minimum waves per SIMD.
// EXT: the scene has book-2 primitives; their code is compiled into separate
// instances so that reference scenes keep the kernel's register allocation.
#ifndef RT_KSCENE
#define RT_KSCENE 1
#endif
// Minimum waves per SIMD of the 256-thread instances (4 = 128 VGPRs: 3 and 5 measured slower);
// the book-2 ones at 3 (168 VGPRs: ~90 spilled VGPRs at 4; final_scene on them +27 %).
#ifndef RT_NARROW_WAVES
#define RT_NARROW_WAVES 4
#endif
constexpr int kNarrowWaves = RT_NARROW_WAVES;
#ifndef RT_NARROW_WAVES_EXT
#define RT_NARROW_WAVES_EXT 3
#endif

template <int THREADS, int MODE, bool EXT>
__global__ __launch_bounds__(THREADS, THREADS >= kTraceThreadsWide3 ? 1 : (EXT ? RT_NARROW_WAVES_EXT : kNarrowWaves))
void trace_kernel(KParams P) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  typedef typename Node4Sel<EXT>::T N4;
  N4* lds_nodes = reinterpret_cast<N4*>(lds_raw);
  DPrim* lds_prims = reinterpret_cast<DPrim*>(lds_raw + (size_t)P.scene.n_lds_nodes4 * sizeof(N4));
  const DPerlin* lds_perlin = (MODE == kSceneLds && P.scene.n_lds_perlin > 0)
                                  ? reinterpret_cast<const DPerlin*>(lds_prims + P.scene.n_lds_prims)
                                  : nullptr;
  unsigned char* stk_base = lds_raw + (size_t)P.scene.n_lds_nodes4 * sizeof(N4) +
                            (MODE == kSceneLds ? (size_t)P.scene.n_lds_prims * sizeof(DPrim) +
                                                     (size_t)P.scene.n_lds_perlin * sizeof(DPerlin) +
                                                     (size_t)P.scene.n_lds_mats * sizeof(DMat) +
                                                     (size_t)P.scene.n_lds_texs * sizeof(DTex)
                                               : 0);
  unsigned* stk = reinterpret_cast<unsigned*>(stk_base) + tid;  // [stack_depth4][THREADS] packed entries
  stage_nodes4<MODE>(P.scene, lds_nodes, lds_prims);
  // the material and texture tables: the scene-in-LDS block's copies (after the Perlin tables: the host
  // places the primitives in LDS only together with them), else global memory.  Unconditional per
  // instance, so the compiler reads the LDS copies with ds_read (a runtime choice made every read a FLAT
  // load).
  const DMat* mats = P.scene.mats;
  const DTex* texs = P.scene.texs;
  if constexpr (MODE == kSceneLds) {
    mats = reinterpret_cast<const DMat*>(reinterpret_cast<const DPerlin*>(lds_prims + P.scene.n_lds_prims) +
                                         P.scene.n_lds_perlin);
    texs = reinterpret_cast<const DTex*>(mats + P.scene.n_lds_mats);
  }

  const DCamera& C = P.cam;
  const DWork& W = P.work;
  const uint64_t seed = W.seed;
  const int lane = __lane_id();

  // wave-uniform window of unit indices
  unsigned long long w_next = 0, w_end = 0;
  bool exhausted = false;
  // units are taken from per-block segments of the unit space (stealing from other segments once the
  // block's is empty) when DWork.n_segs != 0, else from one global queue.
  // the block's segment, XCD-major: blocks are dealt round-robin to the 8 XCDs, so block b (on XCD
  // b % 8) owns segment (b % 8) * ceil(n / 8) + b / 8 — an XCD's blocks own adjacent segments
  uint32_t seg;
  {
    const uint32_t per_xcd = (W.n_segs + 7u) / 8u, s0 = (blockIdx.x % 8u) * per_xcd + blockIdx.x / 8u;
    seg = s0 < W.n_segs ? s0 : blockIdx.x % max(W.n_segs, 1u);
  }

  // lane state
  // (kept lean: every loop-carried VGPR here competes with the 128-VGPR budget of 4 waves per SIMD)
  bool has_unit = false, active = false;
  uint32_t pxy = 0;   // px | py << 16 of the unit's pixel (the host keeps width, height <= 65535)
  int s_end = 0;      // the unit's samples are [.., s_end); the current one is rng.sample
  uint32_t part_index = 0;  // partial-buffer slot of the unit (the host keeps slots < 2^32)
  v3 sum = V(0, 0, 0), o = V(0, 0, 0), d = V(0, 0, 0), att = V(0, 0, 0), em = V(0, 0, 0);
  int depth_left = 0;
  Rng rng{0, 0, 0, 0, 0};
  unsigned long long n_seg = 0, n_samp = 0;  // wave-uniform (SGPRs): popcounts of ballots
  unsigned visits = 0, ptests = 0;           // per lane; flushed to the counters before 2^31

#ifdef RT_PHASE_TIMING
  // wave-uniform clock stamps at wave-uniform points of the loop (SGPR sums): the iteration's time by
  // phase (kPh* buckets), plus the traversal step statistics
  unsigned long long ph_t[kPhBuckets] = {}, ph_last = clock64(), ph_lane_steps = 0, ph_wave_steps = 0;
#define PH_STAMP(b)                               \
  do {                                            \
    const unsigned long long ph_now = clock64();  \
    ph_t[b] += ph_now - ph_last;                  \
    ph_last = ph_now;                             \
  } while (0)
#else
#define PH_STAMP(b) \
  do {              \
  } while (0)
#endif
#ifdef RT_TIMELINE
  const unsigned wave_gid = blockIdx.x * (THREADS / kWave) + tid / kWave;
  bool ph_exh_seen = false;
  if (lane == 0 && wave_gid < (unsigned)kTimelineWaves) g_wave_t0[wave_gid] = __builtin_amdgcn_s_memrealtime();
#endif
  // One iteration: (1) a ray_color segment for every lane holding a path (closest hit, record,
  // material); (2) lanes whose path ends here (sky or a light) or that hold none take the next sample
  // of their unit or a new unit; (3) one wave-wide sampler draws everything the iteration needs — the
  // scatters' unit-sphere points, the dielectrics' uniforms and the new samples' jitter + lens points;
  // (4) shading; ended lanes add their radiance and publish finished units; new samples' camera rays.
  for (;;) {
#if defined(RT_PHASE_TIMING) && !defined(RT_PHASE_NO_EVENTS)
    const unsigned long long ph_before = ph_lane_steps;
#endif
    // the scene record: the kernel argument's copy for every instance.  (Round 5 had the book-2 instances
    // re-read it from the pass's KBlock with scalar loads each iteration, +0.2 % then; with the extended
    // objects' tests moved out of the traversal loop the argument copy is +1.1 % on final_scene:
    // 1675 / 1676 vs 1657 / 1655 Msamples/s, gpurun_out/r06n)
    const DScene& S = P.scene;
    // 1. one ray_color iteration (render.rs:30-46): closest hit and hit record, the material and the
    // texture leaf of a diffuse / emitting material
    bool hit = false, need_pn = false, need_r = false;
    int prim = -1, face = -1, leaf = -1, mat = 0, ptab = 0, mk = -1;
    double t_best = __builtin_inf(), psc = 0.0;
    Hit h;
    h.point = V(0.0, 0.0, 0.0);
    h.normal = h.point;
    h.t = h.u = h.v = 0.0;
    h.front_face = false;
    PH_COUNT(6);
    n_seg += __popcll(__ballot(active));
    if (active) {
      prim = traverse4<THREADS, MODE, EXT>(S, lds_nodes, lds_prims, o, d, 0.001, t_best, face, stk, rng, seed, visits,
                                      ptests RT_STAT_ARG(ph_lane_steps));
#ifdef RT_PHASE_TIMING
    }  // (instrumented build: the traversal's stamp at a wave-uniform point)
    PH_STAMP(kPhTrav);
    {
#endif
      if (prim >= 0) {
        PH_COUNT(15);
        hit = true;
        const DPrim pr = (MODE == kSceneLds) ? lds_prims[prim] : S.prims[prim];  // (LDS copy when resident)
        hit_record<false, EXT>(S, pr, face, o, d, t_best, rng, seed, h);
        mat = pr.material;
        mk = mats[mat].kind;
        need_r = mk == RT_MAT_LAMBERTIAN || mk == RT_MAT_METAL || mk == RT_MAT_FAIRY_LIGHT || mk == RT_MAT_ISOTROPIC;
        if (mk == RT_MAT_LAMBERTIAN || mk == RT_MAT_FAIRY_LIGHT || mk == RT_MAT_DIFFUSE_LIGHT || mk == RT_MAT_ISOTROPIC) {
          leaf = resolve_texture_t(texs, mats[mat].tex, h.point);
          const DTex& tx = texs[leaf];
          if (tx.kind == RT_TEX_PERLIN) {
            need_pn = true;
            ptab = tx.table;
            psc = tx.scale;
          }
        }
      }
    }
    PH_STAMP(kPhRecord);
    // 2. the path ends at this segment when it misses (the sky) or meets a material that does not
    // scatter (diffuse light): known before shading, so the lane's next sample starts in this iteration
    const bool ends = active && (!hit || mk == RT_MAT_DIFFUSE_LIGHT);
    const bool free_lane = !active || ends;
    // a unit whose last sample ends here is published after shading (its sum is complete then)
    bool publish = false;
    uint32_t pub_index = 0;
    if (free_lane && has_unit && rng.sample + 1u >= (uint32_t)s_end) {
      publish = true;
      pub_index = part_index;
      has_unit = false;
    }
    // lanes without a unit take one from the wave's window (one global atomic per 64 units)
    bool need = free_lane && !has_unit;
    unsigned long long mask = __ballot(need);
    if (mask != 0ull && !exhausted) {
      unsigned long long k = __popcll(mask);
      unsigned long long rank = __popcll(mask & lanemask_lt());
      unsigned long long avail = w_end - w_next;
      unsigned long long idx;
      unsigned win = kSegmentWindow;  // units of the window taken below
      if (avail >= k) {
        idx = w_next + rank;
        w_next += k;
      } else {
        KBlk* kb = kblock(P.kconst);  // (the queue's pointers and sizes, read with scalar loads here)
        unsigned long long nb = kb->work.n_units;
        if (kb->work.n_segs != 0u) {
        // the block's segment (consecutive chunks of neighbouring tiles: coherent lanes, the same
        // subtrees in this XCD's L2), then any segment that still holds units: the 64 lanes read 64
        // candidates' counters at once (device-coherent atomic loads) and the wave takes the first
        // non-empty one.  A failed take means that segment is now empty for good (counters only grow),
        // so the search ends after at most n_segs failures.
        unsigned* ctr = reinterpret_cast<unsigned*>(kb->unit_counter);
        for (;;) {
          unsigned off = 0;
          if (lane == 0) off = atomicAdd(ctr + seg, kSegmentWindow);
          off = (unsigned)__builtin_amdgcn_readfirstlane((int)off);
          const uint32_t seg_len = kb->work.seg_len;
          const unsigned long long n_units = kb->work.n_units;
          if (off < seg_len && (unsigned long long)seg * seg_len + off < n_units) {
            nb = (unsigned long long)seg * seg_len + off;
            break;
          }
          bool found = false;
          const uint32_t n_segs = kb->work.n_segs;
          for (uint32_t base = 0; base < n_segs; base += kWave) {
            uint32_t cand = seg + 1u + base + (uint32_t)lane;
            if (cand >= n_segs) cand -= n_segs;
            bool has = false;
            if (base + (uint32_t)lane < n_segs) {
              const unsigned o = __hip_atomic_load(ctr + cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              has = o < seg_len && (unsigned long long)cand * seg_len + o < n_units;
            }
            const unsigned long long m = __ballot(has);
            if (m != 0ull) {
              seg = (uint32_t)__builtin_amdgcn_readlane((int)cand, (int)__builtin_ctzll(m));
              found = true;
              break;
            }
          }
          if (!found) break;
        }
        } else {  // one shared queue (short units: DWork.n_segs = 0), q_window units per atomic (plan.h)
          win = kb->work.q_window;
          nb = 0;
          if (lane == 0) nb = atomicAdd(kb->unit_counter, (unsigned long long)win);
          nb = ((unsigned long long)__builtin_amdgcn_readfirstlane((int)(nb >> 32)) << 32) |
               (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)nb);
        }
        idx = (rank < avail) ? (w_next + rank) : (nb + (rank - avail));
        w_next = nb + (k - avail);
        w_end = nb + win;
        if (nb >= W.n_units) exhausted = true;
      }
      if (need && idx < W.n_units) {
        KBlk* kb = kblock(P.kconst);
        // unit -> (local tile, chunk, lane-in-tile); tile-major so a window = 64 neighbours.  32-bit
        // quotients (the host keeps n_units < 2^32): far cheaper than 64-bit ones.  The work
        // descriptor and the image size are read here with scalar loads, like the camera below.
        KWork* kw = &kb->work;
        KCamera* kc = &kb->cam;
        const uint32_t pt = (uint32_t)kw->n_chunks * (uint32_t)kTilePixels, i32 = (uint32_t)idx;
        const uint32_t lt = udiv(i32, UDiv{kw->div_unit_tile.m, kw->div_unit_tile.s1, kw->div_unit_tile.s2});  // i32 / pt
        const uint32_t g32 = lt * (uint32_t)kw->tile_world + (uint32_t)kw->tile_rank;
        const uint32_t y32 = udiv(g32, UDiv{kw->div_tiles_x.m, kw->div_tiles_x.s1, kw->div_tiles_x.s2});  // g32 / tiles_x
        const uint32_t rem = i32 - lt * pt;
        const int tx = (int)(g32 - y32 * (uint32_t)kw->tiles_x);
        const int ty = kw->ty0 + (int)y32;
        int chunk = (int)(rem / kTilePixels);
        int lp = (int)(rem % kTilePixels);
        const int px = tx * kTile + (lp % kTile);
        const int py = ty * kTile + (lp / kTile);
        if (px < kc->width && py < kc->height) {
          PH_COUNT(10);
          has_unit = true;
          const int s0 = kw->sample_base + chunk * kw->chunk;
          s_end = min(kw->samples, s0 + kw->chunk);
          rng.sample = (uint32_t)s0 - 1u;  // advanced before each sample (wraps to s0)
          rng.pixel = (uint32_t)py * (uint32_t)kc->width + (uint32_t)px;
          pxy = (uint32_t)px | ((uint32_t)py << 16);
          part_index = (uint32_t)chunk * ((uint32_t)kw->n_tiles_rank * (uint32_t)kTilePixels) +
                       lt * (uint32_t)kTilePixels + (uint32_t)lp;
        }
      }
    }
    // a free lane holding a unit starts its next sample (render.rs:60-65): draws from 0 again
    const bool regen = free_lane && has_unit;
    n_samp += __popcll(__ballot(regen));
    if (regen) {
      rng.sample += 1u;
      rng.draw = 0;
    }
    PH_STAMP(kPhRegen);
    // 3. Perlin marble values for the lanes that need one, by the whole wave (wave-uniform)
    const double pn = lds_perlin ? marble_coop((LdsPerlin*)lds_perlin, need_pn, ptab, psc, h.point)
                                 : marble_coop(S.perlin, need_pn, ptab, psc, h.point);
    PH_STAMP(kPhMarble);
    // every draw of the iteration, by the wave: the scatter's random_in_unit_sphere, the dielectric's
    // uniform, a new sample's jitter and lens point
    const bool scat = active && !ends;
    const int dk = regen ? kDrawCam
                         : (scat && need_r) ? kDrawSphere : (scat && mk == RT_MAT_DIELECTRIC) ? kDrawDiel : kDrawNone;
    double jx = 0.0, jy = 0.0;
    const v3 rs = draws_coop(rng, seed, dk, C.has_lens != 0, pxy, jx, jy);
    // the one normalisation a lane's shading needs, for all lanes at once: unit(r) for a lambertian /
    // fairy light scatter, unit(d) for dielectric, metal and the sky (others: a dummy)
    const v3 un = unit_fast(!active ? V(1.0, 1.0, 1.0) : (scat && need_r && mk != RT_MAT_METAL) ? rs : d);
    PH_STAMP(kPhDraws);
    // 4. emitted + scatter (render.rs:31-45) or the sky; an ended lane's o, d are free once un holds
    // unit(d), so its new sample's camera ray is formed first
    if (regen) {
      PH_COUNT(11);
      // the camera read with scalar loads here (an opaque copy of its address keeps them from being
      // hoisted): held in SGPRs across the loop it spills to VGPR lanes, ~66 v_readlane per iteration
      camera_ray_drawn(kblock(P.kconst)->cam, jx, jy, rs, o, d);
    }
    PH_STAMP(kPhCamera);
    if (active) {
      bool alive, has_emit = false;
      v3 mul = V(1.0, 1.0, 1.0), emit = V(0.0, 0.0, 0.0);
      if (hit) {
        const DMat& m = mats[mat];  // (fields read where used: a copy loaded them all up front and spilled them)
        alive = shade_factor(S, texs, m, leaf, pn, rs, un, rng, o, d, h, prim, face, mul, emit, has_emit);
      } else {
        PH_COUNT(20);
#if RT_KSCENE
        // the sky's kind and colour read with scalar loads here, like the camera (held in SGPRs across
        // the loop they spill to VGPR lanes)
        emit = sky_unit(kblock(P.kconst)->scene, un);
#else
        emit = sky_unit(S, un);
#endif
        has_emit = true;
        alive = false;
      }
      // the path's throughput and radiance, read and written once per segment
      if (has_emit) em = em + hmul(att, emit);
      att = hmul(att, mul);
      if (alive) alive = --depth_left > 0;
      if (!alive) {
        sum = sum + em;  // c += ray_color(...)
        active = false;
      }
    }
    PH_STAMP(kPhShade);
    // a finished unit publishes its in-order sample sum (render.rs:58-69: *buf_c = c)
    if (publish) {
      PH_COUNT(24);
      double* dst = kblock(P.kconst)->partial + (size_t)pub_index * 3;
      dst[0] = sum.x;
      dst[1] = sum.y;
      dst[2] = sum.z;
      sum = V(0.0, 0.0, 0.0);
    }
    if (regen) {
      att = V(1.0, 1.0, 1.0);
      em = V(0.0, 0.0, 0.0);
      depth_left = kblock(P.kconst)->work.max_depth;  // >= 1: max_depth == 0 frames are written by render_window itself
      active = true;
    }
    PH_STAMP(kPhTail);
#ifdef RT_TIMELINE
    if (exhausted && !ph_exh_seen) {
      ph_exh_seen = true;
      if (lane == 0 && wave_gid < (unsigned)kTimelineWaves) g_wave_tx[wave_gid] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    // done when no lane holds a path or a unit and the pool is drained (a lane that fails to get a
    // unit while the pool is not drained — e.g. an edge tile's unit outside the image — retries)
    if (exhausted && !__any(active || has_unit)) break;
#if defined(RT_PHASE_TIMING) && !defined(RT_PHASE_NO_EVENTS)
    {
      unsigned dl = (unsigned)(ph_lane_steps - ph_before);  // this lane's steps (0 when idle)
      if (dl > 0) atomicAdd(&g_visit_hist[min(dl, 63u)], 1ull);
      for (int off = 32; off > 0; off >>= 1) dl = max(dl, (unsigned)__shfl_xor((int)dl, off));
      ph_wave_steps += dl;  // the wave's loop iterations = its slowest lane's steps
      if (lane == 0 && dl > 0) atomicAdd(&g_wave_visit_hist[min(dl, 63u)], 1ull);
    }
#endif
    if (visits > (1u << 30) || ptests > (1u << 30)) {  // (never within a frame of today's sizes)
      DCounters* cs = kblock(P.kconst)->counters + (blockIdx.x % kCounterSlots);
      atomicAdd(&cs->node_visits, (unsigned long long)visits);
      atomicAdd(&cs->prim_tests, (unsigned long long)ptests);
      visits = ptests = 0;
    }
  }
#ifdef RT_TIMELINE
  if (lane == 0 && wave_gid < (unsigned)kTimelineWaves) g_wave_t1[wave_gid] = __builtin_amdgcn_s_memrealtime();
#endif
  // wave-reduce the per-lane counters, one atomic per wave
  unsigned long long n_vis = visits, n_pt = ptests;
  for (int off = 32; off > 0; off >>= 1) {
    n_vis += __shfl_down(n_vis, off);
    n_pt += __shfl_down(n_pt, off);
  }
#ifdef RT_PHASE_TIMING
  for (int off = 32; off > 0; off >>= 1) ph_lane_steps += __shfl_down(ph_lane_steps, off);
  if (lane == 0) atomicAdd(&kblock(P.kconst)->counters[blockIdx.x % kCounterSlots].pad[kPhLaneSteps], ph_lane_steps);
#endif
  if (lane == 0) {
    DCounters* cs = kblock(P.kconst)->counters + (blockIdx.x % kCounterSlots);
    atomicAdd(&cs->segments, n_seg);
    atomicAdd(&cs->samples, n_samp);
    atomicAdd(&cs->node_visits, n_vis);
    atomicAdd(&cs->prim_tests, n_pt);
#ifdef RT_PHASE_TIMING
    for (int b = 0; b < kPhBuckets; ++b)
      if (b != kPhLaneSteps && b != kPhWaveSteps) atomicAdd(&cs->pad[b], ph_t[b]);
    atomicAdd(&cs->pad[kPhWaveSteps], ph_wave_steps);
#endif
  }
}

// Sum the per-chunk partials of each pixel in chunk order and write the Image.data layout
// (row 0 = bottom, image.rs:10-14) or the packed tile layout used by the multi-GPU gather.
// accumulate: a later sample pass of the same call — the sum starts from the value the earlier passes
// left in `out` and goes on adding chunks in order, so the additions are exactly one pass's.
__global__ __launch_bounds__(256) void reduce_kernel(const double* __restrict__ partial, int n_chunks,
                                                     int n_tiles_rank, int tiles_x, int ty0, int tile_rank,
                                                     int tile_world, int width, int row0, int row1, int packed,
                                                     int accumulate, double* __restrict__ out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long n_pix = (long long)n_tiles_rank * kTilePixels;
  if (i >= n_pix) return;
  long long lt = i / kTilePixels;
  int lp = (int)(i % kTilePixels);
  long long gt = lt * tile_world + tile_rank;
  int px = (int)(gt % tiles_x) * kTile + lp % kTile;
  int py = (ty0 + (int)(gt / tiles_x)) * kTile + lp / kTile;
  bool inside = px < width && py >= row0 && py < row1;
  double r = 0.0, g = 0.0, b = 0.0;
  const long long o = packed ? i * 3 : ((long long)(py - row0) * width + px) * 3;
  if (accumulate && (packed || inside)) {
    r = out[o + 0];
    g = out[o + 1];
    b = out[o + 2];
  }
  if (inside) {
    // (unrolled: the loads of 8 chunks in flight at once — a sharded frame's reduce runs few waves per
    // CU over many chunks; the additions stay in chunk order)
#pragma unroll 8
    for (int c = 0; c < n_chunks; ++c) {
      const double* p = partial + ((long long)c * n_pix + i) * 3;
      r += p[0];
      g += p[1];
      b += p[2];
    }
  }
  if (packed || inside) {
    out[o + 0] = r;
    out[o + 1] = g;
    out[o + 2] = b;
  }
}

// Sample-partitioned frames (RT_PARTITION_SAMPLES): a rank's row band holds one partial band per rank,
// parts[r][i]; the band's sums are added in rank order (deterministic for any arrival order).
__global__ __launch_bounds__(256) void sum_parts_kernel(const double* __restrict__ parts, int n_parts, long long n,
                                                        double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = parts[i];
  for (int r = 1; r < n_parts; ++r) s += parts[(long long)r * n + i];
  out[i] = s;
}

// image.rs:31-44 to_image + color.rs:31-38 to_pixel on the device: per channel c * (1/S), sqrt,
// * 255.999 and Rust's saturating `as u8` (NaN -> 0); image row j becomes output row H-1-j.
// One thread per output byte (coalesced stores).
__global__ __launch_bounds__(256) void tonemap_kernel(const double* __restrict__ accum, int width, int height,
                                                      double inv, uint8_t* __restrict__ rgb8) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)width * height * 3;
  if (i >= n) return;
  const long long row = i / ((long long)width * 3), rest = i - row * width * 3;
  const double y = sqrt(accum[((long long)(height - 1 - row) * width) * 3 + rest] * inv) * 255.999;
  rgb8[i] = (y != y || y <= 0.0) ? (uint8_t)0 : (y >= 255.0 ? (uint8_t)255 : (uint8_t)y);
}

// Scatter a gathered [world][max_tiles][64][3] buffer into the [H][W][3] image.
__global__ __launch_bounds__(256) void unpack_kernel(const double* __restrict__ gathered, int world, int max_tiles,
                                                     int n_tiles_total, int tiles_x, int width, int height,
                                                     double* __restrict__ out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)world * max_tiles * kTilePixels;
  if (i >= total) return;
  int lp = (int)(i % kTilePixels);
  long long t = i / kTilePixels;
  int lt = (int)(t % max_tiles);
  int r = (int)(t / max_tiles);
  long long gt = (long long)lt * world + r;
  if (gt >= n_tiles_total) return;
  int px = (int)(gt % tiles_x) * kTile + lp % kTile;
  int py = (int)(gt / tiles_x) * kTile + lp / kTile;
  if (px >= width || py >= height) return;
  long long o = ((long long)py * width + px) * 3;
  out[o + 0] = gathered[i * 3 + 0];
  out[o + 1] = gathered[i * 3 + 1];
  out[o + 2] = gathered[i * 3 + 2];
}

// Closest hit for a batch of rays (rt_scene_hit): one lane per ray, same traversal + record code.
struct HitOut {
  int32_t object, front_face;
  double t, point[3], normal[3], u, v;
};
template <int MODE>
__global__ __launch_bounds__(kHitThreads) void hit_kernel(DScene S, const double* __restrict__ rays, int n,
                                                          double t_min, double t_max, HitOut* __restrict__ out) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  DNode* lds_nodes = reinterpret_cast<DNode*>(lds_raw);
  unsigned char* stk_base = lds_raw + (size_t)S.n_lds_nodes * sizeof(DNode);
  int* stk_node = reinterpret_cast<int*>(stk_base) + tid;
  float* stk_t = reinterpret_cast<float*>(stk_base + (size_t)S.stack_depth * kHitThreads * 4) + tid;
  stage_nodes<MODE>(S, lds_nodes);
  int i = blockIdx.x * kHitThreads + tid;
  if (i >= n) return;
  v3 o = V(rays[i * 6 + 0], rays[i * 6 + 1], rays[i * 6 + 2]);
  v3 d = V(rays[i * 6 + 3], rays[i * 6 + 4], rays[i * 6 + 5]);
  double t_best = t_max;
  int face = -1;
  unsigned visits = 0, ptests = 0;
  // side-stream key of a free ray (book-2 media): pixel = ray index, sample 0, draw 0, seed 0
  const Rng rk{(uint32_t)i, 0u, 0u, 0u, 0u};
  int prim = traverse<kHitThreads, MODE, true>(S, lds_nodes, o, d, t_min, t_best, face, rk, 0ull, stk_node, stk_t, visits,
                                         ptests);
  HitOut r{};
  r.object = prim;
  if (prim >= 0) {
    const DPrim pr = S.prims[prim];
    Hit h;
    hit_record<true, true>(S, pr, face, o, d, t_best, rk, 0ull, h);
    r.front_face = h.front_face ? 1 : 0;
    r.t = h.t;
    r.point[0] = h.point.x; r.point[1] = h.point.y; r.point[2] = h.point.z;
    r.normal[0] = h.normal.x; r.normal[1] = h.normal.y; r.normal[2] = h.normal.z;
    r.u = h.u;
    r.v = h.v;
  }
  out[i] = r;
}

// Closest hit for a batch of rays through the traversal the renderer runs (rt_scene_hit_ex with
// RT_TRAVERSAL_RENDER): the 4-wide tree with conservative f32 (inflated) child boxes, exact f64 leaf
// re-tests and the f64 fallback for far origins (traverse4), with nodes / primitives read from the
// place trace_kernel reads them (MODE) and the trace kernel's EXT instance.  One lane per ray; the
// hit record is rebuilt like hit_kernel's.
template <int MODE, bool EXT>
__global__ __launch_bounds__(kHitThreads) void hit4_kernel(DScene S, const double* __restrict__ rays, int n,
                                                           double t_min, double t_max, HitOut* __restrict__ out) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  typedef typename Node4Sel<EXT>::T N4;
  N4* lds_nodes = reinterpret_cast<N4*>(lds_raw);
  DPrim* lds_prims = reinterpret_cast<DPrim*>(lds_raw + (size_t)S.n_lds_nodes4 * sizeof(N4));
  unsigned char* stk_base = lds_raw + (size_t)S.n_lds_nodes4 * sizeof(N4) +
                            (MODE == kSceneLds ? (size_t)S.n_lds_prims * sizeof(DPrim) +
                                                     (size_t)S.n_lds_perlin * sizeof(DPerlin) +
                                                     (size_t)S.n_lds_mats * sizeof(DMat) +
                                                     (size_t)S.n_lds_texs * sizeof(DTex)
                                               : 0);
  unsigned* stk = reinterpret_cast<unsigned*>(stk_base) + tid;
  stage_nodes4<MODE>(S, lds_nodes, lds_prims);
  const int i = blockIdx.x * kHitThreads + tid;
  if (i >= n) return;
  const v3 o = V(rays[i * 6 + 0], rays[i * 6 + 1], rays[i * 6 + 2]);
  const v3 d = V(rays[i * 6 + 3], rays[i * 6 + 4], rays[i * 6 + 5]);
  double t_best = t_max;
  int face = -1;
  unsigned visits = 0, ptests = 0;
  const Rng rk{(uint32_t)i, 0u, 0u, 0u, 0u};  // side-stream key of a free ray, as hit_kernel's
#ifdef RT_PHASE_TIMING
  unsigned long long steps = 0;
#endif
  const int prim = traverse4<kHitThreads, MODE, EXT>(S, lds_nodes, lds_prims, o, d, t_min, t_best, face, stk, rk, 0ull,
                                                      visits, ptests RT_STAT_ARG(steps));
  HitOut r{};
  r.object = prim;
  if (prim >= 0) {
    const DPrim pr = S.prims[prim];
    Hit h;
    hit_record<true, true>(S, pr, face, o, d, t_best, rk, 0ull, h);
    r.front_face = h.front_face ? 1 : 0;
    r.t = h.t;
    r.point[0] = h.point.x; r.point[1] = h.point.y; r.point[2] = h.point.z;
    r.normal[0] = h.normal.x; r.normal[1] = h.normal.y; r.normal[2] = h.normal.z;
    r.u = h.u;
    r.v = h.v;
  }
  out[i] = r;
}

// rt_probe_segment: one ray_color iteration (render.rs:30-46) per given ray through trace_kernel's own
// steps 1, 3 and 4 for a lane that holds a path — the render traversal, the hit record, the material and
// its texture leaf, the wave's marble and sampler, the one normalisation, shade_factor (or the sky) — on
// the path key (seed, pixel = ray index, sample, draw).  Lanes past n take part in the wave-wide steps
// idle, like a megakernel lane without a path.
struct ProbeOut {
  int32_t object, front_face, scattered, emits;
  uint32_t draw;
  int32_t pad;
  double t, point[3], normal[3], emitted[3], attenuation[3], origin[3], direction[3];
};
static_assert(sizeof(ProbeOut) == 176, "ProbeOut is rt_probe (include/shirley_rt.h)");
template <int MODE, bool EXT>
__global__ __launch_bounds__(kHitThreads) void probe_kernel(DScene S, const double* __restrict__ rays, int n,
                                                            uint64_t seed, uint32_t sample, uint32_t draw0,
                                                            ProbeOut* __restrict__ out) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  typedef typename Node4Sel<EXT>::T N4;
  N4* lds_nodes = reinterpret_cast<N4*>(lds_raw);
  DPrim* lds_prims = reinterpret_cast<DPrim*>(lds_raw + (size_t)S.n_lds_nodes4 * sizeof(N4));
  const DPerlin* lds_perlin = (MODE == kSceneLds && S.n_lds_perlin > 0)
                                  ? reinterpret_cast<const DPerlin*>(lds_prims + S.n_lds_prims)
                                  : nullptr;
  unsigned char* stk_base = lds_raw + (size_t)S.n_lds_nodes4 * sizeof(N4) +
                            (MODE == kSceneLds ? (size_t)S.n_lds_prims * sizeof(DPrim) +
                                                     (size_t)S.n_lds_perlin * sizeof(DPerlin) +
                                                     (size_t)S.n_lds_mats * sizeof(DMat) +
                                                     (size_t)S.n_lds_texs * sizeof(DTex)
                                               : 0);
  unsigned* stk = reinterpret_cast<unsigned*>(stk_base) + tid;
  stage_nodes4<MODE>(S, lds_nodes, lds_prims);
  const int i = blockIdx.x * kHitThreads + tid;
  const bool active = i < n;
  v3 o = V(0.0, 0.0, 0.0), d = V(1.0, 1.0, 1.0);
  if (active) {
    o = V(rays[i * 6 + 0], rays[i * 6 + 1], rays[i * 6 + 2]);
    d = V(rays[i * 6 + 3], rays[i * 6 + 4], rays[i * 6 + 5]);
  }
  Rng rng{(uint32_t)i, sample, draw0, 0u, 0u};
  if (draw0 & 1u) {  // an odd counter reads the odd half of block draw0 / 2 from the cache
    uint64_t e0, e1;
    philox_block(seed, rng.pixel, rng.sample, draw0 >> 1, e0, e1);
    rng.c2 = (uint32_t)e1;
    rng.c3 = (uint32_t)(e1 >> 32);
  }
  unsigned visits = 0, ptests = 0;
#ifdef RT_PHASE_TIMING
  unsigned long long steps = 0;
#endif
  // step 1 (trace_kernel): closest hit, record, material, texture leaf
  bool hit = false, need_pn = false, need_r = false;
  int prim = -1, face = -1, leaf = -1, mat = 0, ptab = 0, mk = -1;
  double t_best = __builtin_inf(), psc = 0.0;
  Hit h;
  h.point = V(0.0, 0.0, 0.0);
  h.normal = h.point;
  h.t = h.u = h.v = 0.0;
  h.front_face = false;
  if (active) {
    prim = traverse4<kHitThreads, MODE, EXT>(S, lds_nodes, lds_prims, o, d, 0.001, t_best, face, stk, rng, seed, visits,
                                              ptests RT_STAT_ARG(steps));
    if (prim >= 0) {
      hit = true;
      const DPrim pr = (MODE == kSceneLds) ? lds_prims[prim] : S.prims[prim];
      hit_record<false, EXT>(S, pr, face, o, d, t_best, rng, seed, h);
      mat = pr.material;
      mk = S.mats[mat].kind;
      need_r = mk == RT_MAT_LAMBERTIAN || mk == RT_MAT_METAL || mk == RT_MAT_FAIRY_LIGHT || mk == RT_MAT_ISOTROPIC;
      if (mk == RT_MAT_LAMBERTIAN || mk == RT_MAT_FAIRY_LIGHT || mk == RT_MAT_DIFFUSE_LIGHT || mk == RT_MAT_ISOTROPIC) {
        leaf = resolve_texture(S, S.mats[mat].tex, h.point);
        const DTex& tx = S.texs[leaf];
        if (tx.kind == RT_TEX_PERLIN) {
          need_pn = true;
          ptab = tx.table;
          psc = tx.scale;
        }
      }
    }
  }
  const bool ends = active && (!hit || mk == RT_MAT_DIFFUSE_LIGHT);
  // step 3: the wave's marble values and draws
  const double pn = lds_perlin ? marble_coop((LdsPerlin*)lds_perlin, need_pn, ptab, psc, h.point)
                               : marble_coop(S.perlin, need_pn, ptab, psc, h.point);
  const bool scat = active && !ends;
  const int dk = (scat && need_r) ? kDrawSphere : (scat && mk == RT_MAT_DIELECTRIC) ? kDrawDiel : kDrawNone;
  double jx = 0.0, jy = 0.0;
  const v3 rs = draws_coop(rng, seed, dk, false, 0u, jx, jy);
  const v3 un = unit_fast(!active ? V(1.0, 1.0, 1.0) : (scat && need_r && mk != RT_MAT_METAL) ? rs : d);
  // step 4: emitted + scatter, or the sky
  if (!active) return;
  ProbeOut r{};
  r.object = prim;
  bool alive = false, has_emit = false;
  v3 mul = V(1.0, 1.0, 1.0), emit = V(0.0, 0.0, 0.0);
  if (hit) {
    const DMat& m = S.mats[mat];
    alive = shade_factor(S, S.texs, m, leaf, pn, rs, un, rng, o, d, h, prim, face, mul, emit, has_emit);
    r.front_face = h.front_face ? 1 : 0;
    r.t = h.t;
    r.point[0] = h.point.x; r.point[1] = h.point.y; r.point[2] = h.point.z;
    r.normal[0] = h.normal.x; r.normal[1] = h.normal.y; r.normal[2] = h.normal.z;
  } else {
    emit = sky_unit(S, un);
    has_emit = true;
  }
  r.scattered = alive ? 1 : 0;
  r.emits = has_emit ? 1 : 0;
  r.draw = rng.draw;
  r.emitted[0] = emit.x; r.emitted[1] = emit.y; r.emitted[2] = emit.z;
  if (alive) {
    r.attenuation[0] = mul.x; r.attenuation[1] = mul.y; r.attenuation[2] = mul.z;
    r.origin[0] = o.x; r.origin[1] = o.y; r.origin[2] = o.z;
    r.direction[0] = d.x; r.direction[1] = d.y; r.direction[2] = d.z;
  }
  out[i] = r;
}

// ------------------------------------------------------------------------------------------
// launch wrappers (called from rt_api.cpp)
// ------------------------------------------------------------------------------------------
// megakernel block LDS: [n_lds_nodes4 x node4_bytes][n_lds_prims x DPrim][n_lds_perlin x DPerlin]
// [stack_depth4 x threads packed entries]
size_t trace_lds_bytes(int n_lds_nodes4, int node4_size, int n_lds_prims, int n_lds_perlin, int stack_depth4,
                       int threads, int n_lds_mats, int n_lds_texs) {
  return (size_t)n_lds_nodes4 * node4_size + (size_t)n_lds_prims * sizeof(DPrim) +
         (size_t)n_lds_perlin * sizeof(DPerlin) + (size_t)n_lds_mats * sizeof(DMat) + (size_t)n_lds_texs * sizeof(DTex) +
         (size_t)stack_depth4 * threads * kStack4EntryBytes;
}
size_t hit_lds_bytes(int n_lds_nodes, int stack_depth) { return lds_bytes(n_lds_nodes, stack_depth, kHitThreads); }

static int node_mode(const DScene& S) {
  return S.n_lds_nodes >= S.n_nodes ? kNodesLds : (S.n_lds_nodes == 0 ? kNodesGlobal : kNodesMixed);
}
static int node_mode4(const DScene& S) {
  return S.n_lds_nodes4 >= S.n_nodes4 ? kNodesLds : (S.n_lds_nodes4 == 0 ? kNodesGlobal : kNodesMixed);
}

template <int THREADS, int MODE, bool EXT>
static hipError_t occupancy_impl1(const DScene& S, int* blocks_per_cu) {
  // allow dynamic LDS beyond the 64 KiB default (gfx950 has 160 KiB per CU)
  const size_t lds = trace_lds_bytes(S.n_lds_nodes4, node4_bytes(S.exts != nullptr), S.n_lds_prims, S.n_lds_perlin, S.stack_depth4, THREADS,
                                     S.n_lds_mats, S.n_lds_texs);
  hipError_t e = hipFuncSetAttribute((const void*)trace_kernel<THREADS, MODE, EXT>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, trace_kernel<THREADS, MODE, EXT>, THREADS, lds);
}
template <int THREADS, int MODE>
static hipError_t occupancy_impl(const DScene& S, int* blocks_per_cu) {
  return S.exts ? occupancy_impl1<THREADS, MODE, true>(S, blocks_per_cu)
                : occupancy_impl1<THREADS, MODE, false>(S, blocks_per_cu);
}
template <int THREADS, int MODE>
static void launch_trace1(const KParams& p, int blocks, size_t lds, hipStream_t stream) {
  if (p.scene.exts)
    hipLaunchKernelGGL((trace_kernel<THREADS, MODE, true>), dim3(blocks), dim3(THREADS), lds, stream, p);
  else
    hipLaunchKernelGGL((trace_kernel<THREADS, MODE, false>), dim3(blocks), dim3(THREADS), lds, stream, p);
}

static hipError_t hit_prepare(const DScene& S) {
  const int lds = (int)hit_lds_bytes(S.n_lds_nodes, S.stack_depth);
  switch (node_mode(S)) {
    case kNodesLds: return hipFuncSetAttribute((const void*)hit_kernel<kNodesLds>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    case kNodesGlobal: return hipFuncSetAttribute((const void*)hit_kernel<kNodesGlobal>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    default: return hipFuncSetAttribute((const void*)hit_kernel<kNodesMixed>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  }
}

// Kernel instances: the wide block only with the whole (4-wide) BVH in LDS.  Also prepares the
// rt_scene_hit kernel for the scene.
hipError_t trace_occupancy(const DScene& S, int threads, int* blocks_per_cu) {
  hipError_t e = hit_prepare(S);
  if (e != hipSuccess) return e;
  if (threads == kTraceThreadsWide && !S.exts) {  // reference scenes only: book-2 scenes take kTraceThreadsWide3
    if (node_mode4(S) != kNodesLds) return hipErrorInvalidValue;
    if (S.n_lds_prims > 0) return occupancy_impl1<kTraceThreadsWide, kSceneLds, false>(S, blocks_per_cu);
    return occupancy_impl1<kTraceThreadsWide, kNodesLds, false>(S, blocks_per_cu);
  }
  if (threads == kTraceThreadsWide3) {  // book-2 scenes only (rt_api.cpp)
    if (node_mode4(S) != kNodesLds || !S.exts) return hipErrorInvalidValue;
    if (S.n_lds_prims > 0) return occupancy_impl1<kTraceThreadsWide3, kSceneLds, true>(S, blocks_per_cu);
    return occupancy_impl1<kTraceThreadsWide3, kNodesLds, true>(S, blocks_per_cu);
  }
  switch (node_mode4(S)) {
    case kNodesLds: return occupancy_impl<kTraceThreads, kNodesLds>(S, blocks_per_cu);
    case kNodesGlobal: return occupancy_impl<kTraceThreads, kNodesGlobal>(S, blocks_per_cu);
    default: return occupancy_impl<kTraceThreads, kNodesMixed>(S, blocks_per_cu);
  }
}

hipError_t launch_trace(const KParams& p, int blocks, int threads, hipStream_t stream) {
  const size_t lds = trace_lds_bytes(p.scene.n_lds_nodes4, node4_bytes(p.scene.exts != nullptr), p.scene.n_lds_prims, p.scene.n_lds_perlin, p.scene.stack_depth4, threads,
                                     p.scene.n_lds_mats, p.scene.n_lds_texs);
  if (threads == kTraceThreadsWide && !p.scene.exts) {
    if (p.scene.n_lds_prims > 0)
      hipLaunchKernelGGL((trace_kernel<kTraceThreadsWide, kSceneLds, false>), dim3(blocks), dim3(threads), lds, stream, p);
    else
      hipLaunchKernelGGL((trace_kernel<kTraceThreadsWide, kNodesLds, false>), dim3(blocks), dim3(threads), lds, stream, p);
    return hipGetLastError();
  }
  if (threads == kTraceThreadsWide3) {
    if (!p.scene.exts) return hipErrorInvalidValue;
    if (p.scene.n_lds_prims > 0)
      hipLaunchKernelGGL((trace_kernel<kTraceThreadsWide3, kSceneLds, true>), dim3(blocks), dim3(threads), lds, stream, p);
    else
      hipLaunchKernelGGL((trace_kernel<kTraceThreadsWide3, kNodesLds, true>), dim3(blocks), dim3(threads), lds, stream, p);
    return hipGetLastError();
  }
  switch (node_mode4(p.scene)) {
    case kNodesLds: launch_trace1<kTraceThreads, kNodesLds>(p, blocks, lds, stream); break;
    case kNodesGlobal: launch_trace1<kTraceThreads, kNodesGlobal>(p, blocks, lds, stream); break;
    default: launch_trace1<kTraceThreads, kNodesMixed>(p, blocks, lds, stream);
  }
  return hipGetLastError();
}

hipError_t launch_hit(const DScene& S, const double* rays, int n, double t_min, double t_max, void* out,
                      hipStream_t stream) {
  int blocks = (n + kHitThreads - 1) / kHitThreads;
  if (blocks == 0) return hipSuccess;
  size_t lds = hit_lds_bytes(S.n_lds_nodes, S.stack_depth);
  HitOut* o = static_cast<HitOut*>(out);
  switch (node_mode(S)) {
    case kNodesLds: hipLaunchKernelGGL(hit_kernel<kNodesLds>, dim3(blocks), dim3(kHitThreads), lds, stream, S, rays, n, t_min, t_max, o); break;
    case kNodesGlobal: hipLaunchKernelGGL(hit_kernel<kNodesGlobal>, dim3(blocks), dim3(kHitThreads), lds, stream, S, rays, n, t_min, t_max, o); break;
    default: hipLaunchKernelGGL(hit_kernel<kNodesMixed>, dim3(blocks), dim3(kHitThreads), lds, stream, S, rays, n, t_min, t_max, o);
  }
  return hipGetLastError();
}

template <int MODE, bool EXT>
static hipError_t launch_hit4_1(const DScene& S, const double* rays, int n, double t_min, double t_max, HitOut* o,
                                int blocks, hipStream_t stream) {
  const size_t lds = trace_lds_bytes(S.n_lds_nodes4, node4_bytes(EXT), MODE == kSceneLds ? S.n_lds_prims : 0,
                                     MODE == kSceneLds ? S.n_lds_perlin : 0, S.stack_depth4, kHitThreads,
                                     MODE == kSceneLds ? S.n_lds_mats : 0, MODE == kSceneLds ? S.n_lds_texs : 0);
  hipError_t e = hipFuncSetAttribute((const void*)hit4_kernel<MODE, EXT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((hit4_kernel<MODE, EXT>), dim3(blocks), dim3(kHitThreads), lds, stream, S, rays, n, t_min, t_max, o);
  return hipGetLastError();
}
template <int MODE>
static hipError_t launch_hit4_m(const DScene& S, const double* rays, int n, double t_min, double t_max, HitOut* o,
                                int blocks, hipStream_t stream) {
  return S.exts ? launch_hit4_1<MODE, true>(S, rays, n, t_min, t_max, o, blocks, stream)
                : launch_hit4_1<MODE, false>(S, rays, n, t_min, t_max, o, blocks, stream);
}

// rt_scene_hit_ex(RT_TRAVERSAL_RENDER): the node / primitive placement the trace kernel uses
// (`wide`: the scene-in-LDS block of launch_trace).
hipError_t launch_hit4(const DScene& S, bool wide, const double* rays, int n, double t_min, double t_max, void* out,
                       hipStream_t stream) {
  const int blocks = (n + kHitThreads - 1) / kHitThreads;
  if (blocks == 0) return hipSuccess;
  HitOut* o = static_cast<HitOut*>(out);
  if (wide) {
    if (S.n_lds_prims > 0) return launch_hit4_m<kSceneLds>(S, rays, n, t_min, t_max, o, blocks, stream);
    return launch_hit4_m<kNodesLds>(S, rays, n, t_min, t_max, o, blocks, stream);
  }
  switch (node_mode4(S)) {
    case kNodesLds: return launch_hit4_m<kNodesLds>(S, rays, n, t_min, t_max, o, blocks, stream);
    case kNodesGlobal: return launch_hit4_m<kNodesGlobal>(S, rays, n, t_min, t_max, o, blocks, stream);
    default: return launch_hit4_m<kNodesMixed>(S, rays, n, t_min, t_max, o, blocks, stream);
  }
}

template <int MODE, bool EXT>
static hipError_t launch_probe_1(const DScene& S, const double* rays, int n, uint64_t seed, uint32_t sample,
                                 uint32_t draw, ProbeOut* o, int blocks, hipStream_t stream) {
  const size_t lds = trace_lds_bytes(S.n_lds_nodes4, node4_bytes(EXT), MODE == kSceneLds ? S.n_lds_prims : 0,
                                     MODE == kSceneLds ? S.n_lds_perlin : 0, S.stack_depth4, kHitThreads,
                                     MODE == kSceneLds ? S.n_lds_mats : 0, MODE == kSceneLds ? S.n_lds_texs : 0);
  hipError_t e = hipFuncSetAttribute((const void*)probe_kernel<MODE, EXT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((probe_kernel<MODE, EXT>), dim3(blocks), dim3(kHitThreads), lds, stream, S, rays, n, seed, sample,
                     draw, o);
  return hipGetLastError();
}
template <int MODE>
static hipError_t launch_probe_m(const DScene& S, const double* rays, int n, uint64_t seed, uint32_t sample,
                                 uint32_t draw, ProbeOut* o, int blocks, hipStream_t stream) {
  return S.exts ? launch_probe_1<MODE, true>(S, rays, n, seed, sample, draw, o, blocks, stream)
                : launch_probe_1<MODE, false>(S, rays, n, seed, sample, draw, o, blocks, stream);
}

// rt_probe_segment: the node / primitive placement the trace kernel uses (`wide`, as launch_hit4)
hipError_t launch_probe(const DScene& S, bool wide, const double* rays, int n, uint64_t seed, uint32_t sample,
                        uint32_t draw, void* out, hipStream_t stream) {
  const int blocks = (n + kHitThreads - 1) / kHitThreads;
  if (blocks == 0) return hipSuccess;
  ProbeOut* o = static_cast<ProbeOut*>(out);
  if (wide) {
    if (S.n_lds_prims > 0) return launch_probe_m<kSceneLds>(S, rays, n, seed, sample, draw, o, blocks, stream);
    return launch_probe_m<kNodesLds>(S, rays, n, seed, sample, draw, o, blocks, stream);
  }
  switch (node_mode4(S)) {
    case kNodesLds: return launch_probe_m<kNodesLds>(S, rays, n, seed, sample, draw, o, blocks, stream);
    case kNodesGlobal: return launch_probe_m<kNodesGlobal>(S, rays, n, seed, sample, draw, o, blocks, stream);
    default: return launch_probe_m<kNodesMixed>(S, rays, n, seed, sample, draw, o, blocks, stream);
  }
}

hipError_t launch_reduce(const double* partial, int n_chunks, int n_tiles_rank, int tiles_x, int ty0, int tile_rank,
                         int tile_world, int width, int row0, int row1, int packed, int accumulate, double* out,
                         hipStream_t stream) {
  long long n = (long long)n_tiles_rank * kTilePixels;
  int blocks = (int)((n + 255) / 256);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(reduce_kernel, dim3(blocks), dim3(256), 0, stream, partial, n_chunks, n_tiles_rank, tiles_x,
                     ty0, tile_rank, tile_world, width, row0, row1, packed, accumulate, out);
  return hipGetLastError();
}

hipError_t launch_sum_parts(const double* parts, int n_parts, long long n, double* out, hipStream_t stream) {
  const long long blocks = (n + 255) / 256;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, parts, n_parts, n, out);
  return hipGetLastError();
}

#ifdef RT_TIMELINE
// timeline build: per-wave exit times of the last launch relative to the first wave's start, and each
// wave's time from seeing the unit pool exhausted to its exit (the frame's tail)
void timeline_dump() {
  {
    static unsigned long long t0[kTimelineWaves], tx[kTimelineWaves], t1[kTimelineWaves];
    if (hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_wave_t0), sizeof t0) == hipSuccess &&
        hipMemcpyFromSymbol(tx, HIP_SYMBOL(g_wave_tx), sizeof tx) == hipSuccess &&
        hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_wave_t1), sizeof t1) == hipSuccess) {
      std::vector<double> ends, tails, firstx;
      unsigned long long tmin = ~0ull;
      for (int i = 0; i < kTimelineWaves; ++i)
        if (t1[i] && t0[i]) tmin = std::min(tmin, t0[i]);
      for (int i = 0; i < kTimelineWaves; ++i)
        if (t1[i] && t0[i] && t1[i] >= tmin) {
          ends.push_back((double)(t1[i] - tmin) * 1e-2);  // 100 MHz ticks -> us
          if (tx[i] && tx[i] <= t1[i]) {
            tails.push_back((double)(t1[i] - tx[i]) * 1e-2);
            firstx.push_back((double)(tx[i] - tmin) * 1e-2);
          }
        }
      auto pct = [](std::vector<double> v, double q) {
        if (v.empty()) return 0.0;
        std::sort(v.begin(), v.end());
        return v[std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1)))];
      };
      fprintf(stderr, "[phase-timeline] waves %zu; exit us p0 %.1f p50 %.1f p90 %.1f p99 %.1f p99.9 %.1f max %.1f; "
              "pool exhausted seen at us p0 %.1f p50 %.1f; exhausted->exit us p50 %.1f p90 %.1f p99 %.1f max %.1f\n",
              ends.size(), pct(ends, 0), pct(ends, 0.5), pct(ends, 0.9), pct(ends, 0.99), pct(ends, 0.999),
              pct(ends, 1), pct(firstx, 0), pct(firstx, 0.5), pct(tails, 0.5), pct(tails, 0.9), pct(tails, 0.99),
              pct(tails, 1));
      std::fill(t0, t0 + kTimelineWaves, 0ull);
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wave_t0), t0, sizeof t0);
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wave_tx), t0, sizeof t0);
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wave_t1), t0, sizeof t0);
    }
  }
}
#endif

#ifdef RT_PHASE_TIMING
// instrumented build: print and clear the event counters (slot 2i: lane events, 2i + 1: wave events)
void phase_counters_dump() {
  unsigned long long h[64];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase_ctr), sizeof h) != hipSuccess) return;
  static const char* names[] = {"visit", "visit_with_leaves", "sphere_iter", "sphere_slab_pass", "rect_iter",
                                "pop_iter", "segment_iter", "box_iter", "marble_round", "draws_coop_round",
                                "unit_fetch", "camera_ray", "philox_A", "philox_B", "marble_sin", "hit_record",
                                "checker_level", "dielectric", "metal", "lambertian", "sky", "diffuse_light",
                                "reflectance", "traverse4", "publish", "tie_resolve"};
  for (int i = 0; i < 26; ++i)
    if (h[2 * i + 1])
      fprintf(stderr, "[phase-ev] %-18s lanes %.4g waves %.4g lanes/wave %.2f\n", names[i], (double)h[2 * i],
              (double)h[2 * i + 1], (double)h[2 * i] / (double)h[2 * i + 1]);
  unsigned long long lh[64], wh[64];
  if (hipMemcpyFromSymbol(lh, HIP_SYMBOL(g_visit_hist), sizeof lh) == hipSuccess &&
      hipMemcpyFromSymbol(wh, HIP_SYMBOL(g_wave_visit_hist), sizeof wh) == hipSuccess) {
    fprintf(stderr, "[phase-hist] visits: lanes / waves (slowest lane)\n");
    for (int i = 1; i < 64; ++i)
      if (lh[i] || wh[i]) fprintf(stderr, "[phase-hist] %2d %.6g %.6g\n", i, (double)lh[i], (double)wh[i]);
  }
  unsigned long long z[64] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_phase_ctr), z, sizeof z);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_visit_hist), z, sizeof z);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wave_visit_hist), z, sizeof z);
}
#endif

hipError_t launch_tonemap(const double* accum, int width, int height, double inv, uint8_t* rgb8, hipStream_t stream) {
  const long long n = (long long)width * height * 3;
  const int blocks = (int)((n + 255) / 256);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(tonemap_kernel, dim3(blocks), dim3(256), 0, stream, accum, width, height, inv, rgb8);
  return hipGetLastError();
}

hipError_t launch_unpack(const double* gathered, int world, int max_tiles, int n_tiles_total, int tiles_x, int width,
                         int height, double* out, hipStream_t stream) {
  long long n = (long long)world * max_tiles * kTilePixels;
  int blocks = (int)((n + 255) / 256);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(unpack_kernel, dim3(blocks), dim3(256), 0, stream, gathered, world, max_tiles, n_tiles_total,
                     tiles_x, width, height, out);
  return hipGetLastError();
}

}  // namespace rt
