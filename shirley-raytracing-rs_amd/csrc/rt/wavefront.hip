// wavefront.hip — wavefront path tracer for the reference's ray_color() loop (MI355X, gfx950).
//
// The bounce loop of render.rs:17-48 is cut into three kernels per iteration over a pool of P path
// slots whose state lives in HBM as structure-of-arrays (coalesced: consecutive lanes = consecutive
// slots):
//   wf_extend  — closest hit for every slot holding a ray (bbox_tree.rs:56-91).  Persistent waves
//                with dynamic ray fetch: a lane whose traversal ends writes its hit and takes the
//                next slot at once, so traversal runs with (almost) full waves; one node step per
//                loop iteration, BVH top levels + per-lane stacks in LDS.
//   wf_shade   — one lane per slot: emitted + scatter (material_type.rs:51-79) with the hit
//                record rebuilt from (t, prim, face); a finished path adds its radiance to its
//                unit's in-order sum and the slot immediately starts its next sample / takes the
//                next unit (render.rs:58-69): path regeneration, no compaction pass needed.
//                Texture values whose leaf is Perlin noise (perlin/mod.rs:162-183, ~7x8 gathers +
//                sin in f64) are NOT evaluated here: they are appended to a queue...
//   wf_texture — ...and evaluated by full, coherent waves, then folded into the slot's throughput /
//                radiance (the next ray does not need them; the next shade does).
// Arithmetic is binary64 and identical to the megakernel (rt_device.h), so both engines produce the
// same pixels; counter-based RNG keyed by (pixel, sample) makes them independent of scheduling.
#include "rt_device.h"

namespace rt {

enum : uint8_t { kSlotIdle = 0, kSlotAlive = 1, kSlotEnded = 2, kSlotRetired = 3 };
enum : int32_t { kDeferLambertian = 0, kDeferFairy = 1, kDeferDiffuse = 2 };
constexpr uint32_t kNoUnit = 0xffffffffu;
constexpr int kExtendThreads = 256;  // 4 waves per block, several blocks per CU
constexpr int kGridThreads = 256;

__device__ __forceinline__ unsigned long long wf_lanemask_lt() {
  unsigned lane = __lane_id();
  return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

// ------------------------------------------------------------------------------------------
// wf_extend
// ------------------------------------------------------------------------------------------
// Next 64-slot window for a wave: queue q first, then the following queues once q is drained.
// Returns the window's first slot, or ~0 when every queue is drained.  Lane 0 does the work.
__device__ __forceinline__ unsigned long long next_window(WfIter* it, int& q, uint32_t qlen, uint32_t win) {
  unsigned long long base = ~0ull;
  int qq = q;
  if (__lane_id() == 0) {
    for (int tries = 0; tries < kWfQueues; ++tries) {
      unsigned long long* cur = &it->fetch[qq][0];
      if (__hip_atomic_load(cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < qlen) {
        const unsigned long long nb = atomicAdd(cur, (unsigned long long)win);
        if (nb < qlen) {
          base = (unsigned long long)qq * qlen + nb;
          break;
        }
      }
      qq = (qq + 1) % kWfQueues;
    }
  }
  q = __shfl(qq, 0);
  return __shfl(base, 0);
}

template <int MODE, bool EXT>
__global__ __launch_bounds__(kExtendThreads) void wf_extend(WfParams P) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  DNode* lds_nodes = reinterpret_cast<DNode*>(lds_raw);
  unsigned char* stk_base = lds_raw + (size_t)P.scene.n_lds_nodes * sizeof(DNode);
  int* stk_node = reinterpret_cast<int*>(stk_base) + tid;
  float* stk_t = reinterpret_cast<float*>(stk_base + (size_t)P.scene.stack_depth * kExtendThreads * 4) + tid;
  stage_nodes<MODE>(P.scene, lds_nodes);
  const DScene& S = P.scene;
  const WfState& st = P.st;
  const int lane = __lane_id();
  const uint32_t qlen = (P.n_slots / kWfQueues + kWave) / kWave * kWave;  // multiple of 64, covers n_slots
  int q = (int)((blockIdx.x * (kExtendThreads / kWave) + tid / kWave) % kWfQueues);

  unsigned long long w_next = 0, w_end = 0;
  bool exhausted = false, active = false;
  int slot = 0;
  v3 o = V(0, 0, 0), d = V(0, 0, 0);
  Trav T;
  Rng rk{0u, 0u, 0u, 0u, 0u};  // side-stream key of the slot's path (read only when the scene has book-2 prims)
  unsigned visits = 0, ptests = 0, rays = 0;
  for (;;) {
    // lanes without a ray take the next slots of the wave's window
    const bool need = !active;
    const unsigned long long mask = __ballot(need);
    if (mask != 0ull && !exhausted) {
      if (w_next == w_end) {
        const unsigned long long nb = next_window(P.it, q, qlen, kWave);
        if (nb == ~0ull) {
          exhausted = true;
        } else {
          w_next = nb;
          w_end = nb + kWave;
        }
      }
      if (!exhausted) {
        const unsigned long long avail = w_end - w_next;
        const unsigned long long rank = __popcll(mask & wf_lanemask_lt());
        const unsigned long long idx = w_next + rank;
        w_next += min((unsigned long long)__popcll(mask), avail);
        if (need && rank < avail && idx < P.n_slots && st.state[idx] == kSlotAlive) {
          slot = (int)idx;
          o = V(st.ox[slot], st.oy[slot], st.oz[slot]);
          d = V(st.dx[slot], st.dy[slot], st.dz[slot]);
          trav_begin(T, d, __builtin_inf());
          if (S.exts) rk = Rng{st.pixel[slot], st.sample[slot], st.draw[slot], 0u, 0u};
          active = true;
          ++rays;
        }
      }
    }
    if (!__any(active)) {
      if (exhausted) break;
      continue;
    }
    if (active && trav_step<kExtendThreads, MODE, EXT>(S, lds_nodes, o, d, 0.001, T, rk, P.work.seed, stk_node, stk_t,
                                                  visits, ptests)) {
      st.ht[slot] = T.t_best;
      st.hprim[slot] = T.best;
      st.hface[slot] = T.face;
      active = false;
    }
  }
  unsigned long long v = visits, pt = ptests, r = rays;
  for (int off = 32; off > 0; off >>= 1) {
    v += __shfl_down(v, off);
    pt += __shfl_down(pt, off);
    r += __shfl_down(r, off);
  }
  if (lane == 0) {
    DCounters* cs = P.counters + ((blockIdx.x * (kExtendThreads / kWave) + tid / kWave) % kCounterSlots);
    atomicAdd(&cs->node_visits, v);
    atomicAdd(&cs->prim_tests, pt);
    atomicAdd(&cs->segments, r);  // ray_color loop iterations that traced a ray (render.rs:31)
  }
}

// wf_extend4: the same closest-hit pass for scenes whose 4-wide tree and primitives fit in LDS next
// to the stacks (the megakernel's wide configuration).  Traversal then issues no global loads, and
// each lane prefetches its NEXT ray (state, origin, direction) while it traverses the current one:
// the refill latency (path state of 2 M slots lives in HBM) is hidden behind the traversal steps.
template <int THREADS, bool EXT>
__global__ __launch_bounds__(THREADS, 1) void wf_extend4(WfParams P) {
  extern __shared__ unsigned char lds_raw[];
  const int tid = threadIdx.x;
  typedef typename Node4Sel<EXT>::T N4;
  N4* lds_nodes = reinterpret_cast<N4*>(lds_raw);
  DPrim* lds_prims = reinterpret_cast<DPrim*>(lds_raw + (size_t)P.scene.n_lds_nodes4 * sizeof(N4));
  unsigned char* stk_base = lds_raw + (size_t)P.scene.n_lds_nodes4 * sizeof(N4) +
                            (size_t)P.scene.n_lds_prims * sizeof(DPrim) + (size_t)P.scene.n_lds_perlin * sizeof(DPerlin);
  unsigned* stk = reinterpret_cast<unsigned*>(stk_base) + tid;  // [stack_depth4][THREADS] packed entries
  stage_nodes4<kSceneLds>(P.scene, lds_nodes, lds_prims);
  const DScene& S = P.scene;
  const WfState& st = P.st;
  const int lane = __lane_id();
  const uint32_t win = P.ext_window;  // slots per cursor claim (a multiple of 64)
  const uint32_t qlen = (P.n_slots / kWfQueues + win) / win * win;
  int q = (int)((blockIdx.x * (THREADS / kWave) + tid / kWave) % kWfQueues);

  unsigned long long w_next = 0, w_end = 0;
  bool exhausted = false, active = false, has_next = false;
  int slot = 0, nslot = 0;
  uint8_t nstate = 0;
  v3 o = V(0, 0, 0), d = V(0, 0, 0), no = V(0, 0, 0), nd = V(0, 0, 0);
  Trav4 T;
  trav4_begin<EXT>(T, S, V(0.0, 0.0, 0.0), V(1.0, 1.0, 1.0), 0.0);
  Rng rk{0u, 0u, 0u, 0u, 0u};  // side-stream key of the slot's path (read only when the scene has book-2 prims)
  unsigned visits = 0, ptests = 0, rays = 0;
  for (;;) {
    // A. a lane without a ray takes its prefetched one (if that slot holds a ray)
    if (!active && has_next) {
      has_next = false;
      if (nstate == kSlotAlive) {
        slot = nslot;
        o = no;
        d = nd;
        trav4_begin<EXT>(T, S, o, d, __builtin_inf());
        if (S.exts) rk = Rng{st.pixel[slot], st.sample[slot], st.draw[slot], 0u, 0u};
        active = true;
        ++rays;
      }
    }
    // B. lanes without a prefetched ray claim the next slot of the wave's window and issue its loads
    const bool need = !has_next;
    const unsigned long long mask = __ballot(need);
    if (mask != 0ull && !exhausted) {
      if (w_next == w_end) {
        const unsigned long long nb = next_window(P.it, q, qlen, win);
        if (nb == ~0ull) {
          exhausted = true;
        } else {
          w_next = nb;
          w_end = nb + win;
        }
      }
      if (!exhausted) {
        const unsigned long long avail = w_end - w_next;
        const unsigned long long rank = __popcll(mask & wf_lanemask_lt());
        const unsigned long long idx = w_next + rank;
        w_next += min((unsigned long long)__popcll(mask), avail);
        if (need && rank < avail && idx < P.n_slots) {
          nslot = (int)idx;
          nstate = st.state[nslot];
          no = V(st.ox[nslot], st.oy[nslot], st.oz[nslot]);
          nd = V(st.dx[nslot], st.dy[nslot], st.dz[nslot]);
          has_next = true;
        }
      }
    }
    if (!__any(active || has_next)) {
      if (exhausted) break;
      continue;
    }
    // C. one node visit for every lane holding a ray
    if (active && trav4_step<THREADS, kSceneLds, EXT>(S, lds_nodes, lds_prims, o, d, 0.001, T, stk, rk, P.work.seed, visits,
                                                 ptests)) {
      st.ht[slot] = T.t_best;
      st.hprim[slot] = T.best;
      st.hface[slot] = T.face;
      active = false;
    }
  }
  unsigned long long v = visits, pt = ptests, r = rays;
  for (int off = 32; off > 0; off >>= 1) {
    v += __shfl_down(v, off);
    pt += __shfl_down(pt, off);
    r += __shfl_down(r, off);
  }
  if (lane == 0) {
    DCounters* cs = P.counters + ((blockIdx.x * (THREADS / kWave) + tid / kWave) % kCounterSlots);
    atomicAdd(&cs->node_visits, v);
    atomicAdd(&cs->prim_tests, pt);
    atomicAdd(&cs->segments, r);
  }
}

// ------------------------------------------------------------------------------------------
// wf_shade (+ path regeneration)
// ------------------------------------------------------------------------------------------
// One lane per slot; the grid covers the slots exactly in whole waves (n_slots % 64 == 0), and the
// wave of slot group g = slots [64 g, 64 g + 64) owns that group's unit window and texture queue.
template <bool EXT>
__global__ __launch_bounds__(kGridThreads) void wf_shade(WfParams P) {
  const DScene& S = P.scene;
  const DCamera& C = P.cam;
  const DWork& W = P.work;
  const WfState& st = P.st;
  const uint64_t seed = W.seed;
  const unsigned long long pix_per_chunk = (unsigned long long)W.n_tiles_rank * kTilePixels;
  const int lane = __lane_id();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = i / kWave;
  const bool valid = i < P.n_slots;
  const int slot = (int)i;
  unsigned n_samp = 0;

  // wf_extend of this round is done with its slot cursors: zero them for the next round
  if (blockIdx.x == 0 && threadIdx.x < kWfQueues) P.it->fetch[threadIdx.x][0] = 0;

  uint8_t state = valid ? st.state[slot] : kSlotRetired;
  bool defer = false;
  int defer_kind = 0, defer_tex = 0;
  double defer_scale = 0.0;
  v3 hp = V(0, 0, 0);

  // 1. shade the traced segment: render.rs:31-45
  if (state == kSlotAlive) {
    v3 o = V(st.ox[slot], st.oy[slot], st.oz[slot]);
    v3 d = V(st.dx[slot], st.dy[slot], st.dz[slot]);
    v3 att = V(st.ax[slot], st.ay[slot], st.az[slot]);
    v3 em = V(st.ex[slot], st.ey[slot], st.ez[slot]);
    Rng rng{st.pixel[slot], st.sample[slot], st.draw[slot], st.c2[slot], st.c3[slot]};
    const int prim = st.hprim[slot];
    bool alive;
    if (prim >= 0) {
      const DPrim pr = S.prims[prim];
      const int face = st.hface[slot];
      const double t = st.ht[slot];
      Hit h;
      hit_record<false, EXT>(S, pr, face, o, d, t, rng, seed, h);
      hp = h.point;
      const DMat& m = S.mats[pr.material];
      if (m.kind == RT_MAT_DIELECTRIC) {  // dielectric.rs:21-49
        double ratio = h.front_face ? (1.0 / m.param) : m.param;
        v3 ud = unit(d);
        double cos_theta = fmin_one(dot(scale(ud, -1.0), h.normal));
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        bool refl = ratio * sin_theta > 1.0;
        if (!refl) refl = reflectance(cos_theta, ratio) > rng_next(rng, seed);  // drawn only if not TIR
        o = h.point;
        d = refl ? reflect(ud, h.normal) : refract(ud, h.normal, ratio);
        alive = true;
      } else if (m.kind == RT_MAT_METAL) {  // metal.rs:26-40 — never absorbs
        v3 r = random_in_unit_sphere(rng, seed);
        v3 reflected = reflect(unit(d), h.normal);
        o = h.point;
        d = reflected + scale(r, m.param);
        att = hmul(att, V(m.albedo[0], m.albedo[1], m.albedo[2]));
        alive = true;
      } else {
        // Lambertian / FairyLight / DiffuseLight: the albedo texture
        const int leaf = resolve_texture(S, m.tex, h.point);
        const bool perlin = S.texs[leaf].kind == RT_TEX_PERLIN;
        v3 a = V(0, 0, 0);
        if (!perlin) {
          const DTex& tx = S.texs[leaf];
          if (tx.kind == RT_TEX_SOLID) {
            a = V(tx.color[0], tx.color[1], tx.color[2]);
          } else {
            const UV uv = hit_uv(pr, face, h);
            a = image_texel(tx, uv.u, uv.v);
          }
        }
        if (m.kind == RT_MAT_DIFFUSE_LIGHT) {  // lighting.rs:21-29: emits, never scatters
          if (perlin) {
            defer = true;
            defer_kind = kDeferDiffuse;
          } else {
            em = em + hmul(att, a);
          }
          alive = false;
        } else {  // lambertian.rs:21-37 / lighting.rs:42-66 / book-2 isotropic
          if (m.kind == RT_MAT_FAIRY_LIGHT) {
            double s = dot(h.normal, scale(d, -1.0));
            if (perlin) {
              defer_scale = s / len(d);
            } else {
              em = em + hmul(att, scale(a, s / len(d)));
              a = unit(a);
            }
          }
          v3 r = random_in_unit_sphere(rng, seed);
          v3 sc = r;  // isotropic: the unit-ball point itself
          if (m.kind != RT_MAT_ISOTROPIC) {
            sc = h.normal + unit(r);
            if (near_zero(sc)) sc = h.normal;
          }
          o = h.point;
          d = sc;
          if (perlin) {
            defer = true;
            defer_kind = (m.kind == RT_MAT_FAIRY_LIGHT) ? kDeferFairy : kDeferLambertian;
          } else {
            att = hmul(att, a);
          }
          alive = true;
        }
        defer_tex = leaf;
      }
    } else {
      em = em + hmul(att, sky(S, d));  // skybox/mod.rs:18-25
      alive = false;
    }
    if (alive) {
      const int dl = st.depth[slot] - 1;
      st.depth[slot] = dl;
      alive = dl > 0;
    }
    st.draw[slot] = rng.draw;
    st.c2[slot] = rng.c2;
    st.c3[slot] = rng.c3;
    st.ax[slot] = att.x; st.ay[slot] = att.y; st.az[slot] = att.z;
    st.ex[slot] = em.x; st.ey[slot] = em.y; st.ez[slot] = em.z;
    if (alive) {
      st.ox[slot] = o.x; st.oy[slot] = o.y; st.oz[slot] = o.z;
      st.dx[slot] = d.x; st.dy[slot] = d.y; st.dz[slot] = d.z;
    } else {
      // the path is finished; a deferred emission must land before its radiance is summed
      state = defer ? kSlotEnded : kSlotIdle;
      if (!defer) {
        st.sx[slot] += em.x;  // c += ray_color(...)  (render.rs:66)
        st.sy[slot] += em.y;
        st.sz[slot] += em.z;
      }
    }
  } else if (state == kSlotEnded) {
    st.sx[slot] += st.ex[slot];
    st.sy[slot] += st.ey[slot];
    st.sz[slot] += st.ez[slot];
    state = kSlotIdle;
  }

  // 2. deferred texture entry, compacted within the group (evaluated by wf_texture)
  {
    const unsigned long long md = __ballot(defer);
    const unsigned q = g * kWave + (unsigned)__popcll(md & wf_lanemask_lt());
    if (defer) {
      P.tq.slot[q] = slot;
      P.tq.tex[q] = defer_tex;
      P.tq.kind[q] = defer_kind;
      P.tq.px[q] = hp.x;
      P.tq.py[q] = hp.y;
      P.tq.pz[q] = hp.z;
      P.tq.scale[q] = defer_scale;
    }
    if (lane == 0 && valid) P.tq.count[g] = (uint32_t)__popcll(md);
  }

  // 3. regeneration: a slot between paths starts its unit's next sample, or publishes the unit's
  //    in-order sum (*buf_c = c, render.rs:68) and takes the next unit
  uint32_t pix = kNoUnit;
  int s_next = 0, s_end = 0;
  const bool regen = state == kSlotIdle;
  if (regen) {
    pix = st.pixel[slot];
    s_next = st.s_next[slot];
    s_end = st.s_end[slot];
    if (pix != kNoUnit && s_next >= s_end) {
      double* dst = P.partial + st.part[slot] * 3;
      dst[0] = st.sx[slot];
      dst[1] = st.sy[slot];
      dst[2] = st.sz[slot];
      pix = kNoUnit;
    }
  }
  const bool need_unit = regen && pix == kNoUnit;
  const unsigned long long mneed = __ballot(need_unit);
  bool retire = false;
  if (mneed) {
    // the group's window of units (one 64-unit refill per atomic, like the megakernel's waves)
    unsigned long long wn, we;
    if (P.first) {
      wn = (unsigned long long)g * kWave;
      we = wn + kWave;
    } else {
      wn = P.win[2 * g];
      we = P.win[2 * g + 1];
    }
    const unsigned long long k = __popcll(mneed), rank = __popcll(mneed & wf_lanemask_lt());
    const unsigned long long avail = we - wn;
    unsigned long long idx;
    if (avail >= k) {
      idx = wn + rank;
      wn += k;
    } else {
      unsigned long long nb = 0;
      if (lane == 0) nb = (unsigned long long)P.n_slots + atomicAdd(P.unit_counter, (unsigned long long)kWave);
      nb = __shfl(nb, 0);
      idx = (rank < avail) ? (wn + rank) : (nb + (rank - avail));
      wn = nb + (k - avail);
      we = nb + kWave;
    }
    if (lane == 0) {
      P.win[2 * g] = wn;
      P.win[2 * g + 1] = we;
    }
    if (need_unit) {
      if (idx < W.n_units) {
        unsigned long long per_tile = (unsigned long long)W.n_chunks * kTilePixels;
        unsigned long long lt = idx / per_tile;
        unsigned long long rem = idx - lt * per_tile;
        int chunk = (int)(rem / kTilePixels);
        int lp = (int)(rem % kTilePixels);
        unsigned long long gt = lt * (unsigned long long)W.tile_world + (unsigned long long)W.tile_rank;
        int tx = (int)(gt % (unsigned long long)W.tiles_x), ty = W.ty0 + (int)(gt / (unsigned long long)W.tiles_x);
        int ppx = tx * kTile + (lp % kTile), ppy = ty * kTile + (lp / kTile);
        if (ppx < C.width && ppy < C.height) {
          pix = (uint32_t)ppy * (uint32_t)C.width + (uint32_t)ppx;
          s_next = W.sample_base + chunk * W.chunk;
          s_end = min(W.samples, s_next + W.chunk);
          st.part[slot] = (unsigned long long)chunk * pix_per_chunk + lt * kTilePixels + (unsigned long long)lp;
          st.sx[slot] = 0.0;
          st.sy[slot] = 0.0;
          st.sz[slot] = 0.0;
          if (W.max_depth == 0) {  // ray_color returns black without drawing (render.rs:30)
            n_samp += (unsigned)(s_end - s_next);
            s_next = s_end;
          }
        }
        // (a unit outside the image is skipped: the slot asks again next round)
      } else {
        state = kSlotRetired;
        retire = true;
      }
    }
  }
  if (state == kSlotIdle && pix != kNoUnit && s_next < s_end) {  // render.rs:60-65
    const int ppx = (int)(pix % (uint32_t)C.width), ppy = (int)(pix / (uint32_t)C.width);
    Rng rng{pix, (uint32_t)s_next, 0u, 0u, 0u};
    double jx = (double)ppx + rng_next(rng, seed);
    double jy = (double)ppy + rng_next(rng, seed);
    v3 o, d;
    camera_ray(C, rng, seed, jx, jy, o, d);
    st.ox[slot] = o.x; st.oy[slot] = o.y; st.oz[slot] = o.z;
    st.dx[slot] = d.x; st.dy[slot] = d.y; st.dz[slot] = d.z;
    st.ax[slot] = 1.0; st.ay[slot] = 1.0; st.az[slot] = 1.0;
    st.ex[slot] = 0.0; st.ey[slot] = 0.0; st.ez[slot] = 0.0;
    st.sample[slot] = rng.sample;
    st.draw[slot] = rng.draw;
    st.c2[slot] = rng.c2;
    st.c3[slot] = rng.c3;
    st.depth[slot] = W.max_depth;
    ++s_next;
    ++n_samp;
    state = kSlotAlive;
  }
  if (valid && regen) {
    st.pixel[slot] = pix;
    st.s_next[slot] = s_next;
    st.s_end[slot] = s_end;
  }
  if (valid) st.state[slot] = state;

  // retirements (termination test on the host) and the samples counter: one atomic per wave/block
  const unsigned long long mr = __ballot(retire);
  if (mr && lane == 0) atomicAdd(P.retired, (unsigned)__popcll(mr));
  __shared__ unsigned red[kGridThreads / kWave];
  unsigned ns = n_samp;
  for (int off = 32; off > 0; off >>= 1) ns += __shfl_down(ns, off);
  if (lane == 0) red[threadIdx.x / kWave] = ns;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    for (int w = 0; w < kGridThreads / kWave; ++w) tot += red[w];
    if (tot) atomicAdd(&P.counters[blockIdx.x % kCounterSlots].samples, tot);
  }
}

// ------------------------------------------------------------------------------------------
// wf_texture: deferred Perlin texture values.  Blocks stride over the slot groups (wave w of a block
// takes group base + w); each block first copies the scene's Perlin tables (9 KB each) into LDS when
// they fit, so the ~210 table gathers of a marble evaluation are LDS reads.
// ------------------------------------------------------------------------------------------
constexpr int kTexLdsTables = 2;

template <bool LDS_TABLES>
__global__ __launch_bounds__(kGridThreads) void wf_texture(WfParams P) {
  __shared__ DPerlin tabs[LDS_TABLES ? kTexLdsTables : 1];
  const DScene& S = P.scene;
  const WfState& st = P.st;
  if (LDS_TABLES) {
    const int4* src = reinterpret_cast<const int4*>(S.perlin);
    int4* dst = reinterpret_cast<int4*>(tabs);
    const int n16 = P.n_perlin * (int)(sizeof(DPerlin) / 16);
    for (int k = threadIdx.x; k < n16; k += blockDim.x) dst[k] = src[k];
    __syncthreads();
  }
  const DPerlin* perlin = LDS_TABLES ? tabs : S.perlin;
  const uint32_t n_groups = P.n_slots / kWave;
  const uint32_t waves = blockDim.x / kWave;
  for (uint32_t g = blockIdx.x * waves + threadIdx.x / kWave; g < n_groups; g += gridDim.x * waves) {
    const uint32_t n = P.tq.count[g];
    if ((uint32_t)__lane_id() >= n) continue;
    const uint32_t i = g * kWave + __lane_id();
    const int slot = P.tq.slot[i];
    const DTex& t = S.texs[P.tq.tex[i]];
    const v3 p = V(P.tq.px[i], P.tq.py[i], P.tq.pz[i]);
    const double nz = marble_inl(perlin + t.table, t.scale, p);  // perlin/mod.rs:162-183
    v3 a = V(nz, nz, nz);
    v3 att = V(st.ax[slot], st.ay[slot], st.az[slot]);
    const int kind = P.tq.kind[i];
    if (kind == kDeferLambertian) {
      att = hmul(att, a);
    } else if (kind == kDeferFairy) {  // emitted (lighting.rs:59-66) before the scatter attenuation
      v3 em = V(st.ex[slot], st.ey[slot], st.ez[slot]);
      em = em + hmul(att, scale(a, P.tq.scale[i]));
      st.ex[slot] = em.x; st.ey[slot] = em.y; st.ez[slot] = em.z;
      att = hmul(att, unit(a));
    } else {  // DiffuseLight
      v3 em = V(st.ex[slot], st.ey[slot], st.ez[slot]);
      em = em + hmul(att, a);
      st.ex[slot] = em.x; st.ey[slot] = em.y; st.ez[slot] = em.z;
    }
    st.ax[slot] = att.x; st.ay[slot] = att.y; st.az[slot] = att.z;
  }
}

// ------------------------------------------------------------------------------------------
// host-side launch helpers (called from rt_api.cpp)
// ------------------------------------------------------------------------------------------
size_t wf_extend_lds(int n_lds_nodes, int stack_depth) {
  return (size_t)n_lds_nodes * sizeof(DNode) + (size_t)stack_depth * kExtendThreads * 8;
}

int wf_extend_threads() { return kExtendThreads; }

static int wf_mode(const DScene& S) {
  return S.n_lds_nodes >= S.n_nodes ? kNodesLds : (S.n_lds_nodes == 0 ? kNodesGlobal : kNodesMixed);
}

size_t wf_extend4_lds(const DScene& S) {
  return (size_t)S.n_lds_nodes4 * node4_bytes(S.exts != nullptr) + (size_t)S.n_lds_prims * sizeof(DPrim) +
         (size_t)S.n_lds_perlin * sizeof(DPerlin) + (size_t)S.stack_depth4 * kTraceThreadsWide * kStack4EntryBytes;
}

// Kernel instances come in pairs: EXT = the scene has book-2 primitives (their out-of-line code
// would otherwise cost every reference scene registers and scratch).
template <class K>
static hipError_t prepare_one(K kernel, int threads, int lds, int* blocks_per_cu) {
  hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, kernel, threads, lds);
}

// The 4-wide, scene-in-LDS extend kernel for scenes where the megakernel runs wide (`S` = that scene).
hipError_t wf_prepare4(const DScene& S, int* extend_blocks_per_cu) {
  const int lds = (int)wf_extend4_lds(S);
  if (lds > kLdsBytes) {  // the megakernel's 768-thread block fits, this 1024-thread one does not
    *extend_blocks_per_cu = 0;
    return hipSuccess;
  }
  return S.exts ? prepare_one(wf_extend4<kTraceThreadsWide, true>, kTraceThreadsWide, lds, extend_blocks_per_cu)
                : prepare_one(wf_extend4<kTraceThreadsWide, false>, kTraceThreadsWide, lds, extend_blocks_per_cu);
}

hipError_t wf_launch_extend4(const WfParams& P, int extend_blocks, hipStream_t s) {
  const size_t lds = wf_extend4_lds(P.scene);
  if (P.scene.exts)
    hipLaunchKernelGGL((wf_extend4<kTraceThreadsWide, true>), dim3(extend_blocks), dim3(kTraceThreadsWide), lds, s, P);
  else
    hipLaunchKernelGGL((wf_extend4<kTraceThreadsWide, false>), dim3(extend_blocks), dim3(kTraceThreadsWide), lds, s, P);
  return hipGetLastError();
}

template <bool EXT>
static hipError_t wf_prepare1(const DScene& S, int lds, int* extend_blocks_per_cu) {
  switch (wf_mode(S)) {
    case kNodesLds: return prepare_one(wf_extend<kNodesLds, EXT>, kExtendThreads, lds, extend_blocks_per_cu);
    case kNodesGlobal: return prepare_one(wf_extend<kNodesGlobal, EXT>, kExtendThreads, lds, extend_blocks_per_cu);
    default: return prepare_one(wf_extend<kNodesMixed, EXT>, kExtendThreads, lds, extend_blocks_per_cu);
  }
}
hipError_t wf_prepare(const DScene& S, int* extend_blocks_per_cu) {
  const int lds = (int)wf_extend_lds(S.n_lds_nodes, S.stack_depth);
  return S.exts ? wf_prepare1<true>(S, lds, extend_blocks_per_cu) : wf_prepare1<false>(S, lds, extend_blocks_per_cu);
}

int wf_grid_threads() { return kGridThreads; }

// One round = wf_launch_extend -> wf_launch_shade -> wf_launch_texture; `P.it` points at the
// round's zeroed counters.
template <bool EXT>
static void wf_launch_extend1(const WfParams& P, int extend_blocks, size_t lds, hipStream_t s) {
  switch (wf_mode(P.scene)) {
    case kNodesLds: hipLaunchKernelGGL((wf_extend<kNodesLds, EXT>), dim3(extend_blocks), dim3(kExtendThreads), lds, s, P); break;
    case kNodesGlobal: hipLaunchKernelGGL((wf_extend<kNodesGlobal, EXT>), dim3(extend_blocks), dim3(kExtendThreads), lds, s, P); break;
    default: hipLaunchKernelGGL((wf_extend<kNodesMixed, EXT>), dim3(extend_blocks), dim3(kExtendThreads), lds, s, P);
  }
}
hipError_t wf_launch_extend(const WfParams& P, int extend_blocks, hipStream_t s) {
  const size_t lds = wf_extend_lds(P.scene.n_lds_nodes, P.scene.stack_depth);
  if (P.scene.exts) wf_launch_extend1<true>(P, extend_blocks, lds, s);
  else wf_launch_extend1<false>(P, extend_blocks, lds, s);
  return hipGetLastError();
}

static void launch_shade1(const WfParams& P, int grid_blocks, hipStream_t s) {
  if (P.scene.exts) hipLaunchKernelGGL(wf_shade<true>, dim3(grid_blocks), dim3(kGridThreads), 0, s, P);
  else hipLaunchKernelGGL(wf_shade<false>, dim3(grid_blocks), dim3(kGridThreads), 0, s, P);
}
hipError_t wf_launch_shade(const WfParams& P, int grid_blocks, hipStream_t s) {
  launch_shade1(P, grid_blocks, s);
  return hipGetLastError();
}

hipError_t wf_launch_texture(const WfParams& P, int grid_blocks, hipStream_t s) {
  if (P.n_perlin <= kTexLdsTables)
    hipLaunchKernelGGL(wf_texture<true>, dim3(grid_blocks), dim3(kGridThreads), 0, s, P);
  else
    hipLaunchKernelGGL(wf_texture<false>, dim3(grid_blocks), dim3(kGridThreads), 0, s, P);
  return hipGetLastError();
}

// First iteration: every slot is Idle -> wf_shade alone assigns units and generates camera rays.
hipError_t wf_start(const WfParams& P, int grid_blocks, hipStream_t s) {
  WfParams Q = P;
  Q.first = 1;
  launch_shade1(Q, grid_blocks, s);
  return hipGetLastError();
}

}  // namespace rt
