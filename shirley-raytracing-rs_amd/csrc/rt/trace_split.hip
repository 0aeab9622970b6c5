// trace_split.hip — the persistent megakernel with its traversal decoupled from its shading
// (MI355X, gfx950): in-block ray queues in LDS.
//
// Why: the megakernel (trace.hip) runs a segment's traversal and shading in the same lanes.  A wave's
// traversal lasts as long as its slowest lane's (8.8 node visits per iteration at 27 of 64 lanes,
// sphere-leaf loops at 7 of 64; PMC lane utilisation 41 % at 98.5 % VALU issue), so the
// kernel is bound by VALU issue spent on idle lanes.  Compacting whole paths across the block is
// impossible (the scene fills the LDS; ~200 B of path state x 1024 lanes would not fit), but the
// traversal only needs a ray in (48 B) and a hit out (16 B).  So one 1024-thread block per CU splits
// its 16 waves into two roles sharing the scene in LDS:
//
//   * NS "shading" waves own the paths exactly like trace_kernel's lanes (units, samples, RNG,
//     throughput, radiance, shading, Perlin / unit-sphere wave cooperation) and, instead of
//     traversing, post their lanes' rays to per-lane LDS slots and a per-wave request mask, then sleep
//     until every requested hit has come back;
//   * NT "traversal" waves keep every lane busy: a lane whose traversal ends writes the hit to the
//     slot, sets its done bit and takes the next pending ray of any shading wave (ballot + rank
//     compaction of the request masks: the north star's per-bounce compaction, done in LDS), so node
//     visits and leaf tests run on (nearly) full waves.
//
// Same device functions as trace_kernel (rt_device.h: traverse4's per-step form, hit record, shading),
// same unit enumeration, counter RNG and in-order unit sums, hence bit-identical frames.
// Hand-off protocol (LDS, workgroup scope): rays / hits are written, then a release fence, then the
// request (atomic or into req[w]) / completion (atomic or into done[w]); the readers acquire after
// observing the mask.  A shading wave posts again only after all its previous rays are done, so
// req[w] and done[w] have one writer-set at a time.  Exit: a shading wave leaves when the unit pool
// is drained and none of its lanes holds a path; it then decrements `live`; traversal waves leave
// when `live` is 0 (no request can be pending then) — every wave reaches its exit.
#include "rt_device.h"

namespace rt {

__device__ __forceinline__ unsigned long long split_lanemask_lt() {
  const unsigned lane = __lane_id();
  return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}
__device__ __forceinline__ unsigned long long lds_load64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned long long bcast64(unsigned long long v) {
  return ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
         (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
}

// LDS layout of a split block (byte offsets; every region 16-B aligned)
struct SplitLds {
  size_t nodes, prims, perlin, stack, rays, hits, ctrl, scratch, total;
};
__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline SplitLds split_lds_layout(int n_nodes4, int n_prims, int n_perlin, int stack_depth4, int nt) {
  const int ns = kTraceThreadsWide / kWave - nt;
  SplitLds L;
  L.nodes = 0;
  L.prims = align16(L.nodes + (size_t)n_nodes4 * sizeof(DNode4F));
  L.perlin = align16(L.prims + (size_t)n_prims * sizeof(DPrim));
  L.stack = align16(L.perlin + (size_t)n_perlin * sizeof(DPerlin));
  L.rays = align16(L.stack + (size_t)stack_depth4 * nt * kWave * kStack4EntryBytes);
  L.hits = align16(L.rays + (size_t)ns * kWave * 48);           // o, d (6 f64) per shading lane
  L.ctrl = align16(L.hits + (size_t)ns * kWave * 16);           // t (f64), prim, face per shading lane
  L.scratch = align16(L.ctrl + (size_t)(2 * ns + 2) * 8);       // req[ns], done[ns], live
  L.total = align16(L.scratch + (size_t)nt * kWave * 4);        // per traversal wave: 64 claimed slot ids
  return L;
}

struct SlotHit {
  double t;
  int32_t prim, face;
};

template <int NT>
__global__ __launch_bounds__(kTraceThreadsWide, 1) void split_kernel(KParams P) {
  constexpr int NS = kTraceThreadsWide / kWave - NT;
  constexpr int kTravLanes = NT * kWave;
  extern __shared__ unsigned char lds_raw[];
  const DScene& S = P.scene;
  const SplitLds L = split_lds_layout(S.n_lds_nodes4, S.n_lds_prims, S.n_lds_perlin, S.stack_depth4, NT);
  DNode4F* lds_nodes = reinterpret_cast<DNode4F*>(lds_raw + L.nodes);
  DPrim* lds_prims = reinterpret_cast<DPrim*>(lds_raw + L.prims);
  double* rays = reinterpret_cast<double*>(lds_raw + L.rays);
  SlotHit* hits = reinterpret_cast<SlotHit*>(lds_raw + L.hits);
  unsigned long long* req = reinterpret_cast<unsigned long long*>(lds_raw + L.ctrl);
  unsigned long long* done = req + NS;
  unsigned* live = reinterpret_cast<unsigned*>(done + NS);
  const int tid = threadIdx.x;
  if (tid < 2 * NS) req[tid] = 0ull;  // req[] and done[]
  if (tid == 0) *live = NS;
  // the scene (nodes, primitives, Perlin tables at L.nodes / L.prims / L.perlin) + __syncthreads
  stage_nodes4<kSceneLds>(S, lds_nodes, lds_prims);

  const int wave = tid / kWave;
  const int lane = __lane_id();
  const uint64_t seed = P.work.seed;

  if (wave < NT) {
    // ------------------------------------------------------------------ traversal waves
    const int tl = tid;  // 0 .. kTravLanes-1
    unsigned* stk = reinterpret_cast<unsigned*>(lds_raw + L.stack) + tl;
    unsigned* scratch = reinterpret_cast<unsigned*>(lds_raw + L.scratch) + wave * kWave;
    bool has_ray = false;
    int slot = 0;
    v3 o = V(0.0, 0.0, 0.0), d = V(1.0, 1.0, 1.0);
    Trav4 T;
    trav4_begin<false>(T, S, o, d, 0.0);
    const Rng rk{0u, 0u, 0u, 0u, 0u};  // reference scenes only (no book-2 media draws)
    unsigned visits = 0, ptests = 0;
    int rot = wave;  // first shading wave this wave looks at (spreads the claims)
    for (;;) {
      unsigned long long idle = __ballot(!has_ray);
      // claim when enough lanes are idle (a claim costs ~40 instructions per candidate wave), or
      // when the whole wave is
      if (idle != 0ull && (__popcll(idle) >= (unsigned)P.split_refill || idle == ~0ull)) {
        // pending requests: lane w < NS reads req[w]
        const unsigned long long r = lane < NS ? lds_load64(&req[lane]) : 0ull;
        unsigned long long pw = __ballot(r != 0ull);
        // rotate the candidate order by `rot` so that the traversal waves do not all claim from
        // the same shading wave first
        pw = (pw >> rot) | (rot ? (pw << (NS - rot)) : 0ull);
        pw &= (NS == 64) ? ~0ull : ((1ull << NS) - 1ull);
        while (idle != 0ull && pw != 0ull) {
          int w = __builtin_ctzll(pw) + rot;
          if (w >= NS) w -= NS;
          pw &= pw - 1ull;
          const unsigned long long snap = bcast64(__shfl(r, w));
          // select the first k = |idle| pending lanes of wave w and claim them
          const unsigned k = (unsigned)__popcll(idle);
          const bool pend = (snap >> lane) & 1ull;
          const bool pick = pend && (unsigned)__popcll(snap & split_lanemask_lt()) < k;
          const unsigned long long sel = __ballot(pick);
          unsigned long long old = 0ull;
          if (lane == 0) old = atomicAnd(&req[w], ~sel);
          const unsigned long long got = bcast64(old) & sel;
          if (got == 0ull) continue;
          // compaction: the q-th claimed lane of wave w -> the q-th idle lane of this wave
          if ((got >> lane) & 1ull) scratch[__popcll(got & split_lanemask_lt())] = (unsigned)(w * kWave + lane);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the claimed rays' data
          const unsigned n = (unsigned)__popcll(got);
          const unsigned rank = (unsigned)__popcll(idle & split_lanemask_lt());
          const bool take = !has_ray && rank < n;
          if (take) {
            slot = (int)scratch[rank];
            const double* rp = rays + (size_t)slot * 6;
            o = V(rp[0], rp[1], rp[2]);
            d = V(rp[3], rp[4], rp[5]);
            trav4_begin<false>(T, S, o, d, __builtin_inf());
            has_ray = true;
          }
          idle &= ~__ballot(take);
          __builtin_amdgcn_wave_barrier();  // scratch is rewritten by the next candidate
        }
        rot = rot + 1 == NS ? 0 : rot + 1;
      }
      if (!__any(has_ray)) {
        if (__hip_atomic_load(live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) break;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      // one node visit per lane holding a ray
      if (has_ray && trav4_step<kTravLanes, kSceneLds, false>(S, lds_nodes, lds_prims, o, d, 0.001, T, stk, rk, seed,
                                                              visits, ptests)) {
        SlotHit hr;
        hr.t = T.t_best;
        hr.prim = T.best;
        hr.face = T.face;
        hits[slot] = hr;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        atomicOr(&done[slot / kWave], 1ull << (slot % kWave));
        has_ray = false;
      }
    }
    unsigned long long n_vis = visits, n_pt = ptests;
    for (int off = 32; off > 0; off >>= 1) {
      n_vis += __shfl_down(n_vis, off);
      n_pt += __shfl_down(n_pt, off);
    }
    if (lane == 0) {
      DCounters* cs = P.counters + (blockIdx.x % kCounterSlots);
      atomicAdd(&cs->node_visits, n_vis);
      atomicAdd(&cs->prim_tests, n_pt);
    }
    return;
  }

  // -------------------------------------------------------------------- shading waves
  const int sw = wave - NT;  // 0 .. NS-1
  const int my_slot = sw * kWave + lane;
  const DCamera& C = P.cam;
  const DWork& W = P.work;
  const DPerlin* lds_perlin = S.n_lds_perlin > 0 ? reinterpret_cast<const DPerlin*>(lds_raw + L.perlin) : nullptr;

  unsigned long long w_next = 0, w_end = 0;
  bool exhausted = false;
  bool has_unit = false, active = false;
  uint32_t pxy = 0;
  int s_end = 0;
  uint32_t part_index = 0;
  v3 sum = V(0, 0, 0), o = V(0, 0, 0), d = V(0, 0, 0), att = V(0, 0, 0), em = V(0, 0, 0);
  int depth_left = 0;
  Rng rng{0, 0, 0, 0, 0};
  unsigned long long n_seg = 0, n_samp = 0;
  const uint32_t pix_per_chunk = (uint32_t)W.n_tiles_rank * (uint32_t)kTilePixels;

  for (;;) {
    // 1. a finished unit publishes its in-order sample sum (render.rs:58-69: *buf_c = c)
    if (has_unit && !active && rng.sample + 1u >= (uint32_t)s_end) {
      double* dst = P.partial + (size_t)part_index * 3;
      dst[0] = sum.x;
      dst[1] = sum.y;
      dst[2] = sum.z;
      has_unit = false;
    }
    // 2. idle lanes take units from the wave's window (as trace_kernel)
    const bool need = !has_unit;
    const unsigned long long mask = __ballot(need);
    if (mask != 0ull && !exhausted) {
      const unsigned long long k = __popcll(mask);
      const unsigned long long rank = __popcll(mask & split_lanemask_lt());
      const unsigned long long avail = w_end - w_next;
      unsigned long long idx;
      if (avail >= k) {
        idx = w_next + rank;
        w_next += k;
      } else {
        unsigned long long nb = 0;
        if (lane == 0) nb = atomicAdd(P.unit_counter, (unsigned long long)kWave);
        nb = bcast64(nb);
        idx = (rank < avail) ? (w_next + rank) : (nb + (rank - avail));
        w_next = nb + (k - avail);
        w_end = nb + kWave;
        if (nb >= W.n_units) exhausted = true;
      }
      if (need && idx < W.n_units) {
        const uint32_t pt = (uint32_t)W.n_chunks * (uint32_t)kTilePixels, i32 = (uint32_t)idx;
        const uint32_t lt = i32 / pt;
        const uint32_t g32 = lt * (uint32_t)W.tile_world + (uint32_t)W.tile_rank;
        const uint32_t y32 = g32 / (uint32_t)W.tiles_x;
        const uint32_t rem = i32 - lt * pt;
        const int tx = (int)(g32 - y32 * (uint32_t)W.tiles_x);
        const int ty = W.ty0 + (int)y32;
        const int chunk = (int)(rem / kTilePixels);
        const int lp = (int)(rem % kTilePixels);
        const int px = tx * kTile + (lp % kTile);
        const int py = ty * kTile + (lp / kTile);
        if (px < C.width && py < C.height) {
          has_unit = true;
          const int s0 = W.sample_base + chunk * W.chunk;
          s_end = min(W.samples, s0 + W.chunk);
          rng.sample = (uint32_t)s0 - 1u;
          rng.pixel = (uint32_t)py * (uint32_t)C.width + (uint32_t)px;
          pxy = (uint32_t)px | ((uint32_t)py << 16);
          part_index = (uint32_t)chunk * pix_per_chunk + lt * (uint32_t)kTilePixels + (uint32_t)lp;
          sum = V(0.0, 0.0, 0.0);
        }
      }
    }
    // 3. lanes between paths start the next sample (render.rs:60-65)
    const bool start = has_unit && !active && rng.sample + 1u < (uint32_t)s_end;
    n_samp += __popcll(__ballot(start));
    if (start) {
      rng.sample += 1u;
      rng.draw = 0;
      const double jx = (double)(pxy & 0xffffu) + rng_next(rng, seed);
      const double jy = (double)(pxy >> 16) + rng_next(rng, seed);
      camera_ray(C, rng, seed, jx, jy, o, d);
      att = V(1.0, 1.0, 1.0);
      em = V(0.0, 0.0, 0.0);
      depth_left = W.max_depth;
      active = depth_left > 0;  // (max_depth == 0 never reaches this kernel: render_window)
    }
    if (!__any(active)) {
      if (exhausted) break;  // as trace_kernel: with max_depth > 0 a held unit is active here
      continue;
    }
    // 4. the closest hit, by the traversal waves: post the ray, sleep until it is back
    const unsigned long long want = __ballot(active);
    n_seg += __popcll(want);
    if (active) {
      double* rp = rays + (size_t)my_slot * 6;
      rp[0] = o.x; rp[1] = o.y; rp[2] = o.z;
      rp[3] = d.x; rp[4] = d.y; rp[5] = d.z;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) atomicOr(&req[sw], want);
    for (;;) {
      const unsigned long long dn = bcast64(lds_load64(&done[sw]));
      if ((dn & want) == want) break;
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane == 0) __hip_atomic_store(&done[sw], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);

    // (a) hit record and the texture leaf of a diffuse / emitting material (as trace_kernel)
    bool hit = false, need_pn = false, need_r = false;
    int prim = -1, face = -1, leaf = -1, mat = 0, ptab = 0, mk = -1;
    double t_best = __builtin_inf(), psc = 0.0;
    Hit h;
    h.point = V(0.0, 0.0, 0.0);
    h.normal = h.point;
    h.t = h.u = h.v = 0.0;
    h.front_face = false;
    if (active) {
      const SlotHit hr = hits[my_slot];
      prim = hr.prim;
      face = hr.face;
      t_best = hr.t;
      if (prim >= 0) {
        hit = true;
        const DPrim pr = S.prims[prim];
        hit_record<false, false>(S, pr, face, o, d, t_best, rng, seed, h);
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
    // (b) Perlin marble values by the whole wave; (b') the scatter's random_in_unit_sphere by the
    // wave; (b'') the one normalisation a lane's shading needs
    const double pn = lds_perlin ? marble_coop((LdsPerlin*)lds_perlin, need_pn, ptab, psc, h.point)
                                 : marble_coop(S.perlin, need_pn, ptab, psc, h.point);
    const v3 rs = random_in_unit_sphere_coop(rng, seed, need_r);
    const v3 un = unit_fast(!active ? V(1.0, 1.0, 1.0) : (need_r && mk != RT_MAT_METAL) ? rs : d);
    // (c) emitted + scatter (render.rs:31-45) or the sky
    if (active) {
      bool alive;
      if (hit) {
        const DMat& m = S.mats[mat];
        alive = shade_pre(S, m, leaf, pn, rs, un, rng, seed, o, d, h, prim, face, att, em);
      } else {
        em = em + hmul(att, sky_unit(S, un));
        alive = false;
      }
      if (alive) alive = --depth_left > 0;
      if (!alive) {
        sum = sum + em;  // c += ray_color(...)
        active = false;
      }
    }
  }
  if (lane == 0) {
    atomicSub(live, 1u);
    DCounters* cs = P.counters + (blockIdx.x % kCounterSlots);
    atomicAdd(&cs->segments, n_seg);
    atomicAdd(&cs->samples, n_samp);
  }
}

// ------------------------------------------------------------------------------------------
// launch wrappers (rt_api.cpp): the split kernel serves reference scenes (no book-2 primitives)
// whose whole scene (4-wide tree, primitives, Perlin tables) fits in LDS next to the traversal
// stacks and the ray slots.
// ------------------------------------------------------------------------------------------
size_t split_lds_bytes(const DScene& S, int nt) {
  return split_lds_layout(S.n_lds_nodes4, S.n_lds_prims, S.n_lds_perlin, S.stack_depth4, nt).total;
}

template <int NT>
static hipError_t split_prepare1(const DScene& S, int* blocks_per_cu) {
  const size_t lds = split_lds_bytes(S, NT);
  hipError_t e = hipFuncSetAttribute((const void*)split_kernel<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, split_kernel<NT>, kTraceThreadsWide, lds);
}

// Supported traversal-wave counts (the rest of the 16 waves shade).
bool split_supported_nt(int nt) { return nt == 4 || nt == 6 || nt == 8; }

hipError_t split_prepare(const DScene& S, int nt, int* blocks_per_cu) {
  *blocks_per_cu = 0;
  if (S.exts || S.n_lds_nodes4 < S.n_nodes4 || S.n_lds_prims < S.n_prims) return hipSuccess;  // not eligible
  if (split_lds_bytes(S, nt) > (size_t)kLdsBytes) return hipSuccess;
  switch (nt) {
    case 4: return split_prepare1<4>(S, blocks_per_cu);
    case 6: return split_prepare1<6>(S, blocks_per_cu);
    case 8: return split_prepare1<8>(S, blocks_per_cu);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_split(const KParams& p, int nt, int blocks, hipStream_t stream) {
  const size_t lds = split_lds_bytes(p.scene, nt);
  switch (nt) {
    case 4: hipLaunchKernelGGL(split_kernel<4>, dim3(blocks), dim3(kTraceThreadsWide), lds, stream, p); break;
    case 6: hipLaunchKernelGGL(split_kernel<6>, dim3(blocks), dim3(kTraceThreadsWide), lds, stream, p); break;
    case 8: hipLaunchKernelGGL(split_kernel<8>, dim3(blocks), dim3(kTraceThreadsWide), lds, stream, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace rt
