// plan.h — how a render call's samples are cut into work units and sample passes (host only, pure:
// no HIP, no context), so the rules can be checked on the CPU (tests/test_plan.py via tools/plan_check).
//
// A work unit is (pixel, chunk of `chunk` consecutive samples of the call's range); a pass traces
// `per_pass` chunks of every pixel and holds their partial sums ([chunks][pixels][3] f64) in scratch.
#pragma once

#include <stdint.h>

#include <algorithm>

#include "../../../include/shirley_rt.h"

namespace rt {

constexpr int kWfDefaultChunk = 8;          // wavefront engine's unit length (its slots regenerate anyway)
// Default bound of a pass's partial sums.  Every extra sample pass costs its launch's ramp and drain on
// MI355X: ~3.9 ms on the headline frame (3 passes of <= 512 MiB: 189.5 ms of trace against 181.7 ms in
// one pass) and ~20 ms on the 1920x1080 @ 2000-spp frames (3 passes of <= 2 GiB: gen_spheres 847 ms and
// final_scene 2902 ms against 803 / 2864 ms in one pass of 6.2 GB).  So the default keeps every BASELINE
// frame in one pass (at most 6.2 GB of the 288 GB); scratch_mb sets a tighter bound (down to one chunk
// per pass) where memory matters more than those milliseconds — the frame is bit-identical either way.
constexpr long long kDefaultScratchMiB = 8192;

// Work units a megakernel wave takes per queue atomic (multiples of the wave size): kSegmentWindow from a
// block's own segment; from the one shared queue kQueueWindow or kSegmentWindow (SamplePlan.queue_window).
constexpr unsigned kSegmentWindow = 64;
constexpr unsigned kQueueWindow = 256;

struct SamplePlan {
  int chunk = 1;          // samples per unit
  int n_chunks = 0;       // chunks of the call's range
  int per_pass = 0;       // chunks per sample pass
  int passes = 0;
  long long partial_bytes = 0;  // scratch of one pass
  bool segments = false;  // megakernel per-block unit segments (units of >= 4 samples)
  unsigned queue_window = kQueueWindow;  // shared queue (segments off): units per queue atomic
  bool ok = true;        // false: a pass cannot index one chunk of the frame in 32 bits
};

// n_pix: pixels of the call's tiles (tiles x 64), count: samples in the range, lanes: resident megakernel
// lanes of the device, sample_chunk: the caller's unit length (0 = automatic), budget: scratch bytes.
inline SamplePlan plan_samples(long long n_pix, int count, int engine, long long lanes, int sample_chunk,
                               long long budget) {
  SamplePlan P;
  // samples per unit: ~256 units per resident lane, so that a wave's last units (its lanes finish at
  // different times) cost little, and no unit longer than 16 samples (MI355X: headline frame chunk
  // 23 -> 8 +0.5 %, final_scene 19 -> 7 +5 %, gen_spheres @ 16 spp 3 -> 1 +24 %; the 1920x1080 @ 2000
  // spp frames 61 -> 16 +1.5-6 %; chunks 25 / 50 on the headline frame -3 / -8 %).  Short units cost
  // only partial-sum traffic (24 B written + read per unit); the scratch they need is bounded by the
  // sample passes below, not by the unit length.
  const int work = std::max(1, count);
  int chunk = sample_chunk;
  if (chunk == 0 && engine == RT_ENGINE_WAVEFRONT) chunk = kWfDefaultChunk;
  if (chunk == 0) {
    const long long want_units = 256 * lanes;
    long long n_chunks = n_pix > 0 ? (want_units + n_pix - 1) / n_pix : 1;
    n_chunks = std::max(1LL, std::min<long long>(n_chunks, work));
    chunk = std::min(16, (int)((work + n_chunks - 1) / n_chunks));
    // the megakernel's per-block unit segments serve units of >= 4 samples: lift a shorter automatic
    // chunk to 4 while that still leaves >= 100 units per lane (measured: the 4-rank frame 47.6 -> 47.1
    // ms; with fewer units per lane — 8 ranks, 57 — the longer units' end costs more than the segments
    // gain, 24.5 -> 24.9 ms)
    if (engine == RT_ENGINE_MEGAKERNEL && chunk < 4 && work >= 4 && n_pix > 0 &&
        n_pix * ((work + 3) / 4) >= 100 * lanes)
      chunk = 4;
  }
  chunk = std::max(1, std::min(chunk, work));
  P.chunk = chunk;
  P.n_chunks = (work + chunk - 1) / chunk;
  // per-block unit segments (trace.hip): for units of >= 4 samples (measured: headline +2 %, gen_spheres
  // +11 %, final_scene +2.4 %, 2 ranks +2.4 %; with 1- or 2-sample units — small frames, 4 and 8 ranks
  // — the shared queue is as fast or faster: cfg1 -17 %, the 8-rank frame -6 % with segments).  A wave
  // takes kSegmentWindow (64) units per queue atomic from its block's segment, kQueueWindow (256) from the
  // shared queue, whose one counter all waves hit — the 8-rank frame (1-sample units)
  // 24.5 -> 23.4 ms with 256-unit windows (512: 23.8, 1024: 25.2; with segments 128 / 256 cost the
  // headline 0.4 / 1.8 %), profiles/r04/shard_scan/.
  P.segments = engine == RT_ENGINE_MEGAKERNEL && chunk >= 4;
  // The shared queue's window: 256 units (4 per lane) per atomic where a lane has >= 128 units (the
  // 8-rank share of the headline, 229: one counter for all waves, 24.1 -> 22.9 ms against 64-unit
  // windows), else 64.  A wave's time is the sum of its windows', whose cost follows the tile they
  // came from (sky vs glass ground): with few units per lane, 4-per-lane windows leave each wave only
  // a few tiles to average over, and the waves end far apart — cfg1 400x225 @ 50 (17.7 units per lane)
  // ran 1490 Msamples/s with 256-unit windows and 1830-1880 with 64 (gpurun_out/r05a, r05f1); serving
  // just the pool's last 1 M units in 64-unit windows from a second counter did not help (r05f1: the
  // imbalance builds up over the whole frame, not at its end), nor did shrinking windows near the end.
  // Each sample pass is its own launch with its own pool, so the rule counts a pass's units (below).

  // sample passes: at most `budget` bytes of [chunks][pixels][3] f64 partial sums per pass
  const long long chunk_bytes = std::max<long long>(1, n_pix * 3 * (long long)sizeof(double));
  long long per_pass = std::max(1LL, std::min<long long>(P.n_chunks, std::max(1LL, budget) / chunk_bytes));
  if (engine == RT_ENGINE_MEGAKERNEL || engine == RT_ENGINE_SPLIT) {
    // the megakernel indexes a pass's units and partial slots (n_pix * chunks) in 32 bits
    const long long max_chunks = n_pix > 0 ? 0xffffffffLL / n_pix : P.n_chunks;
    if (max_chunks < 1) {
      P.ok = false;
      return P;
    }
    per_pass = std::min<long long>(per_pass, max_chunks);
  }
  P.passes = (int)((P.n_chunks + per_pass - 1) / per_pass);
  P.per_pass = (P.n_chunks + P.passes - 1) / P.passes;  // even passes
  P.partial_bytes = std::max<long long>(1, n_pix * P.per_pass * 3) * (long long)sizeof(double);
  {
    const long long units = n_pix * (long long)P.per_pass;  // one pass's launch
    P.queue_window = (lanes > 0 && units >= 128 * lanes) ? kQueueWindow : kSegmentWindow;
  }
  return P;
}

}  // namespace rt
