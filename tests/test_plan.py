"""The work planning of a render call on the CPU (csrc/rt/plan.h through tools/plan_check): unit length
(`sample_chunk`), sample passes and partial-sum scratch for the BASELINE frames and the multi-GPU
partitions, on MI355X's 256 CUs x one 1024-thread block (262 144 resident lanes).  The figures are the
ones DESIGN.md §3.1 / §6 quote and the GPU runs measured (profiles/r03/shard_balance.json: chunk 8 at
N = 1, 4 at N = 2 and 4, 1 at N = 8)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "plan_check.cpp")
HDR = os.path.join(REPO, "shirley-raytracing-rs_amd", "csrc", "rt", "plan.h")
MEGA, WAVE, SPLIT = 1, 2, 3
LANES = 256 * 1024
MIB = 1 << 20
DEFAULT = 8192 * MIB


@pytest.fixture(scope="module")
def plan(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("plan") / "plan_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-o", exe, SRC], check=True, timeout=120)

    def run(*calls):
        args = [str(x) for call in calls for x in call]
        out = subprocess.run([exe] + args, check=True, capture_output=True, text=True, timeout=60).stdout.split("\n")
        keys = ("chunk", "n_chunks", "per_pass", "passes", "partial_bytes", "segments", "ok", "queue_window")
        res = [dict(zip(keys, map(int, line.split()))) for line in out if line.strip()]
        return res if len(res) > 1 else res[0]
    return run


def pixels(w, h):
    return ((w + 7) // 8) * ((h + 7) // 8) * 64


def test_headline_frame_one_pass(plan):
    # random_scene 1200x800 @ 500 spp: 8-sample units, one pass of 1.45 GB, per-block segments
    n = pixels(1200, 800)
    p = plan((n, 500, MEGA, LANES, 0, DEFAULT))
    assert p == dict(chunk=8, n_chunks=63, per_pass=63, passes=1, partial_bytes=n * 63 * 24, segments=1, ok=1,
                     queue_window=256)
    assert p["partial_bytes"] == 1_451_520_000


def test_headline_frame_bounded_scratch(plan):
    # scratch_mb = 512: three even passes of 21 chunks (the measured -4 % A/B of DESIGN §5)
    n = pixels(1200, 800)
    p = plan((n, 500, MEGA, LANES, 0, 512 * MIB))
    assert (p["chunk"], p["passes"], p["per_pass"]) == (8, 3, 21)
    assert p["partial_bytes"] <= 512 * MIB


def test_tile_partition_unit_length(plan):
    # a rank's share of the 150 x 100 tiles: 4-sample units at 2 and 4 ranks (4 ranks: lifted from 2 for
    # the per-block segments), one-sample units and the shared queue at 8 ranks
    n = pixels(1200, 800)
    r2, r4, r8 = plan((n // 2, 500, MEGA, LANES, 0, DEFAULT), (n // 4, 500, MEGA, LANES, 0, DEFAULT),
                      (n // 8, 500, MEGA, LANES, 0, DEFAULT))
    assert (r2["chunk"], r2["segments"]) == (4, 1)
    assert (r4["chunk"], r4["segments"]) == (4, 1)
    assert (r8["chunk"], r8["segments"]) == (1, 0)
    assert all(r["passes"] == 1 for r in (r2, r4, r8))


def test_sample_partition_unit_length(plan):
    # 8 ranks of the sample partition: every pixel, 62 or 63 samples each -> one-sample units
    n = pixels(1200, 800)
    a, b = plan((n, 63, MEGA, LANES, 0, DEFAULT), (n, 62, MEGA, LANES, 0, DEFAULT))
    assert a["chunk"] == b["chunk"] == 1 and a["passes"] == b["passes"] == 1


def test_config5_frames_one_pass_by_default(plan):
    # 1920x1080 @ 2000 spp: units capped at 16 samples, 125 chunks = 6.2 GB in one pass by default; a
    # 2 GiB bound cuts it into 3 even passes of 42 chunks
    n = pixels(1920, 1080)
    d, b = plan((n, 2000, MEGA, LANES, 0, DEFAULT), (n, 2000, MEGA, LANES, 0, 2048 * MIB))
    assert (d["chunk"], d["n_chunks"], d["passes"], d["partial_bytes"]) == (16, 125, 1, 6_220_800_000)
    assert (b["passes"], b["per_pass"]) == (3, 42) and b["partial_bytes"] <= 2048 * MIB


def test_cornell_frame(plan):
    # Cornell 600x600 @ 10 000 spp: 16-sample units, 625 chunks, one pass of 5.4 GB
    p = plan((pixels(600, 600), 10000, MEGA, LANES, 0, DEFAULT))
    assert (p["chunk"], p["n_chunks"], p["passes"]) == (16, 625, 1)


def test_32_bit_unit_limit_splits_passes(plan):
    # 64 pixels x (2^26 + 1) one-sample chunks: more units than a launch indexes in 32 bits, so the
    # megakernel and split engines run passes (tests/test_gpu_parity.py::test_edge_cases runs it)
    calls = [(64, (1 << 26) + 1, e, LANES, 1, 2048 * MIB) for e in (MEGA, SPLIT)]
    for p in plan(*calls):
        assert (p["passes"], p["per_pass"]) == (49, 1369569)
        assert p["per_pass"] * 64 <= 0xFFFFFFFF
    p = plan((64, (1 << 26) + 1, MEGA, LANES, 1, DEFAULT))
    assert p["per_pass"] * 64 <= 0xFFFFFFFF and p["passes"] * p["per_pass"] >= (1 << 26) + 1


def test_frame_too_large_is_refused(plan):
    # 65536 x 65536 pixels: one chunk alone exceeds the 32-bit unit index -> RT_E_UNSUPPORTED
    assert plan((pixels(65536, 65536), 1, MEGA, LANES, 0, DEFAULT))["ok"] == 0


def test_explicit_and_degenerate_chunks(plan):
    wave, clip, empty, small = plan((pixels(64, 64), 100, WAVE, LANES, 0, DEFAULT),
                                    (pixels(64, 64), 10, MEGA, LANES, 100, DEFAULT),
                                    (pixels(64, 64), 0, MEGA, LANES, 0, DEFAULT),
                                    (pixels(64, 64), 40, MEGA, LANES, 1, 1 * MIB))
    assert wave["chunk"] == 8 and wave["segments"] == 0          # the wavefront engine's own unit length
    assert (clip["chunk"], clip["n_chunks"]) == (10, 1)          # a unit never exceeds the range
    assert (empty["chunk"], empty["n_chunks"], empty["passes"]) == (1, 1, 1)
    # tests/test_gpu_ranges.py::test_sample_passes_are_bit_identical: 4 passes of 10 chunks at 1 MiB
    assert (small["passes"], small["per_pass"]) == (4, 10) and small["partial_bytes"] <= MIB


def test_every_pass_fits_its_bound(plan):
    # randomised: passes cover the chunks, fit the bound (unless one chunk alone exceeds it) and the
    # 32-bit index, and are even (no pass holds more than one chunk over another)
    import random
    rng = random.Random(7)
    calls = []
    for _ in range(200):
        n = 64 * rng.randint(1, 40000)
        calls.append((n, rng.randint(0, 20000), rng.choice((MEGA, WAVE, SPLIT)), LANES, rng.choice((0, 0, 1, 3, 16, 64)),
                      rng.choice((1, 64, 512, 2048, 8192)) * MIB))
    for (n, count, engine, _, sc, budget), p in zip(calls, plan(*calls)):
        assert p["ok"] == 1
        work = max(1, count)
        assert p["n_chunks"] == -(-work // p["chunk"]) and 1 <= p["chunk"] <= work
        assert p["passes"] * p["per_pass"] >= p["n_chunks"] > (p["passes"] - 1) * p["per_pass"]
        assert p["partial_bytes"] == n * p["per_pass"] * 24
        assert p["partial_bytes"] <= max(budget, n * 24)
        if engine in (MEGA, SPLIT):
            assert n * p["per_pass"] <= 0xFFFFFFFF
        if sc == 0 and engine != WAVE:
            assert p["chunk"] <= 16


def test_shared_queue_window_follows_units_per_lane(plan):
    # one-sample units on the shared queue: 256-unit windows (4 units per lane per atomic on the one
    # counter) where a lane has >= 128 units — the 8-rank share of the headline (229 per lane: 24.1 -> 22.9
    # ms against 64-unit windows) and its 8-rank sample share (227) —, else 64 — cfg1 400x225 @ 50 (17.7
    # per lane: 1490 Msamples/s with 256-unit windows, 1830-1880 with 64; gpurun_out/r05a, r05f1), where
    # 4-per-lane windows leave each wave too few tiles to average their cost over
    cfg1 = plan((pixels(400, 225), 50, MEGA, LANES, 0, DEFAULT))
    r8t = plan((pixels(1200, 800) // 8, 500, MEGA, LANES, 0, DEFAULT))
    r8s = plan((pixels(1200, 800), 62, MEGA, LANES, 0, DEFAULT))
    for p in (cfg1, r8t, r8s):
        assert p["segments"] == 0 and p["chunk"] == 1
    assert cfg1["queue_window"] == 64 and r8t["queue_window"] == 256 and r8s["queue_window"] == 256
    # the boundary: 128 units per resident lane
    edge = 128 * LANES // 64  # pixels of 64-pixel tiles x 1 chunk
    below, at = plan((edge - 64, 1, MEGA, LANES, 1, DEFAULT), (edge, 1, MEGA, LANES, 1, DEFAULT))
    assert below["queue_window"] == 64 and at["queue_window"] == 64  # (1 chunk: 2 units per lane)
    lo, hi = plan((pixels(1200, 800), 34, MEGA, LANES, 1, DEFAULT), (pixels(1200, 800), 35, MEGA, LANES, 1, DEFAULT))
    assert (lo["queue_window"], hi["queue_window"]) == (64, 256)  # 960000 x 34 < 128 x 262144 <= 960000 x 35
    # a multi-pass frame: the rule counts one pass's units (each pass is its own launch and pool), so the
    # 35-sample frame in passes of 7 chunks (< 128 units per lane each) takes 64-unit windows
    split = plan((pixels(1200, 800), 35, MEGA, LANES, 1, pixels(1200, 800) * 24 * 7))
    assert (split["passes"], split["per_pass"], split["queue_window"]) == (5, 7, 64)
