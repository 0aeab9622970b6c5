"""SURVEY.md §7's statistical check of the RNG, on the CPU through the oracle.

The reference draws every random number from per-worker `thread_rng` streams (main.rs:98,119;
render.rs:61-62; the rejection samplers of core/math.rs:32-81).  This build replaces them, in the oracle
and in the kernels alike, by counter-based Philox4x32-10: draw d of sample s of pixel p under seed k is
half (d & 1) of Philox(counter = (d >> 1, s, p, 0), key = k).  Every GPU parity test
compares the device with the oracle on that same keying, so a keying defect — a counter reused across
draws, samples or pixels, or correlated neighbouring streams — would pass them all.  This file checks the
keying itself:

* the oracle's draws equal an independent numpy restatement of that keying (pins the counter layout the
  GPU tests then hold the device to);
* the counter map is injective over the BASELINE ranges and disjoint from every other stream the build
  draws from (scene construction, Perlin tables, the book-2 time / medium side streams);
* renders under two disjoint groups of seeds converge to the same image: per pixel and channel the
  difference of the two groups' means is consistent with their batch-to-batch spread (z-scores), with no
  spatial correlation between neighbouring pixels' differences — and the same statistic flags a group
  compared with itself (identical streams) as a defect.
"""
import numpy as np
import pytest

import oracle_lib as O
from raytracer import SceneBuilder, scene_camera

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Random123 Philox4x32-10 on uint32 arrays (Salmon et al., SC'11): an independent restatement."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32) for x in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint32).copy()
    k1 = np.asarray(k1, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        for r in range(10):
            if r:
                k0 = k0 + W0
                k1 = k1 + W1
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def path_draw_u64(seed, pixel, sample, draw):
    """The build's path-stream keying: counter (draw >> 1, sample, pixel, 0), key = seed."""
    seed = np.asarray(seed, dtype=np.uint64)
    draw = np.asarray(draw, dtype=np.uint32)
    o0, o1, o2, o3 = philox4x32_10(draw >> np.uint32(1), sample, pixel, np.zeros_like(draw),
                                   (seed & MASK32).astype(np.uint32), (seed >> np.uint64(32)).astype(np.uint32))
    even = o0.astype(np.uint64) | (o1.astype(np.uint64) << np.uint64(32))
    odd = o2.astype(np.uint64) | (o3.astype(np.uint64) << np.uint64(32))
    return np.where((draw & np.uint32(1)) == 0, even, odd)


def test_numpy_philox_matches_random123_kat():
    # the first published Random123 kat_vectors line for philox4x32-10 (ctr 0, key 0), also in test_oracle_kat
    o = philox4x32_10([0], [0], [0], [0], [0], [0])
    assert [int(x[0]) for x in o] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_oracle_draws_follow_the_stated_keying():
    rng = np.random.default_rng(1)
    n = 3000
    seeds = np.concatenate([np.array([0, 0x5EED, 2**64 - 1], dtype=np.uint64),
                            rng.integers(0, 2**64 - 1, n - 3, dtype=np.uint64, endpoint=True)])
    pix = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    smp = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    drw = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    pix[:8], smp[:8], drw[:8] = 0, 0, np.arange(8)  # draws 0..7 of one stream: both halves of 4 blocks
    want = path_draw_u64(seeds, pix, smp, drw)
    L = O.lib()
    got = np.array([L.or_rng_u64(int(k), int(p), int(s), int(d)) for k, p, s, d in zip(seeds, pix, smp, drw)],
                   dtype=np.uint64)
    assert np.array_equal(got, want)
    # the f64 conversion: rand 0.8's Standard, (u64 >> 11) * 2^-53
    f = np.array([L.or_rng_f64(int(k), int(p), int(s), int(d)) for k, p, s, d in zip(seeds[:50], pix[:50], smp[:50],
                                                                                         drw[:50])])
    assert np.array_equal(f, (want[:50] >> np.uint64(11)).astype(np.float64) * 2.0**-53)


# the BASELINE ranges (BASELINE.json configs): the largest frame is 1920x1080, the most samples 10 000
MAX_PIXELS = 1920 * 1080
MAX_SAMPLES = 10000
MAX_DEPTH = 50


def test_counter_map_is_injective_over_baseline_ranges():
    """(pixel, sample, draw) -> (counter, half) puts each index in its own 32-bit word (and the draw's
    low bit in the half), so it is injective while every index fits its word.  Pixel indices (py W + px)
    stay below W H <= 1920 x 1080 < 2^21, samples below 2^14; a path's draw counter (uint32 on the device)
    grows by 3 per unit-sphere attempt and 2 per disk attempt from 4 camera draws: reaching 2^32 would take
    ~2^25 rejected attempts in one bounce (probability 0.48^(2^25)), so it never wraps.  Checked on every
    corner of those ranges plus a random grid: all counters distinct, all 64-bit draws distinct."""
    assert MAX_PIXELS < 2**21 and MAX_SAMPLES < 2**14
    assert 4 + MAX_DEPTH * 3 * 2**20 < 2**32  # a million rejected attempts per bounce still fit
    rng = np.random.default_rng(2)
    corners_p = np.array([0, 1, 1919, 1920, MAX_PIXELS - 1], dtype=np.uint32)
    corners_s = np.array([0, 1, MAX_SAMPLES - 1], dtype=np.uint32)
    corners_d = np.array([0, 1, 2, 3, 2**31, 2**32 - 2, 2**32 - 1], dtype=np.uint32)
    P, S, D = np.meshgrid(corners_p, corners_s, corners_d, indexing="ij")
    p = np.concatenate([P.ravel(), rng.integers(0, MAX_PIXELS, 20000).astype(np.uint32)])
    s = np.concatenate([S.ravel(), rng.integers(0, MAX_SAMPLES, 20000).astype(np.uint32)])
    d = np.concatenate([D.ravel(), rng.integers(0, 4 + MAX_DEPTH * 300, 20000).astype(np.uint32)])
    key = np.unique(np.stack([p, s, d]), axis=1)
    ctr = np.stack([key[2] >> 1, key[1], key[0], np.zeros_like(key[0]), key[2] & 1])
    assert np.unique(ctr, axis=1).shape[1] == key.shape[1]
    v = path_draw_u64(np.full(key.shape[1], 0x5EED, dtype=np.uint64), key[0], key[1], key[2])
    assert np.unique(v).size == v.size


def test_streams_are_disjoint():
    """Counter word 3 (and word 2) separate the build's streams: paths (word 3 = 0), the book-2 ray time
    (0x40000000) and media (0x80000000 | object) side streams (rt_device.h kStream*, oracle.c STREAM_*), and
    scene / Perlin construction (word 2 = 0xFFFFFFFF, word 3 = stream id >= 1, csrc/host/rng.hpp)."""
    path_w3 = {0}
    time_w3 = {0x40000000}
    medium_w3 = {0x80000000 | obj for obj in (0, 1, 1408, 2**20)}
    scene_w3 = {1, 2, 3} | {16 + j for j in range(8)}
    groups = [path_w3, time_w3, medium_w3, scene_w3]
    for i in range(len(groups)):
        for j in range(i + 1, len(groups)):
            assert not (groups[i] & groups[j])
    # scene streams also differ in word 2: a pixel index never reaches 0xFFFFFFFF
    assert MAX_PIXELS - 1 < 0xFFFFFFFF
    assert max(medium_w3) < 2**32 and min(medium_w3) >= 0x80000000 > max(time_w3)


def _render(desc, cam, seed, spp, max_depth=MAX_DEPTH):
    out, _ = O.OracleScene(desc).render(cam, O.params(spp, max_depth, seed))
    return out / spp


def _z_stats(scene, a_seeds, b_seeds, spp, size=32, aspect="square"):
    """Per pixel and channel: z = (mean_A - mean_B) / sqrt(se_A^2 + se_B^2), each group's mean and
    standard error from its batches (one batch per seed, `spp` samples each)."""
    desc = SceneBuilder.builtin(scene, 7).finalize(7)  # fixed geometry and Perlin tables; only the render seed varies
    cam = scene_camera(scene, size, aspect)
    A = np.stack([_render(desc, cam, s, spp) for s in a_seeds])
    B = np.stack([_render(desc, cam, s, spp) for s in b_seeds])
    ma, mb = A.mean(0), B.mean(0)
    va, vb = A.var(0, ddof=1) / len(a_seeds), B.var(0, ddof=1) / len(b_seeds)
    se = np.sqrt(va + vb)
    live = se > 0  # (a pixel whose every sample sees the same constant, e.g. pure sky rows, has no spread)
    z = np.where(live, (ma - mb) / np.where(live, se, 1.0), 0.0)
    return z, live


def _neighbour_corr(z, live):
    """Correlation of horizontally and vertically adjacent pixels' z (channel-averaged)."""
    zc = z.mean(-1)
    lc = live.all(-1)
    out = []
    for a, b, la, lb in ((zc[:, :-1], zc[:, 1:], lc[:, :-1], lc[:, 1:]), (zc[:-1], zc[1:], lc[:-1], lc[1:])):
        m = la & lb
        out.append(float(np.corrcoef(a[m], b[m])[0, 1]))
    return out


# Scenes exercising every sampler: unit-sphere rejection (lambertian, metal), the dielectric's
# conditional uniform, the lens disk, Perlin and checker textures (random); emitters seen directly
# and through deep diffuse paths (cornell).  Two groups of 8 seeds x 64 spp = 512 spp per group.
@pytest.mark.parametrize("scene", ["random", "cornell"])
def test_independent_seed_groups_converge_to_the_same_image(scene):
    z, live = _z_stats(scene, range(1, 9), range(101, 109), spp=64)
    zl = z[live]
    assert zl.size > 0.8 * z.size  # most pixels carry variance
    # the batch-mean z of two 8-batch groups is t-like with ~14 degrees of freedom: mean 0, variance
    # ~14/12; bounds are > 6 standard errors for 3000 channels
    assert abs(float(zl.mean())) < 0.15, zl.mean()
    assert 0.8 < float(zl.var()) < 1.6, zl.var()
    assert float(np.mean(np.abs(zl) > 4.5)) < 0.005  # t14 tail P(|t| > 4.5) ~ 5e-4
    for r in _neighbour_corr(z, live):
        assert abs(r) < 0.15, r  # ~1000 pairs: |r| > 0.15 is ~4.7 standard errors


def test_seed_group_against_itself_is_flagged():
    """The statistic's power against the defect it guards: two groups drawing the same streams (what a
    counter reused across seeds would give) show no spread at all — the variance bound above fails."""
    z, live = _z_stats("random", range(1, 5), range(1, 5), spp=16, size=16)
    assert float(np.var(z[live])) < 1e-12
