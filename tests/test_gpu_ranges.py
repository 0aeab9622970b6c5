"""ABI 6 on the GPU: the sample range of rt_render_params ("tile rect / sample range"),
the sample passes that bound the partial-sum scratch, the sample partition of the multi-GPU calls and the
scene-digest check (reference: the per-pixel sample loop, /root/reference/src/raytracer/render.rs:58-69).

* A range [b, e) renders exactly the samples b..e-1 of every pixel: with sample_chunk >= e - b its
  per-pixel sums equal the oracle's in-order sums over the same range (the oracle's render_scanline
  restatement takes the same range), within the module tolerance of test_gpu_parity.py.
* Splitting [0, S) into ranges changes only the order of additions: sum([0,k)) + sum([k,S)) equals the
  one-call frame within |d| <= 1e-12 |sum| per channel (REASSOC below).
* Sample passes keep every per-pixel addition and its order (reduce_kernel `accumulate`): frames are
  bit-identical for every scratch bound.
"""
import numpy as np
import pytest

import oracle_lib as O
import raytracer as rt
from test_gpu_parity import check_parity

pytestmark = pytest.mark.gpu

SEED = 0x5EED
REASSOC = 1e-12  # relative per-channel bound of a reassociated sum


def _reassoc_close(a, b):
    assert a.shape == b.shape
    assert np.all(np.abs(a - b) <= REASSOC * np.maximum(np.abs(a), np.abs(b)) + 1e-300), \
        f"max rel diff {np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)):.3g}"


@pytest.fixture(scope="module")
def random_scene():
    return rt.scenes.random_scene(SEED).finalize(SEED)


@pytest.mark.parametrize("engine", ["megakernel"])
def test_range_matches_oracle_range(gpu, random_scene, engine):
    spp, b, n = 12, 5, 4  # samples [5, 9) of a 12-spp frame
    cam = rt.default_camera(40, "std16x9")
    gpu.upload(random_scene)
    got = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=n, sample_begin=b, sample_count=n,
                                            engine=engine))
    want, ocnt = O.OracleScene(random_scene).render(cam, O.params(spp, 50, SEED, sample_begin=b, sample_count=n))
    check_parity(got, want, n)
    c = gpu.counters()
    assert c.samples == cam.image_width * cam.image_height * n == ocnt.samples


def test_ranges_sum_to_the_frame(gpu, random_scene):
    spp = 24
    cam = rt.default_camera(48, "std16x9")
    gpu.upload(random_scene)
    s = dict(samples=spp, seed=SEED, sample_chunk=4)
    full = gpu.render(cam, rt.RenderSettings(**s))
    a = gpu.render(cam, rt.RenderSettings(**s, sample_begin=0, sample_count=8))
    b = gpu.render(cam, rt.RenderSettings(**s, sample_begin=8))  # count 0: to the end
    _reassoc_close(a + b, full)
    # chunk-aligned ranges render the frame's own units: the first range's chunk sums are the frame's
    # first two chunk sums, so a frame whose chunks are summed in that order is exact
    c0 = gpu.render(cam, rt.RenderSettings(**s, sample_begin=0, sample_count=4))
    c1 = gpu.render(cam, rt.RenderSettings(**s, sample_begin=4, sample_count=4))
    assert np.array_equal(c0 + c1, a)
    # an empty range is an all-zero frame; a range beyond the frame is refused
    z = gpu.render(cam, rt.RenderSettings(**s, sample_begin=spp))
    assert not z.any() and gpu.counters().samples == 0
    with pytest.raises(rt.RtError, match="sample range"):
        gpu.render(cam, rt.RenderSettings(**s, sample_begin=20, sample_count=5))
    with pytest.raises(rt.RtError, match="sample range"):
        gpu.render(cam, rt.RenderSettings(**s, sample_begin=-1))


@pytest.mark.parametrize("engine", ["megakernel", "wavefront", "split"])
def test_sample_passes_are_bit_identical(gpu, random_scene, engine):
    """scratch_mb = 1 cuts a 64x64 @ 40 spp frame with 1-sample units (98 KB of partials per chunk) into
    4 passes of 10 chunks; the frame is bit-identical to the one-pass frame and the counters add up."""
    cam = rt.default_camera(64, "square")
    gpu.upload(random_scene)
    s = dict(samples=40, seed=SEED, sample_chunk=1, engine=engine)
    one = gpu.render(cam, rt.RenderSettings(**s))
    c1 = gpu.counters()
    assert c1.passes == 1 and c1.n_chunks == 40
    many = gpu.render(cam, rt.RenderSettings(**s, scratch_mb=1))
    c4 = gpu.counters()
    assert c4.passes == 4 and c4.trace_launches == 4 and c4.scratch_bytes <= (1 << 20)
    assert np.array_equal(one, many)
    assert c4.samples == c1.samples and c4.segments == c1.segments
    # the same through a sample range and the packed tile layout
    r1 = gpu.render(cam, rt.RenderSettings(**s, sample_begin=7, sample_count=29))
    r4 = gpu.render(cam, rt.RenderSettings(**s, sample_begin=7, sample_count=29, scratch_mb=1))
    assert gpu.counters().passes == 3
    assert np.array_equal(r1, r4)


def test_scratch_oom_falls_back_to_passes(gpu, random_scene, monkeypatch):
    """A partial buffer the device cannot allocate (simulated: SHIRLEY_SIMULATE_OOM_MB) makes the call halve
    its pass size until it fits: the frame is bit-identical to the one-pass frame, the call succeeds with
    more passes, and no stale error message of the refused allocation is left."""
    cam = rt.default_camera(64, "square")
    gpu.upload(random_scene)
    s = rt.RenderSettings(samples=40, seed=SEED, sample_chunk=1)
    one = gpu.render(cam, s)
    assert gpu.counters().passes == 1
    from raytracer import _native as N
    before = N.rt_lib().rt_last_error(gpu.handle).decode()
    monkeypatch.setenv("SHIRLEY_SIMULATE_OOM_MB", "1")
    lim = gpu.render(cam, s)
    c = gpu.counters()
    assert c.passes >= 4 and c.scratch_bytes <= (1 << 20)
    assert np.array_equal(one, lim)
    assert N.rt_lib().rt_last_error(gpu.handle).decode() == before


def _sample_split(gpu, cam, settings, world):
    """RT_PARTITION_SAMPLES simulated on one device: rank r renders all pixels for its share of the
    frame's samples; the per-rank frames are summed in rank order (what the band sum computes)."""
    spp = settings["samples"]
    parts = []
    for r in range(world):
        b, e = spp * r // world, spp * (r + 1) // world
        if e > b:
            parts.append(gpu.render(cam, rt.RenderSettings(**settings, sample_begin=b, sample_count=e - b)))
        else:
            parts.append(np.zeros((cam.image_height, cam.image_width, 3)))
    out = parts[0].copy()
    for p in parts[1:]:
        out += p
    return out


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sample_split_equals_frame_within_reassociation(gpu, random_scene, world):
    cam = rt.default_camera(40, "std16x9")
    gpu.upload(random_scene)
    s = dict(samples=20, seed=SEED, sample_chunk=20)
    full = gpu.render(cam, rt.RenderSettings(**s))
    _reassoc_close(_sample_split(gpu, cam, s, world), full)


@pytest.mark.parametrize("partition", ["samples", "tiles"])
def test_multi_one_device_partitions(gpu, random_scene, partition):
    """rt_render_multi and rt_render_sharded with either partition on a one-rank communicator: the
    digest check, the render, the exchange (all-to-all + band sum + gather, or the tile gather) all run,
    and the frame equals rt_render's bit for bit (one rank renders everything)."""
    import torch
    cam = rt.default_camera(53, "std16x9")
    gpu.upload(random_scene, "sah")
    s = rt.RenderSettings(samples=5, seed=SEED, partition=partition)
    want = gpu.render(cam, s)
    assert np.array_equal(rt.render_multi([gpu], cam, s), want)
    comm = gpu.comm_init_rank(rt.comm_unique_id(), 1, 0)
    try:
        stream = torch.cuda.current_stream().cuda_stream
        a = torch.full((cam.image_height, cam.image_width, 3), -1.0, dtype=torch.float64, device="cuda")
        gpu.render_sharded(comm, cam, s, a.data_ptr(), stream)
        torch.cuda.synchronize()
        assert np.array_equal(a.cpu().numpy(), want)
        # a sample range is the frame's: the partition splits it
        s2 = rt.RenderSettings(samples=5, seed=SEED, partition=partition, sample_begin=1, sample_count=3)
        gpu.render_sharded(comm, cam, s2, a.data_ptr(), stream)
        torch.cuda.synchronize()
        assert np.array_equal(a.cpu().numpy(), gpu.render(cam, s2))
    finally:
        comm.close()


def test_scene_digest_on_device(gpu, random_scene):
    gpu.upload(random_scene, "sah")
    d = gpu.digest()
    assert d == rt.scene_digest(random_scene, "sah")
    gpu.upload(random_scene, "sah")
    assert gpu.digest() == d
    gpu.upload(rt.scenes.create_cornell_box().finalize(SEED), "sah")
    assert gpu.digest() != d


def test_cli_progressive_checkpoints_and_resume(tmp_path):
    """ray-cli --progressive K renders the frame as K sample ranges and checkpoints the running sums after
    each (--dump-accum FILE + FILE.json); --resume continues a checkpoint.  The resumed run ends with the
    same bits as the uninterrupted one (the same ranges added in the same order), and both equal the
    one-call frame within reassociation."""
    import json
    import os
    import subprocess
    from raytracer import _native as N
    cli = os.path.join(N.BIN_DIR, "ray-cli")
    common = ["render", "random", "-w", "48", "-s", "12", "--seed", "0x5EED", "--sample-chunk", "2"]
    one, full, part = (str(tmp_path / n) for n in ("one.bin", "full.bin", "part.bin"))
    for extra in (["--dump-accum", one],
                  ["--progressive", "3", "--dump-accum", full]):
        r = subprocess.run([cli] + common + ["-o", str(tmp_path / "x.png")] + extra, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    assert json.load(open(full + ".json"))["samples_done"] == 12
    # interrupted after the first of 3 ranges (samples [0, 4)), then resumed for the rest
    r = subprocess.run([cli] + ["render", "random", "-w", "48", "-s", "4", "--seed", "0x5EED", "--sample-chunk", "2",
                                "-o", str(tmp_path / "y.png"), "--progressive", "1", "--dump-accum", part],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert json.load(open(part + ".json"))["samples_done"] == 4
    r = subprocess.run([cli] + common + ["-o", str(tmp_path / "z.png"), "--progressive", "2", "--resume", part,
                                         "--dump-accum", part], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    a = np.fromfile(full)
    assert np.array_equal(np.fromfile(part), a)
    b = np.fromfile(one)
    assert np.all(np.abs(a - b) <= REASSOC * np.abs(b) + 1e-300)
    ck = json.load(open(part + ".json"))
    assert ck["samples_done"] == 12 and ck["max_depth"] == 50 and ck["sample_chunk"] == 2 and len(ck["scene_digest"]) == 16


@pytest.mark.parametrize("change,why", [(["--seed", "0x5EEE"], "seed"), (["-m", "10"], "max_depth"),
                                        (["--sample-chunk", "4"], "sample_chunk"), (["-w", "40"], "x"),
                                        (["--camera-fov", "30"], "camera"), (["-s", "3"], "covers"),
                                        (["@scene", "earth"], "scene")])
def test_cli_resume_refuses_another_frame(tmp_path, change, why):
    """--resume continues only a checkpoint of the same frame — scene digest, camera, size,
    seed, max_depth and unit length equal, and no more samples done than the run renders; anything else
    exits non-zero with the reason instead of adding the sums of another frame.  (The demo scene does not
    depend on the seed, so a changed seed is refused as a seed, not as another scene.)"""
    import os
    import subprocess
    from raytracer import _native as N
    cli = os.path.join(N.BIN_DIR, "ray-cli")
    ck = str(tmp_path / "ck.bin")
    base = ["render", "demo", "-w", "48", "-s", "4", "--seed", "0x5EED", "--sample-chunk", "2"]
    r = subprocess.run([cli] + base + ["-o", str(tmp_path / "a.png"), "--dump-accum", ck], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    argv = base[:] + ["-o", str(tmp_path / "b.png"), "--resume", ck, "--progressive", "1"]
    if change[0] == "@scene":
        argv[1] = change[1]
    elif change[0] in argv:
        argv[argv.index(change[0]) + 1] = change[1]
    else:
        argv += change
    r = subprocess.run([cli] + argv, capture_output=True, text=True)
    assert r.returncode != 0 and why in r.stderr, r.stderr
    # and the same checkpoint resumes as the same frame
    ok = base[:]
    ok[ok.index("-s") + 1] = "6"
    r = subprocess.run([cli] + ok + ["-o", str(tmp_path / "c.png"), "--resume", ck, "--progressive", "1"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
