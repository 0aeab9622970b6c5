"""HIP path vs the f64 CPU oracle, through the C ABI (include/shirley_rt.h).

Tolerance (north star: "within a stated per-channel float tolerance under a fixed RNG seed"):
both sides evaluate the reference's binary64 formulas in the same order with the same counter RNG,
so per-sample colours agree to the last ulp except where the device's transcendentals (ocml sin,
log, acos, atan2, pow) differ from glibc's by an ulp — a last-bit difference in an attenuation — or,
rarely, such an ulp flips a comparison (checker sign, Schlick vs U, texel index) or two objects tie
at exactly the same t, which changes one whole path.  One rule for every GPU-vs-oracle comparison
(check_parity):
  * >= 99 % of pixel channels bit-identical (PARITY_EXACT; sample_chunk = spp: in-order sums like
    render.rs:58-69),
  * every channel within TOL = 1e-10 * spp absolute of the oracle, except at most 0.1 % of pixels
    (PARITY_OUTLIERS: a flipped path changes one sample by up to the path's radiance).
One stated exception: BASELINE config 5's band (CFG5_EXACT below, with its reason).  On top of that rule,
each comparison has its own floor (EXACT_FLOOR): its measured fraction in profiles/r04/parity_fractions.jsonl
(SHIRLEY_PARITY_LOG) minus one channel in a thousand, capped at 0.9995 — so a scene measured bit-identical
(1.0: Cornell, earth, demo, the config bands 3 and 4) fails on a systematic 1-ulp slip that touches more
than 0.05 % of its channels, which the uniform 0.99 would let through.
The trace engines (RT_ENGINE_MEGAKERNEL, RT_ENGINE_WAVEFRONT, RT_ENGINE_SPLIT) run the same binary64
code on the same counter-RNG streams, so their frames must be bit-identical to each other: the
megakernel (the engine the product runs) carries every test; each other engine keeps one smoke parity
test (test_other_engine_matches_oracle_and_megakernel) and its own engine tests.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import raytracer as rt

pytestmark = pytest.mark.gpu

SEED = 0x5EED
ENGINES = ["megakernel"]  # the engine of every test below (RT_ENGINE_AUTO picks it on MI355X)
OTHER_ENGINES = ["wavefront", "split"]  # one smoke parity test each (slower engines)
PARITY_EXACT = 0.99    # bit-identical channel fraction, every comparison
PARITY_OUTLIERS = 0.001  # fraction of pixels allowed beyond 1e-10 * spp
# Per-comparison floors of the bit-identical fraction: min(0.9995, measured - 0.001), from the round-4
# calibration (profiles/r04/parity_fractions.jsonl); never below PARITY_EXACT (exact_floor).
EXACT_FLOOR = {
    # test_render_matches_oracle / test_other_engine_matches_oracle_and_megakernel (48- / 40-wide, 8 spp)
    "random": 0.99566, "random-night": 0.9995, "demo": 0.9995, "perlin": 0.99386, "earth": 0.9995,
    "box-light": 0.99746, "cornell": 0.9995, "final:6:60": 0.99838, "final": 0.9995,
    # test_render_matches_golden (32 x 32 @ 8 spp)
    "golden:random": 0.99437, "golden:cornell": 0.9995, "golden:earth": 0.9995, "golden:final:4:30": 0.9995,
    # test_config_settings_band_matches_oracle (cfg5: its own exception, CFG5_EXACT)
    "cfg1": 0.99451, "cfg3": 0.9995, "cfg3_ground": 0.9995, "cfg4": 0.9995, "cfg4_light": 0.9995,
    "cfg5": 0.98021,
    "spheres": 0.9995, "final_world8": 0.99873,
}


def exact_floor(key, base=PARITY_EXACT):
    """The bit-identical fraction a comparison must reach: its calibrated floor, never below the rule."""
    return max(base, EXACT_FLOOR.get(key, base))
ENGINE_ID = {"megakernel": 1, "wavefront": 2, "split": 3}
# RT_ENGINE_SPLIT serves reference scenes whose whole scene fits in LDS; book-2 scenes fall back to
# the megakernel (rt_counters.engine reports the engine that ran)
SPLIT_FALLBACK = {"final:6:60", "final"}


def engine_ran(cnt, engine, name=""):
    if engine == "split" and name in SPLIT_FALLBACK:
        return cnt.engine == ENGINE_ID["megakernel"]
    return cnt.engine == ENGINE_ID[engine]


def _log_fraction(exact, bad, shape):
    """SHIRLEY_PARITY_LOG=<file>: append each comparison's measured fractions (threshold calibration)."""
    import json
    import os
    path = os.environ.get("SHIRLEY_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", "?"), "exact": float(exact),
                                "bad_px": float(bad), "shape": list(shape)}) + "\n")


def check_parity(gpu_img, ora_img, spp, frac_exact=PARITY_EXACT, frac_outlier=PARITY_OUTLIERS):
    assert gpu_img.shape == ora_img.shape
    assert np.isfinite(gpu_img).all() == np.isfinite(ora_img).all()
    exact = np.mean(gpu_img == ora_img)
    diff = np.abs(gpu_img - ora_img)
    bad_px = np.any(diff > 1e-10 * spp, axis=-1)
    _log_fraction(exact, bad_px.mean(), gpu_img.shape)
    assert exact >= frac_exact, f"only {exact:.5f} of channels bit-identical (max diff {diff.max():.3g})"
    assert bad_px.mean() <= frac_outlier, f"{bad_px.sum()} pixels outside tolerance"


SCENES = [("random", 48, "std16x9"), ("random-night", 48, "std16x9"), ("demo", 48, "std16x9"),
          ("perlin", 48, "std16x9"), ("earth", 48, "square"), ("box-light", 48, "std16x9"),
          ("cornell", 40, "square"),
          # book-2 extensions (absent from the reference; oracle restatement, parity unpinned):
          # reduced final scene (whole scene in LDS) and the full one (1409 objects, nodes in LDS)
          ("final:6:60", 40, "square"), ("final", 32, "square")]



@pytest.mark.parametrize("name,width,aspect", SCENES)
def test_render_matches_oracle(gpu, name, width, aspect):
    spp = 8
    scene = rt.SceneBuilder.builtin(name, SEED).finalize(SEED)
    cam = rt.scene_camera(name, width, aspect)
    gpu.upload(scene)
    ora, ocnt = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED))
    imgs = {}
    for engine in ENGINES:
        img = gpu.render(cam, rt.RenderSettings(samples=spp, max_reflect=50, seed=SEED, sample_chunk=spp,
                                                engine=engine))
        check_parity(img, ora, spp, frac_exact=exact_floor(name))
        cnt = gpu.counters()
        assert engine_ran(cnt, engine, name)
        assert cnt.samples == cam.image_width * cam.image_height * spp == ocnt.samples
        # segment counts follow from the (identical) paths
        assert abs(int(cnt.segments) - int(ocnt.segments)) <= 0.001 * ocnt.segments
        imgs[engine] = img


@pytest.mark.parametrize("engine", OTHER_ENGINES)
@pytest.mark.parametrize("name,width,aspect", [("random", 48, "std16x9"), ("cornell", 40, "square"),
                                               ("perlin", 48, "std16x9"), ("final:6:60", 40, "square")])
def test_other_engine_matches_oracle_and_megakernel(gpu, engine, name, width, aspect):
    """The smoke parity test of each non-default engine: the oracle's tolerance, and the megakernel's
    frame bit for bit (the same device functions on the same streams)."""
    spp = 8
    scene = rt.SceneBuilder.builtin(name, SEED).finalize(SEED)
    cam = rt.scene_camera(name, width, aspect)
    gpu.upload(scene)
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED))
    s = dict(samples=spp, max_reflect=50, seed=SEED, sample_chunk=spp)
    img = gpu.render(cam, rt.RenderSettings(**s, engine=engine))
    assert engine_ran(gpu.counters(), engine, name)
    check_parity(img, ora, spp, frac_exact=exact_floor(name))
    assert np.array_equal(img, gpu.render(cam, rt.RenderSettings(**s, engine="megakernel")))


@pytest.mark.parametrize("name,aspect", [("random", "std16x9"), ("cornell", "square"), ("earth", "square"),
                                         ("final:4:30", "square")])
def test_render_matches_golden(gpu, name, aspect):
    """The committed oracle fixtures (tests/golden/renders.npz, 32x32 @ 8 spp) as the reference data."""
    import os
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "renders.npz"), allow_pickle=False)
    key = name.replace(":", "_").replace("-", "_")
    gpu.upload(rt.SceneBuilder.builtin(name, SEED).finalize(SEED))
    img = gpu.render(rt.scene_camera(name, 32, aspect), rt.RenderSettings(samples=8, max_reflect=50, seed=SEED,
                                                                          sample_chunk=8))
    check_parity(img, gold[key], 8, frac_exact=exact_floor("golden:" + name))


def test_hit_queries_match_golden(gpu):
    import os
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "hits.npz"), allow_pickle=False)
    gpu.upload(rt.scenes.random_scene(SEED).finalize(SEED))
    hits = gpu.hit(gold["rays"], 0.001, float("inf"))
    for i in range(len(gold["rays"])):
        assert hits[i].object == gold["object"][i]
        if gold["object"][i] >= 0:
            g = hits[i]
            assert [g.t, *g.point, *g.normal] == list(gold["record"][i][:7])
            assert abs(g.u - gold["record"][i][7]) < 1e-12 and abs(g.v - gold["record"][i][8]) < 1e-12


@pytest.mark.parametrize("slots", ["64", "4096"])
def test_wavefront_small_slot_pool(gpu, slots, monkeypatch):
    """Far fewer path slots than work units: every slot regenerates many paths and takes many
    units (render.rs:58-69 per slot); chunked sums and path counters equal the megakernel's."""
    monkeypatch.setenv("SHIRLEY_WF_SLOTS", slots)
    spp = 6
    for name, width, aspect in [("perlin", 40, "std16x9"), ("cornell", 24, "square")]:
        scene = rt.SceneBuilder.builtin(name, SEED).finalize(SEED)
        cam = rt.scene_camera(name, width, aspect)
        gpu.upload(scene)
        a = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=2, engine="megakernel"))
        ca = gpu.counters()
        b = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=2, engine="wavefront"))
        cb = gpu.counters()
        assert np.array_equal(a, b)
        assert 64 <= cb.slots <= int(slots) and cb.iterations > 1
        # same paths: same samples and segments (node-test counts differ: the megakernel walks the
        # 4-wide collapse of the tree, the wavefront engine the 2-wide tree)
        assert (ca.samples, ca.segments) == (cb.samples, cb.segments)


def test_wavefront_extend_kernels_agree(gpu, monkeypatch):
    """wf_extend4 (4-wide tree + primitives in LDS, prefetched rays) and wf_extend (2-wide tree via
    L1/L2) give the same frame; the 2-wide kernel is the fallback for scenes too big for LDS."""
    spp = 4
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(64, "std16x9")
    s = rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp, engine="wavefront")  # in-order sums
    a = gpu.upload(scene, "sah").render(cam, s)
    monkeypatch.setenv("SHIRLEY_WF_EXTEND2", "1")
    b = gpu.upload(scene, "sah").render(cam, s)
    assert np.array_equal(a, b)
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED))
    check_parity(a, ora, spp)


def test_wavefront_timing_counters(gpu):
    """Per-launch event timing; the perlin scene has deferred texture work (a scene without Perlin
    textures skips the wf_texture launch)."""
    scene = rt.SceneBuilder.builtin("perlin", SEED).finalize(SEED)
    cam = rt.scene_camera("perlin", 64, "std16x9")
    gpu.upload(scene, "sah")
    a = gpu.render(cam, rt.RenderSettings(samples=4, seed=SEED, engine="wavefront", timing=True))
    c = gpu.counters()
    assert c.engine == 2 and c.iterations > 4
    assert c.extend_ms > 0 and c.shade_ms > 0 and c.texture_ms > 0
    assert c.extend_ms + c.shade_ms + c.texture_ms <= c.kernel_ms * 1.05
    b = gpu.render(cam, rt.RenderSettings(samples=4, seed=SEED, engine="wavefront"))
    assert np.array_equal(a, b)
    assert gpu.counters().extend_ms == 0.0


@pytest.mark.parametrize("engine", ENGINES)
def test_sah_tree_same_image(gpu, engine):
    spp = 4
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(64, "std16x9")
    s = rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp)
    a = gpu.upload(scene, "reference").render(cam, s)
    b = gpu.upload(scene, "sah").render(cam, s)
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED))
    check_parity(a, ora, spp)
    check_parity(b, ora, spp)


@pytest.mark.parametrize("nodes", ["global", "lds", "half-lds"])
@pytest.mark.parametrize("engine", ENGINES)
def test_node_placements_same_image(gpu, engine, nodes):
    """BVH nodes through L1/L2 (default), all in LDS, or split: the same pixels."""
    spp = 3
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(40, "std16x9")
    s = rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp)
    a = gpu.upload(scene, "sah").render(cam, s)
    b = gpu.upload(scene, "sah", nodes).render(cam, s)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("engine", ENGINES)
def test_large_scene_mixed_lds_matches_oracle(gpu, engine):
    """1,728 spheres (gen_spheres side 6): a deeper BVH, both builders, against the oracle."""
    spp = 2
    scene = rt.scenes.gen_spheres(0xDEADBEEF, 6).finalize(1)
    cam = rt.scene_camera("spheres", 40, "std16x9")
    for bvh in ("reference", "sah"):
        img = gpu.upload(scene, bvh).render(cam, rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp))
        ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED))
        check_parity(img, ora, spp, frac_exact=exact_floor("spheres"))


def test_hit_queries_match_oracle(gpu):
    """Per-ray hit records (t, object, normal, u, v) for 4096 rays into the random scene."""
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    gpu.upload(scene)
    osc = O.OracleScene(scene)
    rng = np.random.default_rng(1)
    n = 4096
    orig = np.column_stack([rng.uniform(-12, 12, n), rng.uniform(0.05, 3, n), rng.uniform(-12, 12, n)])
    d = rng.normal(size=(n, 3))
    rays = np.hstack([orig, d])
    hits = gpu.hit(rays, 0.001, float("inf"))
    same = 0
    for i in range(n):
        h = osc.hit(rays[i], 0.001, float("inf"))
        g = hits[i]
        if not h.hit:
            assert g.object == -1
            continue
        assert g.object == h.object
        if (g.t == h.t and list(g.normal) == list(h.normal) and list(g.point) == list(h.point)
                and g.front_face == h.front_face):
            same += 1
        assert abs(g.u - h.u) < 1e-12 and abs(g.v - h.v) < 1e-12
    n_hit = sum(1 for i in range(n) if hits[i].object >= 0)
    assert n_hit > 1000 and same == n_hit


def test_hit_queries_book2_match_oracle(gpu):
    """rt_scene_hit on the book-2 final scene (moving sphere at time 0, media keyed by the ray
    index, rotated + translated cluster): same objects and records as the oracle."""
    scene = rt.scenes.final_scene(SEED, 8, 200).finalize(SEED)
    gpu.upload(scene)
    osc = O.OracleScene(scene)
    rng = np.random.default_rng(2)
    n = 2048
    orig = np.column_stack([rng.uniform(-200, 600, n), rng.uniform(50, 500, n), rng.uniform(-300, 600, n)])
    d = rng.normal(size=(n, 3))
    rays = np.hstack([orig, d])
    hits = gpu.hit(rays, 0.001, float("inf"))
    n_hit = same = n_medium = 0
    for i in range(n):
        h = osc.hit(rays[i], 0.001, float("inf"), index=i)
        g = hits[i]
        assert g.object == (h.object if h.hit else -1)
        if not h.hit:
            continue
        n_hit += 1
        if scene.desc.objects[h.object].medium:
            # free flight -ln(U)/density: ocml's log vs glibc's may differ by an ulp
            n_medium += 1
            assert abs(g.t - h.t) <= 1e-13 * abs(h.t) and np.allclose(list(g.point), list(h.point), rtol=1e-12, atol=1e-9)
        else:
            same += (g.t == h.t and list(g.point) == list(h.point) and list(g.normal) == list(h.normal))
    assert n_hit > 500 and n_medium > 50 and same >= n_hit - n_medium - 2


def test_bbox_tree_unit_cases_on_gpu(gpu):
    """bvh/bbox_tree.rs:94-234 cases through the device traversal."""
    MAX = 1.7976931348623157e308
    cases = [
        ([((0, 0, -10), 0.5)], [0, 0, 0, 1, 0, 0], -1),
        ([((0, 0, -10), 0.5)], [0, 0, 0, 0, 0, -1], 0),
        ([((0, 0, -2), 1.0)], [0, 0, 0, 0.9, 0.9, -1.5], -1),
        ([((0, 0, -2), 1.0)] + [((0, 0, -2.0 * i), 1.0) for i in range(2, 101)], [0, 0, 0, 0, 0, -1], 0),
        ([((0, 0, -2), 1.0), ((2, 2, -4), 1.0)], [0, 0, 0, 0.9, 0.9, -1.5], 1),
        ([((0, 0, -5), -1.0)], [0, 0, 0, 0, 0, -1], -1),
    ]
    for sph, ray, want in cases:
        s = O.SphereScene(sph)
        rt.Device.upload(gpu, type("S", (), {"desc_ptr": s.desc_ptr})())
        got = gpu.hit(np.array([ray], dtype=np.float64), 0.0, MAX)[0]
        assert got.object == want, (sph[:2], ray)


@pytest.mark.parametrize("engine", ENGINES)
def test_scanlines_equal_full_frame(gpu, engine):
    spp = 4
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(40, "std16x9")  # 40 x 22: rows not a multiple of 8
    gpu.upload(scene)
    s = rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp)
    full = gpu.render(cam, s)
    part = gpu.render_scanlines(cam, s, 5, 17)
    assert np.array_equal(part, full[5:17])
    row = np.zeros((cam.image_width, 3))
    cnt = O.or_counters()
    osc = O.OracleScene(scene)
    O.lib().or_render_scanline(osc.h, C.byref(cam), C.byref(O.params(spp, 50, SEED)), 9, row.ctypes.data,
                               C.byref(cnt))
    check_parity(part[4:5], row[None], spp, frac_exact=0.99, frac_outlier=0.05)


@pytest.mark.parametrize("engine", ENGINES)
def test_tiles_gather_unpack_equals_full_frame(gpu, engine):
    """The multi-GPU data path on one device: each rank's packed tiles, concatenated like a
    gather, then unpacked, equal the single-rank frame bit for bit."""
    import torch
    spp, world = 3, 3
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(52, "std16x9")  # 52 x 29: partial tiles on both axes
    gpu.upload(scene)
    full = gpu.render(cam, rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp))
    n_total, max_tiles = rt.tile_layout(cam, world)
    gathered = torch.zeros((world, max_tiles, 64, 3), dtype=torch.float64, device="cuda")
    for r in range(world):
        gpu.render_tiles_device(cam, rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp, tile_rank=r,
                                                       tile_world=world), gathered[r].data_ptr())
    gpu.synchronize()
    accum = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.float64, device="cuda")
    gpu.unpack_tiles_device(cam, world, gathered.data_ptr(), accum.data_ptr())
    gpu.synchronize()
    assert np.array_equal(accum.cpu().numpy(), full)


@pytest.mark.parametrize("engine", ENGINES)
def test_chunked_sums_close_to_in_order(gpu, engine):
    spp = 24
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(32, "std16x9")
    gpu.upload(scene)
    a = gpu.render(cam, rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp))
    b = gpu.render(cam, rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=5))
    assert np.allclose(a, b, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("engine", ENGINES)
def test_edge_cases(gpu, engine):
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    gpu.upload(scene)
    cam = rt.default_camera(8, "square")
    # samples == 0 renders one sample (main.rs:75-80)
    z = gpu.render(cam, rt.RenderSettings(engine=engine, samples=0, seed=SEED))
    one = gpu.render(cam, rt.RenderSettings(engine=engine, samples=1, seed=SEED))
    assert np.array_equal(z, one)
    # max_depth == 0 -> black (ray_color's loop never runs)
    assert not gpu.render(cam, rt.RenderSettings(engine=engine, samples=2, max_reflect=0, seed=SEED)).any()
    # empty scene -> pure sky, equal to the oracle
    empty = O.SphereScene([])
    rt.Device.upload(gpu, type("S", (), {"desc_ptr": empty.desc_ptr})())
    sky = gpu.render(cam, rt.RenderSettings(engine=engine, samples=2, seed=SEED, sample_chunk=2))
    ora, _ = O.OracleScene(empty).render(cam, O.params(2, 50, SEED))
    assert np.array_equal(sky, ora)
    # bad arguments fail loudly with a message
    with pytest.raises(rt.RtError):
        gpu.render(cam, rt.RenderSettings(engine=engine, samples=-1))
    with pytest.raises(rt.RtError):
        gpu.render_scanlines(cam, rt.RenderSettings(engine=engine, samples=1), 5, 100)
    if engine in ("megakernel", "split"):
        # 64 pixels x (2^26 + 1) one-sample units (>= 2^32: more than a launch indexes in 32 bits): the call
        # runs in sample passes (ABI 6) of <= 2 GiB of partial sums — 49 passes of 1369569 one-sample
        # chunks of 64 pixels — instead of being refused
        big = gpu.render(cam, rt.RenderSettings(engine=engine, samples=(1 << 26) + 1, sample_chunk=1, max_reflect=1,
                                                scratch_mb=2048))
        c = gpu.counters()
        assert c.passes == 49 and c.scratch_bytes <= 2048 << 20
        assert c.samples == 64 * ((1 << 26) + 1) and np.isfinite(big).all()


@pytest.mark.parametrize("engine", ENGINES)
def test_full_size_rows_match_oracle(gpu, engine):
    """BASELINE config 2 geometry (1200x800, random_scene) at reduced spp: two full rows against the
    oracle, plus the size-independent property full-frame row == rt_render_scanlines row."""
    spp = 6
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(1200, "std3x2")
    assert (cam.image_width, cam.image_height) == (1200, 800)
    gpu.upload(scene)
    s = rt.RenderSettings(engine=engine, samples=spp, seed=SEED, sample_chunk=spp)
    full = gpu.render(cam, s)
    rows = gpu.render_scanlines(cam, s, 200, 202)
    assert np.array_equal(rows, full[200:202])
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED), 200, 202)
    check_parity(rows, ora, spp)
    assert np.isfinite(full).all() and (full >= 0).all()


def test_device_tonemap_matches_host(gpu):
    """rt_tonemap_device (to_image on the GPU) == the host rt_tonemap, byte for
    byte, on a rendered frame and on synthetic sums with NaN / negative / huge / tiny values."""
    import torch
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(48, "std16x9")
    gpu.upload(scene)
    spp = 3
    frame = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED))
    rng = np.random.default_rng(7)
    synth = rng.uniform(-0.5, 4.0, size=frame.shape) * spp
    flat = synth.reshape(-1)
    flat[::97] = np.nan
    flat[1::89] = np.inf
    flat[2::83] = -np.inf
    flat[3::79] = 5e-324
    flat[4::73] = 0.0
    flat[5::71] = -0.0
    flat[6::67] = spp * (255.0 / 255.999) ** 2  # at the saturation edge
    for accum, s in ((frame, spp), (synth, spp), (synth, 0)):
        want = rt.to_image(accum, s)
        dev = torch.from_numpy(np.ascontiguousarray(accum)).to("cuda")
        out = torch.zeros(accum.shape, dtype=torch.uint8, device="cuda")
        gpu.tonemap_device(dev.data_ptr(), accum.shape[1], accum.shape[0], s, out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)


def test_cli_render_device_output_stage(tmp_path):
    """`ray-cli render random` end to end on the GPU: the default path (sums stay in HBM, to_image on
    the device, RGB8 copied back) writes the same PNG as the host path (--dump-accum: f64 sums copied
    back, host tonemap), and that PNG is to_image of the dumped sums."""
    import os
    import subprocess
    from PIL import Image
    from raytracer import _native as N
    cli = os.path.join(N.BIN_DIR, "ray-cli")
    common = ["render", "random", "-w", "96", "-s", "4", "--seed", "0x5EED", "--camera-aspect-ratio", "std16x9"]
    a, b, acc = str(tmp_path / "dev.png"), str(tmp_path / "host.png"), str(tmp_path / "acc.f64")
    r1 = subprocess.run([cli] + common + ["-o", a], capture_output=True, text=True)
    assert r1.returncode == 0, r1.stderr
    r2 = subprocess.run([cli] + common + ["-o", b, "--dump-accum", acc], capture_output=True, text=True)
    assert r2.returncode == 0, r2.stderr
    img_a, img_b = np.asarray(Image.open(a)), np.asarray(Image.open(b))
    assert np.array_equal(img_a, img_b)
    sums = np.fromfile(acc, dtype=np.float64).reshape(img_a.shape[0], img_a.shape[1], 3)
    assert np.array_equal(rt.to_image(sums, 4), img_a)


def test_headline_settings_band_matches_oracle(gpu):
    """BASELINE config 2 exactly as bench.py runs it: 1200x800 @ 500 spp, max_depth 50, SAH tree,
    rt_render_device with sample_chunk = 0 (auto: several chunks per pixel, so each pixel's sum is
    added per chunk and the chunk sums in order — not render.rs:58-69's one running sum).  A 16-row
    band of that frame against (1) the GPU's in-order sums of the same samples: only the addition order
    differs, every channel within 1e-12 relative (500 non-negative terms: <= 499 ulp-level roundings);
    (2) the oracle's in-order render: the stated parity tolerance, with the exact-bit gate."""
    import torch
    spp, r0, r1 = 500, 392, 408
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(1200, "std3x2")
    gpu.upload(scene, "sah")
    accum = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.float64, device="cuda")
    gpu.render_device(cam, rt.RenderSettings(samples=spp, max_reflect=50, seed=SEED), accum.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = gpu.counters()
    assert 1 < c.sample_chunk < spp and c.n_chunks == -(-spp // c.sample_chunk) > 1
    band = accum[r0:r1].cpu().numpy()
    inorder = gpu.render_scanlines(cam, rt.RenderSettings(samples=spp, max_reflect=50, seed=SEED, sample_chunk=spp),
                                   r0, r1)
    assert gpu.counters().n_chunks == 1
    assert np.all(np.abs(band - inorder) <= 1e-12 * np.abs(inorder))
    ora, cnt = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED), r0, r1, threads=16)
    assert cnt.samples == 1200 * (r1 - r0) * spp
    check_parity(inorder, ora, spp, frac_exact=0.99)
    # the bench frame's own band: reordering tolerance, plus the flipped-path allowance of check_parity
    bad = np.any(np.abs(band - ora) > 1e-12 * np.abs(ora) + 1e-10 * spp * (band != inorder), axis=-1)
    assert bad.mean() <= 0.001


# The other BASELINE configs at their stated frame size and spp, as bench.py's `configs` block runs
# them (auto sample chunk, SAH tree): (key, scene, width, aspect, spp, rows of the centre band checked).
# Gate: the module's one rule, except config 5 (CFG5_EXACT below).
# Row bands: first row (None: centred) and row count; row 0 is the bottom of the picture.
CONFIG_BANDS = [("cfg1", "random", 400, "std16x9", 50, None, 225),      # the whole frame
                ("cfg3", "earth", 800, "square", 1000, None, 8),        # through the earth sphere
                ("cfg3_ground", "earth", 800, "square", 1000, 196, 8),  # the checker ground (sin signs)
                ("cfg4", "cornell", 600, "square", 10000, None, 4),
                # the ceiling light (scenes.rs:23-63: xz_rect 213..343 x 227..332 at y = 554, seen in rows
                # ~501-521 of 600): direct emitter pixels and the deepest paths of the frame
                ("cfg4_light", "cornell", 600, "square", 10000, 508, 4),
                ("cfg5", "final", 1920, "std16x9", 2000, None, 8)]      # book-2 extension scene
# The exception, config 5: a pixel's channel is bit-identical only if none of its 2000 paths meets an
# ulp-level libm difference (the marble's sin, the media's log, the sphere u, v's acos / atan2 on the
# earth and the cluster), so at 2000 samples per pixel ~2 % of channels carry one; the same 0.1 %
# outlier-pixel bound still holds.  Measured fractions: profiles/r04/parity_fractions.jsonl (cfg5: 0.981)
# (DESIGN.md §2).
CFG5_EXACT = 0.975


@pytest.mark.parametrize("key,name,width,aspect,spp,first,rows", CONFIG_BANDS)
def test_config_settings_band_matches_oracle(gpu, key, name, width, aspect, spp, first, rows):
    """BASELINE configs 1, 3, 4 and 5 at their own sizes and spp, like test_headline_settings_band_matches_
    oracle for config 2: the bench's frame (auto chunk) against the GPU's in-order sums of the same rows
    (reassociation only: <= 1e-12 relative), and those against the oracle's in-order render of the rows
    (the stated parity tolerance)."""
    import torch
    scene = rt.SceneBuilder.builtin(name, SEED).finalize(SEED)
    cam = rt.scene_camera(name, width, aspect)
    H = cam.image_height
    r0 = (H - rows) // 2 if first is None else first
    r1 = r0 + rows
    gpu.upload(scene, "sah")
    accum = torch.zeros((H, cam.image_width, 3), dtype=torch.float64, device="cuda")
    gpu.render_device(cam, rt.RenderSettings(samples=spp, max_reflect=50, seed=SEED), accum.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    # the automatic unit is at most 16 samples here (cfg4 / cfg5: 54 / 61 cut to 16, rt_api.cpp), so the
    # large-spp frames are checked at the many-chunk summation order the bench runs
    c = gpu.counters()
    assert c.sample_chunk <= 16 and c.n_chunks == -(-spp // c.sample_chunk)
    band = accum[r0:r1].cpu().numpy()
    if key == "cfg4_light":  # the band sees the emitter directly: FairyLight 15 (scenes.rs:30) seen at
        # n.(-d)/|d| ~ 0.26 from the camera, ~3.9 per channel before its own scattered light
        assert (band[..., 0] / spp > 3.0).sum() >= 20
    inorder = gpu.render_scanlines(cam, rt.RenderSettings(samples=spp, max_reflect=50, seed=SEED, sample_chunk=spp),
                                   r0, r1)
    assert np.all(np.abs(band - inorder) <= 1e-12 * np.abs(inorder))
    ora, cnt = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED), r0, r1, threads=16)
    assert cnt.samples == cam.image_width * rows * spp
    check_parity(inorder, ora, spp, frac_exact=exact_floor(key, CFG5_EXACT if key == "cfg5" else PARITY_EXACT))


def test_max_depth_zero_partial_units(gpu):
    """max_depth 0 (ray_color's loop never runs: black, render.rs:30) with units that end at different
    iterations: a width that is not a multiple of 8 (edge tiles with idle lanes), and a sample chunk
    shorter than spp with a short last chunk — every unit must still publish (all-zero image, no stale
    partial sums)."""
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    gpu.upload(scene)
    cam = rt.default_camera(37, "std16x9")
    # leave garbage in the partial buffer first
    gpu.render(cam, rt.RenderSettings(samples=7, seed=SEED, sample_chunk=3))
    for engine in ENGINES:
        for chunk in (0, 1, 3, 7):
            img = gpu.render(cam, rt.RenderSettings(engine=engine, samples=7, max_reflect=0, seed=SEED,
                                                    sample_chunk=chunk))
            assert not img.any(), (engine, chunk)
            assert gpu.counters().samples == cam.image_width * cam.image_height * 7


def test_final_scene_tile_sharded_world8(gpu):
    """BASELINE config 5's data path on one device: book-2 final_scene (1409 objects, EXT kernels; its
    4-wide tree in the 768-thread block's LDS since the cluster is flattened) rendered as the 8 ranks' interleaved tiles (rt_render_tiles_device), gathered
    rank-major and scattered back (rt_unpack_tiles_device): bit-identical to the full frame."""
    import torch
    spp, world = 3, 8
    scene = rt.scenes.final_scene(SEED).finalize(SEED)
    cam = rt.scene_camera("final", 61, "square")  # 61 x 61: partial edge tiles
    gpu.upload(scene)
    full = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp))
    n_total, max_tiles = rt.tile_layout(cam, world)
    assert n_total == 64 and max_tiles == 8
    gathered = torch.zeros((world, max_tiles, 64, 3), dtype=torch.float64, device="cuda")
    for r in range(world):
        gpu.render_tiles_device(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp, tile_rank=r,
                                                       tile_world=world), gathered[r].data_ptr())
    gpu.synchronize()
    accum = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.float64, device="cuda")
    gpu.unpack_tiles_device(cam, world, gathered.data_ptr(), accum.data_ptr())
    gpu.synchronize()
    assert np.array_equal(accum.cpu().numpy(), full)
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED), threads=16)
    check_parity(full, ora, spp, frac_exact=exact_floor("final_world8"))


@pytest.mark.parametrize("bvh", ["reference", "sah"])
def test_gen_spheres_side11_matches_oracle(gpu, bvh):
    """The config-5 stand-in at full scale: gen_spheres side 11 = 22^3 = 10,648 spheres
    (benches/my_benchmark.rs:35-60), tree through L1/L2 (too large for LDS), both builders."""
    spp = 2
    scene = rt.scenes.gen_spheres(0xDEADBEEF, 11).finalize(1)
    assert scene.desc.n_objects == 10648
    cam = rt.scene_camera("spheres", 48, "std16x9")
    gpu.upload(scene, bvh)
    assert gpu.stats().wide_block == 0
    img = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp))
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED), threads=16)
    check_parity(img, ora, spp, frac_exact=exact_floor("spheres"))


def test_final_scene_on_the_narrow_block(gpu, monkeypatch):
    """The book-2 256-thread instances (a book-2 scene whose tree does not fit the wide block's LDS; 3 waves
    per SIMD, trace.hip RT_NARROW_WAVES_EXT): final_scene forced onto them (SHIRLEY_NO_WIDE, read at upload)
    renders the wide block's frame bit for bit, and the oracle's within the parity rule."""
    spp = 4
    scene = rt.scenes.final_scene(SEED).finalize(SEED)
    cam = rt.scene_camera("final", 32, "square")
    gpu.upload(scene)
    assert gpu.stats().wide_block == 1
    wide = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp))
    monkeypatch.setenv("SHIRLEY_NO_WIDE", "1")
    gpu.upload(scene)
    assert gpu.stats().wide_block == 0
    narrow = gpu.render(cam, rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp))
    monkeypatch.delenv("SHIRLEY_NO_WIDE")
    gpu.upload(scene)  # (the next test's device: the default block again)
    assert np.array_equal(narrow, wide)
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED), threads=16)
    check_parity(narrow, ora, spp, frac_exact=exact_floor("final"))


@pytest.mark.parametrize("name,width,aspect", [("random", 48, "std16x9"), ("cornell", 40, "square"),
                                               ("earth", 48, "square"), ("final:6:60", 40, "square")])
def test_lds_material_tables_change_nothing(gpu, monkeypatch, name, width, aspect):
    """The scene-in-LDS block keeps the material and texture tables in LDS after the Perlin tables (rt_api.cpp
    n_lds_mats): the frame is the one the global-memory tables give (SHIRLEY_NO_LDS_MATS, read
    at upload), bit for bit."""
    spp = 4
    scene = rt.SceneBuilder.builtin(name, SEED).finalize(SEED)
    cam = rt.scene_camera(name, width, aspect)
    s = rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp)
    gpu.upload(scene)
    lds = gpu.render(cam, s)
    monkeypatch.setenv("SHIRLEY_NO_LDS_MATS", "1")
    gpu.upload(scene)
    glob = gpu.render(cam, s)
    monkeypatch.delenv("SHIRLEY_NO_LDS_MATS")
    gpu.upload(scene)
    assert np.array_equal(lds, glob)


@pytest.mark.parametrize("name,width,aspect", [("random", 48, "std16x9"), ("cornell", 40, "square"),
                                               ("box-light", 48, "std16x9"), ("spheres", 48, "std16x9")])
def test_collapse_choice_changes_nothing(gpu, monkeypatch, name, width, aspect):
    """The 4-wide collapse is picked per scene at upload (rt_api.cpp rt_scene_upload: the optimal collapse for
    scene-in-LDS reference scenes, greedy otherwise).  The tree only orders and culls the
    node tests — every leaf test stays exact — so the optimal, the greedy and the automatic choice give the
    same frame, bit for bit, and that frame is the oracle's within the parity gate."""
    spp = 4
    scene = rt.SceneBuilder.builtin(name, SEED).finalize(SEED)
    cam = rt.scene_camera(name, width, aspect)
    s = rt.RenderSettings(samples=spp, seed=SEED, sample_chunk=spp)
    frames = {}
    for mode in ("auto", "0", "1"):
        if mode == "auto":
            monkeypatch.delenv("SHIRLEY_COLLAPSE_DP", raising=False)
        else:
            monkeypatch.setenv("SHIRLEY_COLLAPSE_DP", mode)
        gpu.upload(scene)
        frames[mode] = gpu.render(cam, s)
    monkeypatch.delenv("SHIRLEY_COLLAPSE_DP", raising=False)
    gpu.upload(scene)
    assert np.array_equal(frames["auto"], frames["0"])
    assert np.array_equal(frames["auto"], frames["1"])
    ora, _ = O.OracleScene(scene).render(cam, O.params(spp, 50, SEED), threads=16)
    check_parity(frames["auto"], ora, spp, frac_exact=PARITY_EXACT)


def test_rotated_sphere_instances(gpu):
    """a rotated sphere instance whose material reads u, v (earth texture) keeps per-ray
    instancing; a rotated solid one is flattened, and rt_scene_hit still reports the instance's u, v
    (object frame).  Query records and a frame against the oracle (which flattens by the same rule)."""
    from test_book2_ext import rotated_sphere_rays, rotated_sphere_scene
    scene = rotated_sphere_scene()
    gpu.upload(scene)
    rays = rotated_sphere_rays()
    osc = O.OracleScene(scene)
    seen = {0: 0, 1: 0}
    for i, g in enumerate(gpu.hit(rays)):
        h = osc.hit(rays[i], index=i)
        assert g.object == (h.object if h.hit else -1), i
        if g.object >= 0:
            seen[g.object] += 1
            assert abs(g.t - h.t) <= 1e-12 * h.t
            assert abs(g.u - h.u) < 1e-12 and abs(g.v - h.v) < 1e-12
    assert min(seen.values()) > 50
    spp = 8
    cam = rt.default_camera(32, "square")
    ora, _ = osc.render(cam, O.params(spp, 50, SEED))
    img = gpu.render(cam, rt.RenderSettings(samples=spp, max_reflect=50, seed=SEED, sample_chunk=spp))
    check_parity(img, ora, spp)
