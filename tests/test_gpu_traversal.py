"""Per-ray parity of the traversal the trace kernel RUNS (rt_scene_hit_ex, RT_TRAVERSAL_RENDER).

The renderer walks the 4-wide collapse of the BVH with conservative f32 child boxes (inflated by the
scene's inflation distance, rounded outward), re-tests every hit leaf exactly in f64 (the reference's
Aabb::hit2 on the object's own bounding box, bvh/aabb.rs:62-79, then the object test), and falls back
to f64 box arithmetic for rays whose origin lies beyond rt_scene_stats.origin_limit.  The reference
(bvh/bbox_tree.rs:56-91) visits every node whose f64 box passes hit2; these tests hold that the render
traversal returns the same closest hit — object AND the full hit record, bit for bit — as
  * the reference's own bbox_tree.rs:94-227 cases,
  * the committed golden hit records (tests/golden/hits.npz, oracle-generated),
  * the oracle on 4,096 random rays,
  * the oracle on rays whose origins lie beyond origin_limit (the f64 fallback branch),
for each node placement the trace kernel can run with (whole scene in LDS, nodes in L1/L2, split).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import raytracer as rt

pytestmark = pytest.mark.gpu

SEED = 0x5EED
PLACEMENTS = ["auto", "global", "half-lds"]  # auto = the renderer's choice (random_scene: scene in LDS)


def _same_record(g, h):
    return (g.t == h.t and list(g.point) == list(h.point) and list(g.normal) == list(h.normal)
            and bool(g.front_face) == bool(h.front_face))


def _check_against_oracle(hits, rays, osc, min_hits):
    n_hit = 0
    for i in range(len(rays)):
        h = osc.hit(rays[i], 0.001, float("inf"))
        g = hits[i]
        if not h.hit:
            assert g.object == -1, (i, g.object)
            continue
        n_hit += 1
        assert g.object == h.object, (i, g.object, h.object)
        assert _same_record(g, h), (i, g.t, h.t)
        assert abs(g.u - h.u) < 1e-12 and abs(g.v - h.v) < 1e-12
    assert n_hit >= min_hits
    return n_hit


@pytest.mark.parametrize("nodes", PLACEMENTS)
def test_render_traversal_golden_hits(gpu, nodes):
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "hits.npz"), allow_pickle=False)
    gpu.upload(rt.scenes.random_scene(SEED).finalize(SEED), "sah", nodes)
    st = gpu.stats()
    assert st.wide_block == (1 if nodes == "auto" else 0)
    hits = gpu.hit(gold["rays"], 0.001, float("inf"), traversal="render")
    for i in range(len(gold["rays"])):
        assert hits[i].object == gold["object"][i], i
        if gold["object"][i] >= 0:
            g = hits[i]
            assert [g.t, *g.point, *g.normal] == list(gold["record"][i][:7])
            assert abs(g.u - gold["record"][i][7]) < 1e-12 and abs(g.v - gold["record"][i][8]) < 1e-12


@pytest.mark.parametrize("bvh", ["reference", "sah"])
@pytest.mark.parametrize("nodes", PLACEMENTS)
def test_render_traversal_matches_oracle(gpu, nodes, bvh):
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    gpu.upload(scene, bvh, nodes)
    osc = O.OracleScene(scene)
    rng = np.random.default_rng(1)
    n = 4096
    orig = np.column_stack([rng.uniform(-12, 12, n), rng.uniform(0.05, 3, n), rng.uniform(-12, 12, n)])
    rays = np.hstack([orig, rng.normal(size=(n, 3))])
    hits = gpu.hit(rays, 0.001, float("inf"), traversal="render")
    _check_against_oracle(hits, rays, osc, 1000)
    # and identical to the 2-wide f64 traversal, record for record
    hb = gpu.hit(rays, 0.001, float("inf"), traversal="binary")
    for a, b in zip(hits, hb):
        assert a.object == b.object and (a.object < 0 or _same_record(a, b))


@pytest.mark.parametrize("nodes", PLACEMENTS)
def test_render_traversal_far_origins(gpu, nodes):
    """Origins beyond origin_limit take node4_keys' f64 branch (rt_device.h, `!r.fast`); the result
    must still be the reference's closest hit."""
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    gpu.upload(scene, "sah", nodes)
    lim = gpu.stats().origin_limit
    assert lim >= 16.0
    osc = O.OracleScene(scene)
    rng = np.random.default_rng(3)
    n = 2048
    # aim at points among the small spheres from far away (distance 1.5x .. 1000x the limit)
    target = np.column_stack([rng.uniform(-11, 11, n), rng.uniform(0.0, 1.5, n), rng.uniform(-11, 11, n)])
    u = rng.normal(size=(n, 3))
    u[:, 1] = np.abs(u[:, 1])  # from above the ground
    u /= np.linalg.norm(u, axis=1)[:, None]
    dist = lim * np.exp(rng.uniform(np.log(1.5), np.log(1000.0), n))
    orig = target + u * dist[:, None]
    assert (np.abs(orig).max(axis=1) > lim).all()
    d = target - orig
    d *= rng.uniform(0.5, 2.0, n)[:, None]  # directions are not normalised (camera/mod.rs:122-131)
    rays = np.hstack([orig, d])
    hits = gpu.hit(rays, 0.001, float("inf"), traversal="render")
    _check_against_oracle(hits, rays, osc, 500)


def test_render_traversal_bbox_tree_unit_cases(gpu):
    """bvh/bbox_tree.rs:94-234 cases through the render traversal (t in [0, f64::MAX])."""
    MAX = 1.7976931348623157e308
    cases = [
        ([((0, 0, -10), 0.5)], [0, 0, 0, 1, 0, 0], -1),
        ([((0, 0, -10), 0.5)], [0, 0, 0, 0, 0, -1], 0),
        ([((0, 0, -2), 1.0)], [0, 0, 0, 0.9, 0.9, -1.5], -1),
        ([((0, 0, -2), 1.0)] + [((0, 0, -2.0 * i), 1.0) for i in range(2, 101)], [0, 0, 0, 0, 0, -1], 0),
        ([((0, 0, -2), 1.0), ((2, 2, -4), 1.0)], [0, 0, 0, 0.9, 0.9, -1.5], 1),
        ([((0, 0, -5), -1.0)], [0, 0, 0, 0, 0, -1], -1),
        ([], [0, 0, 0, 0, 0, -1], -1),
    ]
    for sph, ray, want in cases:
        s = O.SphereScene(sph)
        rt.Device.upload(gpu, type("S", (), {"desc_ptr": s.desc_ptr})())
        got = gpu.hit(np.array([ray], dtype=np.float64), 0.0, MAX, traversal="render")[0]
        assert got.object == want, (sph[:2], ray)
        if want >= 0:
            assert _same_record(got, O.OracleScene(s).hit(ray, 0.0, MAX))


@pytest.mark.parametrize("nodes", PLACEMENTS)
@pytest.mark.parametrize("name", ["cornell", "box-light", "final:6:60"])
def test_render_traversal_rect_box_and_book2_scenes(gpu, name, nodes):
    """Rect / RectBox leaves (the renderer's second and third leaf loops) and book-2 extended leaves
    (EXT kernel instance, whose 4-wide nodes use the compact 112-B layout; reference scenes the 160-B
    lo/hi/lo rows — rt_layout.h), in every node placement: render traversal == 2-wide traversal, record
    for record, and == the oracle for reference primitives."""
    scene = rt.SceneBuilder.builtin(name, SEED).finalize(SEED)
    gpu.upload(scene, nodes=nodes)
    cam = rt.scene_camera(name, 32, "square")
    eye = np.array(cam.origin)
    nodes, root = O.OracleScene(scene).tree()
    box = np.array(nodes[root][0])
    lo, hi = box[:3], box[3:]
    if (hi - lo).max() > 5000:  # a huge ground sphere: aim at the region around the origin
        lo, hi = np.maximum(lo, -50.0), np.minimum(hi, 50.0)
    rng = np.random.default_rng(5)
    n = 2048
    target = lo + (hi - lo) * rng.uniform(size=(n, 3))
    # half the rays from around the camera towards points of the scene box, half from inside the box
    orig = np.where((np.arange(n) % 2 == 0)[:, None], eye + rng.normal(scale=1.0, size=(n, 3)),
                    lo + (hi - lo) * rng.uniform(size=(n, 3)))
    rays = np.hstack([orig, target - orig])
    a = gpu.hit(rays, 0.001, float("inf"), traversal="render")
    b = gpu.hit(rays, 0.001, float("inf"), traversal="binary")
    n_hit = 0
    for x, y in zip(a, b):
        assert x.object == y.object
        if x.object >= 0:
            n_hit += 1
            assert _same_record(x, y) and x.u == y.u and x.v == y.v
    assert n_hit > 200
    if not name.startswith("final"):
        _check_against_oracle(a, rays, O.OracleScene(scene), 200)


def test_hit_ex_rejects_bad_traversal(gpu):
    gpu.upload(rt.scenes.random_scene(SEED).finalize(SEED))
    import raytracer._native as N
    out = (N.rt_hit * 1)()
    r = np.zeros(6)
    assert N.rt_lib().rt_scene_hit_ex(gpu.handle, r.ctypes.data, 1, 0.001, 1e300, 7, out) == N.RT_E_INVALID
