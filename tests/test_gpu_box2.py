"""The two-pass RectBox face test of the book-2 instances (rt_device.h box_t2, RT_BOX_TWO_PASS) on the GPU:
adversarial rays at a RectBox — aimed at its faces, edges and corners (where faces of two axes meet at one
t, and entry meets exit), from outside, from inside and from points on its faces — traced through the
book-2 kernel instance (the scene holds a moving sphere, so the render traversal runs leaf_tests4<EXT>)
must return the oracle's sequential six-face record (rect.rs:132-156) bit for bit, and the same record as
the reference-scene instance (box_t1f: the entry planes, else the six-face sequence) on the scene without
the moving sphere.
tests/box_pass_check.c proves the same on the CPU over ~11 M draws."""
import numpy as np
import pytest

import oracle_lib as O
import raytracer as rt
from raytracer import _native as N
from test_scatter_kat import KatScene

pytestmark = pytest.mark.gpu
GREY = {"kind": N.RT_TEX_SOLID, "color": (0.5, 0.5, 0.5)}
MATS = [(N.RT_MAT_LAMBERTIAN, 0, (0, 0, 0), 0.0)]
BOX = (N.RT_GEOM_RECT_BOX, 0, [-1.0, -0.25, -3.0, 1.5, 0.5, -1.0])


def _moving_sphere_far():
    s = (N.RT_GEOM_MOVING_SPHERE, 0, [60.0, 60.0, 60.0, 1.0])
    return s


def _scene(with_ext):
    sc = KatScene([BOX] + ([_moving_sphere_far()] if with_ext else []), MATS, [GREY])
    if with_ext:
        o = sc.objs[1]
        o.q[:] = [60.0, 61.0, 60.0, 0.0, 1.0]
    return sc


def _rays(n, seed):
    rng = np.random.default_rng(seed)
    lo, hi = np.array(BOX[2][:3]), np.array(BOX[2][3:])
    tg = rng.uniform(lo, hi, size=(n, 3))
    kind = rng.integers(0, 4, n)  # 0 face, 1 edge, 2 corner, 3 interior point
    for i in range(n):
        axes = rng.permutation(3)
        for a in axes[:min(kind[i] + 1, 3) if kind[i] < 3 else 0]:
            tg[i, a] = hi[a] if rng.integers(2) else lo[a]
    org = np.empty_like(tg)
    where = rng.integers(0, 3, n)  # 0 outside, 1 inside, 2 on a face
    for i in range(n):
        if where[i] == 0:
            org[i] = tg[i] + rng.uniform(-4, 4, 3)
        elif where[i] == 1:
            org[i] = rng.uniform(lo, hi)
        else:
            org[i] = rng.uniform(lo, hi)
            a = rng.integers(3)
            org[i, a] = hi[a] if rng.integers(2) else lo[a]
    d = tg - org
    # a few nearly axis-parallel rays (components down to 1e-12)
    m = rng.random(n) < 0.15
    d[m, rng.integers(0, 3, m.sum())] *= 1e-12
    ok = np.all(np.abs(d) > 0, axis=1)
    return np.hstack([org, d])[ok]


def _records(hits):
    return [(h.object, h.t, tuple(h.point), tuple(h.normal), h.front_face) if h.t == h.t and h.object >= 0 else None
            for h in hits]


def test_two_pass_box_matches_sequential_faces(gpu):
    rays = _rays(4096, 21)
    ext = _scene(True)
    rt.Device.upload(gpu, type("S", (), {"desc_ptr": ext.desc_ptr})())
    dev = gpu.hit(rays, 0.001, float("inf"), traversal="render")
    osc = O.OracleScene(ext.desc)
    n_hit = 0
    for i, ray in enumerate(rays):
        h = osc.hit(ray)
        g = dev[i]
        if not h.hit:
            assert g.object < 0, i
            continue
        n_hit += 1
        assert g.object == 0 and h.object == 0, i
        assert (g.t, list(g.point), list(g.normal), g.front_face) == (h.t, list(h.point), list(h.normal),
                                                                       h.front_face), i
    assert n_hit > 0.5 * len(rays)
    # the reference-scene instance (six faces in sequence) on the same box: the same records
    ref = _scene(False)
    rt.Device.upload(gpu, type("S", (), {"desc_ptr": ref.desc_ptr})())
    dev6 = gpu.hit(rays, 0.001, float("inf"), traversal="render")
    assert _records(dev6) == _records(dev)
