"""Pin the oracle: the reference's own unit tests, restated, plus analytic known answers.

The reference ships 25 inline #[test]s and no fixtures:
  core/fp.rs:30-113 (11), bvh/aabb.rs:89-179 (7), bvh/bbox_tree.rs:94-234 (7).
Each test below names the reference test it restates.  The Philox known-answer vectors are the
published Random123 kat_vectors for philox4x32-10.
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_lib as O

NAN = float("nan")
MAX = 1.7976931348623157e308  # f64::MAX


def L():
    return O.lib()


# ---- core/fp.rs:30-113 -------------------------------------------------------------------------
def test_fp_non_nan_first():
    assert L().or_non_nan(4.3, 50.1) == 4.3


def test_fp_non_nan_second():
    assert L().or_non_nan(NAN, 50.1) == 50.1


def test_fp_non_nan_both():
    assert math.isnan(L().or_non_nan(NAN, NAN))


def test_fp_check_min():
    assert L().or_fmin(4.3, 50.1) == 4.3 and L().or_fmin(50.1, 4.3) == 4.3


def test_fp_check_min_same():
    assert L().or_fmin(4.3, 4.3) == 4.3


def test_fp_check_min_with_nans():
    assert L().or_fmin(4.3, NAN) == 4.3 and L().or_fmin(NAN, 4.3) == 4.3


def test_fp_check_min_nan_both():
    assert math.isnan(L().or_fmin(NAN, NAN))


def test_fp_check_max():
    assert L().or_fmax(4.3, 50.1) == 50.1 and L().or_fmax(50.1, 4.3) == 50.1


def test_fp_check_max_same():
    assert L().or_fmax(4.3, 4.3) == 4.3


def test_fp_check_max_with_nans():
    assert L().or_fmax(4.3, NAN) == 4.3 and L().or_fmax(NAN, 4.3) == 4.3


def test_fp_check_max_nan_both():
    assert math.isnan(L().or_fmax(NAN, NAN))


# ---- bvh/aabb.rs:89-179 ------------------------------------------------------------------------
def surround(a, b):
    out = O._d6()
    L().or_surrounding_box(O.d6(a), O.d6(b), out)
    return list(out)


def test_aabb_combine_two_identical_boxes():
    b1 = [0, 0, 0, 1, 1, 1]
    assert surround(b1, b1) == b1


def test_aabb_combine_two_overlapping_boxes():
    assert surround([-0.5] * 3 + [1] * 3, [0] * 3 + [2] * 3) == [-0.5] * 3 + [2] * 3


def test_aabb_combine_fully_contained_box():
    assert surround([0.5] * 3 + [1] * 3, [0] * 3 + [2] * 3) == [0] * 3 + [2] * 3


BOX = [1.0, -1.0, -1.0, 2.0, 1.0, 1.0]


def test_aabb_check_hit():
    assert L().or_aabb_hit2(O.d6(BOX), O.d6([0, 0, 0, 1, 0, 0]), 0.0, MAX)


def test_aabb_check_miss():
    assert not L().or_aabb_hit2(O.d6(BOX), O.d6([0, 2, 2, 1, 0, 0]), 0.0, MAX)


def test_aabb_check_graze():
    # a ray along the box edge y=1, z=1 must hit (aabb.rs:157-166)
    assert L().or_aabb_hit2(O.d6(BOX), O.d6([0, 1, 1, 1, 0, 0]), 0.0, MAX)


def test_aabb_check_graze_corner():
    # aabb.rs:168-178 asserts nothing ("TODO should point grazing work?"); record what hit2 does
    b = [1.0001, -1.0, -1.0, 2.0, 1.0001, 1.0001]
    assert L().or_aabb_hit2(O.d6(b), O.d6([0, 0, 0, 1, 1, 1]), 0.0, MAX) in (0, 1)


# ---- bvh/bbox_tree.rs:94-234 (BboxTree<Sphere>::hit_workspace) ---------------------------------
def tree_hit(spheres, ray, t_min=0.0, t_max=MAX):
    s = O.SphereScene(spheres)
    return O.OracleScene(s).hit(ray, t_min, t_max)


def test_tree_size_of_tree_node():
    # bbox_tree.rs:102-107 pins the Rust TreeNode at 72 B (bbox 48 + enum).  Its C-ABI counterpart, the
    # inspection record rt_bvh_node (rt_bvh_build_host), is 64 B: box 48 + leaf / lhs / rhs / pad 4 x 4 B
    # (the enum's tag folded into leaf = -1).  The device's own layouts are rt_layout.h's (DNode 112 B,
    # DNode4F 160 B, DNode4C 112 B; checked there by static_assert).
    import raytracer._native as N
    assert C.sizeof(N.rt_bvh_node) == 64


def test_tree_emptybbox():
    s = O.SphereScene([])
    h = O.OracleScene(s).hit([0, 0, 0, 0, 0, 0], 0.0, MAX)
    assert not h.hit


def test_tree_miss_single_obj():
    assert not tree_hit([((0, 0, -10), 0.5)], [0, 0, 0, 1, 0, 0]).hit


def test_tree_hit_single_obj():
    h = tree_hit([((0, 0, -10), 0.5)], [0, 0, 0, 0, 0, -1])
    assert h.hit and h.object == 0


def test_tree_hit_box_but_not_obj():
    sph = [((0, 0, -2), 1.0)]
    ray = [0, 0, 0, 0.9, 0.9, -1.5]
    assert L().or_aabb_hit2(O.d6([-1, -1, -3, 1, 1, -1]), O.d6(ray), 0.0, MAX), "bad test setup"
    assert not tree_hit(sph, ray).hit


def test_tree_hit_first_sphere_in_chain():
    sph = [((0, 0, -2), 1.0)] + [((0, 0, -2.0 * i), 1.0) for i in range(2, 101)]
    h = tree_hit(sph, [0, 0, 0, 0, 0, -1])
    assert h.hit and h.object == 0


def test_tree_hit_obj_behind_first_box():
    sph = [((0, 0, -2), 1.0), ((2, 2, -4), 1.0)]
    ray = [0, 0, 0, 0.9, 0.9, -1.5]
    h = tree_hit(sph, ray)
    assert h.hit and h.object == 1


# the reference's TODOs (bbox_tree.rs:229-233), answered analytically
def test_tree_ray_inside_object():
    h = tree_hit([((0, 0, 0), 2.0)], [0, 0, 0, 0, 0, -1])
    assert h.hit and abs(h.t - 2.0) < 1e-12 and not h.front_face  # exit point, normal flipped inward


def test_tree_inside_box_not_object():
    # origin inside the sphere's box corner region but outside the sphere, pointing away
    h = tree_hit([((0, 0, 0), 1.0)], [0.95, 0.95, 0.95, 1, 1, 1])
    assert not h.hit


def test_tree_t_max_not_far_enough():
    assert not tree_hit([((0, 0, -10), 0.5)], [0, 0, 0, 0, 0, -1], 0.0, 9.0).hit


def test_tree_t_min_too_far():
    h = tree_hit([((0, 0, -10), 0.5)], [0, 0, 0, 0, 0, -1], 10.2, MAX)
    assert h.hit and h.t == 10.5  # near root rejected -> far root (sphere.rs:40-45)
    assert not tree_hit([((0, 0, -10), 0.5)], [0, 0, 0, 0, 0, -1], 10.6, MAX).hit


def test_tree_negative_radius_sphere_is_invisible():
    # sphere.rs:54-60: signed radius -> inverted bbox -> hit2 always rejects
    h = tree_hit([((0, 0, -5), -1.0)], [0, 0, 0, 0, 0, -1])
    assert not h.hit


# ---- analytic known answers --------------------------------------------------------------------
@pytest.mark.parametrize("ctr,key,want", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox4x32_10_random123_kat(ctr, key, want):
    c, k, o = (C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), (C.c_uint32 * 4)()
    L().or_philox4x32_10(c, k, o)
    assert tuple(o) == want


def test_rng_f64_in_unit_interval_and_53_bits():
    vals = [L().or_rng_f64(1234, 7, 3, d) for d in range(2000)]
    assert all(0.0 <= v < 1.0 for v in vals)
    assert all((v * 2 ** 53) == int(v * 2 ** 53) for v in vals)
    assert 0.45 < np.mean(vals) < 0.55


def test_sphere_analytic_t():
    import raytracer._native as N
    o = N.rt_object(geometry=N.RT_GEOM_SPHERE, material=0)
    o.p[:] = [0, 0, -5, 1, 0, 0]
    h = O.or_hit()
    assert L().or_object_hit(C.byref(o), O.d6([0, 0, 0, 0, 0, -2]), 0.001, float("inf"), C.byref(h))
    assert h.t == 2.0 and h.front_face == 1 and list(h.normal) == [0.0, 0.0, 1.0]
    # u,v from the unflipped outward normal (0,0,1): theta = acos(-0) = pi/2, phi = atan2(-1, 0) + pi
    assert abs(h.v - 0.5) < 1e-15 and abs(h.u - 0.25) < 1e-15


def test_rect_and_box_faces():
    import raytracer._native as N
    r = N.rt_object(geometry=N.RT_GEOM_RECT_XZ, material=0)
    r.p[:] = [-1, 1, -1, 1, 0.5, 0]  # xz_rect at y = 0.5
    h = O.or_hit()
    assert L().or_object_hit(C.byref(r), O.d6([0.5, 2, 0, 0, -1, 0]), 0.001, float("inf"), C.byref(h))
    assert h.t == 1.5 and list(h.normal) == [0.0, 1.0, 0.0] and h.u == 0.75 and h.v == 0.5
    b = N.rt_object(geometry=N.RT_GEOM_RECT_BOX, material=0)
    b.p[:] = [-1, -1, -1, 1, 1, 1]
    assert L().or_object_hit(C.byref(b), O.d6([0, 0, 5, 0, 0, -1]), 0.001, float("inf"), C.byref(h))
    assert h.t == 4.0 and list(h.normal) == [0.0, 0.0, 1.0] and h.front_face == 1
    # from inside: the far face, normal flipped to face the ray
    assert L().or_object_hit(C.byref(b), O.d6([0, 0, 0, 1, 0, 0]), 0.001, float("inf"), C.byref(h))
    assert h.t == 1.0 and list(h.normal) == [-1.0, 0.0, 0.0] and h.front_face == 0


def test_rect_bbox_padding():
    import raytracer._native as N
    r = N.rt_object(geometry=N.RT_GEOM_RECT_XY, material=0)
    r.p[:] = [0, 2, 0, 3, 5, 0]
    out = O._d6()
    L().or_object_bbox(C.byref(r), out)
    assert list(out) == [0, 0, 5 - 0.0001, 2, 3, 5 + 0.0001]  # BBOX_WIDTH (rect.rs:9)


def test_sky_only_pixel_matches_closed_form():
    """Empty scene: every sample is skybox(dir) (skybox/mod.rs:5-9), checked in closed form."""
    import raytracer as rt
    s = O.SphereScene([])
    osc = O.OracleScene(s)
    cam = rt.default_camera(8, "square")
    p = O.params(1)
    col, cnt = osc.sample(cam, p, 3, 4, 0)
    ray = O._d6()
    L().or_pixel_ray(C.byref(cam), p.seed, 3, 4, 0, ray)
    d = np.array(ray[3:])
    t = 0.5 * (d[1] / np.sqrt(d @ d) + 1.0)
    assert np.allclose(col, (1 - t) * np.ones(3) + t * np.array([0.5, 0.7, 1.0]), rtol=0, atol=1e-15)
    assert cnt.segments == 1


def test_dielectric_ir1_passes_straight_through():
    """ir = 1.0: refraction ratio 1, Schlick r0 = 0 -> straight through unless grazing (dielectric.rs)."""
    import raytracer as rt
    b = rt.SceneBuilder()
    b.add(rt.RectBox((-1, -1, -1), (1, 1, 1)), rt.Dielectric(1.0))
    s = b.finalize()
    osc = O.OracleScene(s)
    cam = rt.CameraBuilder(width=8, aspect_ratio=(1, 1), vfov=5.0).build(
        rt.CameraPosition((0, 0, 10), (0, 0, 0), (0, 1, 0)))
    p = O.params(1)
    empty = O.OracleScene(O.SphereScene([]))
    col, cnt = osc.sample(cam, p, 4, 4, 0)
    sky, _ = empty.sample(cam, p, 4, 4, 0)
    assert np.allclose(col, sky, rtol=0, atol=1e-12) and cnt.segments == 3


def test_cornell_light_seen_head_on():
    """FairyLight emission = albedo * (n . -d) / |d| (lighting.rs:59-66): head-on -> 15 exactly."""
    import raytracer as rt
    b = rt.SceneBuilder()
    b.set_skybox(rt.SkyBox.Nothing)
    b.add(rt.xz_rect(-1, 1, -1, 1, 0.0), rt.FairyLight(rt.TextureLoader.solid(15, 15, 15)))
    s = b.finalize()
    osc = O.OracleScene(s)
    e = np.zeros(3)
    h = osc.hit([0, 3, 0, 0, -1, 0])
    assert h.hit and list(h.normal) == [0.0, 1.0, 0.0]
    # emitted for this ray: 15 * (n . -d) / |d| = 15 * 1 / 1
    assert 15.0 * (np.dot(h.normal, [0, 1, 0])) / 1.0 == 15.0


def test_max_depth_zero_is_black():
    import raytracer as rt
    s = rt.scenes.random_scene(1).finalize(1)
    osc = O.OracleScene(s)
    cam = rt.default_camera(8, "square")
    col, cnt = osc.sample(cam, O.params(1, max_depth=0), 2, 2, 0)
    assert list(col) == [0.0, 0.0, 0.0] and cnt.segments == 0


def test_oracle_render_rows_threads_agree():
    import raytracer as rt
    s = rt.scenes.random_scene(7).finalize(7)
    osc = O.OracleScene(s)
    cam = rt.default_camera(24, "std16x9")
    a, _ = osc.render(cam, O.params(3), threads=1)
    b, _ = osc.render(cam, O.params(3), threads=4)
    assert np.array_equal(a, b)
    row = np.zeros((cam.image_width, 3))
    cnt = O.or_counters()
    L().or_render_scanline(osc.h, C.byref(cam), C.byref(O.params(3)), 5, row.ctypes.data, C.byref(cnt))
    assert np.array_equal(row, a[5])
