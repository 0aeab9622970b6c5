"""CPU tests of the boundary and the host layer: exported symbols, error behaviour without a GPU,
BVH builders vs the oracle's restatement of constructor.rs, camera math, serde-JSON interchange,
the to_image tonemap, and scene generation (scenes.rs)."""
import ctypes as C
import json
import math
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O
import raytracer as rt
from raytracer import _native as N

REPO = O.REPO
SEED = 0x5EED


def header_functions(path):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:rt|sh)_[a-z0-9_]+)\s*\(", text)))


@pytest.mark.parametrize("header,lib", [("include/shirley_rt.h", "libshirley_rt.so"),
                                        ("include/shirley_host.h", "libshirley_host.so")])
def test_library_exports_every_declared_symbol(header, lib):
    funcs = header_functions(os.path.join(REPO, header))
    assert len(funcs) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(N.LIB_DIR, lib)], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [f for f in funcs if f not in exported]
    assert not missing, missing
    sigs = N.RT_SIGNATURES if lib == "libshirley_rt.so" else N.SH_SIGNATURES
    assert sorted(sigs) == funcs  # the Python binding declares exactly the header's functions


def test_library_loads_and_reports_version():
    assert b"gfx950" in N.rt_lib().rt_version()


def test_hip_kernels_target_gfx950():
    blob = open(os.path.join(N.LIB_DIR, "libshirley_rt.so"), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in blob


def test_no_gpu_errors_are_loud():
    if N.rt_lib().rt_device_count(C.byref(C.c_int32())) == 0:
        n = C.c_int32()
        N.rt_lib().rt_device_count(C.byref(n))
        if n.value == 0:
            with pytest.raises(rt.RtError):
                rt.Device(0)
    # NULL / invalid arguments never crash
    assert N.rt_lib().rt_scene_upload(None, None, 0) == N.RT_E_INVALID
    assert N.rt_lib().rt_render(None, None, None, None) == N.RT_E_INVALID
    assert N.rt_lib().rt_tonemap(None, 0, 0, 1, None) == N.RT_E_INVALID


def oracle_tree(desc_holder):
    nodes, root = O.OracleScene(desc_holder).tree()
    return nodes, root


def product_tree(desc_ptr, builder):
    n = C.c_int32(0)
    assert N.rt_lib().rt_bvh_build_host(desc_ptr, builder, C.byref(n), None, None) == 0
    arr = (N.rt_bvh_node * max(1, n.value))()
    root = C.c_int32()
    assert N.rt_lib().rt_bvh_build_host(desc_ptr, builder, C.byref(n), arr, C.byref(root)) == 0
    return [(tuple(a.box), a.leaf, a.lhs, a.rhs) for a in arr[:n.value]], root.value


@pytest.mark.parametrize("name", ["random", "random-night", "cornell", "demo", "earth", "final:6:60"])
def test_reference_bvh_builder_equals_oracle(name):
    """O(N log N) builder (bvh_build.cpp) == literal restatement of constructor.rs (oracle.c)."""
    scene = rt.SceneBuilder.builtin(name, 0x5EED).finalize(0x5EED)
    assert product_tree(scene.desc_ptr, N.RT_BVH_REFERENCE) == oracle_tree(scene)


def test_reference_bvh_on_gen_spheres():
    s = O.SphereScene([((x + 0.3 * y, y * 0.7, z), 0.4 + 0.01 * (x * 7 % 5)) for x in range(-4, 4)
                       for y in range(-3, 3) for z in range(-2, 3)])
    assert product_tree(s.desc_ptr, N.RT_BVH_REFERENCE) == oracle_tree(s)


def test_sah_tree_covers_every_visible_object():
    scene = rt.scenes.random_scene(3).finalize(3)
    nodes, root = product_tree(scene.desc_ptr, N.RT_BVH_SAH)
    leaves = sorted(n[1] for n in nodes if n[1] >= 0)
    objs = scene.desc.objects
    visible = [i for i in range(scene.desc.n_objects)
               if not (objs[i].geometry == N.RT_GEOM_SPHERE and objs[i].p[3] <= 0)]
    assert leaves == visible
    for box, leaf, l, r in nodes:  # parents contain children
        if leaf < 0:
            for c in (l, r):
                cb = nodes[c][0]
                assert all(box[k] <= cb[k] for k in range(3)) and all(box[k + 3] >= cb[k + 3] for k in range(3))


def test_camera_matches_reference_formulas():
    cam = rt.default_camera(400, "std16x9", 20.0, 1.0, 0.001)
    assert (cam.image_width, cam.image_height) == (400, 225)
    h = math.tan(20.0 * math.pi / 180.0 / 2.0)
    assert cam.height == 2.0 * h and cam.width == (16 / 9) * cam.height
    w = np.array([13.0, 2.0, 3.0])
    fl = math.sqrt((13.0 * 13.0 + 2.0 * 2.0) + 3.0 * 3.0)
    w = w / fl
    u = np.cross([0.0, 1.0, 0.0], w)
    u = u / math.sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2])
    assert list(cam.w) == list(w) and np.allclose(list(cam.u), u, atol=1e-16)
    assert cam.focus_length == 10.0 and cam.has_lens == 1 and cam.lens_radius == 0.0005
    c = rt.cornell_camera(600)
    assert (c.image_width, c.image_height) == (600, 600) and c.lens_radius == 0.000005
    assert rt.default_camera(1200, "std3x2").image_height == 800
    assert rt.default_camera(800, "square").image_height == 800


def test_scene_json_round_trip_and_format():
    b = rt.scenes.random_scene(11)
    text = b.to_json()
    j = json.loads(text)
    assert j["skybox"] == "Above" and len(j["objects"]) == len(b)
    g0 = j["objects"][0]["geometry"]
    assert "RectXZ" in g0 and g0["RectXZ"]["offset"] == -0.02
    box = j["objects"][1]["geometry"]["RectBox"]
    assert box["min"] == {"vec": [-30.0, -0.01, -30.0]} and len(box["xy_sides"]) == 2
    assert j["objects"][1]["material"] == {"Dielectric": {"ir": 1.0}}
    b2 = rt.SceneBuilder.from_json(text)
    assert b2.to_json() == text
    d1, d2 = b.finalize(5).desc, b2.finalize(5).desc
    assert d1.n_objects == d2.n_objects
    for i in range(d1.n_objects):
        assert list(d1.objects[i].p) == list(d2.objects[i].p)


def test_python_builder_matches_builtin_cornell():
    b = rt.SceneBuilder()
    b.set_skybox(rt.SkyBox.Nothing)
    red = rt.Lambertian(rt.TextureLoader.solid(0.65, 0.05, 0.05))
    white = rt.Lambertian(rt.TextureLoader.solid(0.73, 0.73, 0.73))
    green = rt.Lambertian(rt.TextureLoader.solid(0.12, 0.45, 0.15))
    light = rt.FairyLight(rt.TextureLoader.solid(15.0, 15.0, 15.0))
    b.add(rt.yz_rect(0, 555, 0, 555, 555), green)
    b.add(rt.yz_rect(0, 555, 0, 555, 0), red)
    b.add(rt.xz_rect(213, 343, 227, 332, 554), light)
    b.add(rt.xz_rect(0, 555, 0, 555, 0), white)
    b.add(rt.xz_rect(0, 555, 0, 555, 555), white)
    b.add(rt.xy_rect(0, 555, 0, 555, 555), white)
    b.add(rt.RectBox((130, 0, 65), (295, 165, 230)), white)
    b.add(rt.RectBox((265, 0, 295), (430, 330, 460)), white)
    assert b.to_json() == rt.scenes.create_cornell_box().to_json()


def test_random_scene_structure():
    b = rt.scenes.random_scene(0x5EED)
    j = json.loads(b.to_json())
    objs = j["objects"]
    assert len(objs) > 400  # 2 ground + 3 big + ~481 small (scenes.rs:369-425)
    big = [o["geometry"]["Sphere"] for o in objs[2:5]]
    assert [s["radius"] for s in big] == [1.0, 1.0, 1.0]
    kinds = {list(o["material"])[0] for o in objs[5:]}
    assert kinds <= {"Lambertian", "Dielectric", "Metal"}
    for o in objs[5:]:
        s = o["geometry"]["Sphere"]
        r = s["radius"]
        assert r <= 0.25
        c = s["center"]["vec"]
        assert math.dist(c, [3.0, c[1], 0.0]) > 0.9 or r < 0.25  # keep-out (after check_fit_ball sinking)
    assert json.loads(rt.scenes.random_scene(0x5EED).to_json()) == j  # deterministic per seed
    assert json.loads(rt.scenes.random_scene(0x5EEE).to_json()) != j
    desc = b.finalize(0x5EED).desc
    assert desc.n_perlin == 1  # the day ground's noise(1.0) checker child (scenes.rs:256-260)


def test_texture_dedup_matches_texture_manager():
    """TextureManager (loader.rs:113-131) dedups top-level loaders by bitwise key; checker children
    are loaded fresh (loader.rs:47-60), so each checker holding noise() gets its own Perlin table."""
    b = rt.SceneBuilder()
    t = rt.TextureLoader.checker(3.0, rt.TextureLoader.noise(1.0), rt.TextureLoader.solid(0.1, 0.1, 0.1))
    for k in range(3):
        b.add(rt.Sphere((k, 0, 0), 0.5), rt.Lambertian(t))
    b.add(rt.Sphere((5, 0, 0), 0.5), rt.Lambertian(rt.TextureLoader.noise(1.0)))
    b.add(rt.Sphere((6, 0, 0), 0.5), rt.Lambertian(rt.TextureLoader.noise(1.0)))
    d = b.finalize(1).desc
    assert d.n_perlin == 2 and d.n_textures == 4
    assert len({d.materials[i].texture for i in range(3)}) == 1


def test_perlin_tables_are_permutations():
    t = N.rt_perlin_table()
    N.host_check(N.host_lib().sh_perlin_generate(42, 0, C.byref(t)))
    for perm in (t.perm_x, t.perm_y, t.perm_z):
        assert sorted(perm) == list(range(256))
    rf = np.array([list(v) for v in t.ranfloat])
    assert rf.min() >= -1 and rf.max() < 1 and abs(rf.mean()) < 0.1


def test_earth_texture_loads():
    w, h = C.c_int32(), C.c_int32()
    p = C.POINTER(C.c_uint8)()
    path = os.path.join(REPO, "shirley-raytracing-rs_amd/assets/earthmap.rgb8.gz")
    N.host_check(N.host_lib().sh_load_image(path.encode(), C.byref(w), C.byref(h), C.byref(p)))
    assert (w.value, h.value) == (1024, 512)
    a = np.ctypeslib.as_array(p, shape=(512 * 1024 * 3,)).copy()
    N.host_lib().sh_free(p)
    assert 85 < a.mean() < 95


EARTH_CHILD = r"""
import ctypes as C, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from raytracer import _native as N
s = C.c_void_p()
N.host_check(N.host_lib().sh_scene_builtin(b"earth", 0x5EED, C.byref(s)))
d = C.c_void_p()
N.host_check(N.host_lib().sh_scene_finalize(s, 0x5EED, C.byref(d)))
v = N.host_lib().sh_desc_view(d).contents
assert v.n_images == 1, v.n_images
im = v.images[0]
px = np.ctypeslib.as_array(im.rgb, shape=(im.height * im.width * 3,))
print(im.width, im.height, int(px.astype(np.int64).sum()), N.host_lib()._name)
"""


@pytest.mark.parametrize("lib_dir", ["lib", "lib/diag"])
def test_earth_builtin_needs_no_asset_lookup(lib_dir, tmp_path):
    """EarthBuiltin is linked into the library (earth_embed.S, the reference's include_bytes!,
    image_texture.rs:11,18-20): every copy of libshirley_host.so finalises the earth scene with
    SHIRLEY_ASSETS unset, from any working directory, and the texels equal the committed asset."""
    pkg = os.path.join(REPO, "shirley-raytracing-rs_amd")
    env = {k: v for k, v in os.environ.items() if k not in ("SHIRLEY_ASSETS",)}
    env["SHIRLEY_LIB_DIR"] = os.path.join(pkg, lib_dir)
    env["SHIRLEY_NO_TORCH"] = "1"
    r = subprocess.run([sys.executable, "-c", EARTH_CHILD, pkg], env=env, cwd=str(tmp_path),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    w, h, total, name = r.stdout.split()
    assert name.startswith(env["SHIRLEY_LIB_DIR"])
    import gzip
    blob = gzip.open(os.path.join(pkg, "assets", "earthmap.rgb8.gz")).read()
    texels = np.frombuffer(blob[blob.index(b"\n") + 1:], dtype=np.uint8)
    assert (int(w), int(h)) == (1024, 512)
    assert int(total) == int(texels.astype(np.int64).sum())


def test_tonemap_equals_oracle():
    rng = np.random.default_rng(0)
    acc = rng.uniform(0, 3, size=(7, 9, 3)) * 4
    acc[0, 0] = [np.nan, -1.0, 1e9]
    a = rt.to_image(acc, 4)
    b = np.zeros_like(a)
    O.lib().or_tonemap(np.ascontiguousarray(acc).ctypes.data, 9, 7, 4, b.ctypes.data)
    assert np.array_equal(a, b)
    assert list(a[6, 0]) == [0, 0, 255]  # NaN -> 0, negative -> 0, huge -> 255; row flip


def test_png_writer_round_trip(tmp_path):
    from PIL import Image
    img = (np.arange(5 * 7 * 3) % 256).astype(np.uint8).reshape(5, 7, 3)
    p = str(tmp_path / "x.png")
    rt.write_png(p, img)
    assert np.array_equal(np.asarray(Image.open(p)), img)


def test_cli_scene_output_and_test_subcommand(tmp_path):
    cli = os.path.join(N.BIN_DIR, "ray-cli")
    out = subprocess.run([cli, "test"], capture_output=True, text=True)
    assert out.returncode == 0 and "nothing to test" in out.stderr
    bad = subprocess.run([cli, "render", "nonsense"], capture_output=True, text=True)
    assert bad.returncode != 0


def test_multi_gpu_entry_points_reject_bad_arguments_without_a_device():
    """rt_render_multi / rt_render_sharded / rt_comm_* validate before touching a device or RCCL."""
    lib = N.rt_lib()
    assert lib.rt_render_multi(None, 1, None, None, None) == N.RT_E_INVALID
    assert lib.rt_render_multi(None, 0, None, None, None) == N.RT_E_INVALID
    assert lib.rt_render_sharded(None, None, None, None, None, None) == N.RT_E_INVALID
    assert lib.rt_comm_init_rank(None, None, 1, 0, None) == N.RT_E_INVALID
    assert lib.rt_comm_destroy(None) == N.RT_OK
    assert lib.rt_comm_unique_id(None) == N.RT_E_INVALID


def test_scene_digest_is_stable_and_discriminating():
    """rt_scene_digest_host (ABI 6): the digest rt_scene_upload records and the multi-GPU calls compare
    across ranks — equal for equal scenes (rebuilt from scratch), different for any other scene, seed,
    material or builder."""
    a = rt.scenes.random_scene(SEED).finalize(SEED)
    d = rt.scene_digest(a, "sah")
    assert d == rt.scene_digest(a, "sah")
    assert d == rt.scene_digest(rt.scenes.random_scene(SEED).finalize(SEED), "sah")
    assert d != rt.scene_digest(a, "reference")
    assert d != rt.scene_digest(rt.scenes.random_scene(SEED + 1).finalize(SEED + 1), "sah")
    assert d != rt.scene_digest(rt.scenes.random_scene(SEED).finalize(SEED + 1), "sah")  # Perlin tables only
    assert d != rt.scene_digest(rt.scenes.random_scene(SEED, night=True).finalize(SEED), "sah")
    digests = {rt.scene_digest(rt.SceneBuilder.builtin(n, SEED).finalize(SEED)) for n in
               ("random", "demo", "perlin", "earth", "box-light", "cornell", "final:4:30")}
    assert len(digests) == 7
    # a one-field change of one object
    b = rt.scenes.random_scene(SEED).finalize(SEED)
    b.desc_ptr.contents.objects[3].p[3] += 1e-9
    assert rt.scene_digest(b, "sah") != d


def test_render_params_abi6_layout():
    import ctypes as C
    assert C.sizeof(N.rt_render_params) == 48
    assert N.rt_render_params.sample_begin.offset == 32 and N.rt_render_params.scratch_mb.offset == 44
    assert C.sizeof(N.rt_counters) == 112
