"""Known-answer tests of the material, light and texture semantics.

The reference's own unit tests cover only core/fp.rs, bvh/aabb.rs and bvh/bbox_tree.rs; the scatter,
emission and texture functions were pinned only by reading them.  Here each is held to an analytic answer
or to an independent Python restatement of the cited reference lines (binary64, nalgebra's evaluation
order; draws from the numpy Philox restatement of tests/test_rng_streams.py), for two implementations:

  * backend "oracle" (CPU suite): oracle/oracle.c's or_probe_segment / or_texture_value / or_perlin_noise /
    or_reflectance — the checker every GPU parity test trusts;
  * backend "gpu" (-m gpu): rt_probe_segment, one ray_color iteration through the megakernel's own device
    code (render traversal, hit record, texture leaf, the wave's marble and sampler, shade_factor).

A segment's answer is (object, emitted, scatter attenuation, scattered ray, draw counter after it): one
iteration of render.rs:30-46.  Pinned here beyond the 25 reference unit tests:
  metal.rs:26-40        mirror direction at fuzz 0, reflected + fuzz * random_in_unit_sphere, albedo
  dielectric.rs:15-50   Schlick at cos = 1 (r0) and cos = 0 (1), the TIR boundary (no uniform drawn on the
                        TIR side), Snell refraction at 45 degrees, the Schlick-vs-uniform decision
  lighting.rs:21-67     DiffuseLight emits and absorbs; FairyLight's n.(-d)/|d| emission at an oblique
                        angle and unit(albedo) attenuation
  lambertian.rs:21-37   normal + unit(random_in_unit_sphere) with the solid albedo
  checker.rs:27-37      the sign of sin(sx) sin(sy) sin(sz) at points straddling the sines' zeros
  image_texture.rs:34-56  texel index at u, v = 0 and 1, interior points, and the clamp of out-of-range u, v
  perlin/mod.rs:87-124,162-183  noise = 0 at lattice points, an interior point, turbulence and marble
  skybox/mod.rs:5-25    the sky on a miss
  core/math.rs:32-45    random_in_unit_sphere's rejection loop (draw counter advances 3 per attempt)
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_lib as O
from raytracer import _native as N
from test_rng_streams import path_draw_u64

SEED = 0x5EED
SAMPLE = 7


# ---- Python restatement of the reference's arithmetic (binary64, nalgebra order) --------------------
def U(pixel, draw, sample=SAMPLE, seed=SEED):
    """rng.gen::<f64>() on the path key: (u64 >> 11) * 2^-53 (rand 0.8 Standard)."""
    return float(int(path_draw_u64(seed, pixel, sample, draw)) >> 11) * (1.0 / 9007199254740992.0)


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def length(a):
    return math.sqrt(dot(a, a))


def unit(a):
    n = length(a)
    return [a[0] / n, a[1] / n, a[2] / n]


def add(a, b):
    return [a[0] + b[0], a[1] + b[1], a[2] + b[2]]


def sub(a, b):
    return [a[0] - b[0], a[1] - b[1], a[2] - b[2]]


def scale(a, s):
    return [a[0] * s, a[1] * s, a[2] * s]


def reflect(v, n):  # vec3.rs:134-137
    return sub(v, scale(n, 2.0 * dot(v, n)))


def refract(uv, n, eta):  # vec3.rs:139-145
    cos_theta = min(dot(scale(uv, -1.0), n), 1.0)  # fmin_one (no NaN here)
    r_perp = scale(add(scale(n, cos_theta), uv), eta)
    r_par_mag = math.sqrt(abs(1.0 - dot(r_perp, r_perp))) * -1.0
    return add(r_perp, scale(n, r_par_mag))


def reflectance(cosine, ref_idx):  # dielectric.rs:55-59 (powf = libm pow)
    r0 = (1.0 - ref_idx) / (1.0 + ref_idx)
    r0 = r0 * r0
    return r0 + (1.0 - r0) * math.pow(1.0 - cosine, 5.0)


def unit_sphere(pixel, draw):
    """core/math.rs:32-45: (random_real(-1, 1) x 3) until length_squared <= 1; returns (p, draw after)."""
    while True:
        p = [-1.0 + 2.0 * U(pixel, draw + k) for k in range(3)]
        draw += 3
        if dot(p, p) <= 1.0:
            return p, draw


def near_zero(a):
    return all(abs(x) < 1e-8 for x in a)


# ---- scenes built as raw rt_scene_desc (ctypes) ----------------------------------------------------
class KatScene:
    """objects: (geometry, material, p[6]); materials: (kind, texture, albedo, param); textures: dicts."""

    def __init__(self, objects, materials, textures=(), perlin=None, images=(), sky=N.RT_SKY_ABOVE, sky_color=(0, 0, 0)):
        self.objs = (N.rt_object * max(1, len(objects)))()
        for i, (g, m, p) in enumerate(objects):
            self.objs[i].geometry, self.objs[i].material = g, m
            self.objs[i].p[:] = list(p) + [0.0] * (6 - len(p))
        self.mats = (N.rt_material * max(1, len(materials)))()
        for i, (k, t, alb, par) in enumerate(materials):
            self.mats[i].kind, self.mats[i].texture, self.mats[i].param = k, t, par
            self.mats[i].albedo[:] = list(alb)
        self.texs = (N.rt_texture * max(1, len(textures)))()
        for i, t in enumerate(textures):
            self.texs[i].kind = t["kind"]
            self.texs[i].odd, self.texs[i].even, self.texs[i].table = t.get("odd", 0), t.get("even", 0), t.get("table", 0)
            self.texs[i].color[:] = list(t.get("color", (0, 0, 0)))
            self.texs[i].scale = t.get("scale", 0.0)
        self.perlin = None
        if perlin is not None:
            self.perlin = (N.rt_perlin_table * 1)()
            self.perlin[0] = perlin
        self.img_bufs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        self.imgs = (N.rt_image * max(1, len(images)))()
        for i, im in enumerate(self.img_bufs):
            self.imgs[i].height, self.imgs[i].width = im.shape[0], im.shape[1]
            self.imgs[i].rgb = im.ctypes.data_as(C.POINTER(C.c_uint8))
        d = N.rt_scene_desc()
        d.sky = sky
        d.sky_color[:] = list(sky_color)
        d.n_objects, d.objects = len(objects), self.objs
        d.n_materials, d.materials = len(materials), self.mats
        d.n_textures, d.textures = len(textures), self.texs
        if perlin is not None:
            d.n_perlin, d.perlin = 1, self.perlin
        if images:
            d.n_images, d.images = len(images), self.imgs
        self.desc = d
        self.desc_ptr = C.pointer(self.desc)


def perlin_table(seed=3):
    """A Perlin table like perlin/mod.rs:11-38 (random vectors in [-1, 1)^3, three permutations)."""
    rng = np.random.default_rng(seed)
    t = N.rt_perlin_table()
    vecs = rng.uniform(-1.0, 1.0, size=(256, 3))
    for i in range(256):
        t.ranfloat[i][:] = [float(x) for x in vecs[i]]
    for name in ("perm_x", "perm_y", "perm_z"):
        getattr(t, name)[:] = [int(x) for x in rng.permutation(256)]
    return t, vecs


def perlin_noise(tab, p):
    """perlin/mod.rs:87-109 (+ interp 40-63) restated."""
    vecs, px, py, pz = tab
    xf, yf, zf = math.floor(p[0]), math.floor(p[1]), math.floor(p[2])
    u, v, w = p[0] - xf, p[1] - yf, p[2] - zf
    i, j, k = int(xf), int(yf), int(zf)
    uu, vv, ww = u * u * (3.0 - 2.0 * u), v * v * (3.0 - 2.0 * v), w * w * (3.0 - 2.0 * w)
    acc = 0.0
    for di in range(2):
        for dj in range(2):
            for dk in range(2):
                c = vecs[px[(i + di) & 255] ^ py[(j + dj) & 255] ^ pz[(k + dk) & 255]]
                fi, fj, fk = float(di), float(dj), float(dk)
                wgt = [u - fi, v - fj, w - fk]
                acc += ((fi * uu + (1.0 - fi) * (1.0 - uu)) * (fj * vv + (1.0 - fj) * (1.0 - vv)) *
                        (fk * ww + (1.0 - fk) * (1.0 - ww)) * dot([float(x) for x in c], wgt))
    return acc


def turbulence(tab, p, depth=7):  # perlin/mod.rs:111-124
    acc, tp, weight = 0.0, list(p), 1.0
    for _ in range(depth):
        acc += weight * perlin_noise(tab, tp)
        weight *= 0.5
        tp = scale(tp, 2.0)
    return abs(acc)


def marble(tab, sc, p):  # perlin/mod.rs:162-183
    turb = 10.0 * turbulence(tab, p, 7)
    vd = [0.2 * sc * p[0], 0.1 * sc * p[1], 1.0 * sc * p[2]]
    vd = [math.sin(vd[0] + turb), math.sin(vd[1] + turb), math.sin(vd[2] + turb)]
    total = dot(vd, unit([0.0, 0.0, 1.0]))
    return 0.5 * (1.0 + total)


# ---- the two backends ------------------------------------------------------------------------------
@pytest.fixture(params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def probe(request):
    """probe(scene, rays, draw) -> list of rt_probe records (ray i on pixel i, sample SAMPLE)."""
    if request.param == "oracle":
        def run(scene, rays, draw=0):
            osc = O.OracleScene(scene.desc)
            return [osc.probe(r, SEED, i, SAMPLE, draw) for i, r in enumerate(rays)]
        return run
    gpu = request.getfixturevalue("gpu")
    import raytracer as rt

    def run(scene, rays, draw=0):
        rt.Device.upload(gpu, type("S", (), {"desc_ptr": scene.desc_ptr})())
        return list(gpu.probe(np.array(rays, dtype=np.float64), SEED, SAMPLE, draw))
    return run


XZ = N.RT_GEOM_RECT_XZ
FLOOR = [-10.0, 10.0, -10.0, 10.0, 0.0]  # xz_rect(-10, 10, -10, 10, y = 0): normal +y (rect.rs:54-80)


def v(a):
    return [a[0], a[1], a[2]]


def test_metal_fuzz_zero_mirror(probe):
    # metal.rs:26-40 at fuzz 0: unit(d) reflected about the normal, exactly (a = 1/sqrt(2): (a, -a, 0) -> (a, a, 0));
    # random_in_unit_sphere is still drawn (its product with 0 adds +-0)
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_METAL, -1, (0.8, 0.6, 0.2), 0.0)])
    for draw in (0, 1, 6):
        r = probe(scene, [[0.0, 1.0, 0.0, 1.0, -1.0, 0.0]], draw)[0]
        a = 1.0 / math.sqrt(2.0)
        assert (r.object, r.scattered, r.emits, r.front_face) == (0, 1, 0, 1)
        assert (r.t, v(r.point), v(r.normal)) == (1.0, [1.0, 0.0, 0.0], [0.0, 1.0, 0.0])
        assert v(r.origin) == [1.0, 0.0, 0.0] and v(r.direction) == [a, a, 0.0]
        assert v(r.attenuation) == [0.8, 0.6, 0.2]
        assert r.draw == unit_sphere(0, draw)[1]


def test_metal_fuzzed_direction(probe):
    # reflected + random_in_unit_sphere * fuzz, the point from draws d, d+1, d+2, ... (rejection loop)
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_METAL, -1, (0.5, 0.5, 0.5), 0.3)])
    rays = [[0.1 * i, 2.0, 0.3, 0.2, -1.0, 0.1 * (i - 8)] for i in range(16)]
    got = probe(scene, rays, 4)
    for i, (ray, r) in enumerate(zip(rays, got)):
        p, after = unit_sphere(i, 4)
        want = add(reflect(unit(ray[3:]), [0.0, 1.0, 0.0]), scale(p, 0.3))
        assert v(r.direction) == want and r.draw == after


def test_dielectric_total_internal_reflection_boundary(probe):
    # dielectric.rs:21-49 from inside (back face: ratio = ir = 1.5, normal flipped to -y), rays around the
    # critical angle sin = 1/1.5: on the TIR side the uniform is NOT drawn (the || short-circuits) and the
    # ray reflects; on the other side one uniform is drawn and decides reflect vs refract by Schlick
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_DIELECTRIC, -1, (0, 0, 0), 1.5)])
    crit = math.asin(1.0 / 1.5)
    angles = [crit + k * 1e-7 for k in range(-4, 5)] + [0.3, 1.2]
    rays = [[0.0, -1.0, 0.0, math.sin(t), math.cos(t), 0.0] for t in angles]
    for draw in (2, 3):
        got = probe(scene, rays, draw)
        n_tir = 0
        for i, (ray, r) in enumerate(zip(rays, got)):
            ud = unit(ray[3:])
            n = [0.0, -1.0, 0.0]
            assert r.front_face == 0 and v(r.normal) == n
            cos_t = min(dot(scale(ud, -1.0), n), 1.0)
            tir = 1.5 * math.sqrt(1.0 - cos_t * cos_t) > 1.0
            if tir:
                n_tir += 1
                assert r.draw == draw and v(r.direction) == reflect(ud, n)
            else:
                refl = reflectance(cos_t, 1.5) > U(i, draw)
                assert r.draw == draw + 1
                assert v(r.direction) == (reflect(ud, n) if refl else refract(ud, n, 1.5))
            assert v(r.attenuation) == [1.0, 1.0, 1.0]
        assert 3 <= n_tir <= 7


def test_dielectric_snell_refraction_45_degrees(probe):
    # front face (ratio 1 / 1.5) at 45 degrees: the refracted ray obeys Snell (sin_t = sin_i / 1.5) and is
    # the reference's refract() bit for bit; rays whose uniform falls below Schlick's value reflect
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_DIELECTRIC, -1, (0, 0, 0), 1.5)])
    rays = [[0.01 * i, 1.0, 0.0, 1.0, -1.0, 0.0] for i in range(48)]
    got = probe(scene, rays, 0)
    ratio = 1.0 / 1.5
    n_refr = 0
    for i, (ray, r) in enumerate(zip(rays, got)):
        ud, n = unit(ray[3:]), [0.0, 1.0, 0.0]
        cos_t = min(dot(scale(ud, -1.0), n), 1.0)
        refl = reflectance(cos_t, ratio) > U(i, 0)
        want = reflect(ud, n) if refl else refract(ud, n, ratio)
        assert v(r.direction) == want and r.draw == 1
        if not refl:
            n_refr += 1
            sin_t = math.hypot(r.direction[0], r.direction[2]) / length(v(r.direction))
            assert abs(sin_t - math.sqrt(0.5) / 1.5) < 1e-15
            assert abs(length(v(r.direction)) - 1.0) < 1e-15
    assert n_refr >= 40  # Schlick at 45 degrees is ~0.05


def test_schlick_endpoints_oracle():
    # dielectric.rs:55-59: reflectance(1, r) = r0 exactly (pow(0, 5) = 0), reflectance(0, r) = r0 + (1 - r0)
    for ri in (1.5, 1.0 / 1.5, 1.0, 2.4):
        r0 = ((1.0 - ri) / (1.0 + ri)) ** 2
        assert O.lib().or_reflectance(1.0, ri) == r0
        assert O.lib().or_reflectance(0.0, ri) == r0 + (1.0 - r0)


def test_schlick_decisions_at_normal_and_grazing_incidence(probe):
    # cos = 1 exactly (normal incidence): reflect iff r0 = 0.04 > U; cos ~ 1e-9 (grazing): Schlick ~ 1, so
    # every uniform below it reflects
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_DIELECTRIC, -1, (0, 0, 0), 1.5)])
    ratio = 1.0 / 1.5
    normal = [[0.001 * i, 1.0, 0.0, 0.0, -1.0, 0.0] for i in range(200)]
    got = probe(scene, normal, 0)
    n_refl = 0
    for i, r in enumerate(got):
        refl = reflectance(1.0, ratio) > U(i, 0)
        n_refl += refl
        assert v(r.direction) == ([0.0, 1.0, 0.0] if refl else refract([0.0, -1.0, 0.0], [0.0, 1.0, 0.0], ratio))
    assert 1 <= n_refl <= 20
    grazing = [[0.0, 1e-9 * (1 + 0.25 * i), -5.0 + 0.01 * i, 1.0, -1e-9, 0.0] for i in range(32)]
    got = probe(scene, grazing, 0)
    for i, (ray, r) in enumerate(zip(grazing, got)):
        ud = unit(ray[3:])
        cos_t = min(dot(scale(ud, -1.0), [0.0, 1.0, 0.0]), 1.0)
        assert 0.0 < cos_t < 1e-8
        refl = reflectance(cos_t, ratio) > U(i, 0)
        assert refl and v(r.direction) == reflect(ud, [0.0, 1.0, 0.0])


def test_fairy_light_oblique_emission_and_unit_albedo(probe):
    # lighting.rs:42-67: emitted = albedo * (n . -d) / |d| at the hit (oblique d = (1, -2, 0): 2 / sqrt(5)),
    # attenuation = unit(albedo), scatter = normal + unit(random_in_unit_sphere)
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_FAIRY_LIGHT, 0, (0, 0, 0), 0.0)],
                     [{"kind": N.RT_TEX_SOLID, "color": (3.0, 4.0, 0.0)}])
    rays = [[0.0, 2.0, 0.0, 1.0, -2.0, 0.0], [0.5, 1.0, 0.5, -0.3, -1.0, 0.7]]
    got = probe(scene, rays, 0)
    for i, (ray, r) in enumerate(zip(rays, got)):
        d = ray[3:]
        n = [0.0, 1.0, 0.0]
        s = dot(n, scale(d, -1.0))
        assert r.emits == 1 and v(r.emitted) == scale([3.0, 4.0, 0.0], s / length(d))
        assert v(r.attenuation) == unit([3.0, 4.0, 0.0]) == [0.6, 0.8, 0.0]
        p, after = unit_sphere(i, 0)
        sc = add(n, unit(p))
        assert v(r.direction) == (n if near_zero(sc) else sc) and r.draw == after
    assert v(got[0].emitted) == [3.0 * (2.0 / math.sqrt(5.0)), 4.0 * (2.0 / math.sqrt(5.0)), 0.0]


def test_diffuse_light_emits_and_absorbs(probe):
    # lighting.rs:21-29: emitted = the texture's colour, scatter None (the path ends, no draw)
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_DIFFUSE_LIGHT, 0, (0, 0, 0), 0.0)],
                     [{"kind": N.RT_TEX_SOLID, "color": (7.0, 7.0, 7.0)}])
    r = probe(scene, [[0.0, 1.0, 0.0, 0.2, -1.0, 0.1]], 5)[0]
    assert (r.object, r.emits, r.scattered, r.draw) == (0, 1, 0, 5)
    assert v(r.emitted) == [7.0, 7.0, 7.0]


def test_lambertian_scatter_and_sky_on_miss(probe):
    # lambertian.rs:21-37: normal + unit(random_in_unit_sphere), attenuation = albedo; a miss: the sky
    # (skybox/mod.rs:18-25: lerp of white and (0.5, 0.7, 1.0) by 0.5 (unit(d).y + 1)), the path ends
    scene = KatScene([(XZ, 0, FLOOR)], [(N.RT_MAT_LAMBERTIAN, 0, (0, 0, 0), 0.0)],
                     [{"kind": N.RT_TEX_SOLID, "color": (0.25, 0.5, 0.75)}])
    rays = [[1.0, 3.0, -2.0, 0.1, -1.0, 0.2], [0.0, 1.0, 0.0, 0.3, 1.0, 0.2]]
    got = probe(scene, rays, 3)
    p, after = unit_sphere(0, 3)
    assert v(got[0].direction) == add([0.0, 1.0, 0.0], unit(p)) and got[0].draw == after
    assert v(got[0].attenuation) == [0.25, 0.5, 0.75]
    sky = got[1]
    assert (sky.object, sky.emits, sky.scattered, sky.draw) == (-1, 1, 0, 3)
    t = 0.5 * (unit(rays[1][3:])[1] + 1.0)
    assert v(sky.emitted) == add(scale([1.0, 1.0, 1.0], 1.0 - t), scale([0.5, 0.7, 1.0], t))


def _checker_scene(size):
    # (a checker's children precede it in the flattened texture list, as TextureManager::load leaves them)
    return KatScene([(XZ, 0, [-10.0, 10.0, -10.0, 10.0, 0.25])], [(N.RT_MAT_LAMBERTIAN, 2, (0, 0, 0), 0.0)],
                    [{"kind": N.RT_TEX_SOLID, "color": (1.0, 0.0, 0.0)},
                     {"kind": N.RT_TEX_SOLID, "color": (0.0, 1.0, 0.0)},
                     {"kind": N.RT_TEX_CHECKER, "odd": 0, "even": 1, "scale": size}])


def test_checker_sign_straddling_sine_zeros(probe):
    # checker.rs:27-37: odd where sin(s x) sin(s y) sin(s z) < 0.  Vertical rays hit y = 0.25 at exactly
    # (x, 0.25, z); x runs over the doubles next to k pi / s, where sin(s x) changes sign (the reference's
    # libm, glibc here, decides the sign of each factor; sin(0) = +0 makes the product >= 0: even)
    size = 10.0
    xs = []
    for k in range(-3, 4):
        x0 = k * math.pi / size
        xs += [math.nextafter(x0, -math.inf), x0, math.nextafter(x0, math.inf)]
    xs += [0.0, -0.0]
    rays = []
    for x in xs:
        for z in (0.05, -0.05):
            rays.append([x, 1.25, z, 0.0, -1.0, 0.0])
    got = probe(_checker_scene(size), rays, 0)
    n_odd = 0
    for ray, r in zip(rays, got):
        x, z = ray[0], ray[2]
        assert v(r.point) == [x, 0.25, z]
        sines = math.sin(size * x) * math.sin(size * 0.25) * math.sin(size * z)
        odd = sines < 0.0
        n_odd += odd
        assert v(r.attenuation) == ([1.0, 0.0, 0.0] if odd else [0.0, 1.0, 0.0]), (x, z)
    assert 10 <= n_odd <= len(rays) - 10


def test_checker_value_oracle_texture_value():
    # the same rule through or_texture_value at points given directly (no ray): p on the zeros' both sides
    sc = _checker_scene(10.0)
    osc = O.OracleScene(sc.desc)
    out = (C.c_double * 3)()
    for x in (-0.3, math.nextafter(math.pi / 10, 0), math.nextafter(math.pi / 10, 1), 0.0, -0.0):
        for z in (0.05, -0.05, 0.0):
            p = (C.c_double * 3)(x, 0.25, z)
            O.lib().or_texture_value(osc.h, 2, 0.0, 0.0, p, out)
            odd = math.sin(10 * x) * math.sin(2.5) * math.sin(10 * z) < 0.0
            assert list(out) == ([1.0, 0.0, 0.0] if odd else [0.0, 1.0, 0.0])


W_IMG, H_IMG = 5, 4


def _image():
    img = np.zeros((H_IMG, W_IMG, 3), dtype=np.uint8)
    for j in range(H_IMG):
        for i in range(W_IMG):
            img[j, i] = (40 * i + 3, 50 * j + 5, 7 + i + 10 * j)
    return img


def texel(img, u, v_):
    """image_texture.rs:71-92: clamp, v flipped, (x * (dim - 1)) as u32, rgb * (1 / 255)."""
    cl = lambda x: (x if x < 1.0 else 1.0) if x > 0.0 else 0.0  # nalgebra::clamp (NaN -> min)
    uu, vv = cl(u), 1.0 - cl(v_)
    i = int(uu * float(W_IMG - 1))
    j = int(vv * float(H_IMG - 1))
    return [float(c) * (1.0 / 255.0) for c in img[j, i]]


def test_image_texel_index_at_edges(probe):
    # xz_rect(0, 1, 0, 1, y = 0): u = x, v = z (rect.rs:71-72), so vertical rays pick the texel of (x, z):
    # the corners (u, v in {0, 1}), the centre, and points just inside the texel boundaries
    img = _image()
    scene = KatScene([(XZ, 0, [0.0, 1.0, 0.0, 1.0, 0.0])], [(N.RT_MAT_LAMBERTIAN, 0, (0, 0, 0), 0.0)],
                     [{"kind": N.RT_TEX_IMAGE, "table": 0}], images=[img])
    pts = [(0.0, 0.0), (1.0, 0.0), (0.0, 1.0), (1.0, 1.0), (0.5, 0.5), (0.25, 1 / 3), (math.nextafter(0.25, 0), 0.999),
           (math.nextafter(0.75, 1), math.nextafter(1 / 3, 0)), (0.999999, 0.000001)]
    rays = [[x, 1.0, z, 0.0, -1.0, 0.0] for x, z in pts]
    got = probe(scene, rays, 0)
    for (x, z), r in zip(pts, got):
        assert r.object == 0, (x, z)
        assert v(r.attenuation) == texel(img, x, z), (x, z)


def test_image_texel_clamp_oracle():
    # image_texture.rs:73-74: u, v outside [0, 1] (and NaN, which nalgebra::clamp maps to the minimum)
    img = _image()
    scene = KatScene([(XZ, 0, [0.0, 1.0, 0.0, 1.0, 0.0])], [(N.RT_MAT_LAMBERTIAN, 0, (0, 0, 0), 0.0)],
                     [{"kind": N.RT_TEX_IMAGE, "table": 0}], images=[img])
    osc = O.OracleScene(scene.desc)
    out = (C.c_double * 3)()
    p = (C.c_double * 3)(0.0, 0.0, 0.0)
    for u in (-0.5, 0.0, 0.5, 1.0, 1.5, math.nan, -math.inf, math.inf):
        for v_ in (-2.0, 0.0, 0.7, 1.0, 3.0, math.nan):
            O.lib().or_texture_value(osc.h, 0, u, v_, p, out)
            assert list(out) == texel(img, u, v_), (u, v_)


def _perlin_scene(sc):
    t, vecs = perlin_table()
    tab = (vecs, list(t.perm_x), list(t.perm_y), list(t.perm_z))
    scene = KatScene([(XZ, 0, [-10.0, 10.0, -10.0, 10.0, 0.0])], [(N.RT_MAT_LAMBERTIAN, 0, (0, 0, 0), 0.0)],
                     [{"kind": N.RT_TEX_PERLIN, "table": 0, "scale": sc}], perlin=t)
    return scene, tab


def test_perlin_noise_lattice_and_interior_oracle():
    # perlin/mod.rs:87-109: at a lattice point every corner weight but (0,0,0)'s is 0 and (0,0,0)'s gradient
    # is dotted with (0, 0, 0): noise = 0; at (1/2, 1/2, 1/2) all eight corners weigh 1/8
    scene, tab = _perlin_scene(4.0)
    osc = O.OracleScene(scene.desc)
    for p in [(0, 0, 0), (3, -2, 7), (-1, -1, -1), (255, 256, 1000)]:
        assert O.lib().or_perlin_noise(osc.h, 0, (C.c_double * 3)(*map(float, p))) == 0.0
    vecs, px, py, pz = tab
    half = sum(0.125 * dot([float(x) for x in vecs[px[di] ^ py[dj] ^ pz[dk]]], [0.5 - di, 0.5 - dj, 0.5 - dk])
               for di in range(2) for dj in range(2) for dk in range(2))
    got = O.lib().or_perlin_noise(osc.h, 0, (C.c_double * 3)(0.5, 0.5, 0.5))
    assert abs(got - half) <= 1e-15 and got == perlin_noise(tab, [0.5, 0.5, 0.5])
    rng = np.random.default_rng(5)
    for p in rng.uniform(-40, 40, size=(64, 3)):
        p = [float(x) for x in p]
        assert O.lib().or_perlin_noise(osc.h, 0, (C.c_double * 3)(*p)) == perlin_noise(tab, p)
        assert O.lib().or_perlin_turbulence(osc.h, 0, (C.c_double * 3)(*p), 7) == turbulence(tab, p)


def test_marble_at_lattice_and_interior_points(probe):
    # perlin/mod.rs:162-183 through a Lambertian's albedo: at lattice points (x, 0, z integers) every octave
    # of the turbulence is at a lattice point too, so turbulence = 0 and the marble is 0.5 (1 + sin(s z));
    # at (k + 1/2, 0, m + 1/2) only octave 0 is off the lattice.  The sines are libm's (ocml on the
    # device, glibc here): within 2 ulp of 1.
    sc = 4.0
    scene, tab = _perlin_scene(sc)
    pts = [(0.0, 0.0), (3.0, -2.0), (-4.0, 5.0), (0.5, 0.5), (2.5, -1.5), (-3.5, 4.5), (1.25, 0.75)]
    rays = [[x, 1.0, z, 0.0, -1.0, 0.0] for x, z in pts]
    got = probe(scene, rays, 0)
    for (x, z), r in zip(pts, got):
        want = marble(tab, sc, [x, 0.0, z])
        if x == int(x) and z == int(z):
            assert turbulence(tab, [x, 0.0, z]) == 0.0
            assert want == 0.5 * (1.0 + math.sin(sc * z))
        if x == 0.0 and z == 0.0:
            assert v(r.attenuation) == [0.5, 0.5, 0.5]  # sin(0) = 0 exactly on both libms
        assert all(abs(a - want) <= 4.5e-16 for a in v(r.attenuation)), (x, z, v(r.attenuation), want)
