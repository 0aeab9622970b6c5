"""Generate the committed golden fixtures (SURVEY.md §8c "golden vectors to generate").

The reference (Rust) cannot be built or run here and draws from an unseedable thread_rng, so no
fixture can come from the reference itself.  These vectors freeze the oracle (oracle/oracle.c, pinned
by the reference's 25 unit tests and analytic KATs: tests/test_oracle_kat.py) and the C++ host (scene
generator, serde JSON, BVH builder) on fixed seeds, so that any later change to either is caught
(tests/test_golden.py) and the GPU path is checked against stored data as well as against a live
oracle (tests/test_gpu_parity.py::test_render_matches_golden).

    python tests/golden/make_golden.py        # rewrites tests/golden/*.npz, *.json.gz

Fixtures (seed 0x5EED everywhere):
  renders.npz   per-scene 32x32 @ 8 spp f64 accumulations (render_scanline sums, in-order)
  hits.npz      1024 fixed rays into random_scene: object, t, point, normal, u, v, front_face
  textures.npz  Perlin noise / turbulence, checker and image texture samples at fixed points
  bvh.npz       the reference-rule BBox tree of random_scene (bbox_tree.rs layout)
  scene_random.json.gz  SceneBuilder JSON of random_scene(0x5EED) (scenes.rs:281-429, seeded)
"""
import gzip
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402
import raytracer as rt  # noqa: E402

SEED = 0x5EED
SCENES = [("random", "std16x9"), ("random-night", "std16x9"), ("demo", "std16x9"), ("perlin", "std16x9"),
          ("earth", "square"), ("box-light", "std16x9"), ("cornell", "square"), ("final:4:30", "square")]
W, SPP = 32, 8


def scene(name):
    return rt.SceneBuilder.builtin(name, SEED).finalize(SEED)


def fixed_rays(n=1024):
    rng = np.random.default_rng(20241016)
    orig = np.column_stack([rng.uniform(-12, 12, n), rng.uniform(0.05, 3, n), rng.uniform(-12, 12, n)])
    return np.hstack([orig, rng.normal(size=(n, 3))])


def texture_points(n=256):
    rng = np.random.default_rng(7)
    return rng.uniform(-20, 20, size=(n, 3)), rng.uniform(-0.1, 1.1, size=(n, 2))


def make():
    renders = {}
    for name, aspect in SCENES:
        cam = rt.scene_camera(name.split(":")[0] if not name.startswith("final") else name, W, aspect)
        img, cnt = O.OracleScene(scene(name)).render(cam, O.params(SPP, 50, SEED))
        key = name.replace(":", "_").replace("-", "_")
        renders[key] = img
        renders[key + "__segments"] = np.array([cnt.segments], dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "renders.npz"), **renders)

    sc = scene("random")
    osc = O.OracleScene(sc)
    rays = fixed_rays()
    obj = np.full(len(rays), -1, np.int32)
    rec = np.zeros((len(rays), 9))  # t, point xyz, normal xyz, u, v
    ff = np.zeros(len(rays), np.int32)
    for i, r in enumerate(rays):
        h = osc.hit(r, 0.001, float("inf"))
        if h.hit:
            obj[i], ff[i] = h.object, h.front_face
            rec[i] = [h.t, *h.point, *h.normal, h.u, h.v]
    np.savez_compressed(os.path.join(HERE, "hits.npz"), rays=rays, object=obj, record=rec, front_face=ff)

    pts, uv = texture_points()
    d = sc.desc
    perlin_tex = [i for i in range(d.n_textures) if d.textures[i].kind == rt._native.RT_TEX_PERLIN]
    checker_tex = [i for i in range(d.n_textures) if d.textures[i].kind == rt._native.RT_TEX_CHECKER]
    noise = np.array([O.lib().or_perlin_noise(osc.h, 0, (O.C.c_double * 3)(*p)) for p in pts])
    turb = np.array([O.lib().or_perlin_turbulence(osc.h, 0, (O.C.c_double * 3)(*p), 7) for p in pts])

    def tex(s, osc_, t):
        out = np.zeros((len(pts), 3))
        for i, (p, q) in enumerate(zip(pts, uv)):
            o = (O.C.c_double * 3)()
            O.lib().or_texture_value(osc_.h, t, q[0], q[1], (O.C.c_double * 3)(*p), o)
            out[i] = o[:]
        return out
    marble = tex(sc, osc, perlin_tex[0])
    checker = tex(sc, osc, checker_tex[0])
    se = scene("earth")
    oe = O.OracleScene(se)
    img_tex = [i for i in range(se.desc.n_textures) if se.desc.textures[i].kind == rt._native.RT_TEX_IMAGE][0]
    earth = tex(se, oe, img_tex)
    np.savez_compressed(os.path.join(HERE, "textures.npz"), points=pts, uv=uv, noise=noise, turbulence=turb,
                        marble=marble, checker=checker, earth=earth)

    nodes, root = osc.tree()
    np.savez_compressed(os.path.join(HERE, "bvh.npz"), box=np.array([n[0] for n in nodes]),
                        links=np.array([n[1:] for n in nodes], dtype=np.int32), root=np.array([root]))

    js = rt.SceneBuilder.builtin("random", SEED).to_json(pretty=False)
    with gzip.open(os.path.join(HERE, "scene_random.json.gz"), "wt") as f:
        f.write(js)


if __name__ == "__main__":
    make()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
