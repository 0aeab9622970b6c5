"""The committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py) against the
oracle and the C++ host: bit-exact.  They freeze the oracle's renders, hit records and texture values
and the host's scene generator, serde JSON and reference-rule BVH on seed 0x5EED.
Their provenance: the oracle, itself pinned by the reference's unit tests and analytic KATs
(test_oracle_kat.py) — the reference cannot run here, so no fixture comes from it."""
import gzip
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import raytracer as rt
from golden import make_golden as G

GOLD = os.path.dirname(G.__file__)


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.mark.parametrize("name,aspect", G.SCENES)
def test_oracle_renders_match_golden(name, aspect):
    gold = load("renders.npz")
    key = name.replace(":", "_").replace("-", "_")
    cam = rt.scene_camera(name, G.W, aspect)
    img, cnt = O.OracleScene(G.scene(name)).render(cam, O.params(G.SPP, 50, G.SEED))
    assert np.array_equal(img, gold[key])
    assert cnt.segments == int(gold[key + "__segments"][0])


def test_oracle_hits_match_golden():
    gold = load("hits.npz")
    osc = O.OracleScene(G.scene("random"))
    for i, r in enumerate(gold["rays"]):
        h = osc.hit(r, 0.001, float("inf"))
        assert (h.object if h.hit else -1) == gold["object"][i]
        if h.hit:
            assert [h.t, *h.point, *h.normal, h.u, h.v] == list(gold["record"][i])
            assert h.front_face == gold["front_face"][i]


def test_oracle_textures_match_golden():
    gold = load("textures.npz")
    osc = O.OracleScene(G.scene("random"))
    noise = [O.lib().or_perlin_noise(osc.h, 0, (O.C.c_double * 3)(*p)) for p in gold["points"]]
    turb = [O.lib().or_perlin_turbulence(osc.h, 0, (O.C.c_double * 3)(*p), 7) for p in gold["points"]]
    assert np.array_equal(noise, gold["noise"]) and np.array_equal(turb, gold["turbulence"])
    d = osc_desc = G.scene("random")
    perlin = [i for i in range(d.desc.n_textures) if d.desc.textures[i].kind == rt._native.RT_TEX_PERLIN][0]
    checker = [i for i in range(d.desc.n_textures) if d.desc.textures[i].kind == rt._native.RT_TEX_CHECKER][0]
    osc2 = O.OracleScene(osc_desc)
    se = G.scene("earth")
    image = [i for i in range(se.desc.n_textures) if se.desc.textures[i].kind == rt._native.RT_TEX_IMAGE][0]
    oe = O.OracleScene(se)
    for tex, sc, key in ((perlin, osc2, "marble"), (checker, osc2, "checker"), (image, oe, "earth")):
        for p, q, want in zip(gold["points"], gold["uv"], gold[key]):
            out = (O.C.c_double * 3)()
            O.lib().or_texture_value(sc.h, tex, q[0], q[1], (O.C.c_double * 3)(*p), out)
            assert list(out) == list(want)


def test_host_scene_and_bvh_match_golden():
    with gzip.open(os.path.join(GOLD, "scene_random.json.gz"), "rt") as f:
        gold_js = f.read()
    js = rt.SceneBuilder.builtin("random", G.SEED).to_json(pretty=False)
    assert json.loads(js) == json.loads(gold_js)
    gold = load("bvh.npz")
    from test_host_abi import product_tree
    import raytracer._native as N
    nodes, root = product_tree(G.scene("random").desc_ptr, N.RT_BVH_REFERENCE)
    assert root == int(gold["root"][0])
    assert np.array_equal(np.array([n[0] for n in nodes]), gold["box"])
    assert np.array_equal(np.array([n[1:] for n in nodes], dtype=np.int32), gold["links"])
