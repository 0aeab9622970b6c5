"""The exact-tie rule the device implements (rt_device.h resolve_ties), pinned against the oracle's walk
of the reference tree (bbox_tree.rs:56-91, rhs popped before lhs; every node's box, leaves included,
tested with hit2's strict `t_max <= t_min` at the running closest t, aabb.rs:62-79).

Rule: among the primitives hit at exactly t* (the closest t) whose box can pass hit2 at all, the winner is
the lowest-ranked one (rank = in-order position of its leaf, lhs first) whose box passes hit2 at t*; if
none passes, the highest-ranked one (the first one the reference reaches, tested while the running t was
still above t*).  Checked here on CPU, ray by ray, on the random scene with every object duplicated, where
every hit is a tie; test_gpu_ties.py checks the device against the oracle on the same scene."""
import ctypes as C
import json

import numpy as np

import oracle_lib as O
import raytracer as rt

SEED = 0x5EED


def _duplicated_random_scene():
    src = json.loads(rt.scenes.random_scene(SEED).to_json())
    red = {"Lambertian": {"albedo": {"Solid": {"vec": [0.9, 0.1, 0.05]}}}}
    objs = []
    for o in src["objects"]:
        objs.append(o)
        objs.append({**o, "material": red})
    src["objects"] = objs
    return rt.SceneBuilder.from_json(json.dumps(src)).finalize(SEED)


def _ranks(osc, n):
    nodes, root = osc.tree()
    rank, st, k = [-1] * n, [root], 0
    while st:
        x = st.pop()
        _, leaf, lhs, rhs = nodes[x]
        if leaf >= 0:
            rank[leaf] = k
            k += 1
            continue
        st.append(rhs)
        st.append(lhs)
    assert sorted(rank) == list(range(n))
    return rank


def test_tie_rule_matches_the_reference_walk():
    scene = _duplicated_random_scene()
    L, osc, n = O.lib(), O.OracleScene(scene), scene.desc.n_objects
    rank = _ranks(osc, n)
    boxes = []
    for i in range(n):
        bb = O._d6()
        L.or_object_bbox(C.byref(scene.desc.objects[i]), bb)
        boxes.append(bb)
    rng = np.random.default_rng(3)
    rays = np.hstack([np.array([13.0, 2.0, 3.0]) + rng.normal(scale=0.2, size=(48, 3)),
                      rng.uniform([-13.0, -2.5, -3.5], [-9.0, -1.5, 1.5], size=(48, 3))])
    n_ties = 0
    for r in rays:
        h = osc.hit(r)
        if not h.hit:
            continue
        ray, cands = O.d6(r), []
        for i in range(n):
            hi = O.or_hit()
            if (L.or_object_hit(C.byref(scene.desc.objects[i]), ray, 0.001, h.t, C.byref(hi)) and hi.t == h.t
                    and L.or_aabb_hit2(boxes[i], ray, 0.001, float("inf"))):
                cands.append((rank[i], i, bool(L.or_aabb_hit2(boxes[i], ray, 0.001, h.t))))
        passing = [c for c in cands if c[2]]
        win = min(passing)[1] if passing else max(cands)[1]
        assert win == h.object, (r.tolist(), cands, h.object)
        n_ties += len(cands) > 1
    assert n_ties > 30  # every hit is a tie
