"""Diagnostic: the exact-tie marks (rt_device.h mark_tie / resolve_ties) on a reference-primitive scene full
of coplanar box faces — book 2's final_scene ground (20 x 20 RectBoxes of width 100, random heights,
sharing their side planes), a light and a few book-1 spheres, no book-2 objects, so the reference-scene
kernel instances (the ones that mark) run it.  Renders the frame a few times and prints Msamples/s; run
it against exp/<variant> libraries (SHIRLEY_LIB_DIR) to compare, and against an -DRT_PHASE_TIMING build
to count resolves ([phase-ev] tie_resolve).

usage: python tools/tie_marks.py [width] [spp] [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "shirley-raytracing-rs_amd"))
import raytracer as rt  # noqa: E402
from raytracer import scene as S  # noqa: E402


def box_ground_scene(seed=7):
    rng = np.random.default_rng(seed)
    sb = rt.SceneBuilder()
    sb.set_skybox(S.SkyBox.Flat((0.0, 0.0, 0.0)))
    ground = S.Lambertian(S.TextureLoader.solid(0.48, 0.83, 0.53))
    for i in range(20):
        for j in range(20):
            x0, z0 = -1000.0 + i * 100.0, -1000.0 + j * 100.0
            sb.add(S.RectBox((x0, 0.0, z0), (x0 + 100.0, float(rng.uniform(1, 101)), z0 + 100.0)), ground)
    sb.add(S.xz_rect(123.0, 423.0, 147.0, 412.0, 554.0), S.DiffuseLight(S.TextureLoader.solid(7.0, 7.0, 7.0)))
    sb.add(S.Sphere((260.0, 150.0, 45.0), 50.0), S.Dielectric(1.5))
    sb.add(S.Sphere((0.0, 150.0, 145.0), 50.0), S.Metal((0.8, 0.8, 0.9), 1.0))
    sb.add(S.Sphere((400.0, 200.0, 400.0), 100.0), S.Lambertian(S.TextureLoader.noise(0.1)))
    for _ in range(200):
        c = (float(rng.uniform(-100, 265)), float(rng.uniform(270, 435)), float(rng.uniform(295, 460)))
        sb.add(S.Sphere(c, 10.0), S.Lambertian(S.TextureLoader.solid(0.73, 0.73, 0.73)))
    return sb


def main():
    width = int(sys.argv[1]) if len(sys.argv) > 1 else 800
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    scene = box_ground_scene().finalize(7)
    dev = rt.Device(0)
    dev.upload(scene, "sah")
    cam = rt.CameraBuilder(width=width, aspect_ratio=(1, 1), vfov=40.0).build(
        rt.CameraPosition((478.0, 278.0, -600.0), (278.0, 278.0, 0.0)))
    st = rt.RenderSettings(samples=spp, max_reflect=50, seed=0x5EED)
    dev.render(cam, rt.RenderSettings(samples=4, max_reflect=50, seed=0x5EED))  # warm-up
    for _ in range(reps):
        t0 = time.perf_counter()
        dev.render(cam, st)
        dt = time.perf_counter() - t0
        c = dev.counters()  # (an -DRT_PHASE_TIMING build prints its event counts here)
        print(f"box_ground {width}x{width} @ {spp} spp: {width * width * spp / dt / 1e6:.1f} Msamples/s, "
              f"{c.segments} segments", flush=True)


if __name__ == "__main__":
    main()
