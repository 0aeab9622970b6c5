"""Sphere-leaf outcome statistics of a scene (tools/sphere_stats.c; study tool, CPU only).

    python tools/sphere_stats.py [--scene random] [--width 1200] [--rows 40] [--spp 4]

Renders a centre band of the frame with the oracle built with its statistics hook and prints, per sphere
test: the miss (negative discriminant), no-root-in-range and hit fractions, and the fraction an f32
discriminant could reject.  Used in DESIGN.md §5 to price an f32 sphere pre-reject: in the megakernel a
sphere trip runs ~8 of 64 lanes, so the f64 test is skipped only when every active lane rejects."""
import argparse
import ctypes as C
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "shirley-raytracing-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="random")
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--aspect", default="std3x2")
    ap.add_argument("--rows", type=int, default=40)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    args = ap.parse_args()
    so = os.path.join(REPO, "tools", "libsphere_stats.so")
    subprocess.run(["gcc", "-O2", "-std=c11", "-fPIC", "-ffp-contract=off", "-shared", "-o", so,
                    os.path.join(REPO, "tools", "sphere_stats.c"), "-lm", "-lpthread"], check=True)
    import oracle_lib as O
    O.ORACLE_SO = so
    O._lib = None
    import raytracer as rt
    scene = rt.SceneBuilder.builtin(args.scene, args.seed).finalize(args.seed)
    cam = rt.scene_camera(args.scene, args.width, args.aspect)
    H = cam.image_height
    r0 = (H - args.rows) // 2
    lib = O.lib()
    lib.ss_get.argtypes = [C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 4)()
    O.OracleScene(scene).render(cam, O.params(args.spp, 50, args.seed), r0, r0 + args.rows)
    lib.ss_get(out)
    miss, norange, hit, f32rej = out[:]
    n = miss + norange + hit
    p = miss / n
    print(f"{args.scene} {cam.image_width}x{H} rows [{r0}, {r0 + args.rows}) @ {args.spp} spp: {n} sphere tests")
    print(f"  miss (disc < 0) {miss / n:.4f}  no root in range {norange / n:.4f}  hit {hit / n:.4f}")
    print(f"  f32-rejectable misses {f32rej / max(miss, 1):.5f} of the misses")
    for lanes in (1, 4, 8, 16):
        print(f"  all of {lanes:2d} independent lanes reject (skip the f64 test): {p ** lanes:.4f}")


if __name__ == "__main__":
    main()
