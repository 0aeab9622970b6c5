"""Print rt_scene_stats for built-in scenes (tree sizes, whether the wide LDS block is used).
Usage: SHIRLEY_LIB_DIR=<build> python tools/scene_stats.py random final spheres ..."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "shirley-raytracing-rs_amd"))
import raytracer as rt  # noqa: E402

dev = rt.Device(0)
for name in sys.argv[1:] or ["random", "final", "cornell", "earth"]:
    scene = rt.SceneBuilder.builtin(name, 0x5EED).finalize(0x5EED)
    dev.upload(scene, "sah")
    s = dev.stats()
    print(name, {f: getattr(s, f) for f, _ in s._fields_})
