"""raytracer — MI355X-native drop-in for the render hot path of scottschroeder/shirley-raytracing-rs.

Python face of the C++ host layer (libshirley_host.so: scenes, serde JSON, camera) and of the render
C ABI (libshirley_rt.so: HIP kernels for gfx950).  Module names mirror the reference crate
``raytracer`` (src/raytracer/lib.rs).
"""
from ._native import LIB_DIR, BIN_DIR, RtError, rt_lib, host_lib  # noqa: F401
from .scene import (SceneBuilder, Scene, TextureLoader, Metal, Dielectric, Lambertian, DiffuseLight,  # noqa: F401
                    FairyLight, Sphere, RectBox, xy_rect, yz_rect, xz_rect, SkyBox, Vec3,
                    Isotropic, MovingSphere, ConstantMedium, Transform)
from .camera import CameraBuilder, CameraPosition, default_camera, cornell_camera, scene_camera  # noqa: F401
from .render import (Device, RenderSettings, Comm, render_scene, render_multi, comm_unique_id, scene_digest, to_image,  # noqa: F401
                     write_png, tile_layout)
from . import scenes  # noqa: F401
