"""Camera construction (reference: src/raytracer/camera/mod.rs, src/scenes.rs:191-231), computed by
the C++ host layer so Python, the CLI and the tests build bit-identical ``rt_camera`` values."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Tuple

from . import _native as N

ASPECT_RATIOS = {"std3x2": (3, 2), "std16x9": (16, 9), "std16x10": (16, 10), "square": (1, 1),
                 "target-iphone": (1170, 2532)}  # argparse.rs:160-170


@dataclass
class CameraPosition:
    """CameraPosition::look_at (camera/mod.rs:72-86); ``focus_length`` overrides the distance
    when set, like ``pos.focus_length = 10.0`` in scenes.rs:209,229."""
    look_from: Tuple[float, float, float]
    look_at: Tuple[float, float, float]
    up: Tuple[float, float, float] = (0.0, 1.0, 0.0)
    focus_length: Optional[float] = None

    @staticmethod
    def look_at_(camera, target, up) -> "CameraPosition":
        return CameraPosition(tuple(camera), tuple(target), tuple(up))


@dataclass
class CameraBuilder:
    """CameraBuilder (camera/mod.rs:13-61): width + aspect ratio, vfov, focal_length, aperture."""
    width: int = 640
    aspect_ratio: Tuple[int, int] = (3, 2)
    vfov: float = 1.0           # DEFAULT_FOCAL_LENGTH when unset (camera/mod.rs:46)
    focal_length: float = 1.0
    aperture: Optional[float] = None
    shutter: Tuple[float, float] = (0.0, 0.0)  # book-2 extension: (time0, time1)

    def build(self, pos: CameraPosition) -> N.rt_camera:
        s = N.sh_camera_spec()
        s.width = int(self.width)
        s.ratio_num, s.ratio_den = (int(self.aspect_ratio[0]), int(self.aspect_ratio[1]))
        s.vfov, s.focal_length = float(self.vfov), float(self.focal_length)
        s.has_aperture = 0 if self.aperture is None else 1
        s.aperture = 0.0 if self.aperture is None else float(self.aperture)
        s.look_from[:] = [float(x) for x in pos.look_from]
        s.look_at[:] = [float(x) for x in pos.look_at]
        s.up[:] = [float(x) for x in pos.up]
        s.override_focus = 0 if pos.focus_length is None else 1
        s.focus_length = 0.0 if pos.focus_length is None else float(pos.focus_length)
        s.time0, s.time1 = float(self.shutter[0]), float(self.shutter[1])
        cam = N.rt_camera()
        N.host_check(N.host_lib().sh_camera_build(C.byref(s), C.byref(cam)))
        return cam


def default_camera(width: int = 640, aspect_ratio: str = "std3x2", camera_fov: float = 20.0,
                   camera_focal_length: float = 1.0, camera_aperture: float = 0.001) -> N.rt_camera:
    """scenes.rs:214-231: look_at (13,2,3) -> origin, focus_length forced to 10."""
    cam = N.rt_camera()
    N.host_check(N.host_lib().sh_default_camera(width, aspect_ratio.encode(), camera_fov, camera_focal_length,
                                                camera_aperture, C.byref(cam)))
    return cam


def cornell_camera(width: int) -> N.rt_camera:
    """scenes.rs:191-212: vfov 40, 1:1, aperture 1e-5, (278,278,-800) -> (278,278,0), focus 10."""
    cam = N.rt_camera()
    N.host_check(N.host_lib().sh_cornell_camera(width, C.byref(cam)))
    return cam


def scene_camera(scene: str, width: int, aspect_ratio: str = "std3x2", camera_fov: float = 20.0,
                 camera_focal_length: float = 1.0, camera_aperture: float = 0.001) -> N.rt_camera:
    """The camera each scenes.rs entry point renders with (cornell forces its own)."""
    cam = N.rt_camera()
    N.host_check(N.host_lib().sh_scene_camera(scene.encode(), width, aspect_ratio.encode(), camera_fov,
                                              camera_focal_length, camera_aperture, C.byref(cam)))
    return cam
