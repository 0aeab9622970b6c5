"""Python mirror of the reference's scene-construction API (reference: src/raytracer/scene/mod.rs,
material/texture/loader.rs, material/*.rs, geometry/*.rs, skybox/mod.rs).

Objects serialise to the reference's serde JSON and are handed to the C++
host layer (libshirley_host.so), whose ``finalize`` produces the ``rt_scene_desc`` that crosses the
render ABI.  Names follow the Rust API: ``SceneBuilder().add(Sphere(...), Lambertian(TextureLoader.solid(...)))``.
"""
from __future__ import annotations

import ctypes as C
import json
from dataclasses import dataclass, field
from typing import Optional

from . import _native as N


@dataclass(frozen=True)
class Vec3:
    x: float
    y: float
    z: float

    def to_json(self):
        return {"vec": [float(self.x), float(self.y), float(self.z)]}


def _v(v) -> Vec3:
    return v if isinstance(v, Vec3) else Vec3(*v)


# ---- textures (texture/loader.rs:17-28) -------------------------------------------------------
class TextureLoader:
    def __init__(self, js):
        self._js = js

    def to_json(self):
        return self._js

    @staticmethod
    def solid(r: float, g: float, b: float) -> "TextureLoader":
        return TextureLoader({"Solid": Vec3(r, g, b).to_json()})

    @staticmethod
    def solid_from_vec(v) -> "TextureLoader":
        return TextureLoader({"Solid": _v(v).to_json()})

    @staticmethod
    def checker(size: float, odd: "TextureLoader", even: "TextureLoader") -> "TextureLoader":
        return TextureLoader({"Checker": {"size": float(size), "odd": odd.to_json(), "even": even.to_json()}})

    @staticmethod
    def noise(scalar: float) -> "TextureLoader":
        return TextureLoader({"Perlin": float(scalar)})

    @staticmethod
    def image_path(path: str) -> "TextureLoader":
        return TextureLoader({"ImagePath": str(path)})


TextureLoader.EarthBuiltin = TextureLoader("EarthBuiltin")


# ---- materials (material/material_type.rs:20-27) ----------------------------------------------
class Metal:
    """Metal::new (metal.rs:17-23): fuzz None -> 0, clamped to <= 1."""

    def __init__(self, albedo, fuzz: Optional[float] = None):
        f = 0.0 if fuzz is None else float(fuzz)
        self.albedo, self.fuzz = _v(albedo), (1.0 if f > 1.0 else f)

    def to_json(self):
        return {"Metal": {"albedo": self.albedo.to_json(), "fuzz": self.fuzz}}


@dataclass
class Dielectric:
    ir: float

    def to_json(self):
        return {"Dielectric": {"ir": float(self.ir)}}


@dataclass
class Lambertian:
    albedo: TextureLoader

    def to_json(self):
        return {"Lambertian": {"albedo": self.albedo.to_json()}}


@dataclass
class DiffuseLight:
    albedo: TextureLoader

    def to_json(self):
        return {"DiffuseLight": {"albedo": self.albedo.to_json()}}


@dataclass
class FairyLight:
    albedo: TextureLoader

    def to_json(self):
        return {"FairyLight": {"albedo": self.albedo.to_json()}}


@dataclass
class Isotropic:
    """Book-2 extension (absent from the reference): a ConstantMedium's phase function."""
    albedo: TextureLoader

    def to_json(self):
        return {"Isotropic": {"albedo": self.albedo.to_json()}}


# ---- geometry (geometry/object.rs:9-16) -------------------------------------------------------
@dataclass
class Sphere:
    center: Vec3
    radius: float

    def to_json(self):
        return {"Sphere": {"center": _v(self.center).to_json(), "radius": float(self.radius)}}


def _rect(d1_min, d1_max, d2_min, d2_max, offset):
    return {"d1_min": float(d1_min), "d1_max": float(d1_max), "d2_min": float(d2_min),
            "d2_max": float(d2_max), "offset": float(offset)}


@dataclass
class _Rect:
    tag: str
    d1_min: float
    d1_max: float
    d2_min: float
    d2_max: float
    offset: float

    def to_json(self):
        return {self.tag: _rect(self.d1_min, self.d1_max, self.d2_min, self.d2_max, self.offset)}


def xy_rect(d1_min, d1_max, d2_min, d2_max, offset):  # rect.rs:15-23
    return _Rect("RectXY", d1_min, d1_max, d2_min, d2_max, offset)


def yz_rect(d1_min, d1_max, d2_min, d2_max, offset):  # rect.rs:25-33
    return _Rect("RectYZ", d1_min, d1_max, d2_min, d2_max, offset)


def xz_rect(d1_min, d1_max, d2_min, d2_max, offset):  # rect.rs:35-43
    return _Rect("RectXZ", d1_min, d1_max, d2_min, d2_max, offset)


@dataclass
class RectBox:
    """RectBox::new(p0, p1) (rect.rs:111-129)."""
    min: Vec3
    max: Vec3

    def to_json(self):
        p0, p1 = _v(self.min), _v(self.max)
        return {"RectBox": {
            "min": p0.to_json(), "max": p1.to_json(),
            "xy_sides": [_rect(p0.x, p1.x, p0.y, p1.y, p1.z), _rect(p0.x, p1.x, p0.y, p1.y, p0.z)],
            "yz_sides": [_rect(p0.y, p1.y, p0.z, p1.z, p1.x), _rect(p0.y, p1.y, p0.z, p1.z, p0.x)],
            "xz_sides": [_rect(p0.x, p1.x, p0.z, p1.z, p1.y), _rect(p0.x, p1.x, p0.z, p1.z, p0.y)]}}


# ---- book-2 extensions (absent from the reference) ----------------------------
@dataclass
class MovingSphere:
    """moving_sphere.h: centre center0 at time0 moving linearly to center1 at time1."""
    center0: Vec3
    center1: Vec3
    time0: float
    time1: float
    radius: float

    def to_json(self):
        return {"MovingSphere": {"center0": _v(self.center0).to_json(), "center1": _v(self.center1).to_json(),
                                 "time0": float(self.time0), "time1": float(self.time1),
                                 "radius": float(self.radius)}}


@dataclass
class ConstantMedium:
    """constant_medium.h: the object's geometry is the boundary of a medium of this density (its
    material must be Isotropic)."""
    density: float

    def to_json(self):
        return {"density": float(self.density)}


@dataclass
class Transform:
    """translate(rotate_y(object, rotate_y), offset)."""
    rotate_y: float = 0.0
    offset: Vec3 = (0.0, 0.0, 0.0)

    def to_json(self):
        return {"rotate_y": float(self.rotate_y), "offset": _v(self.offset).to_json()}


# ---- skybox (skybox/mod.rs:11-16) ------------------------------------------------------------
class SkyBox:
    Above = ("Above", None)
    Nothing = ("None", None)

    @staticmethod
    def Flat(color) -> tuple:
        return ("Flat", _v(color))


# ---- SceneBuilder (scene/mod.rs:79-110) + finalize -------------------------------------------
class Scene:
    """Finalized scene (scene/mod.rs:140-144): owns the arrays behind ``desc`` (an rt_scene_desc)."""

    def __init__(self, handle):
        self._h = handle
        self.desc = N.host_lib().sh_desc_view(handle).contents
        self.desc._owner = self  # the view must keep the arrays it points into alive

    @property
    def desc_ptr(self):
        return C.pointer(self.desc)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            N.host_lib().sh_desc_free(h)


class SceneBuilder:
    def __init__(self, _handle=None):
        lib = N.host_lib()
        self._h = _handle if _handle is not None else lib.sh_scene_new()

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            N.host_lib().sh_scene_free(h)

    def set_skybox(self, sky) -> "SceneBuilder":
        tag, color = sky
        kind = {"Above": N.RT_SKY_ABOVE, "Flat": N.RT_SKY_FLAT, "None": N.RT_SKY_NONE}[tag]
        col = (C.c_double * 3)(*(color.x, color.y, color.z)) if color is not None else None
        N.host_check(N.host_lib().sh_scene_set_skybox(self._h, kind, col))
        return self

    def add(self, geometry, material, medium: Optional[ConstantMedium] = None,
            transform: Optional[Transform] = None) -> None:
        js = {"geometry": geometry.to_json(), "material": material.to_json()}
        if medium is not None:
            js["medium"] = medium.to_json()
        if transform is not None:
            js["transform"] = transform.to_json()
        obj = json.dumps(js)
        N.host_check(N.host_lib().sh_scene_add_json(self._h, obj.encode()))

    def __len__(self):
        return N.host_lib().sh_scene_len(self._h)

    def to_json(self, pretty: bool = True) -> str:
        lib = N.host_lib()
        need = C.c_size_t(0)
        N.host_check(lib.sh_scene_to_json(self._h, int(pretty), None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        N.host_check(lib.sh_scene_to_json(self._h, int(pretty), buf, need.value, C.byref(need)))
        return buf.value.decode()

    @staticmethod
    def from_json(text: str) -> "SceneBuilder":
        h = C.c_void_p()
        N.host_check(N.host_lib().sh_scene_from_json(text.encode(), C.byref(h)))
        return SceneBuilder(h.value)

    @staticmethod
    def builtin(name: str, seed: int = 0x5EED) -> "SceneBuilder":
        h = C.c_void_p()
        N.host_check(N.host_lib().sh_scene_builtin(name.encode(), C.c_uint64(seed), C.byref(h)))
        return SceneBuilder(h.value)

    def finalize(self, seed: int = 0x5EED) -> Scene:
        h = C.c_void_p()
        N.host_check(N.host_lib().sh_scene_finalize(self._h, C.c_uint64(seed), C.byref(h)))
        return Scene(h.value)
