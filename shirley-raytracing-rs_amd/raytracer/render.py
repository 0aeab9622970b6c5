"""Render path: the MI355X replacement of render_scene's scanline loop (reference: src/main.rs:65-130,
src/raytracer/render.rs:17-70), driven through the C ABI of include/shirley_rt.h.

There is no CPU fallback: without a GPU, ``Device()`` raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _native as N
from .scene import Scene


def _check(ctx, code):
    if code != 0:
        raise N.RtError(code, N.rt_lib().rt_last_error(ctx).decode())


@dataclass
class RenderSettings:
    """RenderSettings (argparse.rs:106-123) + the seed/tiling the reference lacks."""
    samples: int = 100
    max_reflect: int = 50
    seed: int = 0x5EED
    sample_chunk: int = 0
    tile_rank: int = 0
    tile_world: int = 1
    engine: str = "auto"   # auto | megakernel | wavefront | split
    timing: bool = False   # per-launch HIP-event timing of the wavefront kernels (rt_counters *_ms)
    # ABI 6: samples [sample_begin, sample_begin + sample_count) of the frame (0 = to `samples`)
    sample_begin: int = 0
    sample_count: int = 0
    partition: str = "auto"  # multi-GPU: auto | tiles | samples
    scratch_mb: int = 0      # partial-sum scratch bound per call in MiB (0 = the library default)

    ENGINES = {"auto": N.RT_ENGINE_AUTO, "megakernel": N.RT_ENGINE_MEGAKERNEL, "wavefront": N.RT_ENGINE_WAVEFRONT,
               "split": N.RT_ENGINE_SPLIT}
    PARTITIONS = {"auto": N.RT_PARTITION_AUTO, "tiles": N.RT_PARTITION_TILES, "samples": N.RT_PARTITION_SAMPLES}

    def params(self) -> N.rt_render_params:
        p = N.rt_render_params()
        p.samples, p.max_depth, p.seed = int(self.samples), int(self.max_reflect), int(self.seed)
        p.tile_rank, p.tile_world, p.sample_chunk = int(self.tile_rank), int(self.tile_world), int(self.sample_chunk)
        p.engine = self.ENGINES[self.engine] | (N.RT_ENGINE_TIMING if self.timing else 0)
        p.sample_begin, p.sample_count = int(self.sample_begin), int(self.sample_count)
        p.partition, p.scratch_mb = self.PARTITIONS[self.partition], int(self.scratch_mb)
        return p


class Device:
    """One rt_ctx (one MI355X)."""

    def __init__(self, device: int = 0):
        lib = N.rt_lib()
        h = C.c_void_p()
        code = lib.rt_create(int(device), C.byref(h))
        if code != 0:
            raise N.RtError(code, f"rt_create(device={device}) failed: no usable HIP device")
        self._h = h
        self.scene: Optional[Scene] = None

    def close(self):
        if getattr(self, "_h", None):
            N.rt_lib().rt_destroy(self._h)
            self._h = None

    __del__ = close

    @property
    def handle(self):
        return self._h

    def upload(self, scene: Scene, bvh: str = "reference", nodes: str = "auto") -> "Device":
        """rt_scene_upload; `nodes` = auto | global | half-lds | lds (BVH node placement, tests/tuning)."""
        builder = {"reference": N.RT_BVH_REFERENCE, "sah": N.RT_BVH_SAH}[bvh]
        builder |= {"auto": 0, "global": N.RT_BVH_NODES_GLOBAL, "half-lds": N.RT_BVH_NODES_HALF_LDS,
                    "lds": N.RT_BVH_NODES_LDS}[nodes]
        _check(self._h, N.rt_lib().rt_scene_upload(self._h, scene.desc_ptr, builder))
        self.scene = scene
        return self

    def digest(self) -> int:
        """rt_scene_digest: 64-bit digest of the uploaded scene (the multi-GPU calls compare them)."""
        d = C.c_uint64()
        _check(self._h, N.rt_lib().rt_scene_digest(self._h, C.byref(d)))
        return d.value

    def stats(self) -> N.rt_scene_stats:
        s = N.rt_scene_stats()
        _check(self._h, N.rt_lib().rt_scene_stats_get(self._h, C.byref(s)))
        return s

    def render(self, camera: N.rt_camera, settings: RenderSettings) -> np.ndarray:
        """Whole frame -> [H][W][3] f64 per-pixel sums, row 0 = bottom (Image.data layout)."""
        out = np.zeros((camera.image_height, camera.image_width, 3), dtype=np.float64)
        p = settings.params()
        _check(self._h, N.rt_lib().rt_render(self._h, C.byref(camera), C.byref(p), out.ctypes.data))
        return out

    def render_scanlines(self, camera: N.rt_camera, settings: RenderSettings, line_begin: int,
                         line_end: int) -> np.ndarray:
        out = np.zeros((max(0, line_end - line_begin), camera.image_width, 3), dtype=np.float64)
        p = settings.params()
        _check(self._h, N.rt_lib().rt_render_scanlines(self._h, C.byref(camera), C.byref(p), line_begin, line_end,
                                                       out.ctypes.data))
        return out

    def render_device(self, camera, settings: RenderSettings, accum_ptr: int, stream: int = 0):
        p = settings.params()
        _check(self._h, N.rt_lib().rt_render_device(self._h, C.byref(camera), C.byref(p), C.c_void_p(accum_ptr),
                                                    C.c_void_p(stream or None)))

    def render_tiles_device(self, camera, settings: RenderSettings, packed_ptr: int, stream: int = 0):
        p = settings.params()
        _check(self._h, N.rt_lib().rt_render_tiles_device(self._h, C.byref(camera), C.byref(p),
                                                          C.c_void_p(packed_ptr), C.c_void_p(stream or None)))

    def unpack_tiles_device(self, camera, world: int, gathered_ptr: int, accum_ptr: int, stream: int = 0):
        _check(self._h, N.rt_lib().rt_unpack_tiles_device(self._h, C.byref(camera), int(world),
                                                          C.c_void_p(gathered_ptr), C.c_void_p(accum_ptr),
                                                          C.c_void_p(stream or None)))

    def tonemap_device(self, accum_ptr: int, width: int, height: int, samples: int, rgb8_ptr: int,
                       stream: int = 0):
        """rt_tonemap_device: device [H][W][3] f64 sums -> device RGB8, row 0 = top (to_image)."""
        _check(self._h, N.rt_lib().rt_tonemap_device(self._h, C.c_void_p(accum_ptr), int(width), int(height),
                                                     int(samples), C.c_void_p(rgb8_ptr), C.c_void_p(stream or None)))

    def hit(self, rays: np.ndarray, t_min: float = 0.001, t_max: float = float("inf"), traversal: str = "binary"):
        """Closest hits for rays [n][6] (Hittable for Scene, scene/mod.rs:180-190) -> rt_hit array.
        traversal: "binary" (the 2-wide f64 tree, rt_scene_hit) or "render" (the 4-wide f32-inflated
        traversal the trace kernel runs, rt_scene_hit_ex(RT_TRAVERSAL_RENDER))."""
        r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        out = (N.rt_hit * max(1, len(r)))()
        if traversal == "binary":
            code = N.rt_lib().rt_scene_hit(self._h, r.ctypes.data, len(r), float(t_min), float(t_max), out)
        else:
            tv = {"render": N.RT_TRAVERSAL_RENDER}[traversal]
            code = N.rt_lib().rt_scene_hit_ex(self._h, r.ctypes.data, len(r), float(t_min), float(t_max), tv, out)
        _check(self._h, code)
        return out[:len(r)]

    def probe(self, rays: np.ndarray, seed: int, sample: int = 0, draw: int = 0):
        """One iteration of ray_color's loop (render.rs:30-46) per ray through the megakernel's device code
        (rt_probe_segment): ray i on the path key (seed, pixel = i, sample, draw) -> rt_probe array
        (closest object, emitted / scatter of its material or the sky, the draw counter after it)."""
        r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        out = (N.rt_probe * max(1, len(r)))()
        _check(self._h, N.rt_lib().rt_probe_segment(self._h, r.ctypes.data, len(r), int(seed), int(sample),
                                                     int(draw), out))
        return out[:len(r)]

    def synchronize(self):
        _check(self._h, N.rt_lib().rt_synchronize(self._h))

    # ---- multi-GPU (rt_comm_*, rt_render_sharded) ----
    def comm_init_rank(self, unique_id: bytes, world: int, rank: int) -> "Comm":
        """This device as rank `rank` of a `world`-rank RCCL communicator (one process per GPU)."""
        if len(unique_id) != N.RT_COMM_ID_BYTES:
            raise ValueError("unique id must be RT_COMM_ID_BYTES bytes (rt_comm_unique_id)")
        buf = (C.c_uint8 * N.RT_COMM_ID_BYTES).from_buffer_copy(unique_id)
        h = C.c_void_p()
        _check(self._h, N.rt_lib().rt_comm_init_rank(self._h, buf, int(world), int(rank), C.byref(h)))
        return Comm(h, world, rank)

    def render_sharded(self, comm: "Comm", camera, settings: RenderSettings, accum_ptr: int = 0, stream: int = 0):
        """This rank's share of the frame + the RCCL gather; rank 0 receives the [H][W][3] sums at accum_ptr."""
        p = settings.params()
        _check(self._h, N.rt_lib().rt_render_sharded(self._h, comm.handle, C.byref(camera), C.byref(p),
                                                     C.c_void_p(accum_ptr or None), C.c_void_p(stream or None)))

    def counters(self) -> N.rt_counters:
        c = N.rt_counters()
        _check(self._h, N.rt_lib().rt_counters_get(self._h, C.byref(c)))
        return c


class Comm:
    """An rt_comm (one rank of an RCCL communicator)."""

    def __init__(self, handle, world: int, rank: int):
        self.handle, self.world, self.rank = handle, world, rank

    def close(self):
        if getattr(self, "handle", None):
            N.rt_lib().rt_comm_destroy(self.handle)
            self.handle = None

    __del__ = close


def comm_unique_id() -> bytes:
    """rt_comm_unique_id: the RCCL id rank 0 creates and hands to every rank."""
    buf = (C.c_uint8 * N.RT_COMM_ID_BYTES)()
    code = N.rt_lib().rt_comm_unique_id(buf)
    if code:
        raise N.RtError(code, "rt_comm_unique_id failed (RCCL unavailable or no device)")
    return bytes(buf)


def render_multi(devices, camera: N.rt_camera, settings: RenderSettings) -> np.ndarray:
    """rt_render_multi: the whole frame on several devices of this process (RCCL gather to devices[0])."""
    out = np.zeros((camera.image_height, camera.image_width, 3), dtype=np.float64)
    arr = (C.c_void_p * len(devices))(*[d.handle for d in devices])
    p = settings.params()
    _check(devices[0].handle, N.rt_lib().rt_render_multi(arr, len(devices), C.byref(camera), C.byref(p),
                                                         out.ctypes.data))
    return out


def scene_digest(scene: Scene, bvh: str = "reference") -> int:
    """rt_scene_digest_host: the digest rt_scene_upload would record for this scene (no device needed)."""
    builder = {"reference": N.RT_BVH_REFERENCE, "sah": N.RT_BVH_SAH}[bvh]
    d = C.c_uint64()
    code = N.rt_lib().rt_scene_digest_host(scene.desc_ptr, builder, C.byref(d))
    if code:
        raise N.RtError(code, "rt_scene_digest_host: invalid scene")
    return d.value


def tile_layout(camera: N.rt_camera, world: int):
    n, m = C.c_int32(), C.c_int32()
    code = N.rt_lib().rt_tile_layout(C.byref(camera), int(world), C.byref(n), C.byref(m))
    if code:
        raise N.RtError(code, "rt_tile_layout failed")
    return n.value, m.value


def to_image(accum: np.ndarray, samples: int) -> np.ndarray:
    """image::to_image (image.rs:31-44): [H][W][3] sums -> RGB8 with row 0 = top."""
    h, w, _ = accum.shape
    a = np.ascontiguousarray(accum, dtype=np.float64)
    out = np.zeros((h, w, 3), dtype=np.uint8)
    code = N.rt_lib().rt_tonemap(a.ctypes.data, w, h, int(samples), out.ctypes.data)
    if code:
        raise N.RtError(code, "rt_tonemap failed")
    return out


def write_png(path: str, rgb8: np.ndarray):
    a = np.ascontiguousarray(rgb8, dtype=np.uint8)
    N.host_check(N.host_lib().sh_write_png(path.encode(), a.ctypes.data, a.shape[1], a.shape[0]))


def render_scene(settings: RenderSettings, scene: Scene, camera: N.rt_camera, output: Optional[str] = None,
                 device: Optional[Device] = None, bvh: str = "reference") -> np.ndarray:
    """render_scene (main.rs:65-130): samples 0 -> 1, render, to_image + PNG when ``output`` is set."""
    if settings.samples == 0:
        settings = RenderSettings(**{**settings.__dict__, "samples": 1})
    dev = device or Device(0)
    dev.upload(scene, bvh)
    accum = dev.render(camera, settings)
    if output:
        write_png(output, to_image(accum, settings.samples))
    return accum
