"""Multi-GPU frame sharding: interleaved 8x8 tiles per rank + one gather.

tile k of the frame (row-major over the tile grid) belongs to rank k % world; a rank's packed buffer
holds its tiles in order, [max_tiles][64][3] f64, lane l of a tile = pixel (8*tx + l%8, 8*ty + l//8).
The device kernels (rt_render_tiles_device / rt_unpack_tiles_device) and the numpy mirror below use
the same mapping.
"""
from __future__ import annotations

import numpy as np

TILE = 8


def tile_grid(width: int, height: int):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def max_tiles_per_rank(width: int, height: int, world: int) -> int:
    tx, ty = tile_grid(width, height)
    return (tx * ty + world - 1) // world


def rank_slots(width: int, height: int, rank: int, world: int):
    """(py, px, valid) for every packed slot of `rank` ([max_tiles*64] each)."""
    tx, ty = tile_grid(width, height)
    m = max_tiles_per_rank(width, height, world)
    lt = np.repeat(np.arange(m), TILE * TILE)
    lp = np.tile(np.arange(TILE * TILE), m)
    gt = lt * world + rank
    px = (gt % tx) * TILE + lp % TILE
    py = (gt // tx) * TILE + lp // TILE
    valid = (gt < tx * ty) & (px < width) & (py < height)
    return py, px, valid


def unpack_host(gathered: np.ndarray, width: int, height: int, world: int) -> np.ndarray:
    """numpy mirror of unpack_kernel: [world][max_tiles][64][3] -> [H][W][3]."""
    out = np.zeros((height, width, 3), dtype=np.float64)
    g = gathered.reshape(world, -1, 3)
    for r in range(world):
        py, px, valid = rank_slots(width, height, r, world)
        out[py[valid], px[valid]] = g[r][valid]
    return out


def gather_tiles(packed, world: int):
    """All ranks' packed tile buffers -> [world, ...] on every rank (RCCL all_gather over xGMI for
    CUDA tensors; gloo for CPU tensors in the tests)."""
    import torch
    import torch.distributed as dist
    if packed.is_cuda and dist.get_backend() == "nccl":
        out = torch.empty((world,) + tuple(packed.shape), dtype=packed.dtype, device=packed.device)
        dist.all_gather_into_tensor(out, packed.contiguous())
        return out
    # gloo (CPU tests, single-GPU rehearsals): gather host copies, hand back a tensor on the
    # input's device
    host = packed.detach().to("cpu").contiguous()
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host)
    return torch.stack(parts).to(packed.device)


# ---- sample partition (RT_PARTITION_SAMPLES): the same exchange as rt_render_sharded's -------------
def sample_share(begin: int, end: int, rank: int, world: int):
    """Rank `rank`'s part [b, e) of the frame's sample range [begin, end) (rt_api.cpp shard_render)."""
    n = end - begin
    return begin + n * rank // world, begin + n * (rank + 1) // world


def band_rows(height: int, world: int) -> int:
    """Rows of one band: rank b owns image rows [b * band_rows, (b + 1) * band_rows)."""
    return (height + world - 1) // world


def reduce_sample_bands(local, world: int):
    """A rank's whole-frame sums over its samples, [H][W][3] (torch) -> on rank 0 the frame summed over
    the ranks in rank order (None elsewhere): all-to-all of row bands, the rank-order sum of each band on
    its owner (sum_parts_kernel), gather of the bands to rank 0 — what rt_render_sharded does with RCCL."""
    import torch
    import torch.distributed as dist
    h, w, _ = local.shape
    rows = band_rows(h, world)
    padded = torch.zeros((world * rows, w, 3), dtype=local.dtype, device=local.device)
    padded[:h] = local
    parts = torch.empty_like(padded)
    dist.all_to_all_single(parts.view(-1), padded.view(-1))  # parts[r] = rank r's rows of my band
    parts = parts.view(world, rows, w, 3)
    band = parts[0].clone()
    for r in range(1, world):
        band += parts[r]
    bands = [torch.empty_like(band) for _ in range(world)]
    dist.all_gather(bands, band)
    if dist.get_rank() != 0:
        return None
    return torch.cat(bands)[:h]
