"""Load balance of the interleaved 8x8-tile sharding measured on ONE GPU: for each
world size, every rank's share of the headline frame is rendered exactly as that rank would render it
on its own MI355X (rt_render_tiles_device, same auto sample chunk), and its trace-kernel time taken
from the HIP events.  The slowest rank bounds a sharded frame, so
    predicted strong-scaling efficiency(N) = T(1) / (N * max_r T_r(N))
(the gather, 23 MB over xGMI, is not included; it is ~0.1 % of a frame).

usage: python tools/shard_balance.py [out.json] [--spp 500] [--reps 2] [--worlds 1,2,4,8] [--chunk 0]
(--chunk: a fixed sample_chunk instead of the auto choice, to compare unit lengths per world size)
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "shirley-raytracing-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?", default=os.path.join(REPO, "gpurun_out", "shard_balance.json"))
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--chunk", type=int, default=0)
    a = ap.parse_args()
    import torch
    import raytracer as rt
    seed = 0x5EED
    scene = rt.scenes.random_scene(seed).finalize(seed)
    cam = rt.default_camera(1200, "std3x2")
    dev = rt.Device(0)
    dev.upload(scene, "sah")
    res = {"workload": f"random 1200x800 @ {a.spp}spp, SAH, one MI355X", "chunk": a.chunk or "auto", "worlds": {}}
    t1 = None
    for world in [int(w) for w in a.worlds.split(",")]:
        n_tiles, max_tiles = rt.tile_layout(cam, world)
        buf = torch.zeros((max_tiles, 64, 3), dtype=torch.float64, device="cuda")
        ms, segs, chunks = [], [], []
        for r in range(world):
            s = rt.RenderSettings(samples=a.spp, seed=seed, tile_rank=r, tile_world=world, sample_chunk=a.chunk)
            best = None
            for _ in range(a.reps):
                dev.render_tiles_device(cam, s, buf.data_ptr())
                c = dev.counters()
                best = c.kernel_ms if best is None else min(best, c.kernel_ms)
            ms.append(best)
            segs.append(int(c.segments))
            chunks.append(int(c.sample_chunk))
            print(f"world {world} rank {r}: {best:.2f} ms, {c.segments} segments, chunk {c.sample_chunk}", flush=True)
        if world == 1:
            t1 = ms[0]
        mx, mean = max(ms), sum(ms) / len(ms)
        res["worlds"][str(world)] = {
            "rank_kernel_ms": [round(x, 3) for x in ms], "rank_segments": segs, "sample_chunk": sorted(set(chunks)),
            "max_over_mean": round(mx / mean, 4),
            "segments_max_over_mean": round(max(segs) / (sum(segs) / len(segs)), 4),
            "predicted_efficiency": round(t1 / (world * mx), 4) if t1 else None}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))
    dev.close()


if __name__ == "__main__":
    main()
