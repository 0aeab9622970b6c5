"""Load balance of the multi-GPU partitions measured on ONE GPU: for each world size and
partition, every rank's share of the headline frame is rendered exactly as that rank would render it on
its own MI355X, and its device time (trace + reduce, HIP events) taken.
  tiles:   interleaved 8x8 tiles (rt_render_tiles_device with tile_rank / tile_world, auto sample chunk);
  samples: all pixels for the rank's share of the samples (rt_render_device with sample_begin /
           sample_count, auto sample chunk).
The slowest rank bounds a sharded frame; the exchange is added from a link model (xGMI: one link per
peer pair, LINK_GBS effective per direction; tiles: the gather, 23 MB / N per link into rank 0; samples:
all-to-all of row bands + the band sum + the gather of the bands, 2 x 23 MB / N per link + a 23 MB / N
HBM pass), so
    predicted strong-scaling efficiency(N) = T(1) / (N * (max_r T_r(N) + exchange(N)))

usage: python tools/shard_balance.py [out.json] [--spp 500] [--reps 2] [--worlds 1,2,4,8] [--chunk 0]
       [--partitions tiles,samples]
(--chunk: a fixed sample_chunk instead of the auto choice, to compare unit lengths per world size)
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINK_GBS = 100.0   # effective xGMI bandwidth per peer link and direction, GB/s = MB/ms (model; ~153 GB/s raw)
HBM_GBS = 5000.0   # achievable HBM bandwidth of a streaming kernel, MB/ms
sys.path.insert(0, os.path.join(REPO, "shirley-raytracing-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?", default=os.path.join(REPO, "gpurun_out", "shard_balance.json"))
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--partitions", default="tiles,samples")
    a = ap.parse_args()
    import torch
    import raytracer as rt
    seed = 0x5EED
    scene = rt.scenes.random_scene(seed).finalize(seed)
    cam = rt.default_camera(1200, "std3x2")
    dev = rt.Device(0)
    dev.upload(scene, "sah")
    frame_mb = cam.image_width * cam.image_height * 24 / 1e6
    res = {"workload": f"random 1200x800 @ {a.spp}spp, SAH, one MI355X", "chunk": a.chunk or "auto",
           "link_gbs_model": LINK_GBS, "hbm_gbs_model": HBM_GBS, "partitions": {}}
    for part in a.partitions.split(","):
        out = res["partitions"][part] = {}
        t1 = None
        for world in [int(w) for w in a.worlds.split(",")]:
            n_tiles, max_tiles = rt.tile_layout(cam, world)
            if part == "tiles":
                buf = torch.zeros((max_tiles, 64, 3), dtype=torch.float64, device="cuda")
            else:
                buf = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.float64, device="cuda")
            ms, segs, chunks, passes, kms, rms = [], [], [], [], [], []
            for r in range(world):
                if part == "tiles":
                    s = rt.RenderSettings(samples=a.spp, seed=seed, tile_rank=r, tile_world=world, sample_chunk=a.chunk)
                else:
                    b, e = a.spp * r // world, a.spp * (r + 1) // world
                    s = rt.RenderSettings(samples=a.spp, seed=seed, sample_chunk=a.chunk, sample_begin=b,
                                          sample_count=e - b)
                best = None
                for _ in range(a.reps):
                    if part == "tiles":
                        dev.render_tiles_device(cam, s, buf.data_ptr())
                    else:
                        dev.render_device(cam, s, buf.data_ptr())
                    c = dev.counters()
                    t = c.kernel_ms + c.reduce_ms
                    if best is None or t < best:
                        best, bk, br = t, c.kernel_ms, c.reduce_ms
                ms.append(best)
                kms.append(bk)
                rms.append(br)
                segs.append(int(c.segments))
                chunks.append(int(c.sample_chunk))
                passes.append(int(c.passes))
                print(f"{part} world {world} rank {r}: {best:.2f} ms, {c.segments} segments, chunk {c.sample_chunk}, "
                      f"passes {c.passes}", flush=True)
            if world == 1:
                t1 = ms[0]
            # exchange model (ms): per-link volume / LINK_GBS (+ the band sum's HBM pass for samples)
            per_link_mb = frame_mb / world
            if world == 1:
                xch = 0.0
            elif part == "tiles":
                xch = per_link_mb / LINK_GBS
            else:
                xch = 2 * per_link_mb / LINK_GBS + frame_mb / world / HBM_GBS
            mx, mean = max(ms), sum(ms) / len(ms)
            out[str(world)] = {
                "rank_device_ms": [round(x, 3) for x in ms], "rank_trace_ms": [round(x, 3) for x in kms],
                "rank_reduce_ms": [round(x, 3) for x in rms], "rank_segments": segs,
                "sample_chunk": sorted(set(chunks)), "passes": sorted(set(passes)),
                "max_over_mean": round(mx / mean, 4),
                "segments_max_over_mean": round(max(segs) / (sum(segs) / len(segs)), 4),
                "exchange_model_ms": round(xch, 4),
                "predicted_kernel_efficiency": round(t1 / (world * mx), 4) if t1 else None,
                "predicted_efficiency": round(t1 / (world * (mx + xch)), 4) if t1 else None}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))
    dev.close()


if __name__ == "__main__":
    main()
