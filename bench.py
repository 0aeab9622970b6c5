#!/usr/bin/env python3
"""Headline benchmark: Msamples/s on the book-1 random_scene, 1200x800 @ 500 spp, max_depth 50
(BASELINE.json configs[1]; metric "Msamples/sec (whole node)").

One step = one full frame through the hot path (camera rays -> ray_color bounce loop -> per-pixel
sums in HBM).  N GPUs (torchrun, one process per GPU): the frame's 8x8 tiles are dealt round-robin to
ranks; each rank calls rt_render_sharded (C ABI), which renders its tiles into a packed buffer and
gathers them to rank 0 with RCCL (ncclGather over xGMI, the north star's exchange step), where they
are scattered into the [H][W][3] image: strong scaling of one frame.  Scene upload happens before the timed region; inputs are resident in HBM.
Every step ends with the frame's sums copied into pinned host memory ("kernel start to
gathered accumulation on host"); the device-only step time is reported beside it.

Launch: `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N` (the driver's form), or
`python bench.py --gpus N`, which starts that torchrun itself as a child process before anything touches
the GPU.  --gpus must equal WORLD_SIZE under a launcher, and RCCL ranks may not outnumber the visible GPUs:
both exit non-zero with a message instead of printing a mislabelled line.

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` (dominant kernel:
the persistent trace kernel, timed with HIP events on the launch stream) and `cpu_baseline` (the f64
C oracle on the host cores, bounded sample).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "shirley-raytracing-rs_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
FP64_PEAK_TFLOPS = 78.6      # MI355X vector FP64 (spec)
# algorithmic bytes per path segment (SURVEY.md §8d contract): f32 path state 64 B read + 64 B
# written + 8 B hit record written + 8 B read.  The graded roofline uses this figure.
BYTES_PER_SEGMENT = 144
# the same round trip for the reference's f64 path state, reported beside it
BYTES_PER_SEGMENT_F64 = 256


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU): under torchrun it must equal WORLD_SIZE; without a launcher "
                         "N > 1 starts torchrun itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--aspect", default="std3x2")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    ap.add_argument("--scene", default="random")
    ap.add_argument("--bvh", default="sah", choices=["reference", "sah"])
    ap.add_argument("--sample-chunk", type=int, default=0)
    ap.add_argument("--partition", default="auto", choices=["auto", "tiles", "samples"],
                    help="multi-GPU split of the frame (RT_PARTITION_*): interleaved tiles or sample shares")
    ap.add_argument("--scratch-mb", type=int, default=0, help="partial-sum scratch bound per call (0: library default)")
    ap.add_argument("--nodes", default="auto", choices=["auto", "global", "half-lds", "lds"], help="BVH node placement")
    ap.add_argument("--engine", default="auto", choices=["auto", "megakernel", "wavefront", "split"])
    ap.add_argument("--timing", action="store_true", help="per-launch HIP-event timing of the wavefront kernels")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target wall time of each CPU-baseline leg (full frame at reduced spp; centre rows at full spp)")
    ap.add_argument("--cpu-config-seconds", type=float, default=5.0,
                    help="target wall time of each other config's CPU leg (configs 3-5: full frame, reduced spp)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use (cgroup-aware)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the one-frame measurements of BASELINE.json's other configs (N=1 only)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N>1 (gloo only to rehearse several ranks on one GPU)")
    ap.add_argument("--rank-env-only", action="store_true",
                    help="(tests) every rank prints its RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* as JSON and exits "
                         "before touching the GPU")
    return ap.parse_args()


def rank_launch(n, argv, port=None):
    """The torchrun command and environment that run this bench as `n` ranks (one process per GPU) when
    `python bench.py --gpus n` is started without a launcher: (argv, env).  The parent never touches the
    GPU; every rank reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from torchrun."""
    if port is None:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    env.pop("WORLD_SIZE", None)
    return cmd, env


def check_world(args, environ, n_visible):
    """How this process takes part for `--gpus args.gpus`: "single" (one process, N = 1), "launch" (spawn
    N ranks) or "rank" (a rank of a launched job).  Raises SystemExit with a message on a mislabelled run:
    WORLD_SIZE set and != --gpus, or more RCCL ranks than visible GPUs."""
    n = args.gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}: need at least one GPU")
    ws = environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != n:
        raise SystemExit(f"bench.py: --gpus {n} but WORLD_SIZE={ws}: the launcher and the flag disagree")
    if n > 1 and args.dist_backend == "nccl" and n > n_visible:
        raise SystemExit(f"bench.py: --gpus {n} but {n_visible} visible GPU(s): one rank per GPU (RCCL refuses "
                         "two ranks on one device); use --dist-backend gloo only to rehearse")
    if ws is not None:
        return "rank"
    return "launch" if n > 1 else "single"


def host_cpus():
    """CPUs this process may run on: the affinity mask, capped by the cgroup CPU quota (a GPU box shares
    its host: nproc reports the whole machine, the cgroup the box's share).  Returns (usable, info)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = max(1, min(aff, int(quota)) if quota else aff)
    model = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "cpu_model": model}


def cpu_leg(osc, cam, spp_full, args, threads, seconds, O):
    """The oracle on `threads` host cores over the full frame at reduced spp: calibrated on one sample per
    pixel, then sized to ~`seconds` of wall time (at most the config's spp).  (samples, seconds, spp)."""
    t0 = time.perf_counter()
    osc.render(cam, O.params(1, args.max_depth, args.seed + 1), threads=threads)
    per_spp = time.perf_counter() - t0
    spp = int(max(1, min(spp_full, round(seconds / max(per_spp, 1e-3)))))
    t0 = time.perf_counter()
    _, cnt = osc.render(cam, O.params(spp, args.max_depth, args.seed), threads=threads)
    return cnt.samples, time.perf_counter() - t0, spp


def cpu_baseline(scene, cam, args):
    """The oracle (f64 C restatement of the reference path, test infrastructure) timed on the host, on
    every core this process may use (the rayon analogue: row-granular dynamic scheduling), two legs
    (BASELINE.md): the full frame at reduced spp, and a centre band of rows at the full spp.
    Msamples/s is per-sample throughput, so both are comparable with the GPU figure; `value` is the
    full-frame leg (it weighs every pixel like the GPU frame)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    osc = O.OracleScene(scene)
    usable, info = host_cpus()
    threads = args.cpu_threads or usable
    W, H = cam.image_width, cam.image_height
    n_samples, dt, spp = cpu_leg(osc, cam, args.spp, args, threads, args.cpu_seconds, O)
    full = n_samples / dt / 1e6
    # centre band at full spp: rows sized from the full-frame rate
    rows = int(max(1, min(H, round(args.cpu_seconds * full * 1e6 / (W * args.spp)))))
    r0 = (H - rows) // 2
    t0 = time.perf_counter()
    _, cnt2 = osc.render(cam, O.params(args.spp, args.max_depth, args.seed), r0, r0 + rows, threads=threads)
    dt2 = time.perf_counter() - t0
    return {"value": round(full, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{args.scene} {W}x{H} @ {spp} spp (full frame, reduced spp; {n_samples} samples, "
                      f"{dt:.1f} s wall on {threads} threads; f64 C oracle restating the reference path, "
                      f"-O2 -ffp-contract=off; a proxy: the Rust reference cannot be built here)",
            "centre_rows_leg": {"value": round(cnt2.samples / dt2 / 1e6, 4), "unit": "Msamples/s",
                                "sample": f"rows [{r0}, {r0 + rows}) x {W} @ {args.spp} spp (full spp), "
                                          f"{cnt2.samples} samples, {dt2:.1f} s wall"},
            "host": info}


# BASELINE.json configs other than the headline (configs[1]), each one full frame at its stated size
# and spp on this GPU: (key, scene, width, aspect, spp, note).  Config 5's book-2 final_scene is the
# book-2 extension scene (the reference has none); its ~10k-primitive stand-in from the
# reference's own benches (gen_spheres, benches/my_benchmark.rs:35-60) is measured beside it.
OTHER_CONFIGS = [
    ("cfg1", "random", 400, "std16x9", 50, "book-1 random_scene 400x225 @ 50 spp"),
    ("cfg3", "earth", 800, "square", 1000, "earth-texture sphere 800x800 @ 1000 spp"),
    ("cfg4", "cornell", 600, "square", 10000, "Cornell box 600x600 @ 10000 spp"),
    ("cfg5_final", "final", 1920, "std16x9", 2000, "book-2 final_scene 1920x1080 @ 2000 spp, 1 GPU of the 8"),
    ("cfg5_spheres", "spheres", 1920, "std16x9", 2000, "gen_spheres 22^3 = 10648 spheres 1920x1080 @ 2000 spp, 1 GPU"),
]


def configs_block(args, dev, torch, rt):
    """One timed full frame of every other BASELINE config on this GPU, after one untimed frame of the
    same size and spp (it sizes the per-render scratch, so no allocation falls in the timed frame), and
    each config's CPU leg as BASELINE.md specifies it: config 1 the oracle on one thread over the full
    frame at its spp (BASELINE.md:23); configs 3-5 the oracle on every host core over the full frame at
    reduced spp (BASELINE.md:24,33-35), with the GPU / CPU ratio of the per-sample rates."""
    out = {}
    usable, _ = host_cpus()
    threads = args.cpu_threads or usable
    stream = torch.cuda.current_stream()
    for key, name, width, aspect, spp, note in OTHER_CONFIGS:
        scene = rt.SceneBuilder.builtin(name, args.seed).finalize(args.seed)
        cam = rt.scene_camera(name, width, aspect)
        W, H = cam.image_width, cam.image_height
        dev.upload(scene, args.bvh)
        accum = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
        dev.render_device(cam, rt.RenderSettings(samples=spp, max_reflect=args.max_depth, seed=args.seed),
                          accum.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.render_device(cam, rt.RenderSettings(samples=spp, max_reflect=args.max_depth, seed=args.seed),
                          accum.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        c = dev.counters()
        out[key] = {"workload": note, "value": round(W * H * spp / dt / 1e6, 3), "unit": "Msamples/s",
                    "ms_per_frame": round(dt * 1e3, 3), "kernel_ms": round(c.kernel_ms, 3),
                    "segments_per_sample": round(c.segments / max(c.samples, 1), 4),
                    "engine": {1: "megakernel", 2: "wavefront", 3: "split"}.get(c.engine)}
        if key == "cfg1" and not args.no_cpu:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_lib as O
            t0 = time.perf_counter()
            _, cnt = O.OracleScene(scene).render(cam, O.params(spp, args.max_depth, args.seed), threads=1)
            dt = time.perf_counter() - t0
            out[key]["cpu_single_thread"] = {"value": round(cnt.samples / dt / 1e6, 4), "unit": "Msamples/s",
                                             "sample": f"full frame {W}x{H} @ {spp} spp, 1 thread, {dt:.1f} s "
                                                       "(f64 C oracle, a proxy for the Rust reference)"}
        elif not args.no_cpu:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_lib as O
            n, dt, cspp = cpu_leg(O.OracleScene(scene), cam, spp, args, threads, args.cpu_config_seconds, O)
            rate = n / dt / 1e6
            out[key]["cpu_all_cores"] = {"value": round(rate, 4), "unit": "Msamples/s", "cores": threads,
                                         "kind": "port", "spp": cspp,
                                         "sample": f"full frame {W}x{H} @ {cspp} spp (reduced from {spp}), {n} samples, "
                                                   f"{dt:.1f} s wall on {threads} threads (f64 C oracle)"}
            out[key]["gpu_over_cpu"] = round(out[key]["value"] / rate, 1)
    return out


def sharded_config5(args, dev, comm, rank, world, torch, dist, rt, width=None, spp=None, keep=None):
    """BASELINE config 5 as it is stated: book-2 final_scene 1920x1080 @ 2000 spp tile-sharded across the
    job's GPUs with the RCCL gather to rank 0 (rt_render_sharded), one untimed frame (sizes the per-render
    scratch) and one timed frame bracketed by barriers, max over ranks.  Runs after the headline's timed
    region, so the headline number is unaffected."""
    key, name, w0, aspect, spp0, note = OTHER_CONFIGS[3]
    width, spp = width or w0, spp or spp0  # (smaller only in tests/test_gpu_multi.py)
    scene = rt.SceneBuilder.builtin(name, args.seed).finalize(args.seed)
    cam = rt.scene_camera(name, width, aspect)
    W, H = cam.image_width, cam.image_height
    dev.upload(scene, args.bvh)
    settings = rt.RenderSettings(samples=spp, max_reflect=args.max_depth, seed=args.seed, tile_rank=rank,
                                 tile_world=world)
    accum = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda") if rank == 0 else None
    sh = torch.cuda.current_stream().cuda_stream
    ptr = accum.data_ptr() if rank == 0 else 0
    dev.render_sharded(comm, cam, settings, ptr, sh)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev.render_sharded(comm, cam, settings, ptr, sh)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    if keep is not None:
        keep.append(accum)
    return {f"{key}_sharded": {"workload": f"book-2 final_scene {W}x{H} @ {spp} spp, tile-sharded over {world} GPUs, "
                                          "ncclGather of the packed tiles to rank 0",
                               "value": round(W * H * spp / dt / 1e6, 3), "unit": "Msamples/s",
                               "ms_per_frame": round(dt * 1e3, 3), "ranks": world}}


def resolve_partition(requested, environ):
    """The partition rt_render_sharded runs for `requested` (frame_partition in rt_api.cpp): RT_PARTITION_AUTO
    is tiles unless SHIRLEY_PARTITION=samples overrides it."""
    if requested != "auto":
        return requested
    return "samples" if environ.get("SHIRLEY_PARTITION") == "samples" else "tiles"


def compare_frames(ref, got, exact, rel=1e-12):
    """(ok, detail) of a multi-rank frame against the single-device frame: `exact` bit for bit (tiles:
    every pixel's sum is computed on one rank with the same unit length), else per channel
    |got - ref| <= rel * |ref| (samples: the rank-order sum of per-rank shares reassociates the sum)."""
    import numpy as np
    ref = np.ascontiguousarray(ref, dtype=np.float64)
    got = np.ascontiguousarray(got, dtype=np.float64)
    if ref.shape != got.shape:
        return False, f"shape {tuple(got.shape)} != {tuple(ref.shape)}"
    d = np.abs(got - ref)
    worst = float(np.nanmax(d)) if d.size else 0.0
    if exact:
        n = int(np.count_nonzero(ref.view(np.uint64) != got.view(np.uint64)))
        return n == 0, (f"bit-identical ({ref.size} channels)" if n == 0 else
                        f"{n} of {ref.size} channels differ, max |d| {worst:.3g}")
    bad = ~(d <= rel * np.abs(ref))  # (NaN-safe: a NaN difference is bad)
    n = int(np.count_nonzero(bad))
    return n == 0, (f"within {rel:g} relative ({ref.size} channels, max |d| {worst:.3g})" if n == 0 else
                    f"{n} of {ref.size} channels beyond {rel:g} relative, max |d| {worst:.3g}")


def sharded_frame(args, dev, comm, rank, world, torch, rt, cam, settings, part, ran=None):
    """One multi-rank frame through the job's exchange: rt_render_sharded (RCCL) or, in a gloo rehearsal,
    the same exchange by torch.distributed (raytracer/parallel.py).  Rank 0 gets the [H][W][3] sums
    (a CUDA tensor), the other ranks None.  `ran` (a list) records whether this rank launched a render:
    a gloo rank whose sample share is empty (more ranks than samples) launches none, so it has no
    counters (rt_render_sharded runs an empty-range render instead)."""
    from raytracer.parallel import gather_tiles, reduce_sample_bands, sample_share
    W, H = cam.image_width, cam.image_height
    sh = torch.cuda.current_stream().cuda_stream
    out = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda") if rank == 0 else None
    if ran is not None:
        ran[:] = [True]
    if comm is not None:
        dev.render_sharded(comm, cam, settings, out.data_ptr() if rank == 0 else 0, sh)
        return out
    if part == "samples":
        b, e = sample_share(0, settings.samples, rank, world)
        local = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
        if ran is not None:
            ran[:] = [e > b]
        if e > b:
            s = rt.RenderSettings(**{**settings.__dict__, "sample_begin": b, "sample_count": e - b, "tile_rank": 0,
                                     "tile_world": 1})
            dev.render_device(cam, s, local.data_ptr(), sh)
        torch.cuda.synchronize()
        summed = reduce_sample_bands(local.cpu(), world)  # (gloo: host tensors)
        if rank == 0:
            out.copy_(summed)
        return out
    _, max_tiles = rt.tile_layout(cam, world)
    packed = torch.zeros((max_tiles, 64, 3), dtype=torch.float64, device="cuda")
    dev.render_tiles_device(cam, settings, packed.data_ptr(), sh)
    gathered = gather_tiles(packed, world)
    if rank == 0:
        dev.unpack_tiles_device(cam, world, gathered.data_ptr(), out.data_ptr(), sh)
    return out


def multi_rank_check(args, dev, comm, rank, world, torch, rt):
    """After the timed region at N > 1: a small frame of the headline scene (200x112 @ 8 spp, explicit
    8-sample units) through the job's exchange with both partitions; rank 0 compares each with the same
    frame rendered on its device alone (rt_render): tiles bit for bit, samples within 1e-12 relative.
    The whole-machine loop this replaces is main.rs:117-125.  Returns the JSON block (rank 0; {} elsewhere)."""
    cam = rt.scene_camera(args.scene, 200, "std16x9")
    base = dict(samples=8, max_reflect=args.max_depth, seed=args.seed, sample_chunk=8, tile_rank=rank,
                tile_world=world)
    frames = {}
    for part in ("tiles", "samples"):
        out = sharded_frame(args, dev, comm, rank, world, torch, rt, cam, rt.RenderSettings(**base, partition=part),
                            part)
        torch.cuda.synchronize()
        if rank == 0:
            frames[part] = out.cpu().numpy()
    if rank != 0:
        return {}
    ref = dev.render(cam, rt.RenderSettings(samples=8, max_reflect=args.max_depth, seed=args.seed, sample_chunk=8))
    res = {"frame": f"{args.scene} {cam.image_width}x{cam.image_height} @ 8 spp, sample_chunk 8, {world} ranks, "
                    f"{'rccl' if comm is not None else 'gloo rehearsal'}"}
    ok_all = True
    for part in ("tiles", "samples"):
        ok, detail = compare_frames(ref, frames[part], exact=(part == "tiles"))
        res[part] = detail
        ok_all &= ok
    res["status"] = "ok" if ok_all else "mismatch"
    return res


def valu_block(segments, k_ms, W, H, args):
    """The measured ceiling of the trace kernel (VALU issue x lane utilisation), from the committed PMC
    passes (profiles/valu.json, written by tools/pmc_valu.py from profiles/<round>/pmc_valu_*.csv of one
    trace_kernel dispatch): per-segment instruction and f64-FLOP counts scaled by this run's segments
    and kernel time."""
    path = os.path.join(REPO, "profiles", "valu.json")
    if not os.path.exists(path):
        return None
    try:
        v = json.load(open(path))
    except (OSError, ValueError):
        return None
    if v.get("scene") != args.scene or v.get("bvh") != args.bvh or v.get("size") != [W, H]:
        return None
    flops = v["f64_flops_per_segment"] * segments
    return {"bound": "valu", "busy_frac": v["valu_busy_frac"], "lane_util": v["lane_util"],
            "valu_insts_per_segment": v["valu_insts_per_segment"],
            "f64_tflops": round(flops / (k_ms * 1e-3) / 1e12, 3), "f64_peak_tflops": FP64_PEAK_TFLOPS,
            "f64_frac": round(flops / (k_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4), "source": v["source"]}


def main():
    args = parse()
    import torch
    # (device_count does not initialise the GPU on this image: the launching parent stays GPU-free)
    n_dev = torch.cuda.device_count()
    mode = check_world(args, os.environ, n_dev)
    if mode == "launch":
        import subprocess
        cmd, env = rank_launch(args.gpus, sys.argv[1:])
        sys.exit(subprocess.run(cmd, env=env).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rank_env_only:
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                         "MASTER_PORT", "HSA_ENABLE_IPC_MODE_LEGACY")}), flush=True)
        return
    import numpy as np
    import torch.distributed as dist
    import raytracer as rt
    rehearsal = world > n_dev
    # --dist-backend gloo + fewer GPUs than ranks: a rehearsal of the multi-rank path on one box
    # (ranks share GPUs round-robin); the measured configuration is nccl (RCCL over xGMI)
    local = local % max(1, n_dev)
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    scene = rt.SceneBuilder.builtin(args.scene, args.seed).finalize(args.seed)
    cam = rt.scene_camera(args.scene, args.width, args.aspect)
    W, H = cam.image_width, cam.image_height
    dev = rt.Device(local)
    dev.upload(scene, args.bvh, args.nodes)
    settings = rt.RenderSettings(samples=args.spp, max_reflect=args.max_depth, seed=args.seed,
                                 sample_chunk=args.sample_chunk, tile_rank=rank, tile_world=world,
                                 engine=args.engine, timing=args.timing, partition=args.partition,
                                 scratch_mb=args.scratch_mb)
    # a stream of our own: the render calls, the HIP events and the host copy share it (torch's default
    # stream has handle 0, which the C ABI reads as "the ctx's own stream")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    accum = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
    comm = None
    partition = resolve_partition(args.partition, os.environ)
    if world > 1 and args.dist_backend == "nccl":
        # the exchange runs behind the C ABI (rt_render_sharded: ncclGather / ncclAllToAll over xGMI);
        # torch.distributed only carries the communicator id, the barriers and the max-over-ranks clock
        uid = [rt.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = dev.comm_init_rank(uid[0], world, rank)

    # the metric runs from kernel start to the gathered accumulation on the host, so every
    # step ends with the [H][W][3] sums copied into pinned host memory (rank 0: after the gather)
    host_accum = torch.empty((H, W, 3), dtype=torch.float64, pin_memory=True) if rank == 0 else None
    ev_dev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    device_ms = []

    ran = [True]  # this rank launched a render in the step (a gloo rank with an empty sample share: none)

    def step():
        ev_dev[0].record(stream)
        if world == 1:
            dev.render_device(cam, settings, accum.data_ptr(), sh)
        elif comm is not None:
            dev.render_sharded(comm, cam, settings, accum.data_ptr() if rank == 0 else 0, sh)
        else:  # gloo rehearsal (ranks sharing one GPU cannot form an RCCL communicator): the same exchange
            out = sharded_frame(args, dev, None, rank, world, torch, rt, cam,
                                rt.RenderSettings(**{**settings.__dict__, "partition": partition}), partition, ran)
            if rank == 0:
                accum.copy_(out)
        ev_dev[1].record(stream)
        if host_accum is not None:
            host_accum.copy_(accum, non_blocking=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms, segments, samples, laps = [], [], [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        ev_dev[1].synchronize()
        device_ms.append(ev_dev[0].elapsed_time(ev_dev[1]))
        if not ran[0]:
            continue
        c = dev.counters()  # waits for this step's trace + reduce events (no extra work on the GPU)
        kernel_ms.append(c.kernel_ms)
        segments.append(c.segments)
        samples.append(c.samples)
        laps.append((c.engine, c.iterations, c.slots, c.extend_ms, c.shade_ms, c.texture_ms, c.node_visits,
                     c.prim_tests, c.passes, c.scratch_bytes, c.sample_chunk, c.n_chunks))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_samples = W * H * args.spp * args.steps
    value = total_samples / elapsed / 1e6
    # per trace-kernel launch (a frame whose partial sums exceed the scratch bound runs in several sample
    # passes, one launch each): algorithmic bytes of a launch / its average duration.  Rank 0 may have traced
    # nothing (a sample partition with more ranks than samples per pixel): then the kernel figures are null.
    if not laps:
        laps = [(0,) * 12]
        kernel_ms, segments, samples = [0.0], [0], [0]
    launches = max(1, laps[-1][8])
    k_ms = float(np.mean(kernel_ms)) / launches
    seg = float(np.mean(segments)) / launches
    traced = k_ms > 0.0 and seg > 0.0
    achieved = BYTES_PER_SEGMENT * seg / (k_ms * 1e-3) / 1e9 if traced else None
    achieved_f64 = BYTES_PER_SEGMENT_F64 * seg / (k_ms * 1e-3) / 1e9 if traced else None
    traffic = None
    tfile = os.path.join(REPO, "profiles", "traffic.json")
    if world == 1 and os.path.exists(tfile):  # (measured per N=1 launch; a rank's launch is smaller)
        try:
            tj = json.load(open(tfile))
            # (the file's workload may carry the ", max_depth …" suffix of the bench's own label)
            if (str(tj.get("workload", "")).split(",")[0] == f"{args.scene} {W}x{H} @ {args.spp}spp"
                    and tj.get("bvh") == args.bvh):
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    line = {
        "metric": "Msamples/sec (whole node) on book-1 random_scene 1200x800 @ 500spp; 1/2/4/8 GPU",
        "value": round(value, 3), "unit": "Msamples/s", "n_gpus": min(world, n_dev), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        # ms_per_step: kernel start -> sums in pinned host memory; device_ms_per_step: the
        # same step up to the sums in HBM (rank 0's stream, HIP events), without the device-to-host copy
        "device_ms_per_step": round(float(np.mean(device_ms)), 3), "timed_to": "host (pinned, rank 0)",
        "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{args.scene} {W}x{H} @ {args.spp}spp, max_depth {args.max_depth}, seed "
                               f"{args.seed:#x}", "scene": args.scene, "width": W, "height": H, "spp": args.spp,
                   "max_depth": args.max_depth, "bvh": args.bvh, "parallelism": f"tiles8x8/{world}",
                   "ranks": world, "rehearsal": f"gloo, {world} ranks on {n_dev} GPU(s)" if rehearsal else None,
                   "engine": {1: "megakernel", 2: "wavefront", 3: "split"}.get(laps[-1][0]), "rounds": laps[-1][1],
                   "slots": laps[-1][2],
                   "kernel_ms_split": {"extend": round(laps[-1][3], 3), "shade": round(laps[-1][4], 3),
                                       "texture": round(laps[-1][5], 3)} if args.timing else None,
                   "segments_per_sample": round(float(np.mean(segments)) / max(float(np.mean(samples)), 1.0), 4),
                   "sample_chunk": laps[-1][10], "n_chunks": laps[-1][11], "sample_passes": laps[-1][8],
                   "partial_scratch_bytes": laps[-1][9],
                   "partition": partition if world > 1 else None,
                   # counted by the instrumented build only (RT_PHASE_TIMING): null here
                   "node_tests_per_segment": round(laps[-1][6] / max(segments[-1], 1), 3) if laps[-1][6] else None,
                   "prim_tests_per_segment": round(laps[-1][7] / max(segments[-1], 1), 3) if laps[-1][7] else None},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2) if traced else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5) if traced else None,
                     "traffic": traffic,
                     "kernel": "trace_kernel", "kernel_ms": round(k_ms, 3), "launches_per_step": launches,
                     "bytes_per_segment": BYTES_PER_SEGMENT, "segments_per_launch": int(seg),
                     # SURVEY.md §8d's third figure: path segments per second of the trace kernel
                     "segments_per_s": round(seg / (k_ms * 1e-3), 1) if traced else None,
                     "f64_state": {"bytes_per_segment": BYTES_PER_SEGMENT_F64,
                                   "achieved": round(achieved_f64, 2) if traced else None,
                                   "frac": round(achieved_f64 / HBM_PEAK_GBS, 5) if traced else None},
                     "measured_hbm_gbs": round(traffic / (k_ms * 1e-3) / 1e9, 2) if traffic and traced else None,
                     "valu": valu_block(seg, k_ms, W, H, args) if world == 1 and traced else None},
        "cpu_baseline": None,
    }
    mrc = None
    if world > 1:  # (after the timed region: the exchange of this job checked against one device's frame)
        mrc = multi_rank_check(args, dev, comm, rank, world, torch, rt)
        if rank == 0:
            line["multi_rank_check"] = mrc
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(scene, cam, args)
    if world == 1 and not args.no_configs:  # (after the timed region; the headline scene is replaced)
        line["configs"] = configs_block(args, dev, torch, rt)
    if comm is not None and not args.no_configs:  # config 5 at its stated scale: sharded over the job's GPUs
        try:
            line["configs"] = sharded_config5(args, dev, comm, rank, world, torch, dist, rt)
        except Exception as e:  # (an extra leg: it must not cost the headline line)
            line["configs"] = {"cfg5_final_sharded": {"error": repr(e)[:200]}}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    dev.close()
    if world > 1:
        dist.destroy_process_group()
    if mrc and mrc.get("status") != "ok":
        sys.exit(f"bench.py: multi-rank frame differs from the single-device frame: {mrc}")


if __name__ == "__main__":
    main()
