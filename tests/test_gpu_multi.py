"""Multi-GPU entry points of the C ABI (rt_comm_*, rt_render_sharded, rt_render_multi)
on the devices a box has.  A one-GPU box forms one-rank communicators: the tile render, the RCCL gather
(ncclGather to rank 0) and the unpack all run, and the frame must equal rt_render's bit for bit (the
counter RNG is keyed by the global pixel, so the frame does not depend on the world size).  The
several-rank data path is covered by test_gpu_parity.py::test_tiles_gather_unpack_equals_full_frame
(3 and 8 ranks' tiles on one device) and by tests/test_distributed.py (gloo, several processes)."""
import numpy as np
import pytest

import raytracer as rt
from raytracer import _native as N

pytestmark = pytest.mark.gpu

SEED = 0x5EED


def _frame_setup(gpu):
    scene = rt.scenes.random_scene(SEED).finalize(SEED)
    cam = rt.default_camera(53, "std16x9")  # 53 x 29: partial tiles on both axes
    gpu.upload(scene, "sah")
    return scene, cam


def test_render_multi_one_device_equals_render(gpu):
    _, cam = _frame_setup(gpu)
    s = rt.RenderSettings(samples=5, seed=SEED)
    want = gpu.render(cam, s)
    got = rt.render_multi([gpu], cam, s)
    assert np.array_equal(got, want)
    c = gpu.counters()
    assert c.samples == cam.image_width * cam.image_height * 5
    # a second call reuses the cached communicator
    assert np.array_equal(rt.render_multi([gpu], cam, s), want)


def test_render_sharded_one_rank_equals_render_device(gpu):
    import torch
    _, cam = _frame_setup(gpu)
    s = rt.RenderSettings(samples=4, seed=SEED)
    comm = gpu.comm_init_rank(rt.comm_unique_id(), 1, 0)
    try:
        stream = torch.cuda.current_stream().cuda_stream
        a = torch.full((cam.image_height, cam.image_width, 3), -1.0, dtype=torch.float64, device="cuda")
        gpu.render_sharded(comm, cam, s, a.data_ptr(), stream)
        b = torch.zeros_like(a)
        gpu.render_device(cam, s, b.data_ptr(), stream)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        with pytest.raises(rt.RtError, match="NULL on the root"):
            gpu.render_sharded(comm, cam, s, 0, stream)
    finally:
        comm.close()


def test_multi_argument_errors(gpu):
    _, cam = _frame_setup(gpu)
    s = rt.RenderSettings(samples=1, seed=SEED)
    with pytest.raises(rt.RtError, match="appears twice"):
        rt.render_multi([gpu, gpu], cam, s)
    with pytest.raises(rt.RtError, match="tile_world"):
        rt.render_multi([gpu], cam, rt.RenderSettings(samples=1, tile_world=2))
    with pytest.raises(rt.RtError):
        gpu.comm_init_rank(rt.comm_unique_id(), 2, 2)  # rank out of range
    assert N.rt_lib().rt_render_multi(None, 1, None, None, None) == N.RT_E_INVALID


def test_cli_gpus_flag(tmp_path):
    """ray-cli --gpus: one device renders like the default path; more devices than the box has fail
    with a message (rt_create of the missing device)."""
    import os
    import subprocess
    import torch
    cli = os.path.join(N.BIN_DIR, "ray-cli")
    common = ["render", "random", "-w", "64", "-s", "2", "--seed", "0x5EED"]
    a = str(tmp_path / "a.png")
    r = subprocess.run([cli] + common + ["-o", a, "--gpus", "1"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    n = torch.cuda.device_count()
    r = subprocess.run([cli] + common + ["-o", str(tmp_path / "b.png"), "--gpus", str(n + 1)], capture_output=True,
                       text=True)
    assert r.returncode == 1 and "rt_create" in r.stderr


def test_bench_sharded_config5_leg(gpu):
    """bench.py's config-5 leg (final_scene tile-sharded over the job's GPUs, rt_render_sharded + the
    torch.distributed barrier / max-over-ranks clock) on a one-rank job, reduced size: it runs and its
    frame equals rt_render_device's."""
    import importlib.util
    import os
    import socket
    import torch
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    comm = gpu.comm_init_rank(rt.comm_unique_id(), 1, 0)
    try:
        args = bench.argparse.Namespace(seed=SEED, bvh="sah", max_depth=50)
        keep = []
        out = bench.sharded_config5(args, gpu, comm, 0, 1, torch, dist, rt, width=48, spp=3, keep=keep)
        r = out["cfg5_final_sharded"]
        assert r["value"] > 0 and r["ranks"] == 1
        cam = rt.scene_camera("final", 48, "std16x9")
        want = torch.zeros_like(keep[0])
        gpu.render_device(cam, rt.RenderSettings(samples=3, max_reflect=50, seed=SEED), want.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(keep[0], want)
    finally:
        comm.close()
        dist.destroy_process_group()


def test_bench_gpus_flag_on_this_box():
    """bench.py --gpus: 1 runs the single-process bench as before (n_gpus 1, the to-host step time next
    to the device-only one); more ranks than this box's GPUs exit non-zero with a message instead of
    printing a line labelled with the wrong GPU count."""
    import json
    import os
    import subprocess
    import sys
    import torch
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = [sys.executable, os.path.join(repo, "bench.py"), "--steps", "2", "--warmup", "1", "--width", "64",
            "--spp", "4", "--no-cpu", "--no-configs"]
    r = subprocess.run(base + ["--gpus", "1"], capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith('{"metric"')][-1])
    assert line["n_gpus"] == 1 and line["config"]["ranks"] == 1 and line["steps"] == 2
    assert line["ms_per_step"] >= line["device_ms_per_step"] > 0
    n = torch.cuda.device_count()
    r = subprocess.run(base + ["--gpus", str(n + 1)], capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode != 0 and "visible GPU" in r.stderr
