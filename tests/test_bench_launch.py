"""bench.py's multi-rank launch contract on CPU (no GPU touched): `--gpus N` must match WORLD_SIZE under a
launcher, may not ask for more RCCL ranks than visible GPUs, and without a launcher starts N ranks through
torchrun with the per-rank environment the bench reads (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*)."""
import argparse
import importlib.util
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _args(gpus, backend="nccl"):
    return argparse.Namespace(gpus=gpus, dist_backend=backend)


def test_check_world_modes_and_refusals():
    b = _bench()
    assert b.check_world(_args(1), {}, 1) == "single"
    assert b.check_world(_args(8), {}, 8) == "launch"
    assert b.check_world(_args(8), {"WORLD_SIZE": "8"}, 8) == "rank"
    assert b.check_world(_args(1), {"WORLD_SIZE": "1"}, 1) == "rank"
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        b.check_world(_args(8), {"WORLD_SIZE": "4"}, 8)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        b.check_world(_args(1), {"WORLD_SIZE": "2"}, 8)
    with pytest.raises(SystemExit, match="1 visible GPU"):
        b.check_world(_args(2), {}, 1)
    with pytest.raises(SystemExit, match="1 visible GPU"):
        b.check_world(_args(2), {"WORLD_SIZE": "2"}, 1)
    # a gloo rehearsal may put several ranks on one GPU
    assert b.check_world(_args(2, "gloo"), {}, 1) == "launch"
    with pytest.raises(SystemExit):
        b.check_world(_args(0), {}, 1)


def test_rank_launch_command():
    b = _bench()
    cmd, env = b.rank_launch(4, ["--gpus", "4", "--steps", "3"], port=29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29999" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert "WORLD_SIZE" not in env and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def _run(argv, extra_env=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + argv, capture_output=True, text=True,
                          env=env, timeout=240, cwd=REPO)


def test_launcher_per_rank_environment():
    """`python bench.py --gpus 2` (gloo rehearsal, no GPU here) starts two ranks through torchrun; each
    sees its own RANK / LOCAL_RANK, WORLD_SIZE 2 and the 127.0.0.1 rendezvous."""
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--rank-env-only"])
    assert r.returncode == 0, r.stderr[-2000:]
    envs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(e["RANK"] for e in envs) == ["0", "1"]
    assert sorted(e["LOCAL_RANK"] for e in envs) == ["0", "1"]
    assert all(e["WORLD_SIZE"] == "2" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)


def test_mislabelled_runs_exit_nonzero():
    import torch
    n = torch.cuda.device_count()
    r = _run(["--gpus", str(max(n + 1, 2)), "--rank-env-only"])
    assert r.returncode != 0 and "visible GPU" in r.stderr
    r = _run(["--gpus", "2", "--rank-env-only"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_multi_rank_check_comparison():
    """bench.py's multi_rank_check verdicts: tiles bit for bit, samples within 1e-12
    relative; shape changes, single-ulp flips in the tile frame, NaNs and reassociation-sized errors."""
    import numpy as np
    b = _bench()
    rng = np.random.default_rng(7)
    ref = rng.random((112, 200, 3)) * 8.0
    ok, detail = b.compare_frames(ref, ref.copy(), exact=True)
    assert ok and "bit-identical" in detail
    one_ulp = ref.copy()
    one_ulp[5, 7, 1] = np.nextafter(one_ulp[5, 7, 1], np.inf)
    ok, detail = b.compare_frames(ref, one_ulp, exact=True)
    assert not ok and detail.startswith("1 of")
    ok, _ = b.compare_frames(ref, one_ulp, exact=False)  # one ulp is within the reassociation bound
    assert ok
    far = ref.copy()
    far[0, 0, 0] *= 1.0 + 1e-9
    ok, detail = b.compare_frames(ref, far, exact=False)
    assert not ok and "beyond" in detail
    nan = ref.copy()
    nan[3, 3, 2] = np.nan
    assert not b.compare_frames(ref, nan, exact=False)[0]
    assert not b.compare_frames(ref, nan, exact=True)[0]
    zero = np.zeros_like(ref)
    assert b.compare_frames(zero, zero.copy(), exact=False)[0]
    assert not b.compare_frames(ref, ref[:100], exact=True)[0]


def test_resolve_partition():
    b = _bench()
    assert b.resolve_partition("tiles", {}) == "tiles"
    assert b.resolve_partition("samples", {}) == "samples"
    assert b.resolve_partition("auto", {}) == "tiles"
    assert b.resolve_partition("auto", {"SHIRLEY_PARTITION": "samples"}) == "samples"


def test_cpu_leg_sizes_the_frame_to_the_time_budget():
    """bench.py's per-config CPU legs (configs 3-5, BASELINE.md:24,33-35): the oracle over the full frame
    at an spp sized to the time budget, never above the config's own spp."""
    import oracle_lib as O
    from raytracer import SceneBuilder, scene_camera
    b = _bench()
    args = argparse.Namespace(max_depth=50, seed=0x5EED)
    desc = SceneBuilder.builtin("cornell", 0x5EED).finalize(0x5EED)
    cam = scene_camera("cornell", 48, "square")
    n, dt, spp = b.cpu_leg(O.OracleScene(desc), cam, 4, args, 2, 0.2, O)
    assert 1 <= spp <= 4 and n == cam.image_width * cam.image_height * spp and dt > 0
