"""Division replacements of the trace kernel, checked on the CPU (no GPU): the camera's jittered pixel
coordinate x / n by one correction step on x * RN(1 / n) (rt_device.h pixel_coord_div,
tools/camdiv_check.c).  Bit-identity of the shared-reciprocal division on the device itself is checked on
the GPU (tests/test_gpu_divcheck.py)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_camera_coordinate_division_is_exact(tmp_path):
    exe = str(tmp_path / "camdiv_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(REPO, "tools", "camdiv_check.c"), "-lm"],
                   check=True)
    r = subprocess.run([exe, "20000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert r.stdout.strip().startswith("0 of ")
