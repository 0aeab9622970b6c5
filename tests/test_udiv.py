"""The megakernel's unit fetch divides by launch-invariant divisors (n_chunks x 64, tiles_x) with
host-built Granlund-Montgomery multipliers (rt_layout.h make_udiv, applied by rt_device.h udiv).  The
formula and the host construction are checked here exhaustively over small divisors and on 2 M random
pairs (tools/udiv_check.cpp); the GPU image tests exercise the device side on every frame."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_invariant_division_matches_integer_division(tmp_path):
    exe = str(tmp_path / "udiv_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tools", "udiv_check.cpp")],
                   check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout + r.stderr
