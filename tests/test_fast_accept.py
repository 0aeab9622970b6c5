"""The megakernel's sphere-box fast accept (RT_SPHERE_FAST_ACCEPT, rt_device.h leaf_tests4) on the CPU:
tests/fast_accept_check.c draws random and adversarial rays (silhouettes, tangent points, box edges and
corners, axis-parallel directions, t_best at / around the root) and asserts that whenever the rule
clears a sphere hit, the reference's exact box test (bvh/aabb.rs:62-79 hit2, through the oracle) passes —
so skipping that test cannot change which primitive is hit (bbox_tree.rs:60-71's `box && sphere`)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
@pytest.mark.parametrize("seed", ["0x5EED", "0xC0FFEE", "0xBADD1CE"])
def test_fast_accept_never_skips_a_failing_box_test(tmp_path, seed):
    exe = str(tmp_path / "fac")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe,
                    os.path.join(REPO, "tests", "fast_accept_check.c"), "-I" + os.path.join(REPO, "include"),
                    "-L" + os.path.join(REPO, "oracle"), "-loracle", "-Wl,-rpath," + os.path.join(REPO, "oracle"),
                    "-lm"], check=True)
    r = subprocess.run([exe, "3000000", seed], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    f = dict(zip(r.stdout.split()[0::2], map(int, r.stdout.split()[1::2])))
    assert f["violations"] == 0 and f["cleared"] > 0.5 * (f["cleared"] + f["slab_needed"])
