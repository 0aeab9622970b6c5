"""ASan + UBSan (+ float-cast-overflow) run of the CPU side of the boundary: the C++
host layer (serde-JSON loader/saver behind `ray-cli render saved`, reference scenes.rs:128-134;
SceneBuilder::finalize, scene/mod.rs:111-137), both BVH builders (bvh_build.cpp; reference rules of
bvh/bbox_tree/constructor.rs:9-212) and the C oracle, built from their sources by
tools/sanitize/Makefile and driven by tools/sanitize/host_check.cpp: every builtin scene round-trips
through JSON, is finalized, built and rendered; then a seeded mutation fuzzer feeds malformed and
extreme-valued scene JSON through the same steps.  Any sanitizer report aborts the driver."""
import fcntl
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "tools", "sanitize")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan/libubsan")
@pytest.mark.parametrize("seed", ["0x5EED", "0xC0FFEE"])
def test_host_layer_under_asan_ubsan(seed):
    os.makedirs(os.path.join(SAN, "build"), exist_ok=True)
    with open(os.path.join(SAN, "build", ".lock"), "w") as lock:  # (xdist: one build, no relink while another runs)
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", SAN, "build/host_check"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(SAN, "build", "host_check"),
                        os.path.join(REPO, "shirley-raytracing-rs_amd", "assets"), "1500", seed],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
