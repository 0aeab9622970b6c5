import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "shirley-raytracing-rs_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU-oracle runs")


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    """The in-tree libraries must exist (built by __graft_entry__.build / make); build if stale."""
    libs = [os.path.join(PKG, "lib", n) for n in ("libshirley_rt.so", "libshirley_host.so")]
    srcs = []
    for root, _, files in os.walk(os.path.join(PKG, "csrc")):
        srcs += [os.path.join(root, f) for f in files]
    if any(_stale(l, srcs) for l in libs):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    yield


@pytest.fixture(scope="session")
def gpu():
    """One rt_ctx for the GPU tests; fails loudly (never skips silently to a CPU path)."""
    import raytracer as rt
    return rt.Device(0)
