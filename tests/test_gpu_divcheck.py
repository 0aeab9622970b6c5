"""The shared-reciprocal division (rt_device.h recip / div_recip / unit_fast) against the compiler's
binary64 division, and sqrt_rn against the compiler's sqrt, on the GPU: bit-identical on random
operands (tools/divcheck.hip)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "shirley-raytracing-rs_amd", "bin",
                   "divcheck")


def test_shared_reciprocal_division_is_bit_identical():
    assert os.path.exists(BIN), "bin/divcheck not built (make -C shirley-raytracing-rs_amd)"
    r = subprocess.run([BIN, "24", "8"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert (" 0 division mismatches, 0 unit mismatches, 0 sqrt mismatches, 0 inverse-division mismatches, "
            "0 reciprocal mismatches, 0 face-division mismatches") in r.stdout, r.stdout
