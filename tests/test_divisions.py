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


def test_sphere_sure_pass_never_skips_a_rejecting_box_test(tmp_path):
    """The megakernel skips a sphere leaf's exact box test (aabb.rs:62-79 on c -+ r) where the rounding
    margin proves it passes (rt_device.h leaf_tests4).  tests/sphere_sure_check.c draws
    adversarial spheres and rays (hits at the box-face tangent points, rays tangent in the face planes,
    origins on the sphere, axis-parallel directions): among ~190 k sphere hits whose box test rejects, the
    rule must clear none — and it must still clear most hits, or the skip buys nothing.  (With no margin the
    same draws give ~55 k false skips: the check has teeth.)"""
    exe = str(tmp_path / "sphere_sure_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(REPO, "tests", "sphere_sure_check.c"),
                    "-lm"], check=True)
    r = subprocess.run([exe, "8000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    f = {k: int(v) for v, k in [(w.split()[0], " ".join(w.split()[1:])) for w in r.stdout.split(":")[1].split(",")]}
    assert f["sure but box rejects"] == 0, r.stdout
    assert f["box rejects among them"] > 100000, r.stdout
    assert f["sure"] > 0.8 * f["sphere hits"], r.stdout


def test_two_pass_rectbox_test_is_the_sequential_one(tmp_path):
    """The megakernel tests a RectBox's near planes first and its far planes only when the margin does not
    prove they lose (rt_device.h box_t2).  tests/box_pass_check.c compares it with the sequential six-face
    test (rect.rs:132-156) on adversarial boxes and rays — edges, corners (faces tied at one t), grazing
    rays, origins inside and on faces — bit for bit in (face, t).  Without the 2^-50 margins the same draws
    give ~300 mismatches per million: the check has teeth."""
    src = os.path.join(REPO, "tests", "box_pass_check.c")
    for flags, want_bad in (([], False), (["-DNO_MARGIN"], True)):
        exe = str(tmp_path / ("bpc" + "".join(flags)))
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", *flags, "-o", exe, src, "-lm"], check=True)
        r = subprocess.run([exe, "3000000"], capture_output=True, text=True, timeout=120)
        last = r.stdout.strip().split("\n")[-1].replace(",", "").split()
        bad, compared, one_pass, ties = int(last[0]), int(last[2]), int(last[4]), int(last[7])
        assert compared > 800000 and ties > 100000, r.stdout
        if want_bad:
            assert bad > 0, r.stdout
        else:
            assert r.returncode == 0 and bad == 0, r.stdout
            assert one_pass > 0.8 * compared, r.stdout


def test_portable_libm_is_accurate(tmp_path):
    """The diagnostic libm shared by the RT_PORTABLE_LIBM kernels and the OR_PORTABLE_LIBM oracle
    (csrc/rt/portable_libm.h) is within a few ulps of glibc: its frames are plausible images, so their
    bit-identity (tests/test_gpu_libm_isolation.py) is a test of the path, not of a degenerate function."""
    exe = str(tmp_path / "plcheck")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(REPO, "shirley-raytracing-rs_amd", "csrc", "rt"),
                    "-o", exe, os.path.join(REPO, "tools", "portable_libm_check.c"), "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, check=True).stdout.split()
    vals = [float(out[out.index(k) + 1]) for k in ("sin", "log", "atan2", "acos")]
    assert all(v <= 1e-15 for v in vals), out
