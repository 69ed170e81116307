"""The PSS-MLT splat's fixed-point conversion (frt::splat_fixed, round 6)
equals the fp64 expression it replaced, __double2ll_rn((double)x * 2^36) with
the same validity test, for every float tested: a stride through all 2^32 bit
patterns, the rounding ties around each quantum and the range limits.  The
device header compiled for the host (hipcc --cuda-host-only, no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_splat_fixed_matches_fp64(tmp_path):
    exe = str(tmp_path / "splat_fixed_check")
    subprocess.check_call([HIPCC, "-std=c++17", "-O1", "--cuda-host-only",
                           "-I" + os.path.join(ROOT, "first_raytracer_amd", "csrc"), "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "native", "splat_fixed_check.cpp"), "-o", exe])
    p = subprocess.run([exe, "257"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.strip().startswith("0 of")
