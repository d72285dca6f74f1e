"""Regression check for stale LDS reads in the deformation kernels.

Round 3 saw a two-waves-per-SIMD build of the deformation backward produce a few wrong dX rows in
blocks dispatched after an earlier block had run on the same CU -- the signature of a read of shared
memory the block never wrote.  build/variants/liblsr_ldspoison.so is this library with every
deformation kernel filling its LDS with NaN words at block entry (-DLSR_LDS_POISON, csrc/Makefile).
Under it, the deformation parity tests (tests/test_deform_gpu.py: Neu3D-resolution forward and
backward against the float64 oracle, every reference variant against the reference's own outputs and
gradients) must still pass, and a 60k-Gaussian backward (over 900 blocks: many second-residency
blocks per CU) must match the oracle on every row and repeat bit for bit (tools/deform_race.py).
Each runs in a child process, because the library is chosen when it is first loaded."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "4dlangsplat_amd", "build", "variants", "liblsr_ldspoison.so")


def _env():
    assert os.path.exists(LIB), "build the library first (make -C 4dlangsplat_amd/csrc builds the poison variant)"
    return dict(os.environ, LSR_LIBRARY=LIB, PYTHONUNBUFFERED="1")


def test_deform_parity_under_lds_poison():
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
                        "--timeout", "200", "--timeout-method", "thread", "tests/test_deform_gpu.py"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]


def test_deform_backward_many_blocks_under_lds_poison():
    r = subprocess.run([sys.executable, os.path.join("tools", "deform_race.py"), "60000", "3"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=400)
    out = r.stdout
    assert r.returncode == 0, out[-3000:] + r.stderr[-2000:]
    runs = [line for line in out.splitlines() if line.startswith("run ") and "d_means3D" in line]
    assert len(runs) == 3, out[-3000:]
    assert "DIFFERS" not in out, out[-3000:]
    for line in runs:
        assert "(bad rows 0:" in line and "nan" not in line.lower(), line
