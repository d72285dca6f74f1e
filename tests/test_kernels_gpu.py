"""Unit checks of device building blocks on exact integer data (GPU)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_wave_transpose_reduce(tmp_path):
    src = os.path.join(ROOT, "tests", "kernels", "t_transpose_reduce.hip")
    exe = str(tmp_path / "t_tr")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-o", exe, src], check=True)
    r = subprocess.run(["timeout", "-k", "5", "60", exe], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_mfma_bf16_layout(tmp_path):
    src = os.path.join(ROOT, "tests", "kernels", "t_mfma_layout.hip")
    exe = str(tmp_path / "t_mfma")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-o", exe, src], check=True)
    r = subprocess.run(["timeout", "-k", "5", "60", exe], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_mfma16_helpers(tmp_path):
    """16x16x32 bf16 MFMA lane maps, the lane-group transpose and ds_read_tr16 (lsr_mfma.h)."""
    src = os.path.join(ROOT, "tests", "kernels", "t_mfma16.hip")
    exe = str(tmp_path / "t_mfma16")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-o", exe, src], check=True)
    r = subprocess.run(["timeout", "-k", "5", "60", exe], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_radix_sort(tmp_path):
    """Stable device radix sort (sort.hip) vs std::stable_sort at the binning's shapes."""
    src = os.path.join(ROOT, "tests", "kernels", "t_sort.hip")
    exe = str(tmp_path / "t_sort")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-I", os.path.join(ROOT, "4dlangsplat_amd", "csrc"), "-o", exe, src], check=True)
    r = subprocess.run(["timeout", "-k", "5", "120", exe], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_lds_dma_row_gather(tmp_path):
    """LDS-DMA (global_load_lds, 16 B per lane) row gather as the forward compositor's staged
    variant uses it: lane-linear LDS image, per-lane source rows."""
    src = os.path.join(ROOT, "tests", "kernels", "t_glds.hip")
    exe = str(tmp_path / "t_glds")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-o", exe, src], check=True)
    r = subprocess.run(["timeout", "-k", "5", "60", exe], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_packed_fp32_coresident(tmp_path):
    """The deformation backward's SLP-formed packed-fp32 sequence (a broadcast v_pk_mul_f32 with op_sel
    read by the next instruction with no wait state) run at 1, 2 and 4 blocks per CU,
    against exact host products; the printed counts say whether the back-to-back form reproduces the
    lanes-48..63 low-half corruption.  The forms this build relies on (scalar chains, packed ops with
    a wait state) must be exact."""
    src = os.path.join(ROOT, "tests", "kernels", "t_pk_coresident.hip")
    exe = str(tmp_path / "t_pk")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-o", exe, src], check=True)
    r = subprocess.run(["timeout", "-k", "5", "90", exe, "10"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_waitcnt_forcezero_hazard(tmp_path):
    """DESIGN.md 4.5, the -amdgpu-waitcnt-forcezero fault: the same division / sqrt fix-up patterns
    (VALU writes a lane mask -> v_cndmask reads it), built as the library is (the hazard recognizer's
    s_nop wait states) and with the debug flag (whose inserted s_waitcnt the recognizer counts as wait
    states and drops the s_nop).  The library build must be exact; the flag build's count is reported:
    wrong quotients there mean an s_waitcnt with nothing outstanding supplies no wait state, so that
    flag's code under-pads the hazards (in k_pack_weight the quotient is a row index: an out-of-range
    store, the illegal address)."""
    src = os.path.join(ROOT, "tests", "kernels", "t_waitcnt_hazard.hip")
    res = {}
    for name, extra in (("plain", []), ("forcezero", ["-mllvm", "-amdgpu-waitcnt-forcezero"])):
        exe = str(tmp_path / f"t_wc_{name}")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fhip-fp32-correctly-rounded-divide-sqrt", *extra,
                        "-o", exe, src], check=True)
        r = subprocess.run(["timeout", "-k", "5", "60", exe], capture_output=True, text=True)
        print(name, r.returncode, r.stdout)
        assert r.returncode in (0, 1), r.stdout + r.stderr      # 1 = wrong values (reported), never a fault
        res[name] = r.returncode
    assert res["plain"] == 0
