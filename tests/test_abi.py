"""CPU checks of the C ABI: liblsr.so builds for gfx950, loads, and exports exactly what
include/*.h declare; the workspace size queries behave (no GPU compute is called here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include"))) if h.endswith(".h")]


def declared():
    txt = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*(lsr_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for n in ("lsr_forward_preprocess", "lsr_forward_render", "lsr_backward", "lsr_mark_visible",
              "lsr_geom_bytes", "lsr_binning_bytes", "lsr_img_bytes", "lsr_backward_bytes", "lsr_last_error",
              "lsr_version"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from diff_gaussian_rasterization import _lib
    lib = _lib.load()
    for n in declared():
        assert hasattr(lib, n), n
    assert set(declared()) == set(_lib.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (lsr_\w+)", out))
    assert exported == set(declared())


def test_library_has_no_undefined_internal_symbols():
    """Every kernel launch stub the library references is defined in it (a template kernel whose
    host-side instantiation is dropped leaves an undefined __device_stub__ that only fails at
    load time on the GPU box)."""
    from diff_gaussian_rasterization import _lib
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert not [l for l in out.splitlines() if "lsr" in l], out


def test_library_is_built_for_gfx950():
    from diff_gaussian_rasterization import _lib
    out = subprocess.run(["strings", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_size_queries():
    from diff_gaussian_rasterization import _lib
    lib = _lib.load()
    assert lib.lsr_version() == _lib.API_VERSION == 4
    g1, g2 = lib.lsr_geom_bytes(1000), lib.lsr_geom_bytes(2_000_000)
    assert 0 < g1 < g2 and g2 >= 2_000_000 * 60
    assert lib.lsr_binning_bytes(8_600_000) >= 8_600_000 * 16
    assert lib.lsr_img_bytes(1352, 1014) >= 1352 * 1014 * 8
    assert lib.lsr_backward_bytes(2_000_000, 8_600_000, 32, 0) >= 2_000_000 * 48
    assert lib.lsr_backward_bytes(2_000_000, 8_600_000, 32, 1) >= 8_600_000 * 44 * 4
    # the tile-bucket binning: the sort path's layout (the compositors read its point list), then the
    # per-block tile count table and the long buckets' 8-byte merge workspace
    K, P, W, H = 8_600_000, 2_000_000, 1352, 1014
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    tb = lib.lsr_binning_bytes_tb(K, P, W, H)
    assert tb >= lib.lsr_binning_bytes(K) + 8 * K + 4 * tiles * (P // 16384)
    assert lib.lsr_binning_bytes_tb(K, 2 * P, W, H) > tb                  # more Gaussians: more table rows
    assert lib.lsr_binning_bytes_tb(K, P, 0, H) == -1                     # invalid image size


def test_train_glue_argument_checks():
    """The training-step glue (include/lsr_train.h: activations, view repeat / sum, the multi-view L1)
    refuses bad arguments with a message and accepts empty work, before anything touches a device."""
    import ctypes
    from diff_gaussian_rasterization import _lib
    lib = _lib.load()
    err = lambda: lib.lsr_last_error().decode()
    assert lib.lsr_l1_workspace_bytes(1) == 256 * 4 and lib.lsr_l1_workspace_bytes(8) == 8 * 256 * 4
    assert lib.lsr_l1_workspace_bytes(0) == 256 * 4
    p = ctypes.c_void_p(64)                                    # never dereferenced: every call below fails early
    imgs = (ctypes.c_void_p * 9)(*([64] * 9))
    for V, n, stride in ((0, 4, 4), (9, 4, 4), (2, -1, 4), (2, 8, 4)):
        assert lib.lsr_l1_loss_views(V, n, imgs, p, stride, p, p, None) != 0
        assert "1 <= V <= 8" in err()
    assert lib.lsr_l1_loss_views(2, 4, imgs, p, 4, None, p, None) != 0 and "workspace required" in err()
    assert lib.lsr_l1_loss_views_backward(2, 4, imgs, p, 4, None, imgs, None) != 0 and "d_loss" in err()
    holes = (ctypes.c_void_p * 2)(64, None)
    assert lib.lsr_l1_loss_views(2, 4, holes, p, 4, p, p, None) != 0 and "null image" in err()
    assert lib.lsr_l1_loss_views_backward(2, 4, imgs, p, 4, p, holes, None) != 0 and "null gradient" in err()
    assert lib.lsr_activate(-1, None, None, None, None, None, None, None) != 0 and "P >= 0" in err()
    assert lib.lsr_activate(4, p, None, None, None, None, None, None) != 0 and "needs its output" in err()
    assert lib.lsr_activate(4, None, ctypes.c_void_p(72), None, None, ctypes.c_void_p(64), None, None) != 0
    assert "16-byte aligned" in err()
    assert lib.lsr_activate(0, p, p, p, p, p, p, None) == 0    # no rows: no launch
    rt = (_lib.RowTensor * 1)()
    assert lib.lsr_repeat_rows(1, rt, 4, 0, None) != 0 and "n_blocks >= 1" in err()
    assert lib.lsr_sum_row_blocks(1, rt, 4, 2, None) != 0 and "rows of whole floats" in err()
    assert lib.lsr_repeat_rows(0, None, 4, 2, None) == 0 and lib.lsr_sum_row_blocks(1, rt, 0, 2, None) == 0


def test_settings_validation_messages():
    """Upstream's exactly-one-of errors are raised before anything touches a device."""
    import torch
    import diff_gaussian_rasterization as dgr
    rs = dgr.GaussianRasterizationSettings(8, 8, 0.5, 0.5, torch.ones(3), 1.0, torch.eye(4), torch.eye(4), 0,
                                           torch.zeros(3), False, False)
    assert rs.include_feature is True       # dataset_readers.py:502-515 builds it without the field
    r = dgr.GaussianRasterizer(rs)
    m = torch.zeros(4, 3)
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(means3D=m, means2D=m, opacities=torch.ones(4, 1), scales=m, rotations=torch.zeros(4, 4))
    with pytest.raises(Exception, match="exactly one of either scale/rotation pair"):
        r(means3D=m, means2D=m, opacities=torch.ones(4, 1), shs=torch.zeros(4, 16, 3))
    with pytest.raises(RuntimeError, match="GPU only"):
        r(means3D=m, means2D=m, opacities=torch.ones(4, 1), shs=torch.zeros(4, 16, 3), scales=m,
          rotations=torch.zeros(4, 4))


def test_callers_of_another_header_version_are_refused():
    """lsr_require_api: until a caller has declared the lsr.h version it was built against, every
    entry point that reads the structs refuses (no misread trailing fields); a mismatched
    declaration is refused too.  Fresh process: the handshake is per process."""
    import sys
    from diff_gaussian_rasterization import _lib
    code = f"""
import ctypes
L = ctypes.CDLL({_lib.LIB_PATH!r})
L.lsr_last_error.restype = ctypes.c_char_p
k = ctypes.c_int64(0)
rc = L.lsr_forward_preprocess(None, None, None, None, ctypes.byref(k), None)
assert rc == 1 and b"lsr_require_api" in L.lsr_last_error(), (rc, L.lsr_last_error())
assert L.lsr_require_api(3) == 1 and b"mismatch" in L.lsr_last_error()
rc = L.lsr_forward_preprocess(None, None, None, None, ctypes.byref(k), None)
assert rc == 1 and b"lsr_require_api" in L.lsr_last_error()
assert L.lsr_require_api(4) == 0
rc = L.lsr_forward_preprocess(None, None, None, None, ctypes.byref(k), None)
assert rc == 1 and b"null settings" in L.lsr_last_error(), L.lsr_last_error()
# lsr_deform.h has its own handshake (its structs gained a trailing field in version 3)
L.lsr_deform_workspace_bytes.restype = ctypes.c_int64
assert L.lsr_deform_workspace_bytes(None) == -1 and b"lsr_deform_require_api" in L.lsr_last_error()
assert L.lsr_deform_require_api(2) == 1 and b"mismatch" in L.lsr_last_error()
assert L.lsr_deform_workspace_bytes(None) == -1 and b"lsr_deform_require_api" in L.lsr_last_error()
assert L.lsr_deform_require_api(3) == 0
assert L.lsr_deform_workspace_bytes(None) == -1 and b"null deformation net" in L.lsr_last_error()
print("ok")
"""
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr


STRUCTS = {"Settings": "lsr_settings", "FwdIn": "lsr_fwd_in", "FwdOut": "lsr_fwd_out", "BwdIn": "lsr_bwd_in",
           "BwdOut": "lsr_bwd_out", "DeformNet": "lsr_deform_net", "DeformGrads": "lsr_deform_grads",
           "AdamGroup": "lsr_adam_group", "RowTensor": "lsr_row_tensor"}


def test_ctypes_structs_match_the_headers(tmp_path):
    """Every ctypes mirror of an include/*.h struct has the C compiler's field offsets and size
    (a duplicated or misplaced field in a mirror hands the library NULL or shifted pointers)."""
    from diff_gaussian_rasterization import _lib
    lines = ["#include <stddef.h>", "#include <stdio.h>"] + [f'#include "{h}"' for h in HEADERS] + ["int main(void) {"]
    want = {}
    for py, c in STRUCTS.items():
        cls = getattr(_lib, py)
        names = [f[0] for f in cls._fields_]
        assert len(names) == len(set(names)), f"{py}: duplicate fields"
        lines.append(f'printf("{py} size %zu\\n", sizeof({c}));')
        want[(py, "size")] = ctypes_sizeof(cls)
        for n in names:
            lines.append(f'printf("{py} {n} %zu\\n", offsetof({c}, {n}));')
            want[(py, n)] = getattr(cls, n).offset
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        py, n, v = line.split()
        got[(py, n)] = int(v)
    assert got == want


def ctypes_sizeof(cls):
    import ctypes
    return ctypes.sizeof(cls)
