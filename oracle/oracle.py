"""ctypes front end of the CPU oracle (oracle/lsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  The product package (4dlangsplat_amd/) never imports it.

The oracle restates the rasterizer behind /root/reference/gaussian_renderer/__init__.py:219-228
(the un-vendored zrporz/4d-langsplat-rasterization).  PARITY UNPINNED against the CUDA original
(source absent, no reference tests); the SH / camera / covariance twins are pinned by golden
vectors from the reference's own Python (tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "build")


def build(force: bool = False) -> None:
    libs = [os.path.join(_BUILD, n) for n in ("liborc_f32.so", "liborc_f64.so", "liborc_f32_up.so")]
    src = os.path.join(_HERE, "lsr_oracle.c")
    if not force and all(os.path.exists(p) and os.path.getmtime(p) >= os.path.getmtime(src) for p in libs):
        return
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_LIBS: dict = {}


def _lib(double: bool, upstream: bool = False):
    """double: the fp64 build (libm exp); upstream: the float build with libm expf and fma
    contraction (liborc_f32_up.so, the stand-in for the CUDA original's rounding)."""
    key = "f64" if double else ("f32_up" if upstream else "f32")
    if key not in _LIBS:
        build()
        lib = ctypes.CDLL(os.path.join(_BUILD, f"liborc_{key}.so"))
        lib.orc_forward.restype = ctypes.c_void_p
        lib.orc_num_rendered.restype = ctypes.c_int64
        lib.orc_num_rendered.argtypes = [ctypes.c_void_p]
        lib.orc_free.argtypes = [ctypes.c_void_p]
        lib.orc_real_size.restype = ctypes.c_int
        _LIBS[key] = lib
    return _LIBS[key]


def _real_t(double):
    return ctypes.c_double if double else ctypes.c_float


def _settings_struct(double):
    rt = _real_t(double)

    class S(ctypes.Structure):
        _fields_ = [
            ("H", ctypes.c_int), ("W", ctypes.c_int),
            ("tanfovx", rt), ("tanfovy", rt),
            ("bg", rt * 3), ("scale_modifier", rt),
            ("view", rt * 16), ("proj", rt * 16),
            ("sh_degree", ctypes.c_int), ("campos", rt * 3),
            ("include_feature", ctypes.c_int),
        ]
    return S


@dataclass
class OracleSettings:
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: np.ndarray          # [3]
    scale_modifier: float
    viewmatrix: np.ndarray  # [4,4] (world_view_transform, row-vector convention)
    projmatrix: np.ndarray  # [4,4] (full_proj_transform)
    sh_degree: int
    campos: np.ndarray      # [3]
    include_feature: bool = True

    def to_c(self, double):
        S = _settings_struct(double)
        s = S()
        s.H, s.W = int(self.image_height), int(self.image_width)
        s.tanfovx, s.tanfovy = float(self.tanfovx), float(self.tanfovy)
        for i in range(3):
            s.bg[i] = float(np.asarray(self.bg).reshape(-1)[i])
            s.campos[i] = float(np.asarray(self.campos).reshape(-1)[i])
        s.scale_modifier = float(self.scale_modifier)
        v = np.asarray(self.viewmatrix, dtype=np.float64).reshape(-1)
        p = np.asarray(self.projmatrix, dtype=np.float64).reshape(-1)
        for i in range(16):
            s.view[i] = float(v[i])
            s.proj[i] = float(p[i])
        s.sh_degree = int(self.sh_degree)
        s.include_feature = int(bool(self.include_feature))
        return s


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _arr(x, dt, shape=None):
    if x is None:
        return None
    a = np.ascontiguousarray(np.asarray(x), dtype=dt)
    if shape is not None:
        a = a.reshape(shape)
    return a


class OracleResult:
    """Forward outputs + the intermediate state kept for backward (like the upstream byte buffers)."""

    def __init__(self, lib, handle, double, settings, P, M, C, inputs, outs):
        self._lib, self._h, self.double = lib, handle, double
        self.settings, self.P, self.M, self.C = settings, P, M, C
        self.inputs = inputs
        self.color, self.lang, self.depth, self.radii = outs
        self.num_rendered = int(lib.orc_num_rendered(handle))
        self._state = None

    def state(self):
        if self._state is None:
            dt = np.float64 if self.double else np.float32
            P, H, W = self.P, self.settings.image_height, self.settings.image_width
            nt = ((W + 15) // 16) * ((H + 15) // 16)
            K = self.num_rendered
            st = dict(xy=np.zeros((P, 2), dt), depth=np.zeros(P, dt), conic_o=np.zeros((P, 4), dt),
                      rgb=np.zeros((P, 3), dt), clamped=np.zeros((P, 3), np.uint8),
                      tiles=np.zeros(P, np.uint32), point_list=np.zeros(max(K, 1), np.uint32),
                      ranges=np.zeros((nt, 2), np.uint32), final_T=np.zeros((H, W), dt),
                      n_contrib=np.zeros((H, W), np.uint32))
            self._lib.orc_copy_state(ctypes.c_void_p(self._h), *[_ptr(st[k]) for k in (
                "xy", "depth", "conic_o", "rgb", "clamped", "tiles", "point_list", "ranges",
                "final_T", "n_contrib")])
            st["point_list"] = st["point_list"][:K]
            self._state = st
        return self._state

    def backward(self, dL_dcolor, dL_dlang=None, dL_ddepth=None, nthreads=0, abs_terms=False):
        """abs_terms: the directly accumulated outputs (lang, opacity, means2D) hold the sums of the
        absolute per-pixel terms instead (orc_set_abs_terms: each element's rounding-error scale);
        the other outputs are then meaningless."""
        self._lib.orc_set_abs_terms(ctypes.c_int(1 if abs_terms else 0))
        try:
            return self._backward(dL_dcolor, dL_dlang, dL_ddepth, nthreads)
        finally:
            self._lib.orc_set_abs_terms(ctypes.c_int(0))

    def _backward(self, dL_dcolor, dL_dlang=None, dL_ddepth=None, nthreads=0):
        dt = np.float64 if self.double else np.float32
        P, M, C = self.P, self.M, self.C
        H, W = self.settings.image_height, self.settings.image_width
        inp = self.inputs
        g_color = _arr(dL_dcolor, dt, (3, H, W))
        g_lang = _arr(dL_dlang, dt, (C, H, W)) if (dL_dlang is not None and C > 0) else (np.zeros((max(C, 1), H, W), dt))
        g_depth = _arr(dL_ddepth, dt, (H, W)) if dL_ddepth is not None else None
        out = dict(means3D=np.zeros((P, 3), dt), means2D=np.zeros((P, 3), dt), colors=np.zeros((P, 3), dt),
                   lang=np.zeros((P, max(C, 1)), dt), opacity=np.zeros((P, 1), dt), cov3D=np.zeros((P, 6), dt),
                   sh=np.zeros((P, max(M, 1), 3), dt), scales=np.zeros((P, 3), dt), rotations=np.zeros((P, 4), dt))
        s = self.settings.to_c(self.double)
        self._lib.orc_backward(
            ctypes.c_void_p(self._h), ctypes.byref(s),
            _ptr(inp["means3D"]), _ptr(inp["shs"]), _ptr(inp["colors_precomp"]), _ptr(inp["lang"]),
            _ptr(inp["opacities"]), _ptr(inp["scales"]), _ptr(inp["rotations"]), _ptr(inp["cov3D_precomp"]),
            _ptr(g_color), _ptr(g_lang), _ptr(g_depth),
            _ptr(out["means3D"]), _ptr(out["means2D"]), _ptr(out["colors"]), _ptr(out["lang"]),
            _ptr(out["opacity"]), _ptr(out["cov3D"]), _ptr(out["sh"] if M > 0 else None),
            _ptr(out["scales"]), _ptr(out["rotations"]), ctypes.c_int(nthreads))
        if C == 0:
            out["lang"] = out["lang"][:, :0]
        return out

    def close(self):
        if self._h:
            self._lib.orc_free(ctypes.c_void_p(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def forward(settings: OracleSettings, means3D, opacities, shs=None, colors_precomp=None, lang=None,
            scales=None, rotations=None, cov3D_precomp=None, double=False, nthreads=0,
            upstream_arith=False) -> OracleResult:
    """Restated forward.  Inputs are numpy (or anything np.asarray accepts); activated values,
    exactly what GaussianRasterizer receives (gaussian_renderer/__init__.py:191-228).
    upstream_arith: float build with libm expf + fma contraction instead of the reproducible
    orc_exp / orc_power (drift bound tests only; the parity checks use the default build)."""
    lib = _lib(double, upstream_arith and not double)
    dt = np.float64 if double else np.float32
    means3D = _arr(means3D, dt, (-1, 3))
    P = means3D.shape[0]
    opacities = _arr(opacities, dt, (P,))
    shs = _arr(shs, dt)
    M = 0
    if shs is not None:
        shs = shs.reshape(P, -1, 3)
        M = shs.shape[1]
    colors_precomp = _arr(colors_precomp, dt, (P, 3)) if colors_precomp is not None else None
    if lang is not None and np.asarray(lang).size > 0:
        lang = _arr(lang, dt).reshape(P, -1)
        C = lang.shape[1]
    else:
        lang, C = None, 0
    scales = _arr(scales, dt, (P, 3)) if scales is not None else None
    rotations = _arr(rotations, dt, (P, 4)) if rotations is not None else None
    cov3D_precomp = _arr(cov3D_precomp, dt, (P, 6)) if cov3D_precomp is not None else None
    H, W = settings.image_height, settings.image_width
    color = np.zeros((3, H, W), dt)
    lang_out = np.zeros((C, H, W), dt)
    depth = np.zeros((1, H, W), dt)
    radii = np.zeros(P, np.int32)
    s = settings.to_c(double)
    h = lib.orc_forward(ctypes.byref(s), ctypes.c_int(P), ctypes.c_int(M), ctypes.c_int(C),
                        _ptr(means3D), _ptr(shs), _ptr(colors_precomp), _ptr(lang), _ptr(opacities),
                        _ptr(scales), _ptr(rotations), _ptr(cov3D_precomp),
                        _ptr(color), _ptr(lang_out) if C > 0 else None, _ptr(depth), _ptr(radii),
                        ctypes.c_int(nthreads))
    inputs = dict(means3D=means3D, shs=shs, colors_precomp=colors_precomp, lang=lang, opacities=opacities,
                  scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp)
    return OracleResult(lib, h, double, settings, P, M, C, inputs, (color, lang_out, depth, radii))


def sh_colors(deg, sh, pos, campos, double=False):
    lib = _lib(double)
    dt = np.float64 if double else np.float32
    pos = _arr(pos, dt, (-1, 3))
    N = pos.shape[0]
    sh = _arr(sh, dt).reshape(N, -1, 3)
    M = sh.shape[1]
    campos = _arr(campos, dt, (3,))
    rgb = np.zeros((N, 3), dt)
    clamped = np.zeros((N, 3), np.uint8)
    lib.orc_sh_colors(ctypes.c_int(N), ctypes.c_int(deg), ctypes.c_int(M), _ptr(pos), _ptr(campos), _ptr(sh),
                      _ptr(rgb), _ptr(clamped))
    return rgb, clamped


def cov3d(scales, rotations, mod=1.0, double=False):
    lib = _lib(double)
    dt = np.float64 if double else np.float32
    scales = _arr(scales, dt, (-1, 3))
    N = scales.shape[0]
    rotations = _arr(rotations, dt, (N, 4))
    cov = np.zeros((N, 6), dt)
    lib.orc_cov3d(ctypes.c_int(N), _ptr(scales), (ctypes.c_double if double else ctypes.c_float)(mod),
                  _ptr(rotations), _ptr(cov))
    return cov


def mark_visible(means3D, viewmatrix, double=False):
    lib = _lib(double)
    dt = np.float64 if double else np.float32
    means3D = _arr(means3D, dt, (-1, 3))
    view = _arr(viewmatrix, dt, (16,))
    out = np.zeros(means3D.shape[0], np.uint8)
    lib.orc_mark_visible(ctypes.c_int(means3D.shape[0]), _ptr(means3D), _ptr(view), _ptr(out))
    return out.astype(bool)
