"""ctypes binding of liblsr.so (include/lsr.h).  No torch types cross the boundary: only device
pointers, sizes and the HIP stream handle.

The library is built in-tree (4dlangsplat_amd/csrc/Makefile -> 4dlangsplat_amd/build/liblsr.so).
There is no fallback: if the library is missing, importing the rasterizer raises.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("LSR_LIBRARY", os.path.join(_PKG, "build", "liblsr.so"))

c_float_p = ctypes.c_void_p  # device pointers are passed as opaque addresses
API_VERSION = 4               # LSR_API_VERSION of the include/lsr.h these structs mirror
DEFORM_API_VERSION = 3        # LSR_DEFORM_API_VERSION of include/lsr_deform.h (DeformNet, DeformGrads)


class Settings(ctypes.Structure):
    _fields_ = [
        ("image_height", ctypes.c_int32), ("image_width", ctypes.c_int32),
        ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
        ("bg", ctypes.c_void_p), ("scale_modifier", ctypes.c_float),
        ("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p),
        ("sh_degree", ctypes.c_int32), ("campos", ctypes.c_void_p),
        ("prefiltered", ctypes.c_int32), ("debug", ctypes.c_int32), ("include_feature", ctypes.c_int32),
    ]


class FwdIn(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int32), ("M", ctypes.c_int32), ("C", ctypes.c_int32),
        ("means3D", ctypes.c_void_p), ("shs", ctypes.c_void_p), ("colors_precomp", ctypes.c_void_p),
        ("language_feature", ctypes.c_void_p), ("opacities", ctypes.c_void_p), ("scales", ctypes.c_void_p),
        ("rotations", ctypes.c_void_p), ("cov3D_precomp", ctypes.c_void_p),
        ("language_feature_split", ctypes.c_void_p),
    ]


class FwdOut(ctypes.Structure):
    _fields_ = [("out_color", ctypes.c_void_p), ("out_language_feature", ctypes.c_void_p),
                ("radii", ctypes.c_void_p), ("out_depth", ctypes.c_void_p)]


class BwdIn(ctypes.Structure):
    _fields_ = [("dL_dout_color", ctypes.c_void_p), ("dL_dout_language_feature", ctypes.c_void_p),
                ("dL_dout_depth", ctypes.c_void_p), ("deterministic", ctypes.c_int32)]


class BwdOut(ctypes.Structure):
    _fields_ = [("dL_dmeans3D", ctypes.c_void_p), ("dL_dmeans2D", ctypes.c_void_p), ("dL_dcolors", ctypes.c_void_p),
                ("dL_dlanguage_feature", ctypes.c_void_p), ("dL_dopacity", ctypes.c_void_p),
                ("dL_dcov3D", ctypes.c_void_p), ("dL_dsh", ctypes.c_void_p), ("dL_dscales", ctypes.c_void_p),
                ("dL_drotations", ctypes.c_void_p)]


# every symbol include/lsr.h declares, with its ctypes signature
class DeformNet(ctypes.Structure):
    """include/lsr_deform.h lsr_deform_net (LSR_DEFORM_API_VERSION 3)"""
    _fields_ = [("n_scales", ctypes.c_int32), ("channels", ctypes.c_int32), ("width", ctypes.c_int32),
                ("res", ctypes.c_int32 * 4), ("multires", ctypes.c_int32 * 4), ("depth", ctypes.c_int32),
                ("heads", ctypes.c_uint32), ("apply_rotation", ctypes.c_int32), ("lang_mode", ctypes.c_int32),
                ("lang_dim", ctypes.c_int32), ("centers", ctypes.c_int32), ("time_pe", ctypes.c_int32),
                ("aabb", ctypes.c_void_p), ("planes", (ctypes.c_void_p * 6) * 4),
                ("w_feat", ctypes.c_void_p * 4), ("b_feat", ctypes.c_void_p * 4),
                ("w1", ctypes.c_void_p * 6), ("b1", ctypes.c_void_p * 6), ("w2", ctypes.c_void_p * 6),
                ("b2", ctypes.c_void_p * 6), ("w_lang", ctypes.c_void_p * 3), ("b_lang", ctypes.c_void_p * 3)]


class DeformGrads(ctypes.Structure):
    """include/lsr_deform.h lsr_deform_grads"""
    _fields_ = [("planes", (ctypes.c_void_p * 6) * 4), ("w_feat", ctypes.c_void_p * 4), ("b_feat", ctypes.c_void_p * 4),
                ("w1", ctypes.c_void_p * 6), ("b1", ctypes.c_void_p * 6), ("w2", ctypes.c_void_p * 6),
                ("b2", ctypes.c_void_p * 6), ("w_lang", ctypes.c_void_p * 3), ("b_lang", ctypes.c_void_p * 3),
                ("aabb", ctypes.c_void_p)]


class AdamGroup(ctypes.Structure):
    """include/lsr_train.h lsr_adam_group"""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_int64), ("lr", ctypes.c_double),
                ("step", ctypes.c_int64)]


class RowTensor(ctypes.Structure):
    """include/lsr_train.h lsr_row_tensor"""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("row_bytes", ctypes.c_int64),
                ("zero_from", ctypes.c_int64)]


ADAM_MAX_GROUPS = 16        # LSR_ADAM_MAX_GROUPS
GATHER_MAX_TENSORS = 32     # LSR_GATHER_MAX_TENSORS

_vp = ctypes.c_void_p
SIGNATURES = {
    "lsr_adam_step": (ctypes.c_int, [ctypes.POINTER(AdamGroup), ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, _vp]),
    "lsr_densify_stats": (ctypes.c_int, [ctypes.c_int32, _vp, _vp, ctypes.c_int32, _vp, _vp, _vp, _vp]),
    "lsr_train_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32]),
    "lsr_densify_plan": (ctypes.c_int, [ctypes.c_int32, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_int32, _vp, _vp, _vp, _vp]),
    "lsr_prune_plan": (ctypes.c_int, [ctypes.c_int32, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                      _vp, _vp, _vp, _vp]),
    "lsr_gather_rows": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(RowTensor), _vp, ctypes.c_int64, _vp]),
    "lsr_split_fixup": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp]),
    "lsr_reset_opacity": (ctypes.c_int, [ctypes.c_int32, _vp, _vp, _vp, _vp]),
    "lsr_activate": (ctypes.c_int, [ctypes.c_int32] + [_vp] * 7),
    "lsr_l1_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32]),
    "lsr_l1_loss_views": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, _vp, _vp, ctypes.c_int64, _vp, _vp, _vp]),
    "lsr_l1_loss_views_backward": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, _vp, _vp, ctypes.c_int64, _vp, _vp,
                                                  _vp]),
    "lsr_repeat_rows": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(RowTensor), ctypes.c_int64, ctypes.c_int32, _vp]),
    "lsr_sum_row_blocks": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(RowTensor), ctypes.c_int64, ctypes.c_int32,
                                          _vp]),
    "lsr_activate_backward": (ctypes.c_int, [ctypes.c_int32] + [_vp] * 10),
    "lsr_version": (ctypes.c_int, []),
    "lsr_require_api": (ctypes.c_int, [ctypes.c_int32]),
    "lsr_deform_require_api": (ctypes.c_int, [ctypes.c_int32]),
    "lsr_last_error": (ctypes.c_char_p, []),
    "lsr_geom_bytes": (ctypes.c_int64, [ctypes.c_int32]),
    "lsr_binning_bytes": (ctypes.c_int64, [ctypes.c_int64]),
    "lsr_img_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "lsr_backward_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "lsr_forward_preprocess": (ctypes.c_int, [ctypes.POINTER(Settings), ctypes.POINTER(FwdIn), ctypes.POINTER(FwdOut),
                                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "lsr_forward_preprocess_async": (ctypes.c_int, [ctypes.POINTER(Settings), ctypes.POINTER(FwdIn),
                                                    ctypes.POINTER(FwdOut), ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p]),
    "lsr_forward_preprocess_views_async": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                          ctypes.POINTER(FwdIn), ctypes.POINTER(ctypes.POINTER(FwdOut)),
                                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                                          ctypes.c_void_p]),
    "lsr_forward_preprocess_views_split_async": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32,
                                                                ctypes.POINTER(ctypes.POINTER(Settings)),
                                                                ctypes.POINTER(FwdIn),
                                                                ctypes.POINTER(ctypes.POINTER(FwdOut)),
                                                                ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                                                ctypes.c_void_p]),
    "lsr_forward_preprocess_views_rows_async": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                               ctypes.POINTER(ctypes.POINTER(Settings)),
                                                               ctypes.POINTER(FwdIn),
                                                               ctypes.POINTER(ctypes.POINTER(FwdOut)),
                                                               ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "lsr_forward_depth_order_views_async": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                           ctypes.POINTER(FwdIn), ctypes.POINTER(ctypes.c_void_p),
                                                           ctypes.c_void_p, ctypes.c_void_p]),
    "lsr_forward_binning_views": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                 ctypes.POINTER(FwdIn), ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "lsr_binning_bytes_tb": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "lsr_forward_preprocess_views_tb_async": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                             ctypes.POINTER(ctypes.POINTER(Settings)),
                                                             ctypes.POINTER(FwdIn),
                                                             ctypes.POINTER(ctypes.POINTER(FwdOut)),
                                                             ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "lsr_forward_instance_scan_views_async": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                             ctypes.POINTER(FwdIn), ctypes.POINTER(ctypes.c_void_p),
                                                             ctypes.c_void_p, ctypes.c_void_p]),
    "lsr_forward_binning_views_tb": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                    ctypes.POINTER(FwdIn), ctypes.POINTER(ctypes.c_void_p),
                                                    ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                                    ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "lsr_forward_render": (ctypes.c_int, [ctypes.POINTER(Settings), ctypes.POINTER(FwdIn), ctypes.POINTER(FwdOut),
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p]),
    "lsr_forward_binning": (ctypes.c_int, [ctypes.POINTER(Settings), ctypes.POINTER(FwdIn), ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "lsr_forward_composite": (ctypes.c_int, [ctypes.POINTER(Settings), ctypes.POINTER(FwdIn), ctypes.POINTER(FwdOut),
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_void_p]),
    "lsr_forward_composite_views": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                   ctypes.POINTER(FwdIn), ctypes.POINTER(ctypes.POINTER(FwdOut)),
                                                   ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                                   ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                                                   ctypes.c_void_p]),
    "lsr_backward_composite_views": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                    ctypes.POINTER(FwdIn), ctypes.POINTER(ctypes.POINTER(BwdIn)),
                                                    ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                                    ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                                    ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "lsr_backward": (ctypes.c_int, [ctypes.POINTER(Settings), ctypes.POINTER(FwdIn), ctypes.POINTER(BwdIn),
                                    ctypes.POINTER(BwdOut), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]),
    "lsr_backward_views": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)), ctypes.POINTER(FwdIn),
                                          ctypes.POINTER(ctypes.POINTER(BwdIn)), ctypes.POINTER(BwdOut),
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                                          ctypes.c_int32, ctypes.c_void_p]),
    "lsr_backward_composite": (ctypes.c_int, [ctypes.POINTER(Settings), ctypes.POINTER(FwdIn), ctypes.POINTER(BwdIn),
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int64, ctypes.c_void_p]),
    "lsr_backward_preprocess_views": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                     ctypes.POINTER(FwdIn), ctypes.POINTER(BwdOut),
                                                     ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, ctypes.c_void_p]),
    "lsr_backward_preprocess_views_rows": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Settings)),
                                                          ctypes.POINTER(FwdIn), ctypes.POINTER(BwdOut),
                                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32,
                                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    "lsr_language_split": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "lsr_radii_max": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                     ctypes.c_int32, ctypes.c_void_p]),
    "lsr_mark_visible": (ctypes.c_int, [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "lsr_profile_enable": (ctypes.c_int, [ctypes.c_int32]),
    "lsr_profile_phases": (ctypes.c_int, [ctypes.c_uint32]),
    "lsr_knn_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32]),
    "lsr_knn_mean_dist": (ctypes.c_int, [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "lsr_deform_workspace_bytes": (ctypes.c_int64, [ctypes.POINTER(DeformNet)]),
    "lsr_deform_prepare": (ctypes.c_int, [ctypes.POINTER(DeformNet), ctypes.c_void_p, ctypes.c_void_p]),
    "lsr_deform_forward": (ctypes.c_int, [ctypes.POINTER(DeformNet), ctypes.c_void_p, ctypes.c_int32]
                           + [ctypes.c_void_p] * 14 + [ctypes.c_void_p]),
    "lsr_deform_backward_scratch_bytes": (ctypes.c_int64, [ctypes.POINTER(DeformNet), ctypes.c_int32]),
    "lsr_deform_backward": (ctypes.c_int, [ctypes.POINTER(DeformNet), ctypes.c_void_p, ctypes.c_int32]
                            + [ctypes.c_void_p] * 14 + [ctypes.POINTER(DeformGrads), ctypes.c_void_p, ctypes.c_void_p]),
    "lsr_profile_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.c_int32]),
}

PHASES = ["preprocess", "depth_sort", "instance_scan", "emit", "tile_sort", "tile_ranges", "render_fwd",
          "render_bwd", "preprocess_bwd", "preprocess_bwd_views"]


def profile_enable(on=True, phases=None):
    """Start (resetting the totals) or stop event timing; `phases` limits it to those names."""
    L = load()
    L.lsr_profile_phases(0xFFFFFFFF if phases is None else sum(1 << PHASES.index(p) for p in phases))
    L.lsr_profile_enable(1 if on else 0)


def profile_read():
    """{phase: (total_ms, launches)} of the event-timed phases since profile_enable()."""
    n = len(PHASES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    load().lsr_profile_read(ms, cnt, n)
    return {PHASES[i]: (ms[i], cnt[i]) for i in range(n)}

_LIB = None


def load():
    """Load liblsr.so (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        path = os.environ.get("LSR_LIBRARY", LIB_PATH)   # variant builds for profiling experiments
        if not os.path.exists(path):
            raise ImportError(f"liblsr.so not found at {LIB_PATH}; build it with `make -C 4dlangsplat_amd/csrc` "
                              "(or __graft_entry__.build()).  There is no CPU fallback.")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.lsr_require_api(API_VERSION) != 0 or lib.lsr_deform_require_api(DEFORM_API_VERSION) != 0:
            raise ImportError(f"{path}: {lib.lsr_last_error().decode()} (rebuild it: make -C 4dlangsplat_amd/csrc)")
        _LIB = lib
    return _LIB


def check(rc: int, what: str):
    if rc != 0:
        msg = load().lsr_last_error()
        raise RuntimeError(f"{what} failed (code {rc}): {msg.decode() if msg else ''}")
