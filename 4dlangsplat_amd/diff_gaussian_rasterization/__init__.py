"""diff_gaussian_rasterization -- drop-in Python surface of the 4D-LangSplat rasterizer, backed by
the MI355X-native liblsr.so (HIP, gfx950) through its C ABI (include/lsr.h).

Mirrors what the reference imports and calls (the submodule zrporz/4d-langsplat-rasterization is
un-vendored, so the surface is taken from its call sites):
  from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
      gaussian_renderer/__init__.py:15, scene/dataset_readers.py:492
  GaussianRasterizationSettings(image_height, image_width, tanfovx, tanfovy, bg, scale_modifier,
      viewmatrix, projmatrix, sh_degree, campos, prefiltered, debug, include_feature)
      gaussian_renderer/__init__.py:49-63 (include_feature defaults to True because
      scene/dataset_readers.py:502-515 builds the settings without it)
  rasterizer(means3D=, means2D=, shs=, colors_precomp=, language_feature_precomp=, opacities=,
      scales=, rotations=, cov3D_precomp=) -> (color [3,H,W], language_feature [C,H,W],
      radii int32 [P], depth [1,H,W])            gaussian_renderer/__init__.py:219-228
  rasterizer.markVisible(positions) -> bool [P]
Errors follow upstream: exactly one of shs / colors_precomp, exactly one of (scales, rotations) /
cov3D_precomp, else an Exception with the upstream message; native failures raise RuntimeError.
means2D's values are ignored; its .grad receives the screen-space gradient (NDC units).
"""
from __future__ import annotations

import ctypes
import functools
from typing import NamedTuple, Optional

import torch
import torch.nn as nn

from . import _lib

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "RasterizerState",
           "forward_native", "backward_native", "backward_views_native", "backward_composite_native",
           "backward_preprocess_views_native", "preprocess_views_native", "binning_views_native",
           "render_views_native", "backward_composite_views_native", "language_split_native", "rasterize_views",
           "radii_max_native"]

_lib.load()   # fail loudly at import if the native library is missing
_BINNING_DELAY_CYCLES = 0   # tests only: GPU cycles slept on the stream before a side-stream binning


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    include_feature: bool = True


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _opt(t):
    """upstream passes torch.Tensor([]) for 'not provided'"""
    if t is None or t.numel() == 0:
        return None
    return t


def _f32(t, device):
    return t.detach().to(device=device, dtype=torch.float32).contiguous()


class _NativeSettings:
    """Keeps the device copies of the small settings tensors alive for the duration of a call."""

    def __init__(self, rs: GaussianRasterizationSettings, device):
        self.bg = _f32(rs.bg, device).reshape(-1)
        self.view = _f32(rs.viewmatrix, device).reshape(-1)
        self.proj = _f32(rs.projmatrix, device).reshape(-1)
        self.campos = _f32(rs.campos, device).reshape(-1)
        if self.bg.numel() != 3 or self.view.numel() != 16 or self.proj.numel() != 16 or self.campos.numel() != 3:
            raise ValueError("bg/campos must have 3 elements and view/proj matrices 16")
        s = _lib.Settings()
        s.image_height, s.image_width = int(rs.image_height), int(rs.image_width)
        s.tanfovx, s.tanfovy = float(rs.tanfovx), float(rs.tanfovy)
        s.bg, s.scale_modifier = self.bg.data_ptr(), float(rs.scale_modifier)
        s.viewmatrix, s.projmatrix = self.view.data_ptr(), self.proj.data_ptr()
        s.sh_degree, s.campos = int(rs.sh_degree), self.campos.data_ptr()
        s.prefiltered, s.debug = int(bool(rs.prefiltered)), int(bool(rs.debug))
        s.include_feature = int(bool(rs.include_feature))
        self.c = s


class RasterizerState:
    """What the forward leaves for the backward (upstream: num_rendered + geom/binning/img buffers)."""

    def __init__(self, settings, inputs, fin, geom, binning, img, num_rendered, radii):
        self.settings, self.inputs, self.fin = settings, inputs, fin
        self.geom, self.binning, self.img = geom, binning, img
        self.num_rendered, self.radii = num_rendered, radii
        self.composited = False           # backward_composite_native ran (it may run once)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class PendingForward:
    """Phase 1 of a forward (preprocess, depth order, instance count) done; render_native finishes
    it.  Holds the inputs, the geom workspace and num_rendered (K)."""

    def __init__(self, raster_settings, settings, fin, inputs, geom, radii, K, device, H, W):
        self.raster_settings, self.settings, self.fin, self.inputs = raster_settings, settings, fin, inputs
        self.geom, self.radii, self.num_rendered, self.device, self.H, self.W = geom, radii, K, device, H, W
        self.binning = self.img = None     # set when the binning already ran (preprocess_native(binning=True))
        self.ready = None                  # event recorded after that binning
        self.ready_stream = None           # the stream `ready` was recorded on
        self.count_host = None             # deferred count (preprocess_native(defer_count=True)): pinned
        self.counted = None                # [K, reserved], valid once `counted` (an event) has passed
        self.stream = None
        self.count_batch = None            # (pinned [n, 2] counts of a batch, this view's row)
        self.tile_bucket = False           # phase 1 prepared the tile-bucket binning (id-order counts)

    def resolve(self, binning=False):
        """Deferred-count forwards: wait for the instance count (host waits on the event only, not
        the stream), then optionally enqueue the binning on the preprocess stream.  No-op otherwise."""
        if self.counted is None:
            return self
        self.counted.synchronize()
        self.counted = None
        self.num_rendered = int(self.count_host[0])
        if binning:
            _run_binning(self, self.stream)
        return self


def _dump_forward(raster_settings, inputs):
    if raster_settings.debug:
        torch.save({k: (None if v is None else v.cpu()) for k, v in inputs.items()
                    if k in ("means3D", "opacities", "shs", "colors_precomp", "scales", "rotations")},
                   "snapshot_fw.dump")
        print("\nAn error occured in forward. Writing snapshot_fw.dump for debugging.")


def _check_device(t):
    if t.device.type != "cuda":
        raise RuntimeError("the rasterizer runs on the GPU only (no CPU fallback); got tensors on " + str(t.device))
    return t.device


def _fwd_inputs(means3D, opacities, shs, colors_precomp, language_feature, scales, rotations, cov3D_precomp):
    """fp32 contiguous device inputs and their lsr_fwd_in; returns (fin, inputs, P)."""
    device = _check_device(means3D)
    P = means3D.shape[0]
    means3D = _f32(means3D, device)
    opacities = _f32(opacities, device)
    shs = _opt(shs)
    colors_precomp = _opt(colors_precomp)
    language_feature = _opt(language_feature)
    scales, rotations, cov3D_precomp = _opt(scales), _opt(rotations), _opt(cov3D_precomp)
    shs = _f32(shs, device) if shs is not None else None
    colors_precomp = _f32(colors_precomp, device) if colors_precomp is not None else None
    language_feature = _f32(language_feature, device).reshape(P, -1) if language_feature is not None else None
    scales = _f32(scales, device) if scales is not None else None
    rotations = _f32(rotations, device) if rotations is not None else None
    cov3D_precomp = _f32(cov3D_precomp, device) if cov3D_precomp is not None else None
    M = shs.reshape(P, -1, 3).shape[1] if shs is not None else 0
    C = language_feature.shape[1] if language_feature is not None else 0
    fin = _lib.FwdIn()
    fin.P, fin.M, fin.C = P, M, C
    fin.means3D, fin.shs, fin.colors_precomp = means3D.data_ptr(), _ptr(shs), _ptr(colors_precomp)
    fin.language_feature, fin.opacities = _ptr(language_feature), opacities.data_ptr()
    fin.scales, fin.rotations, fin.cov3D_precomp = _ptr(scales), _ptr(rotations), _ptr(cov3D_precomp)
    inputs = dict(means3D=means3D, opacities=opacities, shs=shs, colors_precomp=colors_precomp,
                  language_feature=language_feature, scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp)
    return fin, inputs, P


def preprocess_native(raster_settings, means3D, opacities, shs=None, colors_precomp=None, language_feature=None,
                      scales=None, rotations=None, cov3D_precomp=None, stream=None, binning=False,
                      defer_count=False):
    """Forward phase 1 through liblsr.so (lsr_forward_preprocess) on `stream` (a torch stream,
    default: the current one).  Synchronises that stream once to read num_rendered (as upstream).
    binning=True also runs the tile binning there (lsr_forward_binning), so that render_native
    only composites.  Workspaces are allocated on `stream`; render_native may run on another
    stream.

    defer_count=True (lsr_forward_preprocess_async) does not synchronise: the count lands in pinned
    host memory and PendingForward.resolve(binning) reads it later (render_native resolves too),
    so a caller can enqueue this view's preprocess ahead of another view's work on the same stream."""
    device = _check_device(means3D)
    L = _lib.load()
    stream = stream or torch.cuda.current_stream(device)
    st = _NativeSettings(raster_settings, device)
    fin, inputs, P = _fwd_inputs(means3D, opacities, shs, colors_precomp, language_feature, scales, rotations,
                                 cov3D_precomp)
    H, W = int(raster_settings.image_height), int(raster_settings.image_width)
    with torch.cuda.stream(stream):
        radii = torch.empty(P, dtype=torch.int32, device=device)
        geom = torch.empty(int(L.lsr_geom_bytes(P)), dtype=torch.uint8, device=device)
    fout = _lib.FwdOut()
    fout.radii = radii.data_ptr()
    if defer_count:
        count = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        try:
            _lib.check(L.lsr_forward_preprocess_async(ctypes.byref(st.c), ctypes.byref(fin), ctypes.byref(fout),
                                                      ctypes.c_void_p(geom.data_ptr()),
                                                      ctypes.c_void_p(count.data_ptr()),
                                                      ctypes.c_void_p(stream.cuda_stream)),
                       "lsr_forward_preprocess_async")
        except RuntimeError:
            _dump_forward(raster_settings, inputs)
            raise
        pf = PendingForward(raster_settings, st, fin, inputs, geom, radii, None, device, H, W)
        pf.count_host, pf.stream = count, stream
        pf.counted = torch.cuda.Event()
        pf.counted.record(stream)
        return pf
    K = ctypes.c_int64(0)
    try:
        _lib.check(L.lsr_forward_preprocess(ctypes.byref(st.c), ctypes.byref(fin), ctypes.byref(fout),
                                            ctypes.c_void_p(geom.data_ptr()), ctypes.byref(K),
                                            ctypes.c_void_p(stream.cuda_stream)), "lsr_forward_preprocess")
    except RuntimeError:
        _dump_forward(raster_settings, inputs)
        raise
    pf = PendingForward(raster_settings, st, fin, inputs, geom, radii, K.value, device, H, W)
    if binning:
        _run_binning(pf, stream)
    return pf


def _run_binning(pf, stream):
    """lsr_forward_binning of a preprocessed view on `stream`; render_native's stream waits for it."""
    L = _lib.load()
    device, H, W, K = pf.device, pf.H, pf.W, pf.num_rendered
    if _BINNING_DELAY_CYCLES:             # test hook: holds the binning back to expose missing waits
        with torch.cuda.stream(stream):
            torch.cuda._sleep(_BINNING_DELAY_CYCLES)
    with torch.cuda.stream(stream):
        pf.binning = torch.empty(int(L.lsr_binning_bytes(K)), dtype=torch.uint8, device=device)
        pf.img = torch.empty(int(L.lsr_img_bytes(W, H)), dtype=torch.uint8, device=device)
    try:
        _lib.check(L.lsr_forward_binning(ctypes.byref(pf.settings.c), ctypes.byref(pf.fin),
                                         ctypes.c_void_p(pf.geom.data_ptr()), ctypes.c_void_p(pf.binning.data_ptr()),
                                         ctypes.c_void_p(pf.img.data_ptr()), ctypes.c_int64(K),
                                         ctypes.c_void_p(stream.cuda_stream)), "lsr_forward_binning")
    except RuntimeError:
        _dump_forward(pf.raster_settings, pf.inputs)
        raise
    pf.ready = torch.cuda.Event()
    pf.ready.record(stream)               # render_native's stream waits for the binning
    pf.ready_stream = stream


def language_split_native(language_feature, stream=None, out=None):
    """lsr_language_split: [P,32] fp32 -> [P,64] int16 holding the bf16 bit patterns (hi channels,
    then lo) that the compositors' matrix-core operands use; lsr_fwd_in.language_feature_split.
    `out` may be a preallocated [P,64] int16 tensor."""
    L = _lib.load()
    device = _check_device(language_feature)
    P, C = language_feature.shape
    stream = stream or torch.cuda.current_stream(device)
    lang = language_feature.detach().to(torch.float32).contiguous()
    if out is None:
        with torch.cuda.stream(stream):
            out = torch.empty(P, 2 * C, dtype=torch.int16, device=device)
    elif out.shape != (P, 2 * C) or out.dtype != torch.int16 or not out.is_contiguous():
        raise ValueError("language_split_native: out must be a contiguous [P, 2C] int16 tensor")
    _lib.check(L.lsr_language_split(P, C, ctypes.c_void_p(lang.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(stream.cuda_stream)), "lsr_language_split")
    return out


def preprocess_views_native(raster_settings_list, means3D, opacities, shs=None, colors_precomp=None,
                            language_feature=None, scales=None, rotations=None, cov3D_precomp=None, stream=None,
                            split_language=True, split_behind_counts=True, split_stream=None, order_first=None,
                            order_stream=None, row_chunks=None, tile_bucket=False):
    """Forward phase 1 of several views of the same Gaussians as one batch
    (lsr_forward_preprocess_views_async: one preprocess launch per 8 views reads each Gaussian once,
    the views' depth sorts and instance scans share their launches) on `stream`.  No host
    synchronisation: returns one deferred-count PendingForward per view; binning_views_native
    resolves them all with one wait.  Same results as preprocess_native per view.

    split_language (C == 32): the language rows' bf16 hi / lo operands are made once here for all
    the batch's views (lsr_language_split) instead of per entry in every compositor wave (same
    bits, same results).  split_behind_counts: enqueue that split behind the batch's count event, so
    it runs while the host waits for the counts (False: ahead of the preprocess; an A/B switch).
    split_stream: enqueue the split there instead (after that stream waits for `stream`); the caller
    orders the compositors after it.

    order_first = k < n with order_stream: only the first k views are depth-ordered and counted on
    `stream` (lsr_forward_preprocess_views_split_async); the other views' depth orders and counts run
    on order_stream behind the preprocess (lsr_forward_depth_order_views_async), so the first views'
    binning and compositing start before the later views' sorts.  Those views carry their own count
    batch (binning_views_native waits for it on their first binning); same results.

    row_chunks = [(r0, r1, before), ...] covering [0, P) in order (r0 multiples of 256): the
    preprocess runs one launch per row chunk (lsr_forward_preprocess_views_rows_async), each after
    before() (which makes `stream` wait for that chunk's rows, e.g. the sharded optimizer's
    all-gather of them), and the depth orders follow once every chunk is in; same results.

    tile_bucket: prepare the tile-bucket binning instead (lsr_forward_preprocess_views_tb_async +
    lsr_forward_instance_scan_views_async: no depth sort; binning_views_native then buckets the
    instances by tile and sorts each bucket in LDS, lsr_forward_binning_views_tb).  Same lists, same
    results; the split into first views and order_stream views applies to the instance scans."""
    device = _check_device(means3D)
    L = _lib.load()
    stream = stream or torch.cuda.current_stream(device)
    fin, inputs, P = _fwd_inputs(means3D, opacities, shs, colors_precomp, language_feature, scales, rotations,
                                 cov3D_precomp)
    if row_chunks:   # validated before anything is enqueued (both binning paths)
        covered = 0
        for r0, r1, _ in row_chunks:
            if r0 != covered or r1 < r0 or r0 % 256:
                raise ValueError("row_chunks must cover [0, P) in order, each r0 a multiple of 256")
            covered = r1
        if covered != P:
            raise ValueError("row_chunks must cover [0, P) in order, each r0 a multiple of 256")
    split = split_language and fin.C == 32 and P > 0
    if split:   # allocated now (fin carries the pointer), written behind the batch's count event
        with torch.cuda.stream(stream):
            inputs["language_feature_split"] = torch.empty(P, 64, dtype=torch.int16, device=device)
        fin.language_feature_split = inputs["language_feature_split"].data_ptr()
        # with row_chunks the language rows may still be arriving (each chunk's before() waits for
        # them): the split is then always enqueued behind the chunk loop
        if not split_behind_counts and not row_chunks:
            language_split_native(inputs["language_feature"], stream=stream, out=inputs["language_feature_split"])
            split = False
    n = len(raster_settings_list)
    sts = [_NativeSettings(rs, device) for rs in raster_settings_list]
    with torch.cuda.stream(stream):
        radii = [torch.empty(P, dtype=torch.int32, device=device) for _ in range(n)]
        geoms = [torch.empty(int(L.lsr_geom_bytes(P)), dtype=torch.uint8, device=device) for _ in range(n)]
    fouts = [_lib.FwdOut() for _ in range(n)]
    for fo, r in zip(fouts, radii):
        fo.radii = r.data_ptr()
    k = n if (order_first is None or order_stream is None) else max(0, min(int(order_first), n))
    counts = torch.zeros(k, 2, dtype=torch.int32, pin_memory=True) if k > 0 else None
    s_arr = (ctypes.POINTER(_lib.Settings) * n)(*[ctypes.pointer(x.c) for x in sts])
    o_arr = (ctypes.POINTER(_lib.FwdOut) * n)(*[ctypes.pointer(fo) for fo in fouts])
    g_arr = (ctypes.c_void_p * n)(*[g.data_ptr() for g in geoms])
    try:
        if tile_bucket:
            for r0, r1, before in (row_chunks or [(0, P, None)]):
                if before is not None:
                    before()
                _lib.check(L.lsr_forward_preprocess_views_tb_async(n, int(r0), int(r1), s_arr, ctypes.byref(fin), o_arr,
                                                                   g_arr, ctypes.c_void_p(stream.cuda_stream)),
                           "lsr_forward_preprocess_views_tb_async")
            if k > 0:
                _lib.check(L.lsr_forward_instance_scan_views_async(k, s_arr, ctypes.byref(fin), g_arr,
                                                                   ctypes.c_void_p(counts.data_ptr()),
                                                                   ctypes.c_void_p(stream.cuda_stream)),
                           "lsr_forward_instance_scan_views_async")
        elif row_chunks:
            for r0, r1, before in row_chunks:
                if before is not None:
                    before()
                _lib.check(L.lsr_forward_preprocess_views_rows_async(n, int(r0), int(r1), s_arr, ctypes.byref(fin),
                                                                     o_arr, g_arr, ctypes.c_void_p(stream.cuda_stream)),
                           "lsr_forward_preprocess_views_rows_async")
            if k > 0:
                _lib.check(L.lsr_forward_depth_order_views_async(k, s_arr, ctypes.byref(fin), g_arr,
                                                                 ctypes.c_void_p(counts.data_ptr()),
                                                                 ctypes.c_void_p(stream.cuda_stream)),
                           "lsr_forward_depth_order_views_async")
        else:
            _lib.check(L.lsr_forward_preprocess_views_split_async(n, k, s_arr, ctypes.byref(fin), o_arr, g_arr,
                                                                  ctypes.c_void_p(counts.data_ptr() if k else 0),
                                                                  ctypes.c_void_p(stream.cuda_stream)),
                       "lsr_forward_preprocess_views_split_async")
    except RuntimeError:
        _dump_forward(raster_settings_list[0], inputs)
        raise
    ev = torch.cuda.Event()
    ev.record(stream)
    late = None
    if k < n:   # the later views' depth orders and counts on order_stream, behind the preprocess
        order_stream.wait_event(ev)
        for g in geoms[k:]:
            g.record_stream(order_stream)
        counts_b = torch.zeros(n - k, 2, dtype=torch.int32, pin_memory=True)
        fn, what = ((L.lsr_forward_instance_scan_views_async, "lsr_forward_instance_scan_views_async") if tile_bucket
                    else (L.lsr_forward_depth_order_views_async, "lsr_forward_depth_order_views_async"))
        try:
            _lib.check(fn(n - k, (ctypes.POINTER(_lib.Settings) * (n - k))(*s_arr[k:]), ctypes.byref(fin),
                          (ctypes.c_void_p * (n - k))(*g_arr[k:]), ctypes.c_void_p(counts_b.data_ptr()),
                          ctypes.c_void_p(order_stream.cuda_stream)), what)
        except RuntimeError:
            _dump_forward(raster_settings_list[0], inputs)
            raise
        ev_b = torch.cuda.Event()
        ev_b.record(order_stream)
        late = (counts_b, ev_b)
    if split and split_stream is not None:   # on the caller's side stream, beside the binning
        split_stream.wait_stream(stream)
        inputs["language_feature_split"].record_stream(split_stream)
        language_split_native(inputs["language_feature"], stream=split_stream, out=inputs["language_feature_split"])
    elif split:   # only the compositors read it: it runs while the host waits for the counts
        language_split_native(inputs["language_feature"], stream=stream, out=inputs["language_feature_split"])
    out = []
    for v, rs in enumerate(raster_settings_list):
        H, W = int(rs.image_height), int(rs.image_width)
        pf = PendingForward(rs, sts[v], fin, inputs, geoms[v], radii[v], None, device, H, W)
        pf.tile_bucket = bool(tile_bucket)
        if v < k:
            pf.count_host, pf.stream, pf.counted = counts[v], stream, ev
            pf.count_batch = (counts, v)      # binning_views_native reads the whole batch at once
        else:
            pf.count_host, pf.stream, pf.counted = late[0][v - k], order_stream, late[1]
            pf.count_batch = (late[0], v - k)
        out.append(pf)
    return out


def _align(nbytes, a=256):
    return (nbytes + a - 1) // a * a


@functools.lru_cache(maxsize=4096)
def _binning_bytes(K):   # pure size queries, asked on the device's critical path (the count wait)
    return _align(int(_lib.load().lsr_binning_bytes(K)))


@functools.lru_cache(maxsize=4096)
def _binning_bytes_tb(K, P, W, H):
    return _align(int(_lib.load().lsr_binning_bytes_tb(K, P, W, H)))


@functools.lru_cache(maxsize=64)
def _img_bytes(W, H):
    return _align(int(_lib.load().lsr_img_bytes(W, H)))


def binning_views_native(pendings, stream=None):
    """Resolve the deferred counts of preprocess_views_native's views (one host wait) and run their
    tile binning as one batch (lsr_forward_binning_views) on `stream` (default: theirs), so that
    render_native only composites each view."""
    if not pendings:
        return
    L = _lib.load()
    stream = stream or pendings[0].stream
    # the device idles from the counts' arrival to the emission launch, so this stretch is kept
    # short: one wait and one read for a batch's counts, one allocation for all workspaces
    batch = pendings[0].count_batch
    if batch is not None and all(pf.count_batch is not None and pf.count_batch[0] is batch[0] for pf in pendings):
        pendings[0].counted.synchronize()
        rows = batch[0].tolist()
        for pf in pendings:
            pf.num_rendered, pf.counted = rows[pf.count_batch[1]][0], None
    else:
        for pf in pendings:
            pf.resolve()
    n = len(pendings)
    device = pendings[0].device
    tb = pendings[0].tile_bucket
    if any(pf.tile_bucket != tb for pf in pendings):
        raise ValueError("binning_views_native: a batch mixes tile-bucket and sort-path views")
    sizes = []
    for pf in pendings:
        sizes += [_binning_bytes_tb(pf.num_rendered, pf.fin.P, pf.W, pf.H) if tb else _binning_bytes(pf.num_rendered),
                  _img_bytes(pf.W, pf.H)]
    with torch.cuda.stream(stream):
        ws = torch.empty(sum(sizes), dtype=torch.uint8, device=device)
    off = 0
    for i, pf in enumerate(pendings):
        pf.binning = ws[off:off + sizes[2 * i]]
        off += sizes[2 * i]
        pf.img = ws[off:off + sizes[2 * i + 1]]
        off += sizes[2 * i + 1]
    s_arr = (ctypes.POINTER(_lib.Settings) * n)(*[ctypes.pointer(pf.settings.c) for pf in pendings])
    g_arr = (ctypes.c_void_p * n)(*[pf.geom.data_ptr() for pf in pendings])
    b_arr = (ctypes.c_void_p * n)(*[pf.binning.data_ptr() for pf in pendings])
    i_arr = (ctypes.c_void_p * n)(*[pf.img.data_ptr() for pf in pendings])
    k_arr = (ctypes.c_int64 * n)(*[pf.num_rendered for pf in pendings])
    fn, what = ((L.lsr_forward_binning_views_tb, "lsr_forward_binning_views_tb") if tb
                else (L.lsr_forward_binning_views, "lsr_forward_binning_views"))
    try:
        _lib.check(fn(n, s_arr, ctypes.byref(pendings[0].fin), g_arr, b_arr, i_arr, k_arr,
                      ctypes.c_void_p(stream.cuda_stream)), what)
    except RuntimeError:
        _dump_forward(pendings[0].raster_settings, pendings[0].inputs)
        raise
    ev = torch.cuda.Event()
    ev.record(stream)
    for pf in pendings:
        pf.ready, pf.ready_stream = ev, stream


def render_native(pending: PendingForward):
    """Forward phase 2 (binning unless preprocess_native already did it, then compositing) on the
    current stream.  Returns (color, language_feature, radii, depth, state)."""
    L = _lib.load()
    if pending.tile_bucket and pending.binning is None:   # lsr_forward_render bins the sort path's way
        binning_views_native([pending], stream=torch.cuda.current_stream(pending.device))
    pending.resolve()
    device, H, W, C = pending.device, pending.H, pending.W, pending.fin.C
    stream = torch.cuda.current_stream(device)
    pending.geom.record_stream(stream)    # allocated on the preprocess stream, used from here on
    pending.radii.record_stream(stream)
    color = torch.empty(3, H, W, dtype=torch.float32, device=device)
    lang_out = torch.empty(C, H, W, dtype=torch.float32, device=device)
    depth = torch.empty(1, H, W, dtype=torch.float32, device=device)
    fout = _lib.FwdOut()
    fout.out_color, fout.out_language_feature = color.data_ptr(), _ptr(lang_out) if C > 0 else None
    fout.radii, fout.out_depth = pending.radii.data_ptr(), depth.data_ptr()
    K = pending.num_rendered
    binned = pending.binning is not None
    if binned:
        binning, img = pending.binning, pending.img
        if pending.ready_stream != stream:   # same stream: already ordered (a wait idles the device)
            waited = getattr(pending.ready, "_lsr_waited_by", None)
            if waited is None or stream.cuda_stream not in waited:   # views binned together share one event
                stream.wait_event(pending.ready)
                try:
                    pending.ready._lsr_waited_by = (waited or set()) | {stream.cuda_stream}
                except AttributeError:
                    pass
        binning.record_stream(stream)
        img.record_stream(stream)
    else:
        binning = torch.empty(int(L.lsr_binning_bytes(K)), dtype=torch.uint8, device=device)
        img = torch.empty(int(L.lsr_img_bytes(W, H)), dtype=torch.uint8, device=device)
    fn, what = (L.lsr_forward_composite, "lsr_forward_composite") if binned else (L.lsr_forward_render,
                                                                                   "lsr_forward_render")
    try:
        _lib.check(fn(ctypes.byref(pending.settings.c), ctypes.byref(pending.fin), ctypes.byref(fout),
                      ctypes.c_void_p(pending.geom.data_ptr()), ctypes.c_void_p(binning.data_ptr()),
                      ctypes.c_void_p(img.data_ptr()), ctypes.c_int64(K), _stream(device)), what)
    except RuntimeError:
        _dump_forward(pending.raster_settings, pending.inputs)
        raise
    state = RasterizerState(pending.settings, pending.inputs, pending.fin, pending.geom, binning, img, K, pending.radii)
    return color, lang_out, pending.radii, depth, state


def radii_max_native(radii, out, accumulate=False, stream=None):
    """lsr_radii_max: out = max(out if accumulate, radii[0], ..., radii[n-1]) elementwise, int32 [P]
    device tensors, one launch per 8 views on `stream` (default: current): the radii MAX over a
    batch's views (train.py:270) without a stack copy or one launch per view."""
    if not radii:
        return out
    L = _lib.load()
    P = out.shape[0]
    rs = [r.contiguous() for r in radii]
    for r in rs:
        if r.dtype != torch.int32 or r.shape != (P,) or r.device != out.device:
            raise ValueError("radii_max_native: int32 [P] tensors on out's device")
    if out.dtype != torch.int32 or not out.is_contiguous():
        raise ValueError("radii_max_native: out must be a contiguous int32 tensor")
    stream = stream or torch.cuda.current_stream(out.device)
    arr = (ctypes.c_void_p * len(rs))(*[r.data_ptr() for r in rs])
    _lib.check(L.lsr_radii_max(P, len(rs), arr, ctypes.c_void_p(out.data_ptr()), 1 if accumulate else 0,
                               ctypes.c_void_p(stream.cuda_stream)), "lsr_radii_max")
    return out


def render_views_native(pendings):
    """render_native for several views of the same Gaussians and image size, their compositing as
    ONE launch per 8 views (lsr_forward_composite_views: a view's last waves run beside the next
    view's first ones).  Views not binned yet are binned first, as one batch.  Same results as
    render_native per view.  Returns a list of (color, language_feature, radii, depth, state)."""
    if not pendings:
        return []
    L = _lib.load()
    unbinned = [pf for pf in pendings if pf.binning is None]
    if unbinned:
        binning_views_native(unbinned, stream=torch.cuda.current_stream(unbinned[0].device))
    device = pendings[0].device
    stream = torch.cuda.current_stream(device)
    waited = set()
    outs, fouts = [], []
    for pf in pendings:
        if pf.device != device or (pf.H, pf.W) != (pendings[0].H, pendings[0].W):
            raise ValueError("render_views_native: the views must share the device and image size")
        if pf.ready_stream is not None and pf.ready_stream != stream and id(pf.ready) not in waited:
            stream.wait_event(pf.ready)   # one wait per binning batch (a wait idles the device)
            waited.add(id(pf.ready))
        for t in (pf.geom, pf.radii, pf.binning, pf.img):
            t.record_stream(stream)
        H, W, C = pf.H, pf.W, pf.fin.C
        color = torch.empty(3, H, W, dtype=torch.float32, device=device)
        lang_out = torch.empty(C, H, W, dtype=torch.float32, device=device)
        depth = torch.empty(1, H, W, dtype=torch.float32, device=device)
        fout = _lib.FwdOut()
        fout.out_color, fout.out_language_feature = color.data_ptr(), _ptr(lang_out) if C > 0 else None
        fout.radii, fout.out_depth = pf.radii.data_ptr(), depth.data_ptr()
        outs.append((color, lang_out, depth))
        fouts.append(fout)
    n = len(pendings)
    s_arr = (ctypes.POINTER(_lib.Settings) * n)(*[ctypes.pointer(pf.settings.c) for pf in pendings])
    o_arr = (ctypes.POINTER(_lib.FwdOut) * n)(*[ctypes.pointer(f) for f in fouts])
    vp = ctypes.c_void_p * n
    try:
        _lib.check(L.lsr_forward_composite_views(n, s_arr, ctypes.byref(pendings[0].fin), o_arr,
                                                 vp(*[pf.geom.data_ptr() for pf in pendings]),
                                                 vp(*[pf.binning.data_ptr() for pf in pendings]),
                                                 vp(*[pf.img.data_ptr() for pf in pendings]),
                                                 (ctypes.c_int64 * n)(*[pf.num_rendered for pf in pendings]),
                                                 _stream(device)), "lsr_forward_composite_views")
    except RuntimeError:
        _dump_forward(pendings[0].raster_settings, pendings[0].inputs)
        raise
    res = []
    for pf, (color, lang_out, depth) in zip(pendings, outs):
        state = RasterizerState(pf.settings, pf.inputs, pf.fin, pf.geom, pf.binning, pf.img, pf.num_rendered, pf.radii)
        res.append((color, lang_out, pf.radii, depth, state))
    return res


def forward_native(raster_settings, means3D, opacities, shs=None, colors_precomp=None, language_feature=None,
                   scales=None, rotations=None, cov3D_precomp=None):
    """Forward through liblsr.so on the current stream.  Returns (color, language_feature, radii,
    depth, state)."""
    return render_native(preprocess_native(raster_settings, means3D, opacities, shs=shs, colors_precomp=colors_precomp,
                                           language_feature=language_feature, scales=scales, rotations=rotations,
                                           cov3D_precomp=cov3D_precomp))


def backward_native(state: RasterizerState, grad_color, grad_lang=None, grad_depth=None, out=None,
                    accumulate=False, need=None, deterministic=False):
    """Backward through liblsr.so.  `out` may hold preallocated gradient buffers (dict); with
    accumulate=True they are added to.  deterministic=True selects the fixed-order reduction
    (bitwise reproducible gradients).  Returns the dict of gradient tensors."""
    L = _lib.load()
    inp = state.inputs
    means3D = inp["means3D"]
    device = means3D.device
    P, M, C = state.fin.P, state.fin.M, state.fin.C
    H, W = state.settings.c.image_height, state.settings.c.image_width
    need = need or {}

    def buf(name, shape, wanted=True):
        if not wanted:
            return None
        if out is not None and name in out and out[name] is not None:
            return out[name]
        return torch.zeros(shape, dtype=torch.float32, device=device) if accumulate else \
            torch.empty(shape, dtype=torch.float32, device=device)

    g = dict(
        means3D=buf("means3D", (P, 3), need.get("means3D", True)),
        means2D=buf("means2D", (P, 3), need.get("means2D", True)),
        colors=buf("colors", (P, 3), need.get("colors", True)),
        language_feature=buf("language_feature", (P, C), need.get("language_feature", True) and C > 0),
        opacities=buf("opacities", (P, 1), need.get("opacities", True)),
        cov3D=buf("cov3D", (P, 6), need.get("cov3D", True) and inp["cov3D_precomp"] is not None),
        sh=buf("sh", (P, max(M, 1), 3), need.get("sh", True) and M > 0),
        scales=buf("scales", (P, 3), need.get("scales", True) and inp["scales"] is not None),
        rotations=buf("rotations", (P, 4), need.get("rotations", True) and inp["rotations"] is not None),
    )
    gc = grad_color.detach().to(torch.float32).contiguous() if grad_color is not None else \
        torch.zeros(3, H, W, dtype=torch.float32, device=device)
    gl = grad_lang.detach().to(torch.float32).contiguous() if (grad_lang is not None and C > 0) else None
    gd = grad_depth.detach().to(torch.float32).contiguous() if grad_depth is not None else None
    gin = _lib.BwdIn()
    gin.dL_dout_color, gin.dL_dout_language_feature, gin.dL_dout_depth = gc.data_ptr(), _ptr(gl), _ptr(gd)
    gin.deterministic = 1 if deterministic else 0
    gout = _lib.BwdOut()
    gout.dL_dmeans3D, gout.dL_dmeans2D, gout.dL_dcolors = _ptr(g["means3D"]), _ptr(g["means2D"]), _ptr(g["colors"])
    gout.dL_dlanguage_feature, gout.dL_dopacity = _ptr(g["language_feature"]), _ptr(g["opacities"])
    gout.dL_dcov3D, gout.dL_dsh = _ptr(g["cov3D"]), _ptr(g["sh"])
    gout.dL_dscales, gout.dL_drotations = _ptr(g["scales"]), _ptr(g["rotations"])
    scratch = torch.empty(int(L.lsr_backward_bytes(P, state.num_rendered, C, 1 if deterministic else 0)),
                          dtype=torch.uint8, device=device)
    rc = L.lsr_backward(ctypes.byref(state.settings.c), ctypes.byref(state.fin), ctypes.byref(gin), ctypes.byref(gout),
                        ctypes.c_void_p(state.geom.data_ptr()), ctypes.c_void_p(state.binning.data_ptr()),
                        ctypes.c_void_p(state.img.data_ptr()), ctypes.c_void_p(scratch.data_ptr()),
                        ctypes.c_int64(state.num_rendered), ctypes.c_int32(1 if accumulate else 0), _stream(device))
    if rc != 0 and state.settings.c.debug:
        print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.")
        torch.save(dict(grad_color=gc.cpu()), "snapshot_bw.dump")
    _lib.check(rc, "lsr_backward")
    return g


def backward_views_native(states, grad_colors, grad_langs=None, grad_depths=None, out=None, accumulate=False,
                          need=None):
    """Backward of several views of the SAME Gaussians through liblsr.so (lsr_backward_views):
    the gradients of every view are summed, as train.py's loss.backward() sums its per-view renders
    (train.py:242-268,339).  Each view's compositor backward runs, then one preprocess backward
    per 8 views reads the Gaussian rows and writes the gradient rows once.  Float-atomic reduction
    (for bitwise-reproducible gradients use backward_native(deterministic=True) per view).
    `states` are the RasterizerState of the views' forwards; grad_* are per-view lists (entries may
    be None).  Returns the dict of gradient tensors (out's buffers when given)."""
    L = _lib.load()
    n = len(states)
    if n == 0:
        raise ValueError("backward_views_native needs at least one view")
    for s in states:
        if s.composited:
            raise RuntimeError("a view's forward was already backpropagated through its workspace accumulators "
                               "(backward_composite_native / backward_views_native run once per forward)")
    st0 = states[0]
    inp = st0.inputs
    for s in states[1:]:
        if s.inputs["means3D"].data_ptr() != inp["means3D"].data_ptr():
            raise ValueError("all views must render the same Gaussians")
    device = inp["means3D"].device
    P, M, C = st0.fin.P, st0.fin.M, st0.fin.C
    need = need or {}
    grad_langs = grad_langs or [None] * n
    grad_depths = grad_depths or [None] * n

    def buf(name, shape, wanted=True):
        if not wanted:
            return None
        if out is not None and name in out and out[name] is not None:
            return out[name]
        return torch.zeros(shape, dtype=torch.float32, device=device) if accumulate else \
            torch.empty(shape, dtype=torch.float32, device=device)

    g = dict(
        means3D=buf("means3D", (P, 3), need.get("means3D", True)),
        means2D=buf("means2D", (P, 3), need.get("means2D", True)),
        colors=buf("colors", (P, 3), need.get("colors", True)),
        language_feature=buf("language_feature", (P, C), need.get("language_feature", True) and C > 0),
        opacities=buf("opacities", (P, 1), need.get("opacities", True)),
        cov3D=buf("cov3D", (P, 6), need.get("cov3D", True) and inp["cov3D_precomp"] is not None),
        sh=buf("sh", (P, max(M, 1), 3), need.get("sh", True) and M > 0),
        scales=buf("scales", (P, 3), need.get("scales", True) and inp["scales"] is not None),
        rotations=buf("rotations", (P, 4), need.get("rotations", True) and inp["rotations"] is not None),
    )
    keep = []
    gins = []
    for v, s in enumerate(states):
        H, W = s.settings.c.image_height, s.settings.c.image_width
        gc = grad_colors[v].detach().to(torch.float32).contiguous() if grad_colors[v] is not None else \
            torch.zeros(3, H, W, dtype=torch.float32, device=device)
        gl = grad_langs[v].detach().to(torch.float32).contiguous() if (grad_langs[v] is not None and C > 0) else None
        gd = grad_depths[v].detach().to(torch.float32).contiguous() if grad_depths[v] is not None else None
        keep += [gc, gl, gd]
        gi = _lib.BwdIn()
        gi.dL_dout_color, gi.dL_dout_language_feature, gi.dL_dout_depth = gc.data_ptr(), _ptr(gl), _ptr(gd)
        gi.deterministic = 0
        gins.append(gi)
    gout = _lib.BwdOut()
    gout.dL_dmeans3D, gout.dL_dmeans2D, gout.dL_dcolors = _ptr(g["means3D"]), _ptr(g["means2D"]), _ptr(g["colors"])
    gout.dL_dlanguage_feature, gout.dL_dopacity = _ptr(g["language_feature"]), _ptr(g["opacities"])
    gout.dL_dcov3D, gout.dL_dsh = _ptr(g["cov3D"]), _ptr(g["sh"])
    gout.dL_dscales, gout.dL_drotations = _ptr(g["scales"]), _ptr(g["rotations"])
    SP = ctypes.POINTER(_lib.Settings)
    BP = ctypes.POINTER(_lib.BwdIn)
    s_arr = (SP * n)(*[ctypes.pointer(s.settings.c) for s in states])
    g_arr = (BP * n)(*[ctypes.pointer(gi) for gi in gins])
    vp = ctypes.c_void_p * n
    geom = vp(*[s.geom.data_ptr() for s in states])
    binning = vp(*[s.binning.data_ptr() for s in states])
    img = vp(*[s.img.data_ptr() for s in states])
    K = (ctypes.c_int64 * n)(*[s.num_rendered for s in states])
    _lib.check(L.lsr_backward_views(n, s_arr, ctypes.byref(st0.fin), g_arr, ctypes.byref(gout), geom, binning, img,
                                    K, 1 if accumulate else 0, _stream(device)), "lsr_backward_views")
    for s in states:
        s.composited = True
    return g


class CompositeGrad:
    """A view whose compositor backward ran (backward_composite_native): its forward state and the
    upstream gradients; the per-Gaussian screen-space sums that backward_preprocess_views_native
    consumes live in the state's geom buffer."""

    def __init__(self, state, keep):
        self.state, self._keep = state, keep


def backward_composite_native(state: RasterizerState, grad_color, grad_lang=None, grad_depth=None,
                              dL_dlanguage=None) -> CompositeGrad:
    """First half of backward_views_native for ONE view (lsr_backward_composite), on the current
    stream: the compositor backward; the language gradient is ADDED to dL_dlanguage [P,C] (the
    caller zeroes it once per batch).  Finish a batch with backward_preprocess_views_native."""
    L = _lib.load()
    if state.composited:
        raise RuntimeError("backward_composite_native already ran on this forward: its screen-space sums are "
                           "accumulated in the forward's workspace, so a second run would double them")
    device = state.inputs["means3D"].device
    P, C = state.fin.P, state.fin.C
    H, W = state.settings.c.image_height, state.settings.c.image_width
    gc = grad_color.detach().to(torch.float32).contiguous() if grad_color is not None else \
        torch.zeros(3, H, W, dtype=torch.float32, device=device)
    gl = grad_lang.detach().to(torch.float32).contiguous() if (grad_lang is not None and C > 0) else None
    gd = grad_depth.detach().to(torch.float32).contiguous() if grad_depth is not None else None
    gi = _lib.BwdIn()
    gi.dL_dout_color, gi.dL_dout_language_feature, gi.dL_dout_depth = gc.data_ptr(), _ptr(gl), _ptr(gd)
    gi.deterministic = 0
    if dL_dlanguage is not None and (dL_dlanguage.shape != (P, C) or not dL_dlanguage.is_contiguous()):
        raise ValueError("dL_dlanguage must be a contiguous [P, C] tensor")
    _lib.check(L.lsr_backward_composite(ctypes.byref(state.settings.c), ctypes.byref(state.fin), ctypes.byref(gi),
                                        _ptr(dL_dlanguage if C > 0 else None), ctypes.c_void_p(state.geom.data_ptr()),
                                        ctypes.c_void_p(state.binning.data_ptr()),
                                        ctypes.c_void_p(state.img.data_ptr()),
                                        ctypes.c_int64(state.num_rendered), _stream(device)), "lsr_backward_composite")
    state.composited = True
    return CompositeGrad(state, (gc, gl, gd))


def backward_composite_views_native(states, grad_colors, grad_langs=None, grad_depths=None,
                                    dL_dlanguage=None):
    """backward_composite_native for several views of the same Gaussians and image size, their
    compositor backward as ONE launch per 8 views (lsr_backward_composite_views; one launch for
    their tile orders too).  grad_* are per-view lists (entries may be None).  Returns a list of
    CompositeGrad for backward_preprocess_views_native."""
    if not states:
        return []
    L = _lib.load()
    for s in states:
        if s.composited:
            raise RuntimeError("backward_composite_native already ran on this forward: its screen-space sums are "
                               "accumulated in the forward's workspace, so a second run would double them")
    st0 = states[0]
    device = st0.inputs["means3D"].device
    P, C = st0.fin.P, st0.fin.C
    n = len(states)
    grad_langs = grad_langs or [None] * n
    grad_depths = grad_depths or [None] * n
    if dL_dlanguage is not None and (dL_dlanguage.shape != (P, C) or not dL_dlanguage.is_contiguous()):
        raise ValueError("dL_dlanguage must be a contiguous [P, C] tensor")
    gins, keeps = [], []
    for v, s in enumerate(states):
        if s.inputs["means3D"].data_ptr() != st0.inputs["means3D"].data_ptr():
            raise ValueError("all views must render the same Gaussians")
        H, W = s.settings.c.image_height, s.settings.c.image_width
        gc = grad_colors[v].detach().to(torch.float32).contiguous() if grad_colors[v] is not None else \
            torch.zeros(3, H, W, dtype=torch.float32, device=device)
        gl = grad_langs[v].detach().to(torch.float32).contiguous() if (grad_langs[v] is not None and C > 0) else None
        gd = grad_depths[v].detach().to(torch.float32).contiguous() if grad_depths[v] is not None else None
        gi = _lib.BwdIn()
        gi.dL_dout_color, gi.dL_dout_language_feature, gi.dL_dout_depth = gc.data_ptr(), _ptr(gl), _ptr(gd)
        gi.deterministic = 0
        gins.append(gi)
        keeps.append((gc, gl, gd))
    s_arr = (ctypes.POINTER(_lib.Settings) * n)(*[ctypes.pointer(s.settings.c) for s in states])
    g_arr = (ctypes.POINTER(_lib.BwdIn) * n)(*[ctypes.pointer(gi) for gi in gins])
    vp = ctypes.c_void_p * n
    _lib.check(L.lsr_backward_composite_views(n, s_arr, ctypes.byref(st0.fin), g_arr,
                                              _ptr(dL_dlanguage if C > 0 else None),
                                              vp(*[s.geom.data_ptr() for s in states]),
                                              vp(*[s.binning.data_ptr() for s in states]),
                                              vp(*[s.img.data_ptr() for s in states]),
                                              (ctypes.c_int64 * n)(*[s.num_rendered for s in states]),
                                              _stream(device)), "lsr_backward_composite_views")
    for s in states:
        s.composited = True
    return [CompositeGrad(s, k) for s, k in zip(states, keeps)]


def backward_preprocess_views_native(parts, out=None, accumulate=False, need=None, row_chunks=None, on_rows=None):
    """Second half of backward_views_native (lsr_backward_preprocess_views): the preprocess backward
    of every view in `parts` (CompositeGrad), summed into one set of gradient rows.  The language
    gradient is not touched here (the composite halves added it).  Returns the dict of gradients.

    row_chunks: [(r0, r1), ...] covering [0, P) in order (r0 multiples of 256): one launch per chunk
    (lsr_backward_preprocess_views_rows), and on_rows(r0, r1) is called right after each chunk's
    launch is enqueued, so a data-parallel caller can start that chunk's all-reduce while the next
    chunk computes."""
    L = _lib.load()
    n = len(parts)
    if n == 0:
        raise ValueError("backward_preprocess_views_native needs at least one view")
    st0 = parts[0].state
    inp = st0.inputs
    for p_ in parts[1:]:
        if p_.state.inputs["means3D"].data_ptr() != inp["means3D"].data_ptr():
            raise ValueError("all views must render the same Gaussians")
    device = inp["means3D"].device
    need = dict(need or {})
    need["language_feature"] = False
    g = _grad_buffers(st0, out, accumulate, need)
    gout = _bwd_out(g)
    SP = ctypes.POINTER(_lib.Settings)
    vp = ctypes.c_void_p * n
    s_arr = (SP * n)(*[ctypes.pointer(p_.state.settings.c) for p_ in parts])
    geoms = vp(*[p_.state.geom.data_ptr() for p_ in parts])
    if row_chunks is None:
        _lib.check(L.lsr_backward_preprocess_views(n, s_arr, ctypes.byref(st0.fin), ctypes.byref(gout), geoms,
                                                   1 if accumulate else 0, _stream(device)),
                   "lsr_backward_preprocess_views")
    else:
        P = st0.fin.P
        expect = 0
        for r0, r1 in row_chunks:
            if r0 != expect or r1 < r0 or r1 > P:
                raise ValueError(f"row_chunks must tile [0, {P}) in order, got {list(row_chunks)}")
            expect = r1
            part = {k: (v[r0:r1] if v is not None else None) for k, v in g.items()}
            gc = _bwd_out(part)
            _lib.check(L.lsr_backward_preprocess_views_rows(n, s_arr, ctypes.byref(st0.fin), ctypes.byref(gc), geoms,
                                                            1 if accumulate else 0, r0, r1 - r0, _stream(device)),
                       "lsr_backward_preprocess_views_rows")
            if on_rows is not None:
                on_rows(r0, r1)
        if expect != P:
            raise ValueError(f"row_chunks must tile [0, {P}) in order, got {list(row_chunks)}")
    return g


def _grad_buffers(state, out, accumulate, need):
    inp = state.inputs
    device = inp["means3D"].device
    P, M, C = state.fin.P, state.fin.M, state.fin.C

    def buf(name, shape, wanted=True):
        if not wanted:
            return None
        if out is not None and name in out and out[name] is not None:
            return out[name]
        return torch.zeros(shape, dtype=torch.float32, device=device) if accumulate else \
            torch.empty(shape, dtype=torch.float32, device=device)

    return dict(
        means3D=buf("means3D", (P, 3), need.get("means3D", True)),
        means2D=buf("means2D", (P, 3), need.get("means2D", True)),
        colors=buf("colors", (P, 3), need.get("colors", True)),
        language_feature=buf("language_feature", (P, C), need.get("language_feature", True) and C > 0),
        opacities=buf("opacities", (P, 1), need.get("opacities", True)),
        cov3D=buf("cov3D", (P, 6), need.get("cov3D", True) and inp["cov3D_precomp"] is not None),
        sh=buf("sh", (P, max(M, 1), 3), need.get("sh", True) and M > 0),
        scales=buf("scales", (P, 3), need.get("scales", True) and inp["scales"] is not None),
        rotations=buf("rotations", (P, 4), need.get("rotations", True) and inp["rotations"] is not None),
    )


def _bwd_out(g):
    gout = _lib.BwdOut()
    gout.dL_dmeans3D, gout.dL_dmeans2D, gout.dL_dcolors = _ptr(g["means3D"]), _ptr(g["means2D"]), _ptr(g["colors"])
    gout.dL_dlanguage_feature, gout.dL_dopacity = _ptr(g["language_feature"]), _ptr(g["opacities"])
    gout.dL_dcov3D, gout.dL_dsh = _ptr(g["cov3D"]), _ptr(g["sh"])
    gout.dL_dscales, gout.dL_drotations = _ptr(g["scales"]), _ptr(g["rotations"])
    return gout


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings):
        color, lang, radii, depth, state = forward_native(
            raster_settings, means3D, opacities, shs=sh, colors_precomp=colors_precomp,
            language_feature=language_feature_precomp if raster_settings.include_feature else None,
            scales=scales, rotations=rotations, cov3D_precomp=cov3Ds_precomp)
        if not raster_settings.include_feature and language_feature_precomp is not None \
                and language_feature_precomp.numel() > 0:
            # base stages: the caller passes zeros [P, hiddendim] and discards the output
            lang = torch.zeros((language_feature_precomp.shape[-1],) + tuple(color.shape[1:]),
                               dtype=color.dtype, device=color.device)
        ctx.state = state
        ctx.shapes = dict(sh=None if sh is None else sh.shape, opacities=opacities.shape,
                          lang=None if language_feature_precomp is None else language_feature_precomp.shape)
        ctx.include_feature = raster_settings.include_feature
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)
        return color, lang, radii, depth

    @staticmethod
    def backward(ctx, grad_color, grad_lang, grad_radii, grad_depth):
        return _raster_backward(ctx.state, ctx.shapes, ctx.include_feature, ctx.needs_input_grad[:9], grad_color,
                                grad_lang, grad_depth) + (None,)


def _raster_backward(st, shp, include_feature, ng, grad_color, grad_lang, grad_depth):
    """The 9 input gradients of one view's rasterization (means3D, means2D, sh, colors_precomp,
    language_feature_precomp, opacities, scales, rotations, cov3D_precomp); ng: which are needed."""
    need = dict(means3D=ng[0], means2D=ng[1], sh=ng[2], colors=True, language_feature=ng[4], opacities=ng[5],
                scales=ng[6], rotations=ng[7], cov3D=ng[8])
    # torch.use_deterministic_algorithms(True) selects the fixed-order reduction (bitwise
    # reproducible gradients, lsr_backward's deterministic mode) instead of float atomics
    g = backward_native(st, grad_color, grad_lang if include_feature else None, grad_depth, need=need,
                        deterministic=torch.are_deterministic_algorithms_enabled())

    def like(t, shape):
        return None if (t is None or shape is None) else t.reshape(shape)

    grad_lang_in = None
    if ng[4] and shp["lang"] is not None and len(shp["lang"]) > 0:
        if g["language_feature"] is not None:
            grad_lang_in = g["language_feature"].reshape(shp["lang"])
        else:
            grad_lang_in = torch.zeros(shp["lang"], dtype=torch.float32, device=st.inputs["means3D"].device)
    return (g["means3D"] if ng[0] else None,
            g["means2D"] if ng[1] else None,
            like(g["sh"], shp["sh"]) if ng[2] else None,
            g["colors"] if ng[3] else None,
            grad_lang_in,
            like(g["opacities"], shp["opacities"]) if ng[5] else None,
            g["scales"] if ng[6] else None,
            g["rotations"] if ng[7] else None,
            g["cov3D"] if ng[8] else None)


class _RasterizeViews(torch.autograd.Function):
    """_RasterizeGaussians for several views with their own Gaussians (a batch's deformed copies,
    gaussian_scene.render_views): every view's preprocess is enqueued first with its instance count
    deferred, then each view is binned and composited, so the host waits on view v's count while the
    device runs the later views' preprocesses (one stream synchronisation per view in a row before:
    the device idled through each).  Same kernels per view, same results; per-view backward."""

    @staticmethod
    def forward(ctx, settings_list, *flat):
        pfs = []
        for v, rs in enumerate(settings_list):
            m3, _, sh, cp, lang, op, sc, rot, cov = flat[9 * v:9 * v + 9]
            pfs.append(preprocess_native(rs, m3, op, shs=sh, colors_precomp=cp,
                                         language_feature=lang if rs.include_feature else None, scales=sc,
                                         rotations=rot, cov3D_precomp=cov, defer_count=True))
        outs, radii_all = [], []
        ctx.views = []
        for v, (rs, pf) in enumerate(zip(settings_list, pfs)):
            color, lang, radii, depth, state = render_native(pf)
            lang_in, sh, op = flat[9 * v + 4], flat[9 * v + 2], flat[9 * v + 5]
            if not rs.include_feature and lang_in is not None and lang_in.numel() > 0:
                lang = torch.zeros((lang_in.shape[-1],) + tuple(color.shape[1:]), dtype=color.dtype,
                                   device=color.device)
            ctx.views.append((state, dict(sh=None if sh is None else sh.shape, opacities=op.shape,
                                          lang=None if lang_in is None else lang_in.shape), rs.include_feature))
            outs += [color, lang, radii, depth]
            radii_all.append(radii)
        ctx.mark_non_differentiable(*radii_all)
        ctx.set_materialize_grads(False)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        res = []
        for v, (state, shapes, include_feature) in enumerate(ctx.views):
            gc, gl, _, gd = grads[4 * v:4 * v + 4]
            res.extend(_raster_backward(state, shapes, include_feature, ctx.needs_input_grad[1 + 9 * v:10 + 9 * v],
                                        gc, gl, gd))
        return (None,) + tuple(res)


def rasterize_views(settings_list, views):
    """GaussianRasterizer forward for several views, each with its own inputs: views[v] =
    dict(means3D=, means2D=, shs=, colors_precomp=, language_feature_precomp=, opacities=, scales=,
    rotations=, cov3D_precomp=).  Returns [(color, language_feature, radii, depth)] per view
    (_RasterizeViews: the views' preprocesses enqueued ahead of their count waits)."""
    flat = []
    for rs, kw in zip(settings_list, views):
        if (kw.get("shs") is None) == (kw.get("colors_precomp") is None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((kw.get("scales") is None or kw.get("rotations") is None) == (kw.get("cov3D_precomp") is None)):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        flat += [kw["means3D"], kw["means2D"], kw.get("shs"), kw.get("colors_precomp"),
                 kw.get("language_feature_precomp"), kw["opacities"], kw.get("scales"), kw.get("rotations"),
                 kw.get("cov3D_precomp")]
    out = _RasterizeViews.apply(list(settings_list), *flat)
    return [tuple(out[4 * v:4 * v + 4]) for v in range(len(settings_list))]


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, language_feature_precomp, opacities,
                                     scales, rotations, cov3Ds_precomp, raster_settings)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            rs = self.raster_settings
            pos = _f32(positions, positions.device)
            view = _f32(rs.viewmatrix, positions.device).reshape(-1)
            proj = _f32(rs.projmatrix, positions.device).reshape(-1)
            out = torch.empty(pos.shape[0], dtype=torch.uint8, device=positions.device)
            L = _lib.load()
            _lib.check(L.lsr_mark_visible(pos.shape[0], ctypes.c_void_p(pos.data_ptr()), ctypes.c_void_p(view.data_ptr()),
                                          ctypes.c_void_p(proj.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                          _stream(positions.device)), "lsr_mark_visible")
            return out.bool()

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, language_feature_precomp=None,
                scales=None, rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = torch.Tensor([])
        return rasterize_gaussians(means3D, means2D, shs if shs is not None else empty,
                                   colors_precomp if colors_precomp is not None else empty,
                                   language_feature_precomp if language_feature_precomp is not None else empty,
                                   opacities, scales if scales is not None else empty,
                                   rotations if rotations is not None else empty,
                                   cov3D_precomp if cov3D_precomp is not None else empty, rs)
