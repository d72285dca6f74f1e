"""GPU-side helpers for the parity tests: run the native rasterizer (through the C ABI) and the
oracle on the same seeded inputs, and decode the native workspaces (layout of lsr_api.hip)."""
import numpy as np
import torch

import diff_gaussian_rasterization as dgr
import oracle
from helpers import oracle_settings

ALIGN = 256


def _al(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


def raster_settings(cam, bg=(1.0, 1.0, 1.0), sh_degree=3, include_feature=True, scale_modifier=1.0, debug=False):
    dev = "cuda"
    return dgr.GaussianRasterizationSettings(
        image_height=cam.image_height, image_width=cam.image_width, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.tensor(bg, dtype=torch.float32, device=dev), scale_modifier=scale_modifier,
        viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev),
        sh_degree=sh_degree, campos=cam.camera_center.to(dev), prefiltered=False, debug=debug,
        include_feature=include_feature)


def decode_img(state):
    """ranges [tiles,2], tile_max [tiles], final_T [H,W], n_contrib [H,W] from the img workspace."""
    W, H = state.settings.c.image_width, state.settings.c.image_height
    gx, gy = (W + 15) // 16, (H + 15) // 16
    nt = gx * gy
    raw = state.img.cpu().numpy()
    off = 0
    ranges = raw[off:off + nt * 8].view(np.uint32).reshape(nt, 2); off += _al(nt * 8)
    tmax = raw[off:off + nt * 4].view(np.uint32); off += _al(nt * 4)
    fT = raw[off:off + W * H * 4].view(np.float32).reshape(H, W); off += _al(W * H * 4)
    nc = raw[off:off + W * H * 4].view(np.uint32).reshape(H, W)
    return ranges, tmax, fT, nc


def decode_point_list(state):
    K = state.num_rendered
    W, H = state.settings.c.image_width, state.settings.c.image_height
    nt = ((W + 15) // 16) * ((H + 15) // 16)
    bits = 1
    while (1 << bits) < nt:
        bits += 1
    in_b = ((bits + 7) // 8) % 2 == 1
    raw = state.binning.cpu().numpy()
    blk = _al(K * 4)
    off = 3 * blk if in_b else 2 * blk
    return raw[off:off + K * 4].view(np.uint32)


def run_native(scene, cam, bg=(1.0, 1.0, 1.0), include_feature=True, use_precomp_cov=False, colors_precomp=None,
               sh_degree=3):
    dev = "cuda"
    rs = raster_settings(cam, bg=bg, sh_degree=sh_degree, include_feature=include_feature)
    kw = {}
    if use_precomp_cov:
        kw["cov3D_precomp"] = torch.tensor(oracle.cov3d(scene.scales.numpy(), scene.rotations.numpy())).to(dev)
    else:
        kw["scales"], kw["rotations"] = scene.scales.to(dev), scene.rotations.to(dev)
    if colors_precomp is not None:
        kw["colors_precomp"] = torch.as_tensor(colors_precomp).to(dev)
    else:
        kw["shs"] = scene.shs.to(dev)
    lang = scene.lang.to(dev) if scene.lang.numel() > 0 else None
    return dgr.forward_native(rs, scene.means3D.to(dev), scene.opacities.to(dev), language_feature=lang, **kw)


def run_oracle(scene, cam, bg=(1.0, 1.0, 1.0), include_feature=True, use_precomp_cov=False, colors_precomp=None,
               sh_degree=3, nthreads=0):
    s = oracle_settings(cam, bg=bg, sh_degree=sh_degree, include_feature=include_feature)
    kw = {}
    if use_precomp_cov:
        kw["cov3D_precomp"] = oracle.cov3d(scene.scales.numpy(), scene.rotations.numpy())
    else:
        kw["scales"], kw["rotations"] = scene.scales.numpy(), scene.rotations.numpy()
    if colors_precomp is not None:
        kw["colors_precomp"] = np.asarray(colors_precomp)
    else:
        kw["shs"] = scene.shs.numpy()
    lang = scene.lang.numpy() if scene.lang.numel() > 0 else None
    return oracle.forward(s, scene.means3D.numpy(), scene.opacities.numpy(), lang=lang, nthreads=nthreads, **kw)


def grad_err(native, ref):
    """max |native - ref| relative to max |ref| (per tensor)"""
    native = np.asarray(native, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-12)
    return float(np.abs(native - ref).max() / scale)
