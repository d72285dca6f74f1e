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


def decode_point_words(state):
    """Raw point-list words: Gaussian id in the low 28 bits, the quadrant bits on top."""
    K = state.num_rendered
    W, H = state.settings.c.image_width, state.settings.c.image_height
    nt = ((W + 15) // 16) * ((H + 15) // 16)
    bits = 1
    while (1 << bits) <= nt:
        bits += 1
    in_b = ((bits + 7) // 8) % 2 == 1
    raw = state.binning.cpu().numpy()
    blk = _al(K * 4)
    off = 3 * blk if in_b else 2 * blk
    return raw[off:off + K * 4].view(np.uint32)


def decode_point_list(state):
    K = state.num_rendered
    W, H = state.settings.c.image_width, state.settings.c.image_height
    nt = ((W + 15) // 16) * ((H + 15) // 16)
    bits = 1
    while (1 << bits) <= nt:        # tile keys 0..nt-1 (instances reaching no quadrant are dropped)
        bits += 1
    in_b = ((bits + 7) // 8) % 2 == 1
    raw = state.binning.cpu().numpy()
    blk = _al(K * 4)
    off = 3 * blk if in_b else 2 * blk
    return raw[off:off + K * 4].view(np.uint32) & 0x0FFFFFFF   # low 28 bits: Gaussian id


def check_binning_against_upstream(state, ref_state, W, H):
    """The native binning drops (Gaussian, tile) instances whose splat cannot pass the alpha
    prefilter at any pixel of the tile (preprocess.hip, binning rectangle).  Checks, against the
    oracle's upstream binning: every tile list is an ordered subsequence of upstream's; every dropped
    entry has alpha < 1/255 at every pixel of its tile (so dropping it changes nothing); and each
    pixel's last contributor (n_contrib, a list position) is the same Gaussian."""
    ranges, _, fT, nc = decode_img(state)
    pl = decode_point_list(state).astype(np.int64)
    rr, rpl, rnc = ref_state["ranges"], ref_state["point_list"].astype(np.int64), ref_state["n_contrib"]
    xy, co = ref_state["xy"].astype(np.float64), ref_state["conic_o"].astype(np.float64)
    gx = (W + 15) // 16
    assert ranges[:, 1].max(initial=0) <= len(pl) and len(pl) <= len(rpl)
    dropped_total = 0
    for t in range(len(ranges)):
        g = pl[ranges[t, 0]:ranges[t, 1]]
        u = rpl[rr[t, 0]:rr[t, 1]]
        pos = {gid: k for k, gid in enumerate(u)}
        idx = np.array([pos[gid] for gid in g], dtype=np.int64)       # KeyError: entry not upstream
        assert (np.diff(idx) > 0).all(), f"tile {t}: order differs from upstream"
        dropped = np.setdiff1d(u, g)
        dropped_total += len(dropped)
        tx, ty = t % gx, t // gx
        px, py = np.meshgrid(np.arange(16 * tx, min(16 * tx + 16, W)), np.arange(16 * ty, min(16 * ty + 16, H)))
        px, py = px.ravel().astype(np.float64), py.ravel().astype(np.float64)
        if len(dropped):
            dx = xy[dropped, 0][:, None] - px[None]
            dy = xy[dropped, 1][:, None] - py[None]
            a, b, c, o = (co[dropped, k][:, None] for k in range(4))
            power = -0.5 * (a * dx * dx + c * dy * dy) - b * dx * dy
            alpha = np.minimum(0.99, o * np.exp(np.minimum(power, 0.0)))
            assert (alpha < (1.0 / 255.0) * (1 - 1e-6)).all(), f"tile {t}: a dropped entry contributes"
        # last contributor of each pixel of the tile: the same Gaussian
        for yy, xx in zip(py.astype(int), px.astype(int)):
            n, rn = int(nc[yy, xx]), int(rnc[yy, xx])
            assert (n == 0) == (rn == 0), (t, yy, xx)
            if n:
                assert g[n - 1] == u[rn - 1], (t, yy, xx)
    np.testing.assert_array_equal(fT, ref_state["final_T"])
    return dropped_total


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
