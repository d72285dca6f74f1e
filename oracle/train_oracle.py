"""CPU restatement (numpy, float32) of the training-step glue.

TEST INFRASTRUCTURE ONLY: imported by tests/ (never by the product path, which is
include/lsr_train.h in liblsr.so).  Each function follows the reference lines it cites:

  adam_step            torch.optim.Adam(..., eps=1e-15) as built at scene/gaussian_model.py:301 and
                       stepped at train.py:420 (the foreach element sequence: lerp, mul, addcmul,
                       sqrt, div, add, addcdiv; bias corrections in double as torch's Python floats)
  densify_stats        train.py:388-389 + scene/gaussian_model.py:746-748
  densify_plan         scene/gaussian_model.py:726-731 (densify), 607-627 (clone), 575-605 (split),
                       541-573 (postfix), 487-508 (prune of the split originals)
  split_rows           scene/gaussian_model.py:587-593 with build_rotation utils/general_utils.py:84-110
  prune_plan           scene/gaussian_model.py:714-723
  reset_opacity        scene/gaussian_model.py:391-394 (inverse_sigmoid utils/general_utils.py:18-19)
  expon_lr             utils/general_utils.py:35-66 (get_expon_lr_func)

Pinning: adam_step is checked against torch.optim.Adam itself (the reference's optimizer) in
tests/test_train_oracle.py; the densify / prune / split restatements have no reference fixtures
(GaussianModel does not import here: open3d, plyfile, simple_knn are absent, and it allocates on
"cuda"), so they are pinned only by the line-by-line restatement and hand-checked cases: parity
unpinned against the running reference.
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32


def adam_step(p, g, m, v, lr, step, beta1=0.9, beta2=0.999, eps=1e-15):
    """In place on float32 arrays; `step` counts this update (1 on the first)."""
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    w1, b2, w2 = F(1.0 - beta1), F(beta2), F(1.0 - beta2)
    bc2s, ss, e = F(math.sqrt(bc2)), F(-(lr / bc1)), F(eps)
    m[...] = m + w1 * (g - m)
    v[...] = v * b2
    v[...] = v + w2 * (g * g)
    den = np.sqrt(v) / bc2s + e
    p[...] = p + ss * (m / den)


def densify_stats(radii, grad2d, max_radii2D, accum, denom):
    """radii [P] int (max over views); grad2d [P, >=2]; the three stats updated in place."""
    vis = radii > 0
    max_radii2D[vis] = np.maximum(max_radii2D[vis], radii[vis].astype(np.float32))
    gx, gy = grad2d[vis, 0], grad2d[vis, 1]
    accum[vis] += np.sqrt(gx * gx + gy * gy)
    denom[vis] += F(1.0)


def _max_scale(scaling):
    return np.exp(scaling.astype(np.float32)).max(axis=1)


def densify_plan(accum, denom, scaling, grad_threshold, percent_dense, extent, n_copies=2):
    """Row map of the densified model: (index, kept, n_clone, n_split)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        g = (accum / denom).astype(np.float32)
    g[np.isnan(g)] = 0.0
    s = _max_scale(scaling)
    limit = F(percent_dense) * F(extent)
    clone = (np.abs(g) >= F(grad_threshold)) & (s <= limit)
    split = (g >= F(grad_threshold)) & (s > limit)
    rows = np.arange(len(g), dtype=np.int32)
    index = np.concatenate([rows[~split], rows[clone]] + [rows[split]] * n_copies).astype(np.int32)
    return index, int((~split).sum()), int(clone.sum()), int(split.sum())


def build_rotation(q):
    q = q.astype(np.float32)
    n = np.sqrt(q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1] + q[:, 2] * q[:, 2] + q[:, 3] * q[:, 3])
    r, x, y, z = (q[:, k] / n for k in range(4))
    R = np.empty((len(q), 3, 3), np.float32)
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - r * z)
    R[:, 0, 2] = 2 * (x * z + r * y)
    R[:, 1, 0] = 2 * (x * y + r * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - r * x)
    R[:, 2, 0] = 2 * (x * z - r * y)
    R[:, 2, 1] = 2 * (y * z + r * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def split_rows(xyz, scaling, rotation, src, samples, n_copies=2):
    """New positions and log-scales of split rows taken from source rows `src` (in output order)."""
    std = np.exp(scaling[src].astype(np.float32))
    smp = std * samples.astype(np.float32)
    R = build_rotation(rotation[src])
    new_xyz = np.einsum("nij,nj->ni", R, smp).astype(np.float32) + xyz[src]
    new_sc = np.log(std / F(0.8 * n_copies)).astype(np.float32)
    return new_xyz, new_sc


def prune_plan(opacity, max_radii2D, scaling, min_opacity, max_screen_size, extent):
    o = (1.0 / (1.0 + np.exp(-opacity.reshape(-1).astype(np.float32)))).astype(np.float32)
    prune = o < F(min_opacity)
    if max_screen_size:
        prune |= max_radii2D > F(max_screen_size)
        prune |= _max_scale(scaling) > F(0.1) * F(extent)
    return np.nonzero(~prune)[0].astype(np.int32)


def reset_opacity(opacity):
    o = np.minimum((1.0 / (1.0 + np.exp(-opacity.astype(np.float32)))).astype(np.float32), F(0.01))
    return np.log(o / (F(1.0) - o)).astype(np.float32)


def expon_lr(step, lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
        return 0.0
    if lr_delay_steps > 0:
        delay = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
    else:
        delay = 1.0
    t = np.clip(step / max_steps, 0, 1)
    return float(delay * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t))
