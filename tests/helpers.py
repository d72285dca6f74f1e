"""Shared helpers for the parity tests (scene -> oracle settings, comparisons)."""
import math

import numpy as np

import oracle
import synthetic


def oracle_settings(cam, bg=(1.0, 1.0, 1.0), sh_degree=3, include_feature=True, scale_modifier=1.0):
    return oracle.OracleSettings(cam.image_height, cam.image_width, cam.tanfovx, cam.tanfovy,
                                 np.asarray(bg, np.float32), scale_modifier, cam.world_view_transform.numpy(),
                                 cam.full_proj_transform.numpy(), sh_degree, cam.camera_center.numpy(),
                                 include_feature)


def small_case(P=2000, W=128, H=96, C=8, seed=0, tanfovx=0.6, big_frac=0.01, logscale_mean=-4.0):
    tanfovy = tanfovx * H / W
    sc = synthetic.make_scene(P, C=C, tanfovx=tanfovx, tanfovy=tanfovy, seed=seed, big_frac=big_frac,
                              logscale_mean=logscale_mean)
    cam = synthetic.origin_camera(W, H, tanfovx)
    return sc, cam


def axis_camera(W=33, H=33, tanfov=0.5):
    return synthetic.make_camera(np.eye(3), np.zeros(3), 2 * math.atan(tanfov), 2 * math.atan(tanfov), W, H)


def image_drift(a, b):
    """Per-pixel max |a - b| over channels ([C,H,W] images): (max, 99.99th percentile, fraction of
    pixels above 1e-4 and above 1e-3)."""
    d = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))
    d = d.reshape(d.shape[0], -1).max(0) if d.size else np.zeros(1)
    return float(d.max()), float(np.quantile(d, 0.9999)), float((d > 1e-4).mean()), float((d > 1e-3).mean())
