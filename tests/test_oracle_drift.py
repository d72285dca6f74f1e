"""How far the reproducible arithmetic can drift from the CUDA original's rounding (CPU only).

The parity oracle (liborc_f32) and the HIP kernels share orc_exp / orc_power (degree-5 minimax exp,
two fma), so the GPU tests' exact T / n_contrib checks compare like with like.  The CUDA original
uses libm-quality expf and nvcc's fma contraction instead.  Its source is absent (parity unpinned,
SURVEY 8c), so this test bounds the drift with two stand-ins at headline resolution (400k
Gaussians, 1352 x 1014, C = 32):
  * liborc_f32_up: float, libm expf, the upstream falloff expression, fma contraction on;
  * liborc_f64:    double, libm exp (the exact answer to float tolerance).
A contributor decision (alpha >= 1/255, T (1 - alpha) >= 1e-4) that flips between two float
builds moves a pixel by up to ~alpha T |c| (~4e-3 here): no two float implementations agree to the
north star's 1e-4 at every pixel of a 1.4M-pixel frame.  What is asserted is that the reproducible
arithmetic is no further from the exact answer than the upstream arithmetic is, and that flips stay
rare (measured: 39 of 1.37M pixels above 1e-4 RGB vs upstream arithmetic; upstream arithmetic vs
fp64: 66).
"""
import numpy as np
import pytest

import oracle
import synthetic
from helpers import image_drift, oracle_settings


@pytest.fixture(scope="module")
def renders():
    sc = synthetic.make_scene(400_000, C=32)
    cam = synthetic.origin_camera()
    s = oracle_settings(cam)
    args = dict(shs=sc.shs.numpy(), lang=sc.lang.numpy(), scales=sc.scales.numpy(), rotations=sc.rotations.numpy())
    out = {}
    for name, kw in (("repro", {}), ("upstream", dict(upstream_arith=True)), ("f64", dict(double=True))):
        r = oracle.forward(s, sc.means3D.numpy(), sc.opacities.numpy(), **args, **kw)
        out[name] = (r.color, r.lang, r.radii)
        r.close()
    return out


def test_reproducible_arithmetic_drift_is_bounded(renders):
    rep, up, ex = renders["repro"], renders["upstream"], renders["f64"]
    # radii / visibility: no exp involved, identical in every build
    assert np.array_equal(rep[2], up[2]) and np.array_equal(rep[2], ex[2])
    ru = image_drift(rep[0], up[0])          # RGB: reproducible vs upstream arithmetic
    ue = image_drift(up[0], ex[0])           # RGB: upstream arithmetic vs fp64
    re = image_drift(rep[0], ex[0])
    lu = image_drift(rep[1], up[1])          # language
    le = image_drift(up[1], ex[1])
    # 99.99 % of pixels inside the north-star tolerances; the rest are decision flips
    assert ru[1] <= 1e-4 and re[1] <= 1e-4 and ue[1] <= 1e-4, (ru, re, ue)
    assert lu[1] <= 1e-3 and le[1] <= 1e-3, (lu, le)
    # flips are rare and no larger than one near-threshold contribution
    assert ru[2] <= 1e-4 and ru[0] <= 1e-2 and lu[0] <= 1e-2, (ru, lu)
    # the reproducible build is as close to the exact answer as the upstream arithmetic is
    assert re[2] <= 2.0 * ue[2] + 1e-5, (re, ue)
