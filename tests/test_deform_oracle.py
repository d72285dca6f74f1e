"""The deformation oracle (oracle/deform_oracle.py) against the reference module's own outputs and
autograd gradients (tests/golden/deform_golden.npz, made by tests/golden/make_deform_golden.py)."""
import os

import numpy as np
import pytest

from deform_oracle import DeformOracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "deform_golden.npz"))


def _oracle(z):
    params = {k[len("param/"):]: z[k] for k in z.files if k.startswith("param/")}
    return DeformOracle(params, z["aabb"])


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def test_forward_matches_reference(golden):
    z = golden
    o = _oracle(z)
    out = o.forward(z["means3D"], z["scales"], z["rotations"], z["opacity"], z["shs"], z["lang"], z["time"])
    for k in ("means3D", "scales", "rotations", "opacity", "shs", "lang"):
        assert _rel(out[k], z["out_" + k]) < 1e-12, k


def test_backward_matches_reference(golden):
    z = golden
    o = _oracle(z)
    o.forward(z["means3D"], z["scales"], z["rotations"], z["opacity"], z["shs"], z["lang"], z["time"])
    g_in, g_p = o.backward(z["up_means3D"], z["up_scales"], z["up_rotations"], z["up_opacity"], z["up_shs"])
    for k in ("means3D", "scales", "rotations", "opacity", "shs"):
        assert _rel(g_in[k], z["grad_" + k]) < 1e-10, k
    for k in z.files:
        if k.startswith("grad/"):
            name = k[len("grad/"):]
            assert _rel(g_p[name], z[k]) < 1e-10, name


def test_golden_exercises_border_and_time(golden):
    z = golden
    a0, a1 = z["aabb"]
    pn = (z["means3D"] - a0) * (2.0 / (a1 - a0)) - 1.0
    assert (np.abs(pn) > 1).any(axis=1).sum() > 20          # points outside the box (border clamp)
    assert len(np.unique(z["time"])) > 10 and (np.abs(z["time"]) > 1).any()
