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


VARIANTS = ("hypernerf", "lang", "noresnet", "discrete", "deep")
OUTS = ("means3D", "scales", "rotations", "opacity", "shs", "lang", "coff")


def variant(z, name):
    """One variant of tests/golden/deform_variants.npz: config, params, inputs, outputs, grads."""
    import ast
    from deform_oracle import DeformConfig
    pre = name + "/"
    cfg = ast.literal_eval(str(z[pre + "config"]))
    d = {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}
    params = {k[len("param/"):]: v for k, v in d.items() if k.startswith("param/")}
    grads = {k[len("grad/"):]: v for k, v in d.items() if k.startswith("grad/")}
    return cfg, DeformConfig.from_golden(cfg), params, grads, d


@pytest.fixture(scope="module")
def variants():
    return np.load(os.path.join(ROOT, "tests", "golden", "deform_variants.npz"))


@pytest.mark.parametrize("name", VARIANTS)
def test_oracle_matches_reference_variant(variants, name):
    """Every switch of scene/deformation.py the reference's configs use (make_deform_variants_golden.py):
    outputs, input gradients and parameter gradients of the reference's autograd."""
    cfg, dc, params, grads, d = variant(variants, name)
    o = DeformOracle(params, d["aabb"], cfg=dc)
    f64 = lambda k: d[k].astype(np.float64)   # noqa: E731
    out = o.forward(f64("means3D"), f64("scales"), f64("rotations"), f64("opacity"), f64("shs"), f64("lang"),
                    f64("time"))
    for k in OUTS:
        if "out_" + k in d:
            assert _rel(out[k], d["out_" + k]) < 1e-6, k
    g_in, g = o.backward(*[f64("up_" + k) for k in OUTS[:5]], up_lang=f64("up_lang"),
                         up_coff=f64("up_coff") if "up_coff" in d else None)
    for k in ("means3D", "scales", "rotations", "opacity", "shs", "lang"):
        assert _rel(g_in[k].reshape(d["grad_" + k].shape), d["grad_" + k]) < 1e-5, k
    assert set(g) == set(grads), set(g) ^ set(grads)
    for k, v in grads.items():
        assert _rel(g[k].reshape(v.shape), v) < 1e-5, k
