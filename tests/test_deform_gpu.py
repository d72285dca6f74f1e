"""Deformation field forward on the GPU (csrc/deform.hip through include/lsr_deform.h) against
the reference module's golden outputs and the float64 oracle (oracle/deform_oracle.py)."""
import os

import numpy as np
import pytest
import torch

from deform_oracle import DeformOracle
from deformation import DeformationField

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("means3D", "scales", "rotations", "opacity", "shs")


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _field(params, res, multires):
    return DeformationField({k: torch.tensor(np.asarray(v, np.float32)) .cuda() for k, v in params.items()}, res, multires)


def _run(field, inp, time):
    out = field.forward(*[torch.tensor(np.asarray(inp[k], np.float32)).cuda() for k in KEYS],
                        torch.zeros(inp["means3D"].shape[0], 3).cuda(),
                        torch.tensor(np.asarray(time, np.float32)).cuda() if np.ndim(time) else float(time))
    return {k: v.cpu().numpy() for k, v in zip(KEYS, out[:5])}


def test_forward_matches_reference_golden():
    z = np.load(os.path.join(ROOT, "tests", "golden", "deform_golden.npz"))
    params = {k[len("param/"):]: z[k] for k in z.files if k.startswith("param/")}
    params["grid.aabb"] = z["aabb"]
    f = _field(params, list(z["res"]), list(z["multires"]))
    out = _run(f, {k: z[k] for k in KEYS}, z["time"][:, 0])
    for k in KEYS:
        # deformed value = input + MLP offset: compare the offsets (what the kernel computes)
        assert _rel(out[k] - z[k], z["out_" + k] - z[k]) < 2e-5, k


def _neu3d_case(P, seed=0):
    rng = np.random.default_rng(seed)
    res, multires = [64, 64, 64, 150], [1, 2]
    params = {}
    for s, m in enumerate(multires):
        rs = [r * m for r in res[:3]] + [res[3]]
        for ci, (c0, c1) in enumerate([(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]):
            params[f"grid.grids.{s}.{ci}"] = rng.uniform(0.1, 1.5, size=(1, 16, rs[c1], rs[c0]))
    params["grid.aabb"] = np.array([[1.5, 1.2, 3.0], [-1.4, -1.1, 0.5]])
    params["feature_out.0.weight"] = rng.normal(scale=0.2, size=(128, 32))
    params["feature_out.0.bias"] = rng.normal(scale=0.05, size=128)
    for name, n in zip(("pos_deform", "scales_deform", "rotations_deform", "opacity_deform", "shs_deform"),
                       (3, 3, 4, 1, 48)):
        params[name + ".1.weight"] = rng.normal(scale=0.1, size=(128, 128))
        params[name + ".1.bias"] = rng.normal(scale=0.05, size=128)
        params[name + ".3.weight"] = rng.normal(scale=0.1, size=(n, 128))
        params[name + ".3.bias"] = rng.normal(scale=0.05, size=n)
    params = {k: np.asarray(v, np.float32).astype(np.float64) for k, v in params.items()}
    lo, hi = params["grid.aabb"][1], params["grid.aabb"][0]
    inp = dict(means3D=rng.uniform(lo - 0.1, hi + 0.1, size=(P, 3)), scales=rng.normal(-4, 0.5, size=(P, 3)),
               rotations=rng.normal(size=(P, 4)), opacity=rng.normal(size=(P, 1)),
               shs=rng.normal(scale=0.3, size=(P, 16, 3)))
    inp = {k: np.asarray(v, np.float32).astype(np.float64) for k, v in inp.items()}
    return params, res, multires, inp


@pytest.mark.parametrize("P,time", [(20000, 0.37), (777, -0.8)])
def test_forward_matches_oracle_at_neu3d_resolution(P, time):
    params, res, multires, inp = _neu3d_case(P)
    f = _field(params, res, multires)
    out = _run(f, inp, time)                      # scalar time (the render() path)
    o = DeformOracle({k: v for k, v in params.items() if k != "grid.aabb"}, params["grid.aabb"])
    ref = o.forward(inp["means3D"], inp["scales"], inp["rotations"], inp["opacity"], inp["shs"], None,
                    np.full((P, 1), time))
    # three chained Linear layers on bf16 hi/lo operands (16 significant bits, ~2^-17 relative per
    # product) and fp32 sampling: held to 1e-4 of each output's range, the north-star RGB bar
    for k in KEYS:
        assert _rel(out[k] - inp[k], ref[k] - inp[k]) < 1e-4, k


# ---- backward (lsr_deform_backward) --------------------------------------------------------------
def test_backward_matches_reference_golden():
    """Input and parameter gradients against the reference module's autograd (float64 golden)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "deform_golden.npz"))
    params = {k[len("param/"):]: z[k] for k in z.files if k.startswith("param/")}
    params["grid.aabb"] = z["aabb"]
    f = _field(params, list(z["res"]), list(z["multires"]))
    t = lambda a: torch.tensor(np.asarray(a, np.float32)).cuda()   # noqa: E731
    f.zero_grad()
    got = f.backward(t(z["means3D"]), t(z["time"][:, 0]), t(z["up_means3D"]), t(z["up_scales"]),
                     t(z["up_rotations"]), t(z["up_opacity"]), t(z["up_shs"]))
    torch.cuda.synchronize()
    for k, g in zip(KEYS, got):
        assert _rel(g.cpu().numpy().reshape(z["grad_" + k].shape), z["grad_" + k]) < 1e-4, k
    for name, g in f.grads.items():
        ref = z["grad/" + name]
        assert _rel(g.cpu().numpy().reshape(ref.shape), ref) < 1e-4, name


def _morton(pts):
    """Order of the points along a 30-bit Morton curve of their bounding box."""
    q = ((pts - pts.min(0)) / np.maximum(np.ptp(pts, 0), 1e-12) * 1023).astype(np.int64)
    code = np.zeros(len(pts), np.int64)
    for bit in range(10):
        for c in range(3):
            code |= ((q[:, c] >> bit) & 1) << (3 * bit + c)
    return np.argsort(code, kind="stable")


@pytest.mark.parametrize("P,time", [(20000, 0.37), (777, -0.8), (3000, 1.0), (3000, -1.0), (20000, "mixed"),
                                    (20000, "views3"), (20000, "views10"), (20000, "morton"),
                                    (20000, "morton_dense"), (20000, "morton_views3")])
def test_backward_matches_oracle_at_neu3d_resolution(P, time):
    """Neu3D resolution (64^3 x 150, multires [1, 2]); gradients accumulate over two calls.  One time
    for all Gaussians (the render path: the time planes go through per-plane x-rows folded into the
    two rows of that time); +-1 put those taps on the clamped border rows (y1 == y0 at +1, weight 0
    on the second row at -1); "mixed": time 0.37 but every 97th Gaussian at -0.55, so that most waves
    take the x-rows and the rest the four-tap scatter; "views3" / "views10": consecutive runs of
    Gaussians at 3 / 10 times (a batched call of several views: the first view's waves take the
    x-rows, the others the four-tap scatter).  "morton*": the Gaussians stored along a Morton curve,
    so that a wave's Gaussians share most of their cells and its atomics add into the same words
    back to back: at time 0.37 over the whole box, squeezed into a box of 1/6 the extent, and at 3
    times (the time planes through the four-tap scatter)."""
    params, res, multires, inp = _neu3d_case(P, seed=3)
    morton = isinstance(time, str) and time.startswith("morton")
    if morton:
        if time == "morton_dense":
            c = inp["means3D"].mean(0)
            inp["means3D"] = c + (inp["means3D"] - c) / 6.0
        time = "views3" if time == "morton_views3" else 0.37
    # the bilinear slope jumps at grid lines: keep the points 1e-3 cells away from every line (and
    # from the clamped borders), where float32 and float64 coordinates could pick different cells
    a0, a1 = params["grid.aabb"][0], params["grid.aabb"][1]
    crd = (inp["means3D"] - a0) * (2.0 / (a1 - a0)) - 1.0
    keep = np.ones(P, bool)
    for m in multires:
        for c in range(3):
            u = (crd[:, c] + 1.0) * 0.5 * (res[c] * m - 1)
            keep &= np.abs(u - np.round(u)) > 1e-3
    inp = {k: v[keep] for k, v in inp.items()}
    P = int(keep.sum())
    if morton:
        order = _morton(inp["means3D"])
        inp = {k: v[order] for k, v in inp.items()}
    scalar = not isinstance(time, str)
    times = np.full((P, 1), time if scalar else 0.37)
    if time == "mixed":
        times[::97] = -0.55
    elif time.startswith("views") if not scalar else False:
        nv = int(time[5:])
        times[:, 0] = np.linspace(-0.9, 0.95, nv)[np.arange(P) * nv // P]
    f = _field(params, res, multires)
    rng = np.random.default_rng(5)
    ups = dict(means3D=rng.normal(size=(P, 3)), scales=rng.normal(size=(P, 3)), rotations=rng.normal(size=(P, 4)),
               opacity=rng.normal(size=(P, 1)), shs=rng.normal(size=(P, 16, 3)) * 0.1)
    o = DeformOracle({k: v for k, v in params.items() if k != "grid.aabb"}, params["grid.aabb"])
    o.forward(inp["means3D"], inp["scales"], inp["rotations"], inp["opacity"], inp["shs"], None, times)
    # A ReLU input within the kernel's error (~1e-5) of 0 may fall on the other side than in float64
    # and legitimately change that Gaussian's gradients: such Gaussians (|pre-activation| < 1e-4 in
    # the oracle) get zero upstream gradients in both runs, which removes their every contribution.
    _, _, h, _, cache, _ = o._cache
    amb = (np.abs(h) < 1e-4).any(axis=1)
    for z, _ in cache.values():
        amb |= (np.abs(z) < 1e-4).any(axis=1)
    assert amb.mean() < 0.3               # 768 pre-activations per Gaussian: ~17% have one that close
    for k in KEYS:
        ups[k][amb] = 0.0
    g_in, g_p = o.backward(*[np.asarray(ups[k], np.float32).astype(np.float64) for k in KEYS])
    t = lambda a: torch.tensor(np.asarray(a, np.float32)).cuda()   # noqa: E731
    f.zero_grad()
    for _ in range(2):
        got = f.backward(t(inp["means3D"]), time if scalar else t(times[:, 0]), *[t(ups[k]) for k in KEYS])
    torch.cuda.synchronize()
    # bf16 hi/lo MFMA products (~2^-17 relative) and fp32 atomics: 1e-4 of each tensor's range
    assert _rel(got[0].cpu().numpy(), g_in["means3D"]) < 1e-4
    for name, g in f.grads.items():
        assert _rel(g.cpu().numpy() / 2.0, g_p[name].reshape(g.shape)) < 1e-4, name


def test_apply_autograd_path():
    """apply(): outputs match forward(), and torch autograd reaches the inputs through the kernel."""
    params, res, multires, inp = _neu3d_case(500, seed=4)
    f = _field(params, res, multires)
    xs = [torch.tensor(np.asarray(inp[k], np.float32)).cuda().requires_grad_(True) for k in KEYS]
    outs = f.apply(*xs, None, 0.25)
    ref = f.forward(*[x.detach() for x in xs], None, 0.25)
    for a, b in zip(outs[:5], ref[:5]):
        assert torch.equal(a.detach(), b)
    f.zero_grad()
    (outs[0].sum() + 2.0 * outs[4].sum()).backward()
    assert torch.equal(xs[4].grad, torch.full_like(xs[4], 2.0)) and torch.equal(xs[1].grad, torch.zeros_like(xs[1]))
    assert xs[0].grad.abs().sum() > 0 and f.grads["pos_deform.3.bias"][0].item() == pytest.approx(500.0)


# ---- every switch of scene/deformation.py (tests/golden/deform_variants.npz) ----------------------
VARIANTS = ("hypernerf", "lang", "noresnet", "discrete", "deep")


def _variant_field(name):
    import ast
    from deformation import LANG_DISCRETE, LANG_NORESNET, LANG_PASS, LANG_RESIDUAL
    z = np.load(os.path.join(ROOT, "tests", "golden", "deform_variants.npz"))
    pre = name + "/"
    cfg = ast.literal_eval(str(z[pre + "config"]))
    d = {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}
    params = {k[len("param/"):]: torch.tensor(v).cuda() for k, v in d.items() if k.startswith("param/")}
    params["grid.aabb"] = torch.tensor(d["aabb"]).cuda()
    mode = LANG_PASS if cfg["no_dlang"] else (LANG_DISCRETE if cfg["discrete"] else
                                              (LANG_NORESNET if cfg["no_resnet"] else LANG_RESIDUAL))
    f = DeformationField(params, cfg["res"], cfg["multires"], depth=cfg["depth"], no_dx=cfg["no_dx"],
                         no_ds=cfg["no_ds"], no_dr=cfg["no_dr"], no_do=cfg["no_do"], no_dshs=cfg["no_dshs"],
                         apply_rotation=cfg["apply_rotation"], lang_mode=mode, lang_dim=cfg["lang_dim"],
                         centers=cfg["centers"], time_pe=cfg["time_pe"])
    return f, cfg, d


@pytest.mark.parametrize("name", VARIANTS)
def test_variant_forward_matches_reference(name):
    """HyperNeRF structure (3 scales, 3 heads), lang_deform with / without the residual, the discrete
    centres + coff head, apply_rotation, no_ds / no_dx, defor_depth 2: every output vs the
    reference module (residual outputs compared as offsets, what the kernels compute)."""
    f, cfg, d = _variant_field(name)
    t = lambda k: torch.tensor(d[k]).cuda()   # noqa: E731
    out = f.forward(t("means3D"), t("scales"), t("rotations"), t("opacity"), t("shs"), t("lang"), t("time")[:, 0])
    names = ("means3D", "scales", "rotations", "opacity", "shs", "lang", "coff")
    for k, o in zip(names, out):
        if "out_" + k not in d:
            assert o is None, k
            continue
        ref = d["out_" + k].astype(np.float64)
        got = o.cpu().numpy().astype(np.float64).reshape(ref.shape)
        if k in ("lang", "coff") or (k == "rotations" and cfg["apply_rotation"]):
            assert _rel(got, ref) < 1e-4, k
        else:
            base = d[k].astype(np.float64).reshape(ref.shape)
            if np.abs(ref - base).max() == 0:           # head off: the input itself
                assert np.array_equal(got, base), k
            else:
                assert _rel(got - base, ref - base) < 1e-4, k


def _kink_masked_oracle(name, d, cfg):
    """The float64 oracle (pinned to the reference's autograd by test_deform_oracle.py) on the
    variant's inputs, with the upstream gradients of every Gaussian that has a ReLU input within
    1e-4 of zero set to zero, and its backward.  Random 128-wide layers put ~1/3 of the golden's
    300 Gaussians that close to a kink somewhere; there float32 / bf16-split pre-activations (error
    ~1e-5) may fall on the other side than float64 and legitimately change that Gaussian's
    gradients (the same masking as test_backward_matches_oracle_at_neu3d_resolution).  The language
    inputs reach the kernel exactly (their ReLU decisions cannot differ) and are not masked on."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_deform_oracle import variant
    _, dc, params, _, _ = variant(np.load(os.path.join(ROOT, "tests", "golden", "deform_variants.npz")), name)
    o = DeformOracle(params, d["aabb"], cfg=dc)
    f64 = lambda k: d[k].astype(np.float64)   # noqa: E731
    o.forward(*[f64(k) for k in ("means3D", "scales", "rotations", "opacity", "shs", "lang", "time")])
    zs = o.preactivations()
    if dc.lang_mode in ("residual", "noresnet"):
        zs[-3] = zs[-3][:, dc.lang_dim:]
    amb = np.zeros(d["means3D"].shape[0], bool)
    for v in zs:
        amb |= (np.abs(v) < 1e-4).any(axis=1)
    ups = {k: d["up_" + k].copy() for k in ("means3D", "scales", "rotations", "opacity", "shs", "lang", "coff")
           if "up_" + k in d}
    for v in ups.values():
        v[amb] = 0.0
    g_in, g_p = o.backward(*[ups[k].astype(np.float64) for k in KEYS], up_lang=ups["lang"].astype(np.float64),
                           up_coff=ups["coff"].astype(np.float64) if "coff" in ups else None)
    return ups, g_in, g_p, amb


@pytest.mark.parametrize("name", VARIANTS)
def test_variant_backward_matches_reference(name):
    """Input gradients (means3D through the HexPlane coordinates, rotations through the quaternion
    product, the language input through lang_deform / the discrete combination) and every
    parameter gradient: within 1e-4 against the reference-pinned oracle once the kink-ambiguous
    Gaussians' upstream is zeroed, and against the reference's autograd on the golden's full
    upstream within 5e-2 of each tensor's range (kink flips, see _kink_masked_oracle)."""
    f, cfg, d = _variant_field(name)
    t = lambda a: torch.tensor(a).cuda() if a is not None else None   # noqa: E731
    names = ("means3D", "scales", "rotations", "opacity", "shs", "lang")

    def run(ups):
        f.zero_grad()
        got = f.backward(t(d["means3D"]), t(d["time"][:, 0]), t(ups["up_means3D"]), t(ups["up_scales"]),
                         t(ups["up_rotations"]), t(ups["up_opacity"]), t(ups["up_shs"]), rotations=t(d["rotations"]),
                         lang=t(d["lang"]), d_lang=t(ups.get("up_lang")), d_coff=t(ups.get("up_coff")))
        torch.cuda.synchronize()
        return [g.cpu().numpy() for g in got], {k: v.cpu().numpy() for k, v in f.grads.items()}

    ups, g_in, g_p, amb = _kink_masked_oracle(name, d, cfg)
    assert amb.mean() < 0.5
    got, grads = run({"up_" + k: v for k, v in ups.items()})
    for k, g in zip(names, got):
        assert _rel(g.reshape(g_in[k].shape), g_in[k]) < 1e-4, k
    for k, v in g_p.items():
        assert _rel(grads[k].reshape(v.shape), v) < 1e-4, k
    # every Gaussian: the reference's own gradients, up to the kink flips (a flipped Gaussian moves
    # whole rows of a weight gradient)
    got, grads = run(d)
    ref_grads = {k[len("grad/"):]: v for k, v in d.items() if k.startswith("grad/")}
    assert set(grads) == set(ref_grads)
    for k, g in zip(names, got):
        assert _rel(g.reshape(d["grad_" + k].shape), d["grad_" + k]) < 5e-2, k
    for k, v in ref_grads.items():
        assert _rel(grads[k].reshape(v.shape), v) < 5e-2, k


def test_variant_apply_autograd():
    """apply() with the discrete language and apply_rotation variants inside autograd: the same
    gradients as backward() on the same upstream."""
    for name in ("discrete", "noresnet"):
        f, cfg, d = _variant_field(name)
        xs = [torch.tensor(d[k]).cuda().requires_grad_(True) for k in ("means3D", "scales", "rotations", "opacity",
                                                                        "shs", "lang")]
        outs = f.apply(*xs, torch.tensor(d["time"][:, 0]).cuda())
        loss = sum((o * torch.tensor(d["up_" + k]).cuda()).sum() for o, k in
                   zip(outs, ("means3D", "scales", "rotations", "opacity", "shs", "lang", "coff")) if o is not None)
        f.zero_grad()
        loss.backward()
        t = lambda k: torch.tensor(d[k]).cuda() if k in d else None   # noqa: E731
        ref = f.backward(t("means3D"), t("time")[:, 0], t("up_means3D"), t("up_scales"), t("up_rotations"),
                         t("up_opacity"), t("up_shs"), rotations=t("rotations"), lang=t("lang"), d_lang=t("up_lang"),
                         d_coff=t("up_coff"))
        for x, r, k in zip(xs, ref, ("means3D", "scales", "rotations", "opacity", "shs", "lang")):
            assert _rel(x.grad.cpu().numpy(), r.cpu().numpy().reshape(x.shape)) < 1e-6, (name, k)



def test_discrete_field_in_a_base_stage():
    """A discrete-language field called as render() calls it in the 'base' stages (no_dlang forced,
    zeros [P, language_feature_hiddendim] as the language; gaussian_renderer/__init__.py:99,121-124):
    the geometry heads are those of the full call, the language passes through, coff is None, and
    the autograd backward runs with finite gradients equal to the full call's under a zero language /
    coff upstream."""
    f, cfg, d = _variant_field("discrete")
    P = d["means3D"].shape[0]
    xs = [torch.tensor(d[k]).cuda() for k in ("means3D", "scales", "rotations", "opacity", "shs")]
    t = torch.tensor(d["time"][:, 0]).cuda()
    zeros = torch.zeros(P, f.lang_dim, device="cuda")
    base = f.forward(*xs, zeros, t, no_dlang=True)
    full = f.forward(*xs, torch.tensor(d["lang"]).cuda(), t)
    for k in range(5):
        assert torch.equal(base[k], full[k]), k
    assert base[6] is None and torch.equal(base[5], zeros)
    xg = [x.clone().requires_grad_(True) for x in xs]
    outs = f.apply(*xg, zeros, t, no_dlang=True)
    assert outs[6] is None
    f.zero_grad()
    sum((o * torch.tensor(d["up_" + k]).cuda()).sum()
        for o, k in zip(outs[:5], ("means3D", "scales", "rotations", "opacity", "shs"))).backward()
    grads_base = {k: v.clone() for k, v in f.grads.items()}
    ref = lambda k: torch.tensor(d[k]).cuda()   # noqa: E731
    f.zero_grad()
    full_g = f.backward(ref("means3D"), t, ref("up_means3D"), ref("up_scales"), ref("up_rotations"),
                        ref("up_opacity"), ref("up_shs"), rotations=ref("rotations"), lang=ref("lang"),
                        d_lang=torch.zeros(P, f.lang_dim, device="cuda"), d_coff=torch.zeros(P, f.centers, device="cuda"))
    for x, r, k in zip(xg, full_g, ("means3D", "scales", "rotations", "opacity", "shs")):
        assert torch.isfinite(x.grad).all(), k
        assert _rel(x.grad.cpu().numpy(), r.cpu().numpy().reshape(x.shape)) < 1e-5, k
    for k, v in f.grads.items():
        if k.startswith("discrete_coff_generator"):
            assert float(grads_base[k].abs().max()) == 0.0, k
        else:
            assert torch.isfinite(grads_base[k]).all(), k
            assert _rel(grads_base[k].cpu().numpy(), v.cpu().numpy()) < 1e-5, k

def test_from_reference_is_strict():
    """deform_network.state_dict() + ModelHiddenParams + env: the unused modules the reference always
    builds are skipped; a key the configuration does not compute raises (a defor_depth 2 state dict
    loaded as depth 1), as do unsupported switches."""
    f, cfg, d = _variant_field("hypernerf")
    sd = {"deformation_net." + k: v for k, v in f.p.items()}
    W = 128
    for h, n in (("opacity_deform", 1), ("shs_deform", 48)):   # built but not computed (no_do, no_dshs)
        sd[f"deformation_net.{h}.1.weight"], sd[f"deformation_net.{h}.1.bias"] = torch.zeros(W, W), torch.zeros(W)
        sd[f"deformation_net.{h}.3.weight"], sd[f"deformation_net.{h}.3.bias"] = torch.zeros(n, W), torch.zeros(n)
    sd["timenet.0.weight"], sd["time_poc"] = torch.zeros(64, 9), torch.zeros(4)
    hidden = dict(kplanes_config={"resolution": cfg["res"], "output_coordinate_dim": 16}, multires=cfg["multires"],
                  defor_depth=1, no_dlang=1, net_width=128)
    g = DeformationField.from_reference(sd, hidden, env={"language_feature_hiddendim": "3"})
    assert g.heads_computed() == ["pos_deform", "scales_deform", "rotations_deform"]
    sd2 = dict(sd, **{"deformation_net.feature_out.2.weight": torch.zeros(W, W)})
    with pytest.raises(ValueError, match="feature_out.2.weight"):
        DeformationField.from_reference(sd2, hidden, env={})
    with pytest.raises(ValueError, match="static_mlp"):
        DeformationField.from_reference(sd, dict(hidden, static_mlp=True), env={})
    with pytest.raises(ValueError, match="unexpected"):
        DeformationField({**f.p, "feature_out.2.weight": torch.zeros(W, W).cuda()}, cfg["res"], cfg["multires"],
                         depth=1, no_do=True, no_dshs=True)
