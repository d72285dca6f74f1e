"""Per-view data-parallel step on the GPU (view_parallel.py): the pipelined
renderer (view v+1's preprocess on a side stream during view v's render and backward) must give
exactly the sequential result, and the accumulated bucket must equal the sum of per-view
gradients."""
import pytest
import torch

import diff_gaussian_rasterization as dgr
import synthetic
from view_parallel import GradBucket, ViewParallelStep, native_view_renderer

pytestmark = pytest.mark.gpu


def _setup(n_views=4, P=20000, W=160, H=120, C=32):
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W, seed=5, logscale_mean=-4.0).to("cuda")
    cams = synthetic.camera_batch(n_views, W, H, tanfovx=0.6, seed=2)
    bg = torch.ones(3, device="cuda")
    settings = [dgr.GaussianRasterizationSettings(H, W, c.tanfovx, c.tanfovy, bg, 1.0, c.world_view_transform.cuda(),
                                                  c.full_proj_transform.cuda(), 3, c.camera_center.cuda(), False,
                                                  False, True) for c in cams]
    g = torch.Generator(device="cpu").manual_seed(7)
    grads = [((torch.randn(3, H, W, generator=g)).cuda(), torch.randn(C, H, W, generator=g).cuda())
             for _ in range(n_views)]
    return sc, settings, grads


def _run(sc, settings, grads, overlap, deterministic, prefill=None, **kw):
    b = GradBucket(sc.means3D.shape[0], sc.shs.shape[1], sc.lang.shape[1], "cuda", densify_stats=True)
    step = ViewParallelStep(b, len(settings))
    r = native_view_renderer(sc, settings, lambda v, c, l, d: (grads[v][0], grads[v][1], None),
                             deterministic=deterministic, overlap=overlap, **kw)
    for _ in range(2):   # second step exercises the pipeline with warm streams and caches
        if prefill is not None:   # whatever the step does not zero or write shows up
            b.flat.fill_(prefill)
            b.radii.fill_(-1)
        step.run(r)
    torch.cuda.synchronize()
    return b.flat.clone(), b.radii.clone()


@pytest.mark.parametrize("mode", [True, "lookahead"])
def test_pipelined_step_equals_sequential(mode):
    """Side-stream pipelining and the one-stream lookahead (deferred instance counts read from
    pinned memory after an event) give the sequential result bit for bit."""
    sc, settings, grads = _setup()
    f0, r0 = _run(sc, settings, grads, overlap=False, deterministic=True)
    f1, r1 = _run(sc, settings, grads, overlap=mode, deterministic=True)
    assert torch.equal(f0, f1) and torch.equal(r0, r1)
    assert float(f0.abs().sum()) > 0 and int((r0 > 0).sum()) > 0


def test_pipelined_step_waits_for_side_stream_binning(monkeypatch):
    """The side stream's binning is held back (about 20 ms per view) so that the main stream would
    composite unfinished lists if it did not wait for it."""
    sc, settings, grads = _setup(n_views=3)
    f0, r0 = _run(sc, settings, grads, overlap=False, deterministic=True)
    monkeypatch.setattr(dgr, "_BINNING_DELAY_CYCLES", 40_000_000)
    f1, r1 = _run(sc, settings, grads, overlap=True, deterministic=True)
    assert torch.equal(f0, f1) and torch.equal(r0, r1)


@pytest.mark.parametrize("mode", [True, "lookahead"])
def test_bucket_is_sum_of_views(mode):
    sc, settings, grads = _setup(n_views=3)
    # batched backward: the flush overwrites every field but the language gradients, which are
    # the only ones zeroed before the views; NaN-filled buckets prove every row is written
    flat, radii = _run(sc, settings, grads, overlap=mode, deterministic=False, prefill=float("nan"))
    assert not torch.isnan(flat).any()
    b = GradBucket(sc.means3D.shape[0], sc.shs.shape[1], sc.lang.shape[1], "cuda", densify_stats=True)
    ref = torch.zeros_like(b.flat)
    rmax = torch.zeros_like(radii)
    for v, rs in enumerate(settings):
        _, _, rad, _, st = dgr.forward_native(rs, sc.means3D, sc.opacities, shs=sc.shs, language_feature=sc.lang,
                                              scales=sc.scales, rotations=sc.rotations)
        g = dgr.backward_native(st, grads[v][0], grads[v][1], None, need=b.need())
        o = 0
        for name in ("means3D", "scales", "rotations", "opacities", "sh", "language_feature", "means2D"):
            t = g[name].reshape(-1, b.views[name].reshape(b.P, -1).shape[1])
            w = t.shape[1]
            ref[o * b.P:(o + w) * b.P] += t.reshape(-1)
            o += w
        rmax = torch.maximum(rmax, rad)
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    assert float((flat - ref).abs().max()) <= 1e-4 * scale
    assert torch.equal(radii, rmax)


def test_language_split_bits():
    """lsr_language_split writes, per Gaussian, bf16(x) for the 32 channels then bf16(x - bf16(x))
    (round to nearest even, as torch's conversion)."""
    g = torch.Generator(device="cpu").manual_seed(3)
    lang = torch.randn(1001, 32, generator=g).cuda()
    lang[0, :4] = torch.tensor([0.0, -0.0, 1e-30, 3.0e38])
    out = dgr.language_split_native(lang)
    hi = lang.to(torch.bfloat16)
    lo = (lang - hi.float()).to(torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :32], hi.view(torch.int16)) and torch.equal(out[:, 32:], lo.view(torch.int16))


def test_batched_forward_with_language_split_is_bit_identical():
    """The batched preprocess + binning with the precomputed bf16 operands (split_language) renders
    every view bit for bit as the single-view forward, whose compositors split the rows themselves;
    the compositor backward's language gradient agrees within float-atomic reordering."""
    sc, settings, grads = _setup(n_views=3)
    args = dict(shs=sc.shs, language_feature=sc.lang, scales=sc.scales, rotations=sc.rotations)
    pfs = dgr.preprocess_views_native(settings, sc.means3D, sc.opacities, **args)
    assert "language_feature_split" in pfs[0].inputs
    dgr.binning_views_native(pfs)
    for v, (rs, pf) in enumerate(zip(settings, pfs)):
        c1, l1, r1, d1, st1 = dgr.render_native(pf)
        c0, l0, r0, d0, st0 = dgr.forward_native(rs, sc.means3D, sc.opacities, **args)
        assert torch.equal(c0, c1) and torch.equal(l0, l1) and torch.equal(r0, r1) and torch.equal(d0, d1)
        g0 = torch.zeros_like(sc.lang)
        g1 = torch.zeros_like(sc.lang)
        dgr.backward_composite_native(st0, grads[v][0], grads[v][1], None, dL_dlanguage=g0)
        dgr.backward_composite_native(st1, grads[v][0], grads[v][1], None, dL_dlanguage=g1)
        torch.cuda.synchronize()
        scale = float(g0.abs().max())
        assert scale > 0 and float((g0 - g1).abs().max()) <= 1e-5 * scale


@pytest.mark.parametrize("early", [1, 2])
def test_batched_side_binning_agrees(early):
    """The batched forward with the later views binned on a side stream (early_views) gives the
    one-stream result: radii exactly, the float-atomic bucket within 1e-5."""
    kw = dict(early_views=early)
    sc, settings, grads = _setup(n_views=4)
    f0, r0 = _run(sc, settings, grads, overlap="batched", deterministic=False, early_views=0)
    f1, r1 = _run(sc, settings, grads, overlap="batched", deterministic=False, prefill=float("nan"), **kw)
    assert not torch.isnan(f1).any() and torch.equal(r0, r1)
    scale = float(f0.abs().max())
    assert scale > 0 and float((f0 - f1).abs().max()) <= 1e-5 * scale


def _away_settings(W=160, H=120):
    """A camera turned 180 degrees about y: every Gaussian of _setup's scene is behind it (K = 0)."""
    import math
    import numpy as np
    fx = 2 * math.atan(0.6)
    fy = 2 * math.atan(0.6 * H / W)
    c = synthetic.make_camera(np.diag([-1.0, 1.0, -1.0]), np.zeros(3), fx, fy, W, H)
    return dgr.GaussianRasterizationSettings(H, W, c.tanfovx, c.tanfovy, torch.ones(3, device="cuda"), 1.0,
                                             c.world_view_transform.cuda(), c.full_proj_transform.cuda(), 3,
                                             c.camera_center.cuda(), False, False, True)


@pytest.mark.parametrize("split", [True, False])
def test_composite_views_equals_per_view(split):
    """lsr_forward_composite_views / lsr_backward_composite_views (one launch for a batch of views,
    one of them with nothing listed) against the per-view launches on the same binned views:
    images, depth and radii bit for bit, the compositor backward's sums within float-atomic
    reordering (language gradients and, through the batched preprocess backward, every other
    gradient)."""
    sc, settings, grads = _setup(n_views=4)
    settings = settings[:2] + [_away_settings()] + settings[2:]
    grads = grads[:2] + [grads[0]] + grads[2:]
    args = dict(shs=sc.shs, language_feature=sc.lang, scales=sc.scales, rotations=sc.rotations)
    outs, gls, bwd = [], [], []
    for batched in (False, True):
        pfs = dgr.preprocess_views_native(settings, sc.means3D, sc.opacities, split_language=split, **args)
        dgr.binning_views_native(pfs)
        res = dgr.render_views_native(pfs) if batched else [dgr.render_native(pf) for pf in pfs]
        gl = torch.zeros_like(sc.lang)
        sts = [r[4] for r in res]
        if batched:
            parts = dgr.backward_composite_views_native(sts, [g[0] for g in grads], [g[1] for g in grads],
                                                        dL_dlanguage=gl)
        else:
            parts = [dgr.backward_composite_native(st, g[0], g[1], None, dL_dlanguage=gl) for st, g in zip(sts, grads)]
        b = GradBucket(sc.means3D.shape[0], sc.shs.shape[1], sc.lang.shape[1], "cuda", densify_stats=True)
        dgr.backward_preprocess_views_native(parts, out=b.views, accumulate=False, need=b.need())
        torch.cuda.synchronize()
        outs.append([(c.clone(), l.clone(), r.clone(), d.clone(), st.num_rendered) for c, l, r, d, st in res])
        gls.append(gl)
        bwd.append(b.flat.clone())
    assert outs[0][2][4] == 0 and all(o[4] > 0 for i, o in enumerate(outs[0]) if i != 2)
    for a, c in zip(outs[0], outs[1]):
        assert a[4] == c[4]
        for x, y in zip(a[:4], c[:4]):
            assert torch.equal(x, y)
    for x, y in ((gls[0], gls[1]), (bwd[0], bwd[1])):
        scale = float(x.abs().max())
        assert scale > 0 and float((x - y).abs().max()) <= 1e-5 * scale


@pytest.mark.parametrize("early,fill_side,order_side", [(0, False, False), (3, False, False), (3, True, False),
                                                       (3, False, True), (1, False, True), ((1, 2), False, False),
                                                       ((1, 1, 1), False, False), ((1, 2), False, True)])
def test_batched_composite_step_agrees(early, fill_side, order_side):
    """ViewParallelStep through render_batch (the bench default: one compositor launch per binning
    batch) against the per-view compositor launches of the same batched pipeline; fill_side: the
    language split, bucket zeroing and radii MAX on the side stream (a NaN-prefilled bucket shows
    any compositor that runs before the zeroing); order_side: the later views' depth sorts on the
    side stream too, binned after the early views' compositing is enqueued; a tuple: several side
    binning batches, each composited once its own binning is done."""
    sc, settings, grads = _setup(n_views=5)
    f0, r0 = _run(sc, settings, grads, overlap="batched", deterministic=False, early_views=early,
                  composite_batch=False)
    f1, r1 = _run(sc, settings, grads, overlap="batched", deterministic=False, prefill=float("nan"),
                  early_views=early, fill_on_side=fill_side, order_on_side=order_side)
    assert not torch.isnan(f1).any() and torch.equal(r0, r1)
    scale = float(f0.abs().max())
    assert scale > 0 and float((f0 - f1).abs().max()) <= 1e-5 * scale


def test_radii_max_native():
    """lsr_radii_max against torch: the vector rows and the scalar tail, more views than one launch
    takes (8), accumulate on and off."""
    g = torch.Generator(device="cpu").manual_seed(4)
    for P in (1, 7, 1001, 4096):
        rs = [torch.randint(0, 50, (P,), generator=g, dtype=torch.int32).cuda() for _ in range(11)]
        out = torch.full((P,), 7, dtype=torch.int32, device="cuda")
        dgr.radii_max_native(rs, out, accumulate=True)
        ref = torch.clamp_min(torch.stack(rs).amax(0), 7)
        assert torch.equal(out, ref)
        dgr.radii_max_native(rs[:3], out)
        assert torch.equal(out, torch.stack(rs[:3]).amax(0))


@pytest.mark.parametrize("C,include", [(0, True), (3, True), (16, True), (32, False)])
def test_composite_views_other_channel_counts(C, include):
    """The batched compositor launches of the other instantiations (VALU channel sums for C <= 16,
    the no-language backward for C = 0 or include_feature off) against the per-view launches."""
    sc, settings, grads = _setup(n_views=3, C=C)
    settings = [s._replace(include_feature=include) for s in settings]
    args = dict(shs=sc.shs, language_feature=sc.lang if C > 0 else None, scales=sc.scales, rotations=sc.rotations)
    outs, gls, bwd = [], [], []
    for batched in (False, True):
        pfs = dgr.preprocess_views_native(settings, sc.means3D, sc.opacities, **args)
        dgr.binning_views_native(pfs)
        res = dgr.render_views_native(pfs) if batched else [dgr.render_native(pf) for pf in pfs]
        gl = torch.zeros(sc.means3D.shape[0], C, device="cuda")
        sts = [r[4] for r in res]
        gcs = [g[0] for g in grads]
        gll = [g[1] if C > 0 else None for g in grads]
        if batched:
            parts = dgr.backward_composite_views_native(sts, gcs, gll, dL_dlanguage=gl if C > 0 else None)
        else:
            parts = [dgr.backward_composite_native(st, a, b, None, dL_dlanguage=gl if C > 0 else None)
                     for st, a, b in zip(sts, gcs, gll)]
        b = GradBucket(sc.means3D.shape[0], sc.shs.shape[1], C, "cuda", densify_stats=True)
        dgr.backward_preprocess_views_native(parts, out=b.views, accumulate=False, need=b.need())
        torch.cuda.synchronize()
        outs.append([(c.clone(), l.clone(), r.clone(), d.clone()) for c, l, r, d, _ in res])
        gls.append(gl)
        bwd.append(b.flat.clone())
    for a, c in zip(outs[0], outs[1]):
        for x, y in zip(a, c):
            assert torch.equal(x, y)
    scale = float(bwd[0].abs().max())
    assert scale > 0 and float((bwd[0] - bwd[1]).abs().max()) <= 1e-5 * scale
    if C > 0 and include:
        s2 = float(gls[0].abs().max())
        assert s2 > 0 and float((gls[0] - gls[1]).abs().max()) <= 1e-5 * s2
