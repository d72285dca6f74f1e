"""The config-5 loop end to end on the GPU (train_step.TrainStep): deformation field (autograd
through lsr_deform_backward) -> rasterizer for 2 views -> L1 -> backward -> densification
statistics -> Adam on the Gaussians (lsr_adam_step) and on the field (TensorAdam), densify and
prune between iterations.  No oracle: the check is that the pieces compose (shapes, gradient
flow, every parameter moves) and that the loss falls when fitting renders of a teacher scene."""
import dataclasses
import math

import numpy as np
import pytest
import torch

import synthetic
from deformation import DeformationField
from gaussian_scene import render, render_views
from gaussian_train import GaussianTrainer
from train_step import TrainStep

pytestmark = pytest.mark.gpu
AABB = [[7.0, 5.5, 10.5], [-7.0, -5.5, 1.5]]
RES, MULTIRES = [16, 16, 16, 10], [1, 2]
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-2, "f_rest": 2.5e-2 / 20, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3}


def _raw(sc, P):
    shs = sc.shs
    return {"xyz": sc.means3D.contiguous(), "f_dc": shs[:, :1].contiguous(), "f_rest": shs[:, 1:].contiguous(),
            "opacity": torch.logit(sc.opacities.reshape(P, 1)).contiguous(),
            "scaling": torch.log(sc.scales).contiguous(), "rotation": sc.rotations.contiguous()}


def test_train_loop_fits_teacher():
    P, W, H = 4000, 160, 120
    dev = torch.device("cuda")
    sc = synthetic.make_scene(P, C=3, tanfovx=0.6, tanfovy=0.6 * H / W, seed=3, logscale_mean=-3.0).to(dev)
    cams = synthetic.camera_batch(2, W, H, tanfovx=0.6, seed=2)
    field_p = DeformationField.init_params(RES, MULTIRES, AABB, seed=1)
    teacher_field = DeformationField({k: v.to(dev) for k, v in field_p.items()}, RES, MULTIRES)
    teacher = GaussianTrainer(_raw(sc, P), LRS)
    with torch.no_grad():
        tscene = TrainStep(teacher, teacher_field).scene()
        gts = torch.stack([render(c, tscene, torch.ones(3, device=dev), stage="fine-base")["render"] for c in cams])
    # student: the same geometry and field, colours perturbed
    raw = _raw(sc, P)
    g = torch.Generator(device="cpu").manual_seed(9)
    raw["f_dc"] = raw["f_dc"] + (torch.randn(P, 1, 3, generator=g) * 0.5).to(dev)
    field = DeformationField({k: v.to(dev) for k, v in field_p.items()}, RES, MULTIRES)
    tr = GaussianTrainer(raw, LRS)
    step = TrainStep(tr, field)
    plane0 = field.p["grid.grids.1.3"].clone()
    w0 = field.p["pos_deform.3.weight"].clone()
    losses = []
    for it in range(16):
        losses.append(float(step(cams, gts)))
        if it == 7:   # the densification / pruning passes between iterations (train.py:388-414)
            n_clone, n_split = tr.densify(1e-9, 0.005, 8.0)
            assert tr.P == P + n_clone + n_split and n_clone + n_split > 0
            tr.prune(1e-9, 0.0, 8.0, None)
    torch.cuda.synchronize()
    assert all(math.isfinite(x) for x in losses), losses
    # the loss falls while fitting; the densify at iteration 7 (every visible Gaussian cloned or split
    # at this threshold) perturbs the fit, after which it falls again
    assert losses[7] < 0.8 * losses[0] and losses[15] < losses[8], losses
    assert tr.steps["f_dc"] == 16 and not torch.equal(field.p["pos_deform.3.weight"], w0)
    assert not torch.equal(field.p["grid.grids.1.3"], plane0)
    assert tr.denom.shape[0] == tr.P and np.isfinite(tr.xyz_gradient_accum.cpu().numpy()).all()


def test_densify_callback_runs_before_the_step():
    """train.py:388-421 order: densification statistics -> densify / prune / reset_opacity ->
    optimizer.step().  On the iterations the callback rebuilds the rows (densify, prune) the
    Gaussian groups have no gradient and Adam skips them, as the reference's optimizer skips its
    fresh nn.Parameters; after a reset only the opacity group is skipped; the field always steps."""
    P, W, H = 3000, 128, 96
    dev = torch.device("cuda")
    sc = synthetic.make_scene(P, C=3, tanfovx=0.6, tanfovy=0.6 * H / W, seed=4, logscale_mean=-3.0).to(dev)
    cams = synthetic.camera_batch(2, W, H, tanfovx=0.6, seed=2)
    field_p = DeformationField.init_params(RES, MULTIRES, AABB, seed=1)
    field = DeformationField({k: v.to(dev) for k, v in field_p.items()}, RES, MULTIRES)
    tr = GaussianTrainer(_raw(sc, P), LRS)
    gts = torch.rand(2, 3, H, W, device=dev)
    calls = []

    def schedule(t, it):
        calls.append((it, t.P))
        if it == 3:
            t.densify(1e-9, 0.005, 8.0)
        if it == 5:
            t.reset_opacity()

    step = TrainStep(tr, field, densify=schedule)
    for _ in range(6):
        step(cams, gts)
    torch.cuda.synchronize()
    assert [c[0] for c in calls] == [1, 2, 3, 4, 5, 6]
    assert tr.P > P and calls[3][1] == tr.P           # rows rebuilt at iteration 3, seen from 4 on
    assert tr.steps["f_dc"] == 5 and tr.steps["xyz"] == 5   # iteration 3 skipped
    assert tr.steps["opacity"] == 4                          # iterations 3 and 5 skipped
    assert all(p.grad is None for p in tr.params.values())


def test_reference_schedule_loop_fits_teacher():
    """The configs[4] loop in miniature (tools/bench_train_loop.py at full size): create_from_pcd
    init, the reference's learning-rate schedules, ReferenceSchedule densify / prune on a shortened
    schedule; the mean loss falls window over window."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench_train_loop", os.path.join(os.path.dirname(__file__), "..", "tools", "bench_train_loop.py"))
    btl = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(btl)
    from train_step import ReferenceSchedule
    args = type("A", (), dict(gaussians=3000, width=160, height=120, cameras=4, frames=2, point_noise=0.02,
                              densify_until_iter=10_000))()
    dev = torch.device("cuda")
    step, _, pool, gts, extent = btl.build(args, dev)
    sched = ReferenceSchedule(extent, densify_from_iter=10, densification_interval=10, pruning_from_iter=10,
                              pruning_interval=20, densify_until_iter=60, min_points=3000)
    step.densify = sched
    g = torch.Generator().manual_seed(1)
    windows, acc = [], 0.0
    for it in range(1, 81):
        idx = torch.randperm(len(pool), generator=g)[:2].tolist()
        acc += float(step([pool[i] for i in idx], gts[idx], iteration=it))
        if it % 20 == 0:
            windows.append(acc / 20)
            acc = 0.0
    kinds = [(e[0], e[1]) for e in sched.events]
    assert kinds[:3] == [(20, "densify"), (20, "prune"), (30, "densify")], sched.events
    assert all(e[0] < 60 for e in sched.events)          # nothing past densify_until_iter
    assert all(b < a for a, b in zip(windows, windows[1:])), windows
    assert step.trainer.denom.shape[0] == step.trainer.P
    assert step.trainer.lrs["xyz"] < 1.6e-4 * extent     # the xyz schedule decays


def test_render_views_matches_per_view_render():
    """render_views (one deformation launch over V * P rows) against render() per view: the field
    is per row, so images and radii are bit-identical; the Gaussians' and the field's gradients
    agree up to the summation order of the atomics and of the views."""
    P, W, H = 3000, 128, 96
    dev = torch.device("cuda")
    sc = synthetic.make_scene(P, C=3, tanfovx=0.6, tanfovy=0.6 * H / W, seed=5, logscale_mean=-3.0).to(dev)
    cams = synthetic.camera_batch(3, W, H, tanfovx=0.6, seed=2)
    cams = [dataclasses.replace(c, time=0.2 + 0.3 * i) for i, c in enumerate(cams)]
    field_p = DeformationField.init_params(RES, MULTIRES, AABB, seed=1)
    gts = torch.rand(len(cams), 3, H, W, device=dev)
    res = []
    for batched in (False, True):
        field = DeformationField({k: v.to(dev) for k, v in field_p.items()}, RES, MULTIRES)
        tr = GaussianTrainer(_raw(sc, P), LRS)
        step = TrainStep(tr, field, batch_views=batched)
        field.zero_grad()
        scene = step.scene()
        outs = render_views(cams, scene, step.bg, stage="fine-base") if batched else \
            [render(c, scene, step.bg, stage="fine-base") for c in cams]
        images = torch.stack([o["render"] for o in outs])
        (images - gts).abs().mean().backward()
        torch.cuda.synchronize()
        res.append(dict(images=images.detach(), radii=torch.stack([o["radii"] for o in outs]),
                        vs=torch.stack([o["viewspace_points"].grad for o in outs]),
                        g={k: v.grad.clone() for k, v in tr.params.items()},
                        f={k: v.clone() for k, v in field.grads.items()}))
    a, b = res
    assert torch.equal(a["images"], b["images"]) and torch.equal(a["radii"], b["radii"])
    torch.testing.assert_close(b["vs"], a["vs"], rtol=1e-4, atol=1e-9)
    for k in a["g"]:   # float atomics and the view sums reorder: max-normalised, as for the field below
        scale = float(a["g"][k].abs().max())
        err = float((b["g"][k] - a["g"][k]).abs().max())
        assert err <= 1e-5 * scale + 1e-12, (k, err, scale)
    for k in a["f"]:
        scale = float(a["f"][k].abs().max())
        err = float((b["f"][k] - a["f"][k]).abs().max())
        assert err <= 1e-4 * scale + 1e-12, (k, err, scale)


def test_configs4_standin_at_size():
    """BASELINE configs[4] at its stand-in size (tools/bench_train_loop.py): 100k
    Gaussians from create_from_pcd + distCUDA2, 2 views of 1352 x 1014 per iteration, the Neu3D field
    (64^3 x 150, multires [1, 2]), ReferenceSchedule with the Neu3D overrides, fine-base, 700
    iterations so the first densify (iteration 600, train.py:388-414 / arguments/neu3d/default.py:24-33)
    fires.  Checks: the window losses fall up to the densify and stay below the first window after it;
    densify events land on the reference iterations; the statistics track P; everything stays finite.
    At iteration 650 one view's rasterizer call is checked against the C oracle: the Gaussian gradients
    the training step's backward produced (inside autograd, on the training inputs) against the
    oracle's backward on the same inputs and upstream gradient."""
    import importlib.util
    import os

    import diff_gaussian_rasterization as dgr
    import oracle
    from lsr_testutil import grad_err

    spec = importlib.util.spec_from_file_location(
        "bench_train_loop", os.path.join(os.path.dirname(__file__), "..", "tools", "bench_train_loop.py"))
    btl = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(btl)
    args = type("A", (), dict(gaussians=100_000, width=1352, height=1014, cameras=8, frames=4, point_noise=0.02,
                              densify_until_iter=10_000))()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    step, sched, pool, gts, extent = btl.build(args, dev)
    P0 = step.trainer.P
    assert P0 == 100_000 and tuple(gts.shape) == (32, 3, 1014, 1352)
    order = torch.Generator().manual_seed(5)
    captured = []
    real_backward = dgr.backward_native

    def capture(state, grad_color, *a, **kw):     # one view of one iteration: inputs, upstream grad, result
        g = real_backward(state, grad_color, *a, **kw)
        captured.append((state.settings, {k: (None if v is None else v.detach().cpu()) for k, v in state.inputs.items()},
                         grad_color.detach().cpu(), {k: (None if v is None else v.detach().cpu()) for k, v in g.items()}))
        return g

    windows, acc, iters, window = [], torch.zeros((), device=dev), 700, 100
    for it in range(1, iters + 1):
        idx = torch.randperm(len(pool), generator=order)[:2].tolist()
        if it == 650:
            dgr.backward_native = capture
        try:
            acc += step([pool[i] for i in idx], gts[idx], iteration=it)
        finally:
            dgr.backward_native = real_backward
        if it == 650:
            cams650 = [pool[i] for i in idx]
        if it % window == 0:
            windows.append(float(acc) / window)
            acc.zero_()
    torch.cuda.synchronize()
    tr = step.trainer
    assert all(math.isfinite(w) for w in windows), windows
    # falls window over window up to the densify at 600; the densify moves the image (clone / split),
    # after which the window stays well below the first
    assert all(b < a for a, b in zip(windows[:6], windows[1:6])), windows
    assert windows[6] < 0.5 * windows[0], windows
    ev = [(e[0], e[1]) for e in sched.events]
    assert ev and ev[0] == (600, "densify") and all(e[0] % 100 == 0 and e[0] > 500 for e in ev), sched.events
    assert sched.events[0][2] == P0 and tr.P == sched.events[-1][3] > P0
    assert tr.denom.shape[0] == tr.P and tr.xyz_gradient_accum.shape[0] == tr.P and tr.max_radii2D.shape[0] == tr.P
    for k, v in tr.params.items():
        assert torch.isfinite(v).all(), k
    for k, v in step.field.p.items():
        assert torch.isfinite(v).all(), k
    # the oracle check on one of iteration 650's two views (matched to its camera by the view matrix)
    assert len(captured) == 2
    st, inp, gcol, g = captured[0]
    view = st.view.detach().cpu().reshape(4, 4)
    cam650 = [cam for cam in cams650 if torch.equal(cam.world_view_transform.detach().cpu().float(), view)]
    assert len(cam650) >= 1
    cam650 = cam650[0]
    c = st.c
    assert inp["colors_precomp"] is None and inp["cov3D_precomp"] is None and inp["language_feature"] is None
    cam_np = lambda t: t.detach().cpu().numpy()   # noqa: E731
    s = oracle.OracleSettings(c.image_height, c.image_width, c.tanfovx, c.tanfovy, np.ones(3, np.float32), 1.0,
                              cam_np(cam650.world_view_transform), cam_np(cam650.full_proj_transform), 3,
                              cam_np(cam650.camera_center), False)
    ref = oracle.forward(s, inp["means3D"].numpy(), inp["opacities"].numpy(), shs=inp["shs"].numpy(),
                         scales=inp["scales"].numpy(), rotations=inp["rotations"].numpy())
    rg = ref.backward(gcol.numpy())
    P = inp["means3D"].shape[0]
    errs = {k: grad_err(g[n].numpy().reshape(P, -1), rg[r].reshape(P, -1))
            for k, n, r in (("means3D", "means3D", "means3D"), ("means2D", "means2D", "means2D"),
                            ("sh", "sh", "sh"), ("opacity", "opacities", "opacity"), ("scales", "scales", "scales"),
                            ("rotations", "rotations", "rotations"))}
    assert max(errs.values()) <= 1e-4, errs


@pytest.mark.parametrize("V,ch", [(2, 3), (4, 4), (1, 3)])
def test_l1_loss_views_matches_torch(V, ch):
    """lsr_l1_loss_views (the base stages' loss over the views' renders, not stacked) against
    (stack(images) - gts[:, :3]).abs().mean(): the loss within float summation order, the images'
    gradients bit for bit (PyTorch's sign(x) * (g * (1 / N))); gts with a fourth channel read through its
    view stride; exact zeros (sign 0) included."""
    from train_step import l1_loss_views
    g = torch.Generator(device="cpu").manual_seed(V)
    H, W = 97, 131
    imgs = [torch.rand(3, H, W, generator=g).cuda().requires_grad_(True) for _ in range(V)]
    gts = torch.rand(V, ch, H, W, generator=g).cuda()
    gts[0, :3, :5] = imgs[0].detach()[:, :5]   # exact zeros
    ref_imgs = [x.detach().clone().requires_grad_(True) for x in imgs]
    got = l1_loss_views(imgs, gts)
    ref = (torch.stack(ref_imgs) - gts[:, :3]).abs().mean()
    torch.testing.assert_close(got, ref, rtol=2e-6, atol=0.0)
    (got * 3.0).backward()
    (ref * 3.0).backward()
    for a, b in zip(imgs, ref_imgs):
        assert torch.equal(a.grad, b.grad)
