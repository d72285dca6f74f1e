#!/usr/bin/env python3
"""BASELINE configs[4] stand-in (the Neu3D flame_steak frames and its COLMAP
point cloud are unavailable offline): train.py's fine-base stage loop for 1000 iterations on the MI355X
pieces, densification on the reference schedule.

  scene        a synthetic teacher (100k Gaussians, S2M-style generator) deformed by a Neu3D field
               (arguments/neu3d/default.py: 16-channel planes 64/64/64/150 x multires [1, 2],
               defor_depth 0, every head) whose time planes vary; ground truth = the teacher's renders
               of a pool of cameras x times at 1352 x 1014 (the dataloader's frames)
  student      create_from_pcd (scene/gaussian_model.py:192-219) on a noisy copy of the teacher's
               points and colours: RGB2SH colour, zero higher SH, log sqrt(distCUDA2) scales (our
               simple_knn), identity rotations, opacity inverse_sigmoid(0.1); a fresh Neu3D field
  iteration    train.py:224-421 via train_step.TrainStep: `views` random cameras of the pool, render,
               L1 (the base-stage loss: train.py:287, 331-337), backward, densification statistics,
               ReferenceSchedule (train.py:388-414 with the Neu3D overrides), Adam on the Gaussians and
               the field, the reference's learning-rate schedules (gaussian_model.py:302-330)

Prints one JSON line: iterations/s over the whole loop (densify / prune included), the mean loss per
window of `window` iterations (the loss must fall window over window), the densify / prune events,
and the deformation's share of an iteration at the final size (the field's forward + backward for
every view and its Adam + repack, event-timed alone, over the iteration time of the last window)."""
import argparse
import dataclasses
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import torch  # noqa: E402

import synthetic  # noqa: E402
from deformation import DeformationField  # noqa: E402
from gaussian_scene import render  # noqa: E402
from gaussian_train import GaussianTrainer  # noqa: E402
from train_step import ReferenceSchedule, TrainStep  # noqa: E402

NEU3D_RES, NEU3D_MULTIRES = [64, 64, 64, 150], [1, 2]
C0 = 0.28209479177387814


def feature_lrs(feature_lr=2.5e-3, opacity_lr=0.05, scaling_lr=5e-3, rotation_lr=1e-3):
    """OptimizationParams (arguments/__init__.py:137-141); xyz is set by the schedule."""
    return {"xyz": 0.0, "f_dc": feature_lr, "f_rest": feature_lr / 20.0, "opacity": opacity_lr,
            "scaling": scaling_lr, "rotation": rotation_lr}


def cameras_extent(cams):
    """scene/dataset_readers.py getNerfppNorm: 1.1 x the largest camera-centre distance from their mean."""
    c = torch.stack([cam.camera_center.double() for cam in cams])
    return float((c - c.mean(0)).norm(dim=1).max()) * 1.1


def teacher(P, W, H, dev, seed=0):
    sc = synthetic.make_scene(P, C=3, tanfovx=0.6, tanfovy=0.6 * H / W, seed=seed, logscale_mean=-4.0).to(dev)
    raw = {"xyz": sc.means3D.contiguous(), "f_dc": sc.shs[:, :1].contiguous(), "f_rest": sc.shs[:, 1:].contiguous(),
           "opacity": torch.logit(sc.opacities.reshape(P, 1)).contiguous(), "scaling": torch.log(sc.scales).contiguous(),
           "rotation": sc.rotations.contiguous()}
    lo, hi = sc.means3D.min(0).values.cpu(), sc.means3D.max(0).values.cpu()
    fp = DeformationField.init_params(NEU3D_RES, NEU3D_MULTIRES, torch.stack([hi, lo]), seed=seed)
    g = torch.Generator().manual_seed(seed)
    for k, v in fp.items():   # time planes off 1 (motion), small head outputs
        if k.startswith("grid.grids") and k[-1] in "245":
            fp[k] = 1.0 + 0.1 * (torch.rand(v.shape, generator=g) - 0.5)
        if k.endswith(".3.weight"):
            fp[k] = v * 0.01
    return raw, fp


def create_from_pcd(points, colors, dev):
    """scene/gaussian_model.py:192-219 on a point cloud (points [N,3], colours [N,3] in [0, 1])."""
    from simple_knn._C import distCUDA2
    N = points.shape[0]
    f_dc = ((colors - 0.5) / C0).reshape(N, 1, 3)                                  # RGB2SH
    dist2 = torch.clamp_min(distCUDA2(points.contiguous()), 1e-7)
    return {"xyz": points.contiguous(), "f_dc": f_dc.contiguous(), "f_rest": torch.zeros(N, 15, 3, device=dev),
            "opacity": torch.full((N, 1), math.log(0.1 / 0.9), device=dev),
            "scaling": torch.log(torch.sqrt(dist2))[:, None].repeat(1, 3).contiguous(),
            "rotation": torch.tensor([1.0, 0, 0, 0], device=dev).repeat(N, 1).contiguous()}


def build(args, dev):
    P, W, H = args.gaussians, args.width, args.height
    t_raw, t_fp = teacher(P, W, H, dev)
    # the dataloader's frames: `cameras` viewpoints x `frames` times
    rig = synthetic.camera_batch(args.cameras, W, H, tanfovx=0.6, seed=1, max_yaw=15.0, sigma_t=0.3)
    # the reference's Camera keeps its matrices on the GPU (scene/cameras.py:56-67, .cuda()): no
    # host-to-device copy (a stream synchronisation) per render
    rig = [dataclasses.replace(c, world_view_transform=c.world_view_transform.to(dev),
                               projection_matrix=c.projection_matrix.to(dev),
                               full_proj_transform=c.full_proj_transform.to(dev),
                               camera_center=c.camera_center.to(dev)) for c in rig]
    pool = [dataclasses.replace(c, time=f / max(1, args.frames - 1)) for f in range(args.frames) for c in rig]
    tfield = DeformationField({k: v.to(dev) for k, v in t_fp.items()}, NEU3D_RES, NEU3D_MULTIRES)
    tstep = TrainStep(GaussianTrainer(t_raw, feature_lrs()), tfield)
    bg = torch.ones(3, device=dev)
    gts = []
    with torch.no_grad():
        tsc = tstep.scene()
        for cam in pool:
            gts.append(render(cam, tsc, bg, stage="fine-base")["render"].clone())
    gts = torch.stack(gts)
    # the student's point cloud: the teacher's points and colours, noisy
    g = torch.Generator(device="cpu").manual_seed(7)
    pts = t_raw["xyz"] + (torch.randn(P, 3, generator=g) * args.point_noise).to(dev)
    rgb = (t_raw["f_dc"].reshape(P, 3) * C0 + 0.5).clamp(0, 1)
    rgb = (rgb + (torch.randn(P, 3, generator=g) * 0.1).to(dev)).clamp(0, 1)
    s_raw = create_from_pcd(pts, rgb, dev)
    lo, hi = pts.min(0).values.cpu(), pts.max(0).values.cpu()
    sfp = DeformationField.init_params(NEU3D_RES, NEU3D_MULTIRES, torch.stack([hi, lo]), seed=11)
    field = DeformationField({k: v.to(dev) for k, v in sfp.items()}, NEU3D_RES, NEU3D_MULTIRES)
    extent = cameras_extent(rig)
    tr = GaussianTrainer(s_raw, feature_lrs())
    sched = ReferenceSchedule(extent, stage="fine-base", densify_until_iter=args.densify_until_iter)
    step = TrainStep(tr, field, densify=sched, stage="fine-base")
    step.set_reference_lr(extent)
    return step, sched, pool, gts, extent


def deformation_ms(step, views, reps=10):
    """The field's share of one iteration at the current size: forward + backward for the views
    (one call over views * P rows as render_views makes it, or one per view as render() does
    when step.batch_views is off) and its Adam + repack, event-timed on the current stream."""
    tr, field = step.trainer, step.field
    sc = step.scene()
    P = tr.P
    args = (sc.xyz.detach(), sc.scaling.detach(), sc.rotation.detach(), sc.opacity.detach(),
            sc.get_features.detach(), None)
    if step.batch_views and views > 1:
        args = tuple(a.repeat(views, *([1] * (a.dim() - 1))) for a in args[:5]) + (None,)
        P, views = P * views, 1
    ups = [torch.randn(P, 3, device=tr.device) * 1e-3, torch.randn(P, 3, device=tr.device) * 1e-3,
           torch.randn(P, 4, device=tr.device) * 1e-3, torch.randn(P, 1, device=tr.device) * 1e-3,
           torch.randn(P, 16, 3, device=tr.device) * 1e-3]
    saved = {k: v.clone() for k, v in field.p.items()}
    opt_state = ({k: v.clone() for k, v in step.field_opt.exp_avg.items()},
                 {k: v.clone() for k, v in step.field_opt.exp_avg_sq.items()}, dict(step.field_opt.steps))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        for v in range(views):
            field.forward(*args, 0.5, no_dlang=True)
    ev[1].record()
    field.zero_grad()
    for _ in range(reps):
        for v in range(views):
            field.backward(args[0], 0.5, *ups, rotations=args[2], no_dlang=True)
    ev[2].record()
    for _ in range(reps):
        step.field_opt.step(field.grads)
        field.prepare()
    ev[3].record()
    torch.cuda.synchronize()
    for k, v in saved.items():   # leave the field as it was
        field.p[k].copy_(v)
    step.field_opt.exp_avg, step.field_opt.exp_avg_sq, step.field_opt.steps = opt_state
    field.prepare()
    return (ev[0].elapsed_time(ev[1]) / reps, ev[1].elapsed_time(ev[2]) / reps, ev[2].elapsed_time(ev[3]) / reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=100_000)
    ap.add_argument("--width", type=int, default=1352)
    ap.add_argument("--height", type=int, default=1014)
    ap.add_argument("--views", type=int, default=2, help="cameras per iteration (Neu3D batch_size is 4)")
    ap.add_argument("--cameras", type=int, default=8)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--window", type=int, default=100)
    ap.add_argument("--point-noise", type=float, default=0.02)
    ap.add_argument("--densify-until-iter", type=int, default=10_000)
    ap.add_argument("--per-view-deform", action="store_true",
                    help="one deformation launch per view (render) instead of one per iteration over all views "
                         "(render_views, TrainStep's default)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    t_setup = time.perf_counter()
    step, sched, pool, gts, extent = build(args, dev)
    step.batch_views = not args.per_view_deform
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    P0 = step.trainer.P
    order = torch.Generator().manual_seed(5)
    windows, window_ms, window_P = [], [], []
    acc = torch.zeros((), device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tw = t0
    for it in range(1, args.iters + 1):
        idx = torch.randperm(len(pool), generator=order)[: args.views].tolist()
        loss = step([pool[i] for i in idx], gts[idx], iteration=it)
        acc += loss
        if it % args.window == 0:
            windows.append(float(acc) / args.window)      # host sync once per window
            now = time.perf_counter()
            window_ms.append((now - tw) * 1e3 / args.window)
            window_P.append(step.trainer.P)
            tw = now
            acc.zero_()
            print(f"iter {it}: window loss {windows[-1]:.5f}  P {step.trainer.P}  {window_ms[-1]:.2f} ms/it",
                  file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    total_s = time.perf_counter() - t0
    f_ms, b_ms, o_ms = deformation_ms(step, args.views)
    deform = f_ms + b_ms + o_ms
    last = window_ms[-1] if window_ms else total_s * 1e3 / args.iters
    monotone = all(b < a for a, b in zip(windows, windows[1:]))
    line = dict(metric="train.py fine-base iterations/s (configs[4] stand-in)", value=round(args.iters / total_s, 2),
                unit="iterations/s", ms_per_iteration=round(total_s * 1e3 / args.iters, 3), iterations=args.iters,
                window=args.window, window_loss=[round(x, 5) for x in windows], loss_falls_every_window=monotone,
                window_ms_per_iteration=[round(x, 3) for x in window_ms], window_gaussians=window_P,
                gaussians_initial=P0, gaussians_final=step.trainer.P,
                schedule_events=[list(e) for e in sched.events],
                deformation=dict(forward_ms=round(f_ms, 3), backward_ms=round(b_ms, 3), adam_repack_ms=round(o_ms, 3),
                                 batched_views=step.batch_views,
                                 ms_per_iteration=round(deform, 3),
                                 share_of_last_window=round(deform / last, 3) if last > 0 else None,
                                 note="forward/backward are per iteration (all views), at the final size"),
                setup_s=round(setup_s, 1), cameras_extent=round(extent, 4),
                config=dict(workload="configs[4] stand-in: synthetic teacher, Neu3D field, fine-base",
                            gaussians=args.gaussians, views_per_iteration=args.views, width=args.width,
                            height=args.height, pool=len(pool), resolution=NEU3D_RES, multires=NEU3D_MULTIRES,
                            deformation_launches="per view" if args.per_view_deform else "one per iteration"),
                data="synthetic")
    print(json.dumps(line))


if __name__ == "__main__":
    main()
