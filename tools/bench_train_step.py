"""Config-5 stand-in: one training iteration of the fine stage on the MI355X pieces
(train_step.TrainStep): 100k Gaussians (random init), Neu3D deformation field (64^3 x 150,
multires [1, 2]), a batch of 2 views at 1352 x 1014, L1 to synthetic ground truth, backward
through rasterizer and field, densification statistics, Adam on the Gaussians and the field.
Prints one JSON line: iterations/s and ms per iteration (HIP events around the timed loop)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import torch  # noqa: E402

import synthetic  # noqa: E402
from deformation import DeformationField  # noqa: E402
from gaussian_train import GaussianTrainer  # noqa: E402
from train_step import TrainStep  # noqa: E402

LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=100_000)
    ap.add_argument("--width", type=int, default=1352)
    ap.add_argument("--height", type=int, default=1014)
    ap.add_argument("--views", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda")
    P, W, H = args.gaussians, args.width, args.height
    sc = synthetic.make_scene(P, C=3, tanfovx=0.6, tanfovy=0.6 * H / W, seed=0, logscale_mean=-4.0).to(dev)
    raw = {"xyz": sc.means3D.contiguous(), "f_dc": sc.shs[:, :1].contiguous(), "f_rest": sc.shs[:, 1:].contiguous(),
           "opacity": torch.logit(sc.opacities.reshape(P, 1)).contiguous(), "scaling": torch.log(sc.scales).contiguous(),
           "rotation": sc.rotations.contiguous()}
    res, multires = [64, 64, 64, 150], [1, 2]
    fp = DeformationField.init_params(res, multires, [[7.0, 5.5, 10.5], [-7.0, -5.5, 1.5]], seed=0)
    field = DeformationField({k: v.to(dev) for k, v in fp.items()}, res, multires)
    tr = GaussianTrainer(raw, LRS)
    step = TrainStep(tr, field)
    cams = synthetic.camera_batch(args.views, W, H, tanfovx=0.6, seed=1)
    gts = torch.rand(args.views, 3, H, W, device=dev)
    for _ in range(3):
        step(cams, gts)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        loss = step(cams, gts)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps(dict(metric="fine-stage training iterations/s (config-5 stand-in)", value=round(1e3 / ms, 2),
                          unit="iterations/s", ms_per_iteration=round(ms, 3), gaussians=P, views_per_iteration=args.views,
                          width=W, height=H, deformation="Neu3D 64^3x150, multires [1,2]", loss=round(float(loss), 5),
                          data="synthetic")))


if __name__ == "__main__":
    main()
