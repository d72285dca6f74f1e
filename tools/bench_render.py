#!/usr/bin/env python3
"""render.py throughput on the BASELINE configs[1] stand-in (the pretrained HyperNeRF
americano scene is unavailable offline): a synthetic 300k-Gaussian model with the HyperNeRF
deformation field (arguments/hypernerf/default.py: 16-channel planes 64/64/64/150 x multires
[1, 2, 4], defor_depth 1, the position / scale / rotation heads), 3 language channels
(language_feature_hiddendim 3, no_dlang 1), written to a model directory in the reference's layout
(point_cloud/fine-lang_iteration_N/{point_cloud.ply, deformation.pth, ...}), loaded back the way
render.py's Scene(load_iteration=-1) does (gaussian_scene.load_model_dir), and rendered frame by
frame at 960 x 540 through render() under no_grad (render.py:67-161, --mode lang and rgb).

Prints one JSON line: frames/s as render.py counts them (frames after the first / elapsed), the
per-frame deformation and rasterizer times (events), and the configuration."""
import argparse
import json
import math
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import numpy as np
import torch  # noqa: E402

import gaussian_scene as gs  # noqa: E402
import synthetic  # noqa: E402
from deformation import DeformationField  # noqa: E402

HYPERNERF = dict(kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                                 "resolution": [64, 64, 64, 150]},
                 multires=[1, 2, 4], defor_depth=1, net_width=128, no_dlang=1, timebase_pe=4)


def synthetic_model(P, C, W, H, seed=2):
    """A GaussianScene (raw parameters) from the S2M-style generator plus a HyperNeRF field."""
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W, seed=seed)
    scene = gs.GaussianScene(xyz=sc.means3D, features_dc=sc.shs[:, :1].contiguous(),
                             features_rest=sc.shs[:, 1:].contiguous(), language_feature=sc.lang,
                             opacity=torch.logit(sc.opacities.clamp(1e-6, 1 - 1e-6)), scaling=torch.log(sc.scales),
                             rotation=sc.rotations)
    lo, hi = sc.means3D.min(0).values, sc.means3D.max(0).values
    params = DeformationField.init_params(HYPERNERF["kplanes_config"]["resolution"], HYPERNERF["multires"],
                                          torch.stack([hi, lo]), depth=1,
                                          heads=("pos_deform", "scales_deform", "rotations_deform"), seed=seed)
    g = torch.Generator().manual_seed(seed)
    for k, v in params.items():   # time planes off 1 (a trained field varies in time), small MLP outputs
        if k.startswith("grid.grids") and k[-1] in "245":
            params[k] = 1.0 + 0.1 * (torch.rand(v.shape, generator=g) - 0.5)
        if k.endswith(".3.weight"):
            params[k] = v * 0.01
    state = {"deformation_net." + k: v for k, v in params.items()}
    return scene, state


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=300_000)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--width", type=int, default=960)
    ap.add_argument("--height", type=int, default=540)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--mode", choices=("lang", "rgb"), default="lang")
    args = ap.parse_args()
    P, C, W, H = args.gaussians, args.channels, args.width, args.height
    scene, state = synthetic_model(P, C, W, H)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "point_cloud", "fine-lang_iteration_10000")
        os.makedirs(path)
        scene.save_ply(os.path.join(path, "point_cloud.ply"))
        torch.save(state, os.path.join(path, "deformation.pth"))
        t0 = time.perf_counter()
        model, it = gs.load_model_dir(d, HYPERNERF, env={"language_feature_hiddendim": str(C)})
        load_s = time.perf_counter() - t0
    cams = synthetic.camera_batch(args.frames, W, H, tanfovx=0.6, seed=3)
    for i, c in enumerate(cams):   # a video path: time sweeps [0, 1]
        c.time = i / max(1, args.frames - 1)
    bg = torch.ones(3, device="cuda")
    key = "render" if args.mode == "rgb" else "language_feature_image"
    kw = dict(stage="fine-lang", language_feature_hiddendim=C)
    with torch.no_grad():
        for c in cams[:3]:
            gs.render(c, model, bg, **kw)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for c in cams:
            out = gs.render(c, model, bg, **kw)[key]
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        # render.py's own loop (render.py:94-134): per frame the render, (x + 1) / 2 for the language
        # output, and to8b -- a device-to-host copy of the frame, which synchronises every frame;
        # its printed FPS is (frames - 1) / the loop's time
        to8b = lambda x: (255 * np.clip(x.cpu().numpy(), 0, 1)).astype(np.uint8)   # noqa: E731 (render.py:48)
        frames8 = []
        h1 = time.perf_counter()
        for c in cams:
            r = gs.render(c, model, bg, **kw)[key]
            if args.mode == "lang":
                r = (r + 1.0) / 2
            frames8.append(to8b(r).transpose(1, 2, 0))
        h2 = time.perf_counter()
        # the deformation alone (the same call render() makes), event-timed
        m, s_, r, o = model.xyz, model.scaling, model.rotation, model.opacity
        sh, lang = model.get_features, model.language_feature
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for c in cams:
            model.deformation(m, s_, r, o, sh, lang, c.time)
        e1.record()
        torch.cuda.synchronize()
        deform_ms = e0.elapsed_time(e1) / len(cams)
    frame_ms = (t2 - t1) / len(cams) * 1e3
    line = dict(metric="render.py frames/s (configs[1] stand-in)", value=round((len(cams) - 1) / (h2 - h1), 2),
                unit="frames/s", measure="render.py's: render + (x+1)/2 + to8b host copy per frame, (frames-1)/time",
                ms_per_frame_with_host_copy=round((h2 - h1) / len(cams) * 1e3, 3),
                device_only=dict(value=round(len(cams) / (t2 - t1), 2), unit="frames/s",
                                 note="render() calls only, one synchronisation at the end"),
                ms_per_frame=round(frame_ms, 3), deformation_ms=round(deform_ms, 3),
                rasterizer_and_host_ms=round(frame_ms - deform_ms, 3), frames=len(cams), mode=args.mode,
                output_shape=list(out.shape), load_model_dir_s=round(load_s, 2), iteration=it,
                config=dict(workload="configs[1] stand-in: synthetic model dir, HyperNeRF field", gaussians=P,
                            width=W, height=H, channels=C, multires=HYPERNERF["multires"],
                            defor_depth=HYPERNERF["defor_depth"], heads=model.deformation.heads_computed()),
                data="synthetic")
    print(json.dumps(line))


if __name__ == "__main__":
    main()
