#!/usr/bin/env python3
"""Diagnostic: does the forward compositor of one group of views, run concurrently with the backward
compositor of another (a second stream), finish the pair sooner than one after the other?  The
backward is latency-bound at 2 waves/SIMD, the forward issue-bound at 4, so a
mix on the CUs could fill the backward's stalls.  Headline scene (2M, 1352x1014, C = 32), 8 views
binned up front; only the compositing is timed (events), alternating the modes:
  one8 : fwd(8 views) ; bwd(8)                       (the bench's early-views-8 shape)
  seq44: fwd(A) ; bwd(A) ; fwd(B) ; bwd(B)           (two groups of 4, one stream)
  conc : fwd(A) ; [bwd(A) || fwd(B) on a side stream] ; bwd(B)
Prints one JSON line with the mean ms per mode."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402


def main():
    P, W, H, C, V = 2_000_000, 1352, 1014, 32, 8
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    split = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda")
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W).to(dev)
    cams = synthetic.camera_batch(V, W, H, tanfovx=0.6, seed=1)
    bg = torch.ones(3, device=dev)
    rss = [dgr.GaussianRasterizationSettings(H, W, c.tanfovx, c.tanfovy, bg, 1.0, c.world_view_transform.to(dev),
                                             c.full_proj_transform.to(dev), 3, c.camera_center.to(dev), False, False,
                                             True) for c in cams]
    g = torch.Generator(device="cpu").manual_seed(123)
    gcol = (torch.randn(3, H, W, generator=g) * 1e-3).to(dev)
    glang = (torch.randn(C, H, W, generator=g) * 1e-3).to(dev)
    dlang = torch.zeros(P, C, device=dev)
    side = torch.cuda.Stream(device=dev)

    def prep():
        pfs = dgr.preprocess_views_native(rss, sc.means3D, sc.opacities, shs=sc.shs, language_feature=sc.lang,
                                          scales=sc.scales, rotations=sc.rotations)
        dgr.binning_views_native(pfs)
        torch.cuda.synchronize()
        return pfs

    def bwd(res):
        n = len(res)
        return dgr.backward_composite_views_native([r[4] for r in res], [gcol] * n, [glang] * n, [None] * n,
                                                   dL_dlanguage=dlang)

    def run(mode, pfs):
        main = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        if mode == "one8":
            bwd(dgr.render_views_native(pfs))
        elif mode == "seq44":
            bwd(dgr.render_views_native(pfs[:split]))
            bwd(dgr.render_views_native(pfs[split:]))
        else:
            ra = dgr.render_views_native(pfs[:split])
            side.wait_stream(main)
            with torch.cuda.stream(side):
                rb = dgr.render_views_native(pfs[split:])
            bwd(ra)
            main.wait_stream(side)
            bwd(rb)
        e1.record(main)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    modes = ("one8", "seq44", "conc")
    for m in modes:   # warm-up
        run(m, prep())
    times = {m: [] for m in modes}
    for _ in range(reps):
        for m in modes:
            times[m].append(run(m, prep()))
    print(json.dumps({"split": split, **{m: round(sum(t) / len(t), 4) for m, t in times.items()},
                      "all": {m: [round(x, 3) for x in t] for m, t in times.items()}}))


if __name__ == "__main__":
    main()
