"""Diagnostic: how the compositor backward's work and atomics would change if quadrant waves were
merged, on the headline scene (2M, 1352x1014, C = 32, the bench's first cameras).

Per tile and 8x8 quadrant q the backward replays list positions [0, R_q), R_q = the largest
n_contrib of the quadrant's pixels, and keeps the entries whose quadrant bit q is set (one
quadrant-entry each: 64 pixel evaluations and one set of gradient atomics).  For a unit of several
quadrants processed by one wave (or one lock-step block) the kept entries are the union over its
quadrants within the largest R, each evaluated at every pixel of the unit and issuing ONE set of
atomics.  Prints, per grouping, the entries that issue atomics and the pixel evaluations, relative
to today's per-quadrant waves."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402
from bwd_stamps import raster_settings  # noqa: E402
from lsr_testutil import decode_img, decode_point_words  # noqa: E402

GROUPS = {
    "quadrant (today)": [[0], [1], [2], [3]],
    "vertical pair (8x16)": [[0, 2], [1, 3]],
    "horizontal pair (16x8)": [[0, 1], [2, 3]],
    "tile (16x16)": [[0, 1, 2, 3]],
}


def main():
    sc = synthetic.make_scene(2_000_000, C=32).to("cuda")
    W, H = 1352, 1014
    gx, gy = (W + 15) // 16, (H + 15) // 16
    out = {}
    for vi, cam in enumerate(synthetic.camera_batch(int(os.environ.get("VIEWS", "2")), seed=1)):
        *_, st = dgr.forward_native(raster_settings(cam), sc.means3D, sc.opacities, shs=sc.shs,
                                    language_feature=sc.lang, scales=sc.scales, rotations=sc.rotations)
        torch.cuda.synchronize()
        ranges, _, _, nc = decode_img(st)
        words = decode_point_words(st)
        # R[t, q]: replay bound of quadrant q of tile t (pixels outside the image have none)
        ncp = np.zeros((gy * 16, gx * 16), np.int64)
        ncp[:H, :W] = nc
        R = ncp.reshape(gy, 2, 8, gx, 2, 8).max(axis=(2, 5))          # [gy, qy, gx, qx]
        R = R.transpose(0, 2, 1, 3).reshape(gy * gx, 4)               # q = 2 qy + qx
        bits = ((words[:, None] >> (28 + np.arange(4))[None, :]) & 1).astype(bool)   # [K, 4]
        tile_of = np.repeat(np.arange(len(ranges)), (ranges[:, 1] - ranges[:, 0]).astype(np.int64))
        starts = ranges[:, 0].astype(np.int64)
        idx = np.concatenate([np.arange(ranges[t, 0], ranges[t, 1]) for t in range(len(ranges)) if ranges[t, 1] > ranges[t, 0]])
        pos = idx - starts[tile_of]                                    # list position in its tile
        res = {}
        for name, groups in GROUPS.items():
            ent = evals = 0
            for g in groups:
                Rg = R[:, g].max(axis=1)[tile_of]
                keep = (pos < Rg) & bits[idx][:, g].any(axis=1)
                n = int(keep.sum())
                ent += n
                evals += n * 64 * len(g)
            res[name] = dict(atomic_entries=ent, pixel_evals=evals)
        base = res["quadrant (today)"]
        for r in res.values():
            r["atomics_rel"] = round(r["atomic_entries"] / base["atomic_entries"], 3)
            r["evals_rel"] = round(r["pixel_evals"] / base["pixel_evals"], 3)
        res["K"] = int(st.num_rendered)
        out[f"view{vi}"] = res
        print(json.dumps({f"view{vi}": res}), flush=True)


if __name__ == "__main__":
    main()
