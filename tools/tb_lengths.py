"""Tile list lengths of the bench workload (2M Gaussians, 1352x1014, 8 views of camera_batch seed 1):
the tile-bucket sort's bucket sizes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "4dlangsplat_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
import diff_gaussian_rasterization as dgr
import synthetic
from lsr_testutil import decode_img, raster_settings

W, H, P = 1352, 1014, 2_000_000
sc = synthetic.make_scene(P, C=32, tanfovx=0.6, tanfovy=0.6 * H / W).to("cuda")
cams = synthetic.camera_batch(8, W, H, tanfovx=0.6, seed=1)
rss = [raster_settings(c) for c in cams]
pfs = dgr.preprocess_views_native(rss, sc.means3D, sc.opacities, language_feature=sc.lang, scales=sc.scales,
                                  rotations=sc.rotations, shs=sc.shs, tile_bucket=True)
dgr.binning_views_native(pfs)
outs = dgr.render_views_native(pfs)
torch.cuda.synchronize()
allL = []
for o in outs:
    r = decode_img(o[4])[0].astype(np.int64)
    L = r[:, 1] - r[:, 0]
    allL.append(L)
    print("K", o[4].num_rendered, "listed", int(L.sum()), "max", int(L.max()), "mean", round(float(L.mean()), 1),
          ">2048", int((L > 2048).sum()), ">4096", int((L > 4096).sum()), "sum>2048", int(L[L > 2048].sum()))
L = np.concatenate(allL)
print("pct", {q: int(np.percentile(L, q)) for q in (10, 50, 90, 99, 99.9)})
print("pow2 padded total", int(sum(max(8, 1 << int(np.ceil(np.log2(max(x, 1))))) for x in L if 0 < x <= 2048)),
      "vs", int(L[(L > 0) & (L <= 2048)].sum()))
