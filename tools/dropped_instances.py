"""Share of emitted (Gaussian, tile) instances that reach no quadrant of their tile (the emission
gives them the past-the-end tile key; they are sorted but never listed) on the headline scene:
K (num_rendered) against the listed entries (the tile ranges' total)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "4dlangsplat_amd"), os.path.join(ROOT, "tools")]
import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402
from bwd_stamps import raster_settings  # noqa: E402


def tile_ranges(st):   # the img workspace starts with the [tiles][2] ranges
    W, H = st.settings.c.image_width, st.settings.c.image_height
    nt = ((W + 15) // 16) * ((H + 15) // 16)
    return st.img[:nt * 8].cpu().numpy().view("uint32").reshape(nt, 2)


def main():
    sc = synthetic.make_scene(2_000_000, C=32).to("cuda")
    for cam in synthetic.camera_batch(3, seed=1):
        rs = raster_settings(cam)
        *_, st = dgr.forward_native(rs, sc.means3D, sc.opacities, shs=sc.shs, language_feature=sc.lang,
                                    scales=sc.scales, rotations=sc.rotations)
        ranges = tile_ranges(st)
        listed = int((ranges[:, 1].astype("int64") - ranges[:, 0]).clip(min=0).sum())
        K = int(st.num_rendered)
        print(f"K {K}  listed {listed}  unlisted {K - listed} ({100.0 * (K - listed) / max(K, 1):.1f} %)")


if __name__ == "__main__":
    main()
