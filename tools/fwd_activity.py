"""Diagnostic: the share of the forward compositor's (entry, pixel) evaluations that blend, on the
headline scene, from the counting build (tools/build_variants.sh fcount:render_fwd_mfma_wave.hip:
-DLSR_FWD_COUNT).  Run with LSR_LIBRARY pointing at that build.  A pair is evaluated when a
quadrant wave processes a compacted entry for a pixel inside the image (all 64 lanes compute it);
it blends when it passes the alpha prefilter before the pixel's termination.  Also counts the
compacted (entry, quadrant) pairs with no blending pixel that lie before the quadrant's last blending
entry: the backward replays them (its range ends at the largest n_contrib) and an exact activity bit
written by the forward would let it skip them (VERDICT r4 item 2's measure-first)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402
from bwd_stamps import raster_settings  # noqa: E402


def main():
    fn = dgr._lib.load().lsr_debug_fwd_count
    fn.restype = ctypes.c_int
    sc = synthetic.make_scene(2_000_000, C=32).to("cuda")
    buf = (ctypes.c_ulonglong * 5)()
    tot = [0, 0, 0, 0, 0]
    Ks = []
    for cam in synthetic.camera_batch(4, seed=1):
        pf = dgr.preprocess_native(raster_settings(cam), sc.means3D, sc.opacities, shs=sc.shs, language_feature=sc.lang,
                                   scales=sc.scales, rotations=sc.rotations, stream=torch.cuda.current_stream(),
                                   binning=True)
        torch.cuda.synchronize()
        fn(buf)   # reset
        *_, st = dgr.render_native(pf)
        torch.cuda.synchronize()
        fn(buf)
        Ks.append(st.num_rendered)
        for i in range(5):
            tot[i] += buf[i]
    print(json.dumps(dict(views=len(Ks), K_mean=sum(Ks) / len(Ks), pairs_evaluated=tot[0], pairs_blended=tot[1],
                          blend_share=round(tot[1] / max(tot[0], 1), 4), waves=tot[2],
                          evaluated_per_frame=tot[0] // len(Ks), blended_per_frame=tot[1] // len(Ks),
                          quadrant_entries=tot[3], inactive_before_last_blend=tot[4],
                          inactive_share=round(tot[4] / max(tot[3], 1), 4),
                          note="inactive_before_last_blend: (entry, quadrant) pairs that pass the conservative "
                               "quadrant bits and are replayed by the backward (before the quadrant's last "
                               "blending entry) but blend no pixel: what exact activity bits would skip")))


if __name__ == "__main__":
    main()
