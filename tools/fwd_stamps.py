"""Diagnostic: per-segment cycle shares of the forward MFMA compositor's group loop on the headline
scene, from the stamp build (tools/build_variants.sh fstamps:render_fwd_mfma_wave.hip:-DLSR_FWD_STAMPS).
Run with LSR_LIBRARY pointing at that build.  Prints shares, not times (stamps cost cycles)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402
from bwd_stamps import raster_settings  # noqa: E402

SEG = ["scan", "stage", "composite", "mfma"]


def main():
    fn = dgr._lib.load().lsr_debug_fwd_stamps
    fn.restype = ctypes.c_int
    sc = synthetic.make_scene(2_000_000, C=32).to("cuda")
    buf = (ctypes.c_ulonglong * 5)()
    tot = [0] * 5
    for cam in synthetic.camera_batch(4, seed=1):
        pf = dgr.preprocess_native(raster_settings(cam), sc.means3D, sc.opacities, shs=sc.shs, language_feature=sc.lang,
                                   scales=sc.scales, rotations=sc.rotations, stream=torch.cuda.current_stream(),
                                   binning=True)
        torch.cuda.synchronize()
        fn(buf)   # reset
        dgr.render_native(pf)
        torch.cuda.synchronize()
        fn(buf)
        for i in range(5):
            tot[i] += buf[i]
    s = sum(tot[:4])
    print("waves", tot[4], "cycles/wave", s / max(tot[4], 1))
    for i, n in enumerate(SEG):
        print(f"{n:10s} {100.0 * tot[i] / s:6.2f} %")


if __name__ == "__main__":
    main()
