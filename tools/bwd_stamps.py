"""Diagnostic: per-segment cycle shares of the compositor backward's group loop on the headline
scene, from the stamp build (tools/build_variants.sh stamps:render_bwd_wave.hip:-DLSR_BWD_STAMPS).
Run with LSR_LIBRARY pointing at that build.  Prints shares, not times (stamps cost cycles)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402


def raster_settings(cam):
    return dgr.GaussianRasterizationSettings(
        image_height=cam.image_height, image_width=cam.image_width, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.ones(3, device="cuda"), scale_modifier=1.0, viewmatrix=cam.world_view_transform.cuda(),
        projmatrix=cam.full_proj_transform.cuda(), sh_degree=3, campos=cam.camera_center.cuda(), prefiltered=False,
        debug=False, include_feature=True)

SEG = ["store_group", "scan_fill", "atomics", "load_group", "mfma1", "replay", "mfma_wt", "stage_moments"]


def main():
    L = dgr._lib.load()
    fn = L.lsr_debug_bwd_stamps
    fn.restype = ctypes.c_int
    sc = synthetic.make_scene(2_000_000, C=32).to("cuda")
    cams = synthetic.camera_batch(4, seed=1)
    buf = (ctypes.c_ulonglong * 14)()
    tot = [0] * 14
    for cam in cams:
        rs = raster_settings(cam)
        color, lang, radii, depth, st = dgr.forward_native(rs, sc.means3D, sc.opacities, shs=sc.shs,
                                                           language_feature=sc.lang, scales=sc.scales,
                                                           rotations=sc.rotations)
        g = torch.Generator(device="cpu").manual_seed(0)
        gc = (torch.randn(color.shape, generator=g) * 1e-3).cuda()
        gl = (torch.randn(lang.shape, generator=g) * 1e-3).cuda()
        torch.cuda.synchronize()
        fn(buf)   # reset
        dl = torch.zeros(sc.means3D.shape[0], 32, device="cuda")
        dgr.backward_composite_native(st, gc, gl, None, dL_dlanguage=dl)
        torch.cuda.synchronize()
        fn(buf)
        for i in range(14):
            tot[i] += buf[i]
    s = sum(tot[:8])
    print("waves", tot[8], "cycles/wave", s / max(tot[8], 1))
    for i, n in enumerate(SEG):
        print(f"{n:14s} {100.0 * tot[i] / s:6.2f} %")
    w = max(tot[8], 1)
    print(f"per wave: life {tot[10] / w:.0f} cycles, setup (entry -> first group) {tot[9] / w:.0f} "
          f"({100.0 * tot[9] / max(tot[10], 1):.1f} % of the lives), group loop {s / w:.0f}")
    print(f"setup parts per wave: pixel loads + replay bound {tot[11] / w:.0f}, G rows {tot[12] / w:.0f}, "
          f"first scan + prefetch {tot[13] / w:.0f}")


if __name__ == "__main__":
    main()
