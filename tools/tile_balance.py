"""Diagnostic: per-tile work of the headline frame and the tail a launch-order list schedule leaves.

Renders the S2M origin view, decodes ranges / n_contrib, and simulates the hardware's in-order
dispatch of the compositor's blocks onto a fixed number of wave slots with cost = list length
(forward) or the quadrant's replay length (backward), in launch order and in
longest-first order.  Prints the makespan of each relative to a perfect balance.
"""
import heapq
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "4dlangsplat_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import synthetic  # noqa: E402
from lsr_testutil import decode_img, run_native  # noqa: E402


def makespan(costs, slots):
    h = [0.0] * slots
    for c in costs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return max(h)


def main():
    W, H, P, C = 1352, 1014, 2_000_000, 32
    scene = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W)
    cam = synthetic.origin_camera(W, H)
    color, lang, radii, depth, st = run_native(scene, cam)
    torch.cuda.synchronize()
    ranges, tmax, fT, nc = decode_img(st)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ntiles = gx * gy
    L = (ranges[:, 1].astype(np.int64) - ranges[:, 0].astype(np.int64))[:ntiles]
    print("K", st.num_rendered, "tiles", ntiles, "list len mean %.1f p50 %d p90 %d p99 %d max %d" % (
        L.mean(), np.percentile(L, 50), np.percentile(L, 90), np.percentile(L, 99), L.max()))
    ncp = np.zeros((gy * 16, gx * 16), np.int64)
    ncp[:H, :W] = nc.reshape(H, W)
    q = ncp.reshape(gy, 2, 8, gx, 2, 8).max(axis=(2, 5))           # [gy, qy, gx, qx]
    qrep = q.transpose(0, 2, 1, 3).reshape(ntiles, 4)              # tile-major, quad = qy*2+qx
    print("bwd replay len per quadrant mean %.1f p99 %d max %d" % (qrep.mean(), np.percentile(qrep, 99), qrep.max()))
    # launch order of the wave kernels: block b -> tile (b>>5)*8 + (b&7), quad (b>>3)&3
    nb = ((ntiles + 7) // 8) * 32
    b = np.arange(nb)
    tile = (b >> 5) * 8 + (b & 7)
    quad = (b >> 3) & 3
    ok = tile < ntiles
    cost_b = np.where(ok, qrep[np.minimum(tile, ntiles - 1), quad], 0).astype(np.float64) + 4.0
    cost_f = np.where(ok, L[np.minimum(tile, ntiles - 1)], 0).astype(np.float64) + 4.0
    for slots in (2048, 4096):
        for name, cost in (("fwd(list len)", cost_f), ("bwd(replay)", cost_b)):
            ideal = cost.sum() / slots
            m_launch = makespan(cost, slots)
            m_lpt = makespan(np.sort(cost)[::-1], slots)
            print(f"slots {slots} {name}: launch-order makespan/ideal {m_launch / ideal:.3f}, "
                  f"longest-first {m_lpt / ideal:.3f}")


if __name__ == "__main__":
    main()
