#!/usr/bin/env python3
"""Deformation field forward throughput (csrc/deform.hip) at the Neu3D structure: P Gaussians,
planes 64/64/64/150 x multires [1, 2] x 16 channels, width-128 MLP with five heads.
Prints one JSON line: Gaussians/s, ms per call, and the matrix-core roofline of the MLP
(useful fp32-equivalent flops; the bf16 hi/lo split issues 3 MFMAs per product)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import torch  # noqa: E402

from deformation import DeformationField, HEADS, HEAD_OUT  # noqa: E402

BF16_DENSE_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 MFMA


def _stamps_fn():
    """lsr_debug_deform_stamps of a -DLSR_DEFORM_STAMPS build (LSR_LIBRARY), else None: read-and-reset."""
    import ctypes
    from diff_gaussian_rasterization import _lib
    try:
        fn = _lib.load().lsr_debug_deform_stamps
    except AttributeError:
        return None
    buf = (ctypes.c_ulonglong * 14)()

    def read():
        fn(buf)
        return list(buf)
    return read


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=2_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-torch", action="store_true", help="skip the eager-PyTorch comparison")
    ap.add_argument("--morton", action="store_true", help="store the Gaussians in Morton order (diagnostic)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    res, multires = [64, 64, 64, 150], [1, 2]
    params = {}
    for s, m in enumerate(multires):
        rs = [r * m for r in res[:3]] + [res[3]]
        for ci, (c0, c1) in enumerate([(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]):
            params[f"grid.grids.{s}.{ci}"] = torch.rand(1, 16, rs[c1], rs[c0], generator=g) * 1.4 + 0.1
    params["grid.aabb"] = torch.tensor([[1.5, 1.2, 10.0], [-1.5, -1.2, 2.0]])
    params["feature_out.0.weight"] = torch.randn(128, 32, generator=g) * 0.2
    params["feature_out.0.bias"] = torch.randn(128, generator=g) * 0.05
    for name, n in zip(HEADS, HEAD_OUT):
        params[name + ".1.weight"] = torch.randn(128, 128, generator=g) * 0.1
        params[name + ".1.bias"] = torch.randn(128, generator=g) * 0.05
        params[name + ".3.weight"] = torch.randn(n, 128, generator=g) * 0.1
        params[name + ".3.bias"] = torch.randn(n, generator=g) * 0.05
    field = DeformationField({k: v.to(dev) for k, v in params.items()}, res, multires)
    P = args.gaussians
    means = (torch.rand(P, 3, generator=g) * torch.tensor([3.0, 2.4, 8.0]) + torch.tensor([-1.5, -1.2, 2.0])).to(dev)
    if args.morton:   # diagnostic: Gaussians stored along a Morton curve (spatially coherent order)
        q = ((means - means.min(0).values) / (means.max(0).values - means.min(0).values) * 1023).long().cpu()
        code = torch.zeros(P, dtype=torch.long)
        for bit in range(10):
            for c in range(3):
                code |= ((q[:, c] >> bit) & 1) << (3 * bit + c)
        means = means[torch.argsort(code).to(dev)].contiguous()
    ins = [means, torch.randn(P, 3, generator=g).to(dev), torch.randn(P, 4, generator=g).to(dev),
           torch.randn(P, 1, generator=g).to(dev), torch.randn(P, 16, 3, generator=g).to(dev),
           torch.zeros(P, 3, device=dev)]
    for _ in range(3):
        field.forward(*ins, 0.4)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        field.forward(*ins, 0.4)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    macs = 32 * 128 + sum(128 * 128 + 128 * n for n in HEAD_OUT)   # per Gaussian
    useful_tflops = 2.0 * macs * P / (ms * 1e-3) / 1e12
    print(json.dumps(dict(metric="deformation forward Gaussians/s (Neu3D structure)", value=round(P / (ms * 1e-3)),
                          unit="Gaussians/s", ms_per_call=round(ms, 4), gaussians=P,
                          roofline=dict(bound="mfma", achieved=round(useful_tflops, 1), unit="TFLOP/s",
                                        peak=BF16_DENSE_PEAK_TFLOPS / 3, note="useful fp32-equivalent flops vs "
                                        "dense bf16 peak / 3 (hi/lo split: 3 MFMAs per product)",
                                        frac=round(useful_tflops / (BF16_DENSE_PEAK_TFLOPS / 3), 4)))))
    # backward: upstream gradients of the five outputs; input + parameter gradients
    ups = [torch.randn(P, 3, generator=g).to(dev), torch.randn(P, 3, generator=g).to(dev),
           torch.randn(P, 4, generator=g).to(dev), torch.randn(P, 1, generator=g).to(dev),
           torch.randn(P, 16, 3, generator=g).to(dev)]
    field.zero_grad()
    for _ in range(2):
        field.backward(means, 0.4, *ups)
    torch.cuda.synchronize()
    stamps = _stamps_fn()            # diagnostic build only (-DLSR_DEFORM_STAMPS)
    if stamps is not None:
        stamps()
    e0.record()
    for _ in range(args.iters // 2):
        field.backward(means, 0.4, *ups)
    e1.record()
    torch.cuda.synchronize()
    bms = e0.elapsed_time(e1) / (args.iters // 2)
    if stamps is not None:
        seg = stamps()
        names = ["features", "chain_fwd", "head_Z1", "head_dZ1_rest", "head_dA", "head_closing_sync",
                 "chain_bwd_dX", "hexplane_bwd", "small_G_loads", "small_first_sync", "sh_G_rows",
                 "sh_sync_GW2", "hexplane_grads"]   # hexplane_bwd: the scatter after hexplane_grads
        tot = sum(seg[:13]) or 1
        print(json.dumps(dict(phase_a_stamps={n: round(v / tot, 4) for n, v in zip(names, seg[:13])},
                              blocks=seg[13], note="wave 0 of each phase-A block, s_memtime cycles; shares")))
    # recompute of the forward MLP + data gradients (2 products per weight) + weight gradients (1)
    bflops = 2.0 * macs * 4 * P
    # rows written by the backward's phase A and read again (deform_api.hip bwd_scratch): the
    # features X (32), the feature_out layer's activation A and its gradient dH (128 each); the five
    # heads' hidden rows are recomputed by the weight-gradient kernels, not saved (round 4)
    saved = P * (32 + 128 + 128) * 4
    print(json.dumps(dict(metric="deformation backward Gaussians/s (Neu3D structure)", value=round(P / (bms * 1e-3)),
                          unit="Gaussians/s", ms_per_call=round(bms, 4), gaussians=P,
                          mlp_tflops=round(bflops / (bms * 1e-3) / 1e12, 1),
                          saved_activation_gb=round(saved / 1e9, 2))))
    if not args.no_torch:
        torch_baseline(params, res, multires, ins, ups, P, args.iters // 2)


def torch_baseline(params, res, multires, ins, ups, P, iters):
    """The same network in eager PyTorch on the same GPU (F.grid_sample bilinear, align_corners,
    border padding, product over the 6 planes, concat over scales, the Linear heads), fwd + autograd
    bwd: what running the reference module on this GPU costs (it cannot travel to the box)."""
    import torch.nn.functional as F
    dev = ins[0].device
    p = {k: v.to(dev).requires_grad_(k != "grid.aabb") for k, v in params.items()}
    combos = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]

    def run(means, scales, rots, opac, shs, t):
        a = p["grid.aabb"]
        pts = (means - a[0]) * (2.0 / (a[1] - a[0])) - 1.0
        q = torch.cat([pts, torch.full_like(means[:, :1], t)], dim=1)
        feats = []
        for s in range(len(multires)):
            prod = 1.0
            for ci, (c0, c1) in enumerate(combos):
                grid = q[:, [c0, c1]].view(1, 1, -1, 2)
                v = F.grid_sample(p[f"grid.grids.{s}.{ci}"], grid, mode="bilinear", padding_mode="border",
                                  align_corners=True).view(16, -1).t()
                prod = prod * v
            feats.append(prod)
        h = F.linear(torch.cat(feats, 1), p["feature_out.0.weight"], p["feature_out.0.bias"])
        outs = []
        for name, inp in zip(HEADS, (means, scales, rots, opac, shs.reshape(P, 48))):
            z = F.linear(torch.relu(h), p[name + ".1.weight"], p[name + ".1.bias"])
            outs.append(inp + F.linear(torch.relu(z), p[name + ".3.weight"], p[name + ".3.bias"]))
        return outs

    xs = [x.detach().clone().requires_grad_(True) for x in ins[:5]]
    gs = [ups[0], ups[1], ups[2], ups[3], ups[4].reshape(P, 48)]
    for _ in range(2):
        torch.autograd.backward(run(*xs, 0.4), gs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        with torch.no_grad():
            run(*xs, 0.4)
    e1.record()
    torch.cuda.synchronize()
    fms = e0.elapsed_time(e1) / iters
    e0.record()
    for _ in range(iters):
        torch.autograd.backward(run(*xs, 0.4), gs)
    e1.record()
    torch.cuda.synchronize()
    fbms = e0.elapsed_time(e1) / iters
    print(json.dumps(dict(metric="deformation, eager PyTorch on the same GPU (reference structure)", gaussians=P,
                          forward_ms=round(fms, 3), forward_backward_ms=round(fbms, 3))))


if __name__ == "__main__":
    main()
