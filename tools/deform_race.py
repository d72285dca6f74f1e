#!/usr/bin/env python3
"""Deformation backward repeatability and oracle agreement (diagnostic): the Neu3D-resolution case of
tests/test_deform_gpu.py (P Gaussians, kink-ambiguous ones masked) run R times; d_means3D involves
no atomics, so any run-to-run difference is a race.  LSR_LIBRARY selects a variant build."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("4dlangsplat_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_deform_gpu as T  # noqa: E402
from deform_oracle import DeformOracle  # noqa: E402


def main():
    P0 = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    time = 0.37
    params, res, multires, inp = T._neu3d_case(P0, seed=3)
    a0, a1 = params["grid.aabb"][0], params["grid.aabb"][1]
    crd = (inp["means3D"] - a0) * (2.0 / (a1 - a0)) - 1.0
    keep = np.ones(P0, bool)
    for m in multires:
        for c in range(3):
            u = (crd[:, c] + 1.0) * 0.5 * (res[c] * m - 1)
            keep &= np.abs(u - np.round(u)) > 1e-3
    inp = {k: v[keep] for k, v in inp.items()}
    P = int(keep.sum())
    rng = np.random.default_rng(5)
    ups = dict(means3D=rng.normal(size=(P, 3)), scales=rng.normal(size=(P, 3)), rotations=rng.normal(size=(P, 4)),
               opacity=rng.normal(size=(P, 1)), shs=rng.normal(size=(P, 16, 3)) * 0.1)
    o = DeformOracle({k: v for k, v in params.items() if k != "grid.aabb"}, params["grid.aabb"])
    o.forward(inp["means3D"], inp["scales"], inp["rotations"], inp["opacity"], inp["shs"], None, np.full((P, 1), time))
    _, _, h, _, cache, _ = o._cache
    amb = (np.abs(h) < 1e-4).any(axis=1)
    for z, _ in cache.values():
        amb |= (np.abs(z) < 1e-4).any(axis=1)
    for k in T.KEYS:
        ups[k][amb] = 0.0
    g_in, g_p = o.backward(*[np.asarray(ups[k], np.float32).astype(np.float64) for k in T.KEYS])
    f = T._field(params, res, multires)
    t = lambda a: torch.tensor(np.asarray(a, np.float32)).cuda()   # noqa: E731
    first = None
    F = 16 * len(multires)
    al = lambda n: ((n * 4 + 255) // 256) * 256    # noqa: E731  (deform_api.hip bwd_scratch: X, A0, dH0)
    segs = {"X": (0, F), "A0": (al(P * F), 128), "dH0": (al(P * F) + al(P * 128), 128)}
    first_seg = {}
    from diff_gaussian_rasterization import _lib
    f_lib = _lib.load()
    try:
        f_lib.lsr_debug_deform_diag
    except AttributeError:
        f_lib = None
    # the forward (same LDS footprint class, features_to_lds) repeated: outputs must repeat bit for bit
    fin = [t(inp[k]) for k in T.KEYS]
    ref_out = None
    for r in range(R):
        out = [o.cpu().numpy() for o in f.forward(*fin, None, time)[:5]]
        if ref_out is None:
            ref_out = out
        else:
            for k, a_, b_ in zip(T.KEYS, out, ref_out):
                if not np.array_equal(a_, b_):
                    rows = np.nonzero((a_ != b_).reshape(P, -1).any(axis=1))[0]
                    print(f"forward run {r}: {k} DIFFERS at {len(rows)} rows {rows[:8].tolist()} (in-block "
                          f"{sorted(set((rows % 64).tolist()))[:16]})", flush=True)
    print("forward repeats checked", flush=True)
    for r in range(R):
        f.zero_grad()
        got = f.backward(t(inp["means3D"]), time, *[t(ups[k]) for k in T.KEYS])
        torch.cuda.synchronize()
        for name, (off, w) in segs.items():   # saved rows run to run: the first stage that differs
            v = f._scratch[off:off + P * w * 4].view(torch.float32).reshape(P, w).cpu().numpy()
            if name not in first_seg:
                first_seg[name] = v.copy()
            elif not np.array_equal(v, first_seg[name]):
                rows = np.nonzero((v != first_seg[name]).any(axis=1))[0]
                cols = np.nonzero((v != first_seg[name]).any(axis=0))[0]
                print(f"run {r}: {name} DIFFERS at {len(rows)} rows {rows[:12].tolist()} (in-block "
                      f"{sorted(set((rows % 64).tolist()))[:16]}) cols {cols[:40].tolist()}", flush=True)
        diag = getattr(f_lib, "lsr_debug_deform_diag", None) if f_lib is not None else None
        if diag is not None:
            buf = (ctypes.c_ulonglong * 8)()
            diag(buf)
            print(f"run {r}: scatter diag bad={buf[0]} by tap {list(buf)[1:5]}", flush=True)
        dm = got[0].cpu().numpy()
        err = T._rel(dm, g_in["means3D"])
        perr = max(T._rel(g.cpu().numpy(), g_p[n].reshape(g.shape)) for n, g in f.grads.items())
        bad = np.abs(dm - g_in["means3D"]).max(axis=1) > 1e-3 * np.abs(g_in["means3D"]).max()
        same = "first" if first is None else ("identical" if np.array_equal(dm, first) else
                                              f"DIFFERS at {int((dm != first).any(axis=1).sum())} rows")
        first = dm if first is None else first
        rows = np.nonzero(bad)[0]
        print(f"run {r}: d_means3D rel {err:.2e} (bad rows {len(rows)}: {rows[:8].tolist()} blocks "
              f"{sorted(set((rows // 64).tolist()))[:8]}), params rel {perr:.2e}, vs run 0: {same}", flush=True)


if __name__ == "__main__":
    main()
