"""simple_knn._C.distCUDA2 on the MI355X (lsr_knn_mean_dist, knn.hip).

distCUDA2(points [P, 3] float32 on the GPU) -> [P] float32: the mean of the squared distances
from each point to its 3 nearest other points (scene/gaussian_model.py:203 clamps it at 1e-7 and
takes log(sqrt(.)) as the initial scale).  Exact 3-NN; GPU only (no CPU fallback).
"""
import ctypes

import torch

from diff_gaussian_rasterization import _lib


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    if points.device.type != "cuda":
        raise RuntimeError("distCUDA2 runs on the GPU only (no CPU fallback); got tensors on " + str(points.device))
    if points.dim() != 2 or points.shape[1] != 3:
        raise ValueError("points must be [P, 3]")
    L = _lib.load()
    pts = points.detach().to(torch.float32).contiguous()
    P = pts.shape[0]
    out = torch.empty(P, dtype=torch.float32, device=pts.device)
    if P == 0:
        return out
    ws = torch.empty(int(L.lsr_knn_workspace_bytes(P)), dtype=torch.uint8, device=pts.device)
    stream = torch.cuda.current_stream(pts.device).cuda_stream
    _lib.check(L.lsr_knn_mean_dist(P, ctypes.c_void_p(pts.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                   ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(stream)), "lsr_knn_mean_dist")
    return out
