"""CPU oracle of simple_knn distCUDA2 (include/lsr_knn.h) -- TEST INFRASTRUCTURE ONLY.

Restates the contract of the un-vendored submodule submodules/simple-knn (.gitmodules:1-3),
called at /root/reference/scene/gaussian_model.py:203: for every point, the mean of the squared
Euclidean distances to its 3 nearest OTHER points (duplicates count at distance 0; fewer than 3
others leave FLT_MAX entries, as upstream initialises its best list).  Brute force in float32
with the kernel's operation order -- d = dx*dx + dy*dy + dz*dz, the three smallest ascending,
(d1 + d2 + d3) / 3 -- so the HIP kernel is compared bit for bit.  PARITY UNPINNED against the
CUDA original (source absent); tests/test_knn_oracle.py checks this restatement against scipy's
KD-tree (an independent exact 3-NN).
"""
import numpy as np

FLT_MAX = np.float32(np.finfo(np.float32).max)


def mean_dist(points, chunk=512):
    p = np.ascontiguousarray(points, dtype=np.float32)
    P = p.shape[0]
    out = np.empty(P, np.float32)
    for s in range(0, P, chunk):
        q = p[s:s + chunk]
        dx = p[None, :, 0] - q[:, None, 0]
        dy = p[None, :, 1] - q[:, None, 1]
        dz = p[None, :, 2] - q[:, None, 2]
        d = dx * dx + dy * dy + dz * dz                       # float32, left to right
        d[np.arange(q.shape[0]), np.arange(s, s + q.shape[0])] = np.inf   # not itself
        k = min(3, P - 1)
        best = np.full((q.shape[0], 3), FLT_MAX, np.float32)
        if k > 0:
            part = np.partition(d, k - 1, axis=1)[:, :k] if P - 1 > k else d[:, :]
            part = np.sort(part, axis=1)[:, :k]
            best[:, :k] = np.minimum(part, FLT_MAX)
        with np.errstate(over="ignore"):
            out[s:s + chunk] = (best[:, 0] + best[:, 1] + best[:, 2]) / np.float32(3.0)
    return out
