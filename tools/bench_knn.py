"""distCUDA2 timing (simple_knn._C, knn.hip) at the config-5 init size (100k points) and at 2M,
beside scipy's KD-tree on the host (exact 3-NN, all cores) as the CPU reference point.
Prints one JSON line per size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from simple_knn._C import distCUDA2  # noqa: E402


def main():
    from scipy.spatial import cKDTree
    for P in (100_000, 2_000_000):
        rng = np.random.default_rng(0)
        pts = rng.uniform(-5, 5, (P, 3)).astype(np.float32)
        x = torch.tensor(pts, device="cuda")
        for _ in range(2):
            distCUDA2(x)
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            distCUDA2(x)
        torch.cuda.synchronize()
        gpu_ms = (time.perf_counter() - t0) / reps * 1e3
        t0 = time.perf_counter()
        cKDTree(pts).query(pts, k=4, workers=-1)
        cpu_ms = (time.perf_counter() - t0) * 1e3
        print(json.dumps(dict(metric="distCUDA2 points/s", points=P, gpu_ms=round(gpu_ms, 3),
                              value=round(P / gpu_ms * 1e3), unit="points/s",
                              cpu_kdtree_ms=round(cpu_ms, 1), cpu_threads=os.cpu_count())))


if __name__ == "__main__":
    main()
