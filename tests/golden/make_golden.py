"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own Python code.

Runs only in the build container, where /root/reference exists (it never travels to the GPU
box).  The fixtures are data: seeded inputs and the reference's outputs.

  sh_golden.npz   utils/sh_utils.py:57-112 eval_sh + gaussian_renderer/__init__.py:201-205
                  (+0.5, clamp_min 0), degrees 0-3, float32 torch CPU.
  cameras.npz     scene/cameras.py:56-67 with utils/graphics_utils.py:38-71
                  (world_view_transform, full_proj_transform, camera_center).
  cov3d.npz       scene/gaussian_model.py:32-36 build_covariance_from_scaling_rotation with
                  utils/general_utils.py:70-116 (build_rotation / build_scaling_rotation /
                  strip_symmetric).  Those functions hard-code device="cuda"
                  (general_utils.py:71,89,108); they are run unchanged on the CPU with that one
                  keyword dropped by a torch proxy.

Usage:  python tests/golden/make_golden.py
"""
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    if not os.path.isdir(REF):
        raise SystemExit("reference tree not present; fixtures are committed, nothing to do")
    sys.path.insert(0, REF)
    from utils import sh_utils, graphics_utils  # noqa: E402
    import utils.general_utils as gu  # noqa: E402

    g = torch.Generator().manual_seed(1234)

    # ---- SH -> RGB -----------------------------------------------------------------------
    sh_out = {}
    N = 512
    for deg in range(4):
        M = 16
        sh = (torch.randn(N, M, 3, generator=g) * 0.4).float()
        pos = (torch.randn(N, 3, generator=g) * 3.0).float()
        campos = torch.tensor([0.3, -0.2, 0.1], dtype=torch.float32)
        shs_view = sh.transpose(1, 2).view(-1, 3, M)
        dir_pp = pos - campos.repeat(N, 1)
        dir_n = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(sh_utils.eval_sh(deg, shs_view, dir_n) + 0.5, 0.0)
        sh_out[f"sh_{deg}"] = sh.numpy()
        sh_out[f"pos_{deg}"] = pos.numpy()
        sh_out[f"campos_{deg}"] = campos.numpy()
        sh_out[f"rgb_{deg}"] = rgb.numpy()
    np.savez(os.path.join(OUT, "sh_golden.npz"), **sh_out)

    # ---- cameras ---------------------------------------------------------------------------
    cams = {}
    specs = [
        (np.eye(3), np.zeros(3), 2 * math.atan(0.6), 2 * math.atan(0.45), 1352, 1014),
        (None, np.array([0.1, -0.05, 0.3]), 2 * math.atan(0.5), 2 * math.atan(0.4), 960, 540),
        (None, np.array([-0.2, 0.02, -0.1]), 1.2, 0.9, 400, 400),
    ]
    rng = np.random.default_rng(7)
    for i, (R, T, fovx, fovy, W, H) in enumerate(specs):
        if R is None:
            a = rng.normal(size=3)
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            w, x, y, z = q
            R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                          [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                          [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
            del a
        wv = torch.tensor(graphics_utils.getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
        pr = graphics_utils.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pr.unsqueeze(0)).squeeze(0)
        center = wv.inverse()[3, :3]
        cams[f"R_{i}"] = R
        cams[f"T_{i}"] = T
        cams[f"fov_{i}"] = np.array([fovx, fovy])
        cams[f"size_{i}"] = np.array([W, H])
        cams[f"view_{i}"] = wv.numpy()
        cams[f"proj_{i}"] = pr.numpy()
        cams[f"full_{i}"] = full.numpy()
        cams[f"center_{i}"] = center.numpy()
    np.savez(os.path.join(OUT, "cameras.npz"), **cams)

    # ---- covariance from (scale, rotation) ---------------------------------------------------
    class _TorchCPU(types.ModuleType):
        def __getattr__(self, name):
            return getattr(torch, name)

        @staticmethod
        def zeros(*a, **k):
            k.pop("device", None)
            return torch.zeros(*a, **k)

    gu.torch = _TorchCPU("torch")
    N = 512
    scales = torch.exp(torch.randn(N, 3, generator=g) * 0.7 - 3.0).float()
    q = torch.randn(N, 4, generator=g).float()
    rots = torch.nn.functional.normalize(q)
    mod = 1.0
    L = gu.build_scaling_rotation(mod * scales, rots)
    cov = gu.strip_symmetric(L @ L.transpose(1, 2))
    np.savez(os.path.join(OUT, "cov3d.npz"), scales=scales.numpy(), rotations=rots.numpy(), mod=np.float32(mod),
             cov=cov.numpy())
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
