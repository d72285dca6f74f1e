"""Generate tests/golden/deform_golden.npz from the REFERENCE deformation network (run in the
build container only; /root/reference does not exist on the GPU box).

Anchors the deformation oracle (oracle/deform_oracle.py) and the HIP kernels (deform.hip) on the
reference's own module: scene/deformation.py `deform_network` with the Neu3D structure
(arguments/neu3d/default.py: 16-channel planes, multires [1, 2], defor_depth 0, net_width 128,
d-opacity and d-SH heads on, language pass-through), on reduced plane resolutions so the fixture
stays small.  Planes are re-drawn at random (the reference initialises time planes to 1, which
would hide the time axis).  Stored: inputs, every parameter, the forward outputs, and the
gradients of a seeded linear loss w.r.t. inputs and parameters (torch autograd, float64).

    python tests/golden/make_deform_golden.py
"""
import os
import sys
import types
from argparse import Namespace

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "deform_golden.npz")
RES = [12, 10, 9, 7]          # x, y, z, t plane resolution (spatial ones scaled by multires)


def main():
    sys.path.insert(0, REF)
    tk = types.ModuleType("tkinter")
    tk.W = "w"                # scene/deformation.py does `from tkinter import W`
    sys.modules.setdefault("tkinter", tk)
    # the scene package's __init__ pulls in the dataset readers (torchvision); the deformation
    # modules need none of it, so register the package namespace without running __init__
    pkg = types.ModuleType("scene")
    pkg.__path__ = [os.path.join(REF, "scene")]
    sys.modules.setdefault("scene", pkg)
    from scene.deformation import deform_network

    args = Namespace(net_width=128, timebase_pe=4, defor_depth=0, posebase_pe=10, scale_rotation_pe=2, opacity_pe=2,
                     timenet_width=64, timenet_output=32, bounds=1.6,
                     kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                                     "resolution": list(RES)},
                     multires=[1, 2], no_dx=False, no_grid=False, no_ds=False, no_dr=False, no_do=False,
                     no_dshs=False, no_dlang=1, empty_voxel=False, grid_pe=0, static_mlp=False, apply_rotation=False)
    torch.manual_seed(0)
    net = deform_network(args).double()
    xyz_max, xyz_min = np.array([1.3, 0.9, 2.1]), np.array([-1.1, -0.7, 0.4])
    net.deformation_net.set_aabb(list(xyz_max), list(xyz_min))
    net.deformation_net.grid.aabb.data = net.deformation_net.grid.aabb.data.double()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for p in net.deformation_net.grid.grids.parameters():
            p.copy_(torch.rand(p.shape, generator=g, dtype=torch.float64) * 1.4 + 0.1)
        for name, p in net.named_parameters():   # biases drawn too (the reference leaves torch defaults)
            if "bias" in name:
                p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float64) * 0.05)

    P = 700
    rng = np.random.default_rng(2)
    lo, hi = xyz_min - 0.15 * (xyz_max - xyz_min), xyz_max + 0.15 * (xyz_max - xyz_min)   # some outside: border clamp
    means = rng.uniform(lo, hi, size=(P, 3))
    scales = rng.normal(-4.0, 0.5, size=(P, 3))
    rots = rng.normal(size=(P, 4))
    opac = rng.normal(size=(P, 1))
    shs = rng.normal(scale=0.3, size=(P, 16, 3))
    lang = rng.normal(size=(P, 3))
    times = np.full((P, 1), 0.3)
    times[: P // 5] = rng.uniform(-1.2, 1.2, size=(P // 5, 1))   # some varied, incl. outside [-1, 1]

    T = lambda a: torch.tensor(a, dtype=torch.float64, requires_grad=True)   # noqa: E731
    tm, ts, tr, to, tsh, tl, tt = T(means), T(scales), T(rots), T(opac), T(shs), T(lang), T(times)
    outs = net(tm, ts, tr, to, tsh, tl, tt)
    m2, s2, r2, o2, sh2, l2, coff = outs
    up = [rng.normal(size=tuple(x.shape)) for x in (m2, s2, r2, o2, sh2)]
    loss = sum((x * torch.tensor(u)).sum() for x, u in zip((m2, s2, r2, o2, sh2), up))
    params = dict(net.deformation_net.named_parameters())
    # parameters on the computed path (language pass-through: lang_deform / coff heads unused)
    wanted = {k: v for k, v in params.items() if v.requires_grad and not k.startswith(("lang_deform", "discrete_coff"))}
    grads = torch.autograd.grad(loss, [tm, ts, tr, to, tsh] + list(wanted.values()), allow_unused=True)

    data = dict(res=np.array(RES), multires=np.array([1, 2]), aabb=net.deformation_net.grid.aabb.detach().numpy(),
                means3D=means, scales=scales, rotations=rots, opacity=opac, shs=shs, lang=lang, time=times,
                out_means3D=m2.detach().numpy(), out_scales=s2.detach().numpy(), out_rotations=r2.detach().numpy(),
                out_opacity=o2.detach().numpy(), out_shs=sh2.detach().numpy(), out_lang=l2.detach().numpy(),
                up_means3D=up[0], up_scales=up[1], up_rotations=up[2], up_opacity=up[3], up_shs=up[4],
                grad_means3D=grads[0].numpy(), grad_scales=grads[1].numpy(), grad_rotations=grads[2].numpy(),
                grad_opacity=grads[3].numpy(), grad_shs=grads[4].numpy())
    for (k, v), gv in zip(wanted.items(), grads[5:]):
        data["param/" + k] = v.detach().numpy()
        data["grad/" + k] = np.zeros(tuple(v.shape)) if gv is None else gv.numpy()
    np.savez_compressed(OUT, **{k: np.asarray(v) for k, v in data.items()})   # float64 kept
    print("wrote", OUT, os.path.getsize(OUT), "bytes;", len(wanted), "parameter tensors")
    for k, v in wanted.items():
        print(f"  {k:60s} {tuple(v.shape)}")


if __name__ == "__main__":
    main()
