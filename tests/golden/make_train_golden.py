"""Generate tests/golden/train_golden.npz from the REFERENCE's own GaussianModel.

Runs only in the build container, where /root/reference exists.  The fixture is data: seeded
inputs and the outputs of the reference's methods, run unchanged on the CPU:

  * torch.optim.Adam(groups, lr=0.0, eps=1e-15) as scene/gaussian_model.py:301 builds it, three
    steps with random gradients (train.py:420-421);
  * the densification statistics of train.py:388-389 (max_radii2D) and
    GaussianModel.add_densification_stats (:746-748), two iterations;
  * GaussianModel.densify (:726-731: densify_and_clone then densify_and_split, N = 2);
  * GaussianModel.prune (:714-723) with a max screen size;
  * GaussianModel.reset_opacity (:391-394);
  * get_expon_lr_func (utils/general_utils.py:35-66) on a grid of steps.

How it runs on the CPU: the module's top-level imports of open3d, plyfile and simple_knn (absent
here, and not used by these methods) are registered as empty modules; the GaussianModel object is
made with __new__ plus setup_functions() and the attributes training_setup would set (its
deformation network is not involved); the module's `torch` (and utils.general_utils's, for
build_rotation) is a proxy that drops device="cuda" from torch.zeros and records the standard
normal draws of torch.normal(mean, std) = mean + std * z, so that the HIP split can be fed the
same z.

Usage:  python tests/golden/make_train_golden.py
"""
import os
import sys
import types

import numpy as np
import torch
from torch import nn

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "train_golden.npz")
P, C = 600, 8
NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation", "language_feature")
ATTR = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
        "scaling": "_scaling", "rotation": "_rotation", "language_feature": "_language_feature"}
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20.0, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3,
       "language_feature": 2.5e-3}


def main():
    if not os.path.isdir(REF):
        raise SystemExit("reference tree not present; the fixture is committed, nothing to do")
    sys.path.insert(0, REF)
    for name in ("open3d", "plyfile", "simple_knn", "simple_knn._C"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["plyfile"].PlyData = sys.modules["plyfile"].PlyElement = None
    sys.modules["simple_knn._C"].distCUDA2 = None
    tk = types.ModuleType("tkinter")
    tk.W = "w"
    sys.modules.setdefault("tkinter", tk)
    pkg = types.ModuleType("scene")
    pkg.__path__ = [os.path.join(REF, "scene")]
    sys.modules.setdefault("scene", pkg)
    import scene.gaussian_model as gmod  # noqa: E402
    import utils.general_utils as gu  # noqa: E402

    draws = []

    class _TorchCPU(types.ModuleType):
        def __getattr__(self, name):
            return getattr(torch, name)

        @staticmethod
        def zeros(*a, **k):
            k.pop("device", None)
            return torch.zeros(*a, **k)

        @staticmethod
        def normal(mean, std):
            z = torch.randn(std.shape, generator=gen)
            draws.append(z.clone())
            return mean + std * z

    proxy = _TorchCPU("torch")
    gmod.torch = proxy
    gu.torch = proxy

    gen = torch.Generator().manual_seed(2024)
    out = {}

    def rnd(*shape, scale=1.0, shift=0.0):
        return (torch.randn(*shape, generator=gen) * scale + shift).float()

    init = {
        "xyz": rnd(P, 3, scale=1.5),
        "f_dc": rnd(P, 1, 3, scale=0.5),
        "f_rest": rnd(P, 15, 3, scale=0.1),
        "opacity": rnd(P, 1, scale=2.0),
        "scaling": rnd(P, 3, scale=0.6, shift=-4.0),
        "rotation": rnd(P, 4),
        "language_feature": rnd(P, C),
    }
    gm = gmod.GaussianModel.__new__(gmod.GaussianModel)
    gm.setup_functions()
    for n in NAMES:
        setattr(gm, ATTR[n], nn.Parameter(init[n].clone().requires_grad_(True)))
        out[f"init_{n}"] = init[n].numpy()
    gm.percent_dense = 0.01
    gm.xyz_gradient_accum = torch.zeros((P, 1))
    gm.denom = torch.zeros((P, 1))
    gm.max_radii2D = torch.zeros((P,))
    gm._deformation_accum = torch.zeros((P, 3))
    gm._deformation_table = torch.rand(P, generator=gen) > 0.3
    out["init_deformation_table"] = gm._deformation_table.numpy()
    groups = [{"params": [getattr(gm, ATTR[n])], "lr": LRS[n], "name": n} for n in NAMES]
    gm.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)

    # ---- three Adam steps (train.py:420-421) ---------------------------------------------------
    for s in range(3):
        for n in NAMES:
            p = getattr(gm, ATTR[n])
            g = rnd(*p.shape, scale=10.0 ** (-1 - s))
            if s == 1:
                g[::7] = 0.0            # rows with zero gradient still move (moments decay)
            p.grad = g
            out[f"grad{s}_{n}"] = g.numpy()
        gm.optimizer.step()
        gm.optimizer.zero_grad(set_to_none=True)
    for n in NAMES:
        out[f"adam_{n}"] = getattr(gm, ATTR[n]).detach().numpy().copy()
        st = gm.optimizer.state[getattr(gm, ATTR[n])]
        out[f"adam_m_{n}"] = st["exp_avg"].numpy().copy()
        out[f"adam_v_{n}"] = st["exp_avg_sq"].numpy().copy()

    # ---- densification statistics (train.py:388-389) --------------------------------------------
    for it in range(2):
        radii = torch.randint(0, 30, (P,), generator=gen, dtype=torch.int32)
        radii[torch.rand(P, generator=gen) < 0.2] = 0
        vgrad = rnd(P, 3, scale=4e-4)
        vis = radii > 0
        gm.max_radii2D[vis] = torch.max(gm.max_radii2D[vis], radii[vis])
        gm.add_densification_stats(vgrad, vis)
        out[f"stats{it}_radii"] = radii.numpy()
        out[f"stats{it}_grad"] = vgrad.numpy()
    out["stats_max_radii2D"] = gm.max_radii2D.numpy().copy()
    out["stats_accum"] = gm.xyz_gradient_accum.numpy().copy()
    out["stats_denom"] = gm.denom.numpy().copy()

    # ---- densify (clone + split) --------------------------------------------------------------
    max_grad, extent = 4e-4, 3.0
    with torch.no_grad():                       # train.py:357: the densification runs under no_grad
        gm.densify(max_grad, 0.005, extent, None, 5, 5, None, None, stage="fine-base")
    out["densify_args"] = np.array([max_grad, gm.percent_dense, extent], np.float32)
    out["densify_z"] = torch.cat(draws).numpy() if draws else np.zeros((0, 3), np.float32)
    for n in NAMES:
        p = getattr(gm, ATTR[n])
        out[f"dens_{n}"] = p.detach().numpy().copy()
        st = gm.optimizer.state[p]
        out[f"dens_m_{n}"] = st["exp_avg"].numpy().copy()
        out[f"dens_v_{n}"] = st["exp_avg_sq"].numpy().copy()
    out["dens_deformation_table"] = gm._deformation_table.numpy().copy()

    # ---- prune (with statistics gathered after the densify) ----------------------------------------
    Pn = gm._xyz.shape[0]
    gm.max_radii2D = torch.randint(0, 40, (Pn,), generator=gen).float()
    gm.xyz_gradient_accum = rnd(Pn, 1).abs()
    gm.denom = torch.randint(0, 5, (Pn, 1), generator=gen).float()
    out["prune_in_max_radii2D"] = gm.max_radii2D.numpy().copy()
    out["prune_in_accum"] = gm.xyz_gradient_accum.numpy().copy()
    out["prune_in_denom"] = gm.denom.numpy().copy()
    min_op, max_screen = 0.08, 20
    with torch.no_grad():
        gm.prune(max_grad, min_op, extent, max_screen, "fine-base")
    out["prune_args"] = np.array([min_op, max_screen, extent], np.float32)
    for n in NAMES:
        p = getattr(gm, ATTR[n])
        out[f"prune_{n}"] = p.detach().numpy().copy()
        st = gm.optimizer.state[p]
        out[f"prune_m_{n}"] = st["exp_avg"].numpy().copy()
        out[f"prune_v_{n}"] = st["exp_avg_sq"].numpy().copy()
    out["prune_deformation_table"] = gm._deformation_table.numpy().copy()
    out["prune_max_radii2D"] = gm.max_radii2D.numpy().copy()
    out["prune_accum"] = gm.xyz_gradient_accum.numpy().copy()
    out["prune_denom"] = gm.denom.numpy().copy()

    # ---- reset_opacity -----------------------------------------------------------------------
    with torch.no_grad():
        gm.reset_opacity()
    st = gm.optimizer.state[gm._opacity]
    out["reset_opacity"] = gm._opacity.detach().numpy().copy()
    out["reset_m"] = st["exp_avg"].numpy().copy()
    out["reset_v"] = st["exp_avg_sq"].numpy().copy()

    # ---- learning-rate schedule (utils/general_utils.py:35-66) ---------------------------------
    steps = np.array([-1, 0, 1, 10, 500, 3000, 14000, 20000, 30000], np.int64)
    cfgs = [(1.6e-4 * 5.0, 1.6e-6 * 5.0, 0, 0.01, 20000), (1.6e-3, 1.6e-4, 100, 0.01, 14000), (0.0, 0.0, 0, 1.0, 100)]
    lr = np.array([[gu.get_expon_lr_func(lr_init=a, lr_final=b, lr_delay_steps=c, lr_delay_mult=d, max_steps=e)(int(s))
                    for s in steps] for a, b, c, d, e in cfgs], np.float64)
    out["lr_steps"] = steps
    out["lr_cfgs"] = np.array(cfgs, np.float64)
    out["lr_values"] = lr

    out["lrs"] = np.array([LRS[n] for n in NAMES], np.float64)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, "densified", out["dens_xyz"].shape[0], "pruned to", out["prune_xyz"].shape[0],
          "split draws", out["densify_z"].shape)


if __name__ == "__main__":
    main()
