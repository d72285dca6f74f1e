"""Generate tests/golden/deform_variants.npz from the REFERENCE deformation network (run in the
build container only; /root/reference does not exist on the GPU box).

deform_golden.npz (make_deform_golden.py) pins the Neu3D structure.  This file pins every other
switch of scene/deformation.py that the reference's configs and scripts use, each as a variant
named by its key prefix:

  hypernerf   arguments/hypernerf/default.py: multires [1, 2, 4], defor_depth 1, the ModelHiddenParams
              defaults no_do = no_dshs = True (three heads), language pass-through (no_dlang 1)
  lang        Neu3D structure, no_dlang 0 (scripts/train_eval.sh:27-31): lang_deform over
              [lang ++ poc_fre(t)] with the residual and re-normalisation (deformation.py:164-180,261-267),
              language_feature_hiddendim 6 (the video features)
  noresnet    lang with env no_resnet=t (:176-177), apply_rotation (quaternion product,
              :135-136, utils/graphics_utils.py:109-132) and no_ds (:120-122)
  discrete    hypernerf structure with env use_discrete_lang_f=t, centers_num 3
              (scripts/train_eval.sh:33-37): discrete_coff_generator head, per-centre normalisation,
              coff-weighted sum, re-normalisation (:156-163); coff is an output too
  deep        defor_depth 2 (feature_out.0, ReLU, feature_out.2: :55-60), no_dx (:114-115)

Each variant stores: config, inputs, every parameter on the computed path (float32 values, so the
kernels see exactly what the reference saw), the forward outputs (pts, scales, rotations, opacity,
shs, lang, coff) and the float64 autograd gradients of a seeded linear loss over all outputs
w.r.t. the inputs and the parameters.

    python tests/golden/make_deform_variants_golden.py            # deform_variants.npz
    python tests/golden/make_deform_variants_golden.py --layout   # deform_state_dict_layout.json
"""
import os
import sys
import types
from argparse import Namespace

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "deform_variants.npz")
RES = [10, 9, 8, 7]           # x, y, z, t plane resolution (spatial ones scaled by multires)
P = 300

VARIANTS = {
    "hypernerf": dict(args=dict(multires=[1, 2, 4], defor_depth=1, no_do=True, no_dshs=True, no_dlang=1),
                      env=dict(language_feature_hiddendim="3")),
    "lang": dict(args=dict(multires=[1, 2], defor_depth=0, no_do=False, no_dshs=False, no_dlang=0),
                 env=dict(language_feature_hiddendim="6")),
    "noresnet": dict(args=dict(multires=[1, 2], defor_depth=0, no_do=False, no_dshs=False, no_dlang=0,
                               apply_rotation=True, no_ds=True),
                     env=dict(language_feature_hiddendim="6", no_resnet="t")),
    "discrete": dict(args=dict(multires=[1, 2, 4], defor_depth=1, no_do=True, no_dshs=True, no_dlang=0),
                     env=dict(language_feature_hiddendim="6", use_discrete_lang_f="t", centers_num="3")),
    "deep": dict(args=dict(multires=[1, 2], defor_depth=2, no_do=False, no_dshs=False, no_dlang=1, no_dx=True),
                 env=dict(language_feature_hiddendim="3")),
}
ENV_KEYS = ("language_feature_hiddendim", "use_discrete_lang_f", "centers_num", "no_resnet", "use_tribute_dlang")


def _import_reference():
    sys.path.insert(0, REF)
    tk = types.ModuleType("tkinter")
    tk.W = "w"                # scene/deformation.py does `from tkinter import W`
    sys.modules.setdefault("tkinter", tk)
    pkg = types.ModuleType("scene")   # register the package without running its __init__ (dataset readers)
    pkg.__path__ = [os.path.join(REF, "scene")]
    sys.modules.setdefault("scene", pkg)
    from scene.deformation import deform_network
    return deform_network


def make_variant(deform_network, name, spec, seed):
    for k in ENV_KEYS:
        os.environ.pop(k, None)
    os.environ.update(spec["env"])
    base = dict(net_width=128, timebase_pe=4, defor_depth=0, posebase_pe=10, scale_rotation_pe=2, opacity_pe=2,
                timenet_width=64, timenet_output=32, bounds=1.6,
                kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                                "resolution": list(RES)},
                multires=[1, 2], no_dx=False, no_grid=False, no_ds=False, no_dr=False, no_do=True, no_dshs=True,
                no_dlang=1, empty_voxel=False, grid_pe=0, static_mlp=False, apply_rotation=False)
    base.update(spec["args"])
    args = Namespace(**base)
    torch.manual_seed(seed)
    net = deform_network(args).double()
    xyz_max, xyz_min = np.array([1.3, 0.9, 2.1]), np.array([-1.1, -0.7, 0.4])
    net.deformation_net.set_aabb(list(xyz_max), list(xyz_min))
    net.deformation_net.grid.aabb.data = net.deformation_net.grid.aabb.data.double()
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.deformation_net.grid.grids.parameters():
            p.copy_(torch.rand(p.shape, generator=g, dtype=torch.float64) * 1.4 + 0.1)
        for pname, p in net.named_parameters():
            if "bias" in pname:
                p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float64) * 0.05)
            p.copy_(p.float().double())          # float32 values: the kernels get exactly these
        net.deformation_net.grid.aabb.copy_(net.deformation_net.grid.aabb.float().double())

    C = int(spec["env"]["language_feature_hiddendim"])
    centers = int(spec["env"].get("centers_num", "3"))
    discrete = spec["env"].get("use_discrete_lang_f") == "t"
    lang_in = C * centers if discrete else C
    rng = np.random.default_rng(seed + 2)
    f32 = lambda a: np.asarray(a, np.float32).astype(np.float64)   # noqa: E731
    lo, hi = xyz_min - 0.15 * (xyz_max - xyz_min), xyz_max + 0.15 * (xyz_max - xyz_min)   # some outside: border clamp
    inp = dict(means3D=f32(rng.uniform(lo, hi, size=(P, 3))), scales=f32(rng.normal(-4.0, 0.5, size=(P, 3))),
               rotations=f32(rng.normal(size=(P, 4))), opacity=f32(rng.normal(size=(P, 1))),
               shs=f32(rng.normal(scale=0.3, size=(P, 16, 3))))
    lang = rng.normal(size=(P, lang_in))
    inp["lang"] = f32(lang / (np.linalg.norm(lang, axis=1, keepdims=True) + 1e-9))   # render()'s pre-normalisation
    times = np.full((P, 1), 0.3)
    times[: P // 4] = rng.uniform(-1.2, 1.2, size=(P // 4, 1))
    inp["time"] = f32(times)

    T = lambda a: torch.tensor(a, dtype=torch.float64, requires_grad=True)   # noqa: E731
    ts = {k: T(v) for k, v in inp.items()}
    outs = net(ts["means3D"], ts["scales"], ts["rotations"], ts["opacity"], ts["shs"], ts["lang"], ts["time"])
    names = ("means3D", "scales", "rotations", "opacity", "shs", "lang", "coff")
    loss = 0.0
    data = {}
    for n, x in zip(names, outs):
        if x is None:
            continue
        u = rng.normal(size=tuple(x.shape))
        data["out_" + n] = x.detach().numpy().astype(np.float32)
        data["up_" + n] = u.astype(np.float32)
        loss = loss + (x * torch.tensor(u.astype(np.float32).astype(np.float64))).sum()
    params = {k: v for k, v in net.deformation_net.named_parameters() if v.requires_grad}
    keys_in = ("means3D", "scales", "rotations", "opacity", "shs", "lang")
    grads = torch.autograd.grad(loss, [ts[k] for k in keys_in] + list(params.values()), allow_unused=True)
    for k, gv in zip(keys_in, grads[:6]):
        data["grad_" + k] = (np.zeros(inp[k].shape) if gv is None else gv.numpy()).astype(np.float32)
    used = 0
    for (k, v), gv in zip(params.items(), grads[6:]):
        if gv is None:            # off the computed path (a disabled head, the unused lang modules)
            continue
        used += 1
        data["param/" + k] = v.detach().numpy().astype(np.float32)
        data["grad/" + k] = gv.numpy().astype(np.float32)
    for k, v in inp.items():
        data[k] = v.astype(np.float32)
    data["aabb"] = net.deformation_net.grid.aabb.detach().numpy().astype(np.float32)
    cfg = dict(res=RES, multires=base["multires"], depth=base["defor_depth"], no_dx=base["no_dx"],
               no_ds=base["no_ds"], no_dr=base["no_dr"], no_do=base["no_do"], no_dshs=base["no_dshs"],
               no_dlang=base["no_dlang"], apply_rotation=base["apply_rotation"], lang_dim=C,
               centers=centers if discrete else 0, discrete=discrete, no_resnet=spec["env"].get("no_resnet") == "t",
               time_pe=base["timebase_pe"])
    data["config"] = np.array(repr(cfg))
    for k in ENV_KEYS:
        os.environ.pop(k, None)
    return {f"{name}/{k}": v for k, v in data.items()}, used


def state_dict_layout(deform_network):
    """Keys and shapes of deform_network(...).state_dict() for the HyperNeRF and Neu3D configs (what
    a trained model directory's deformation.pth holds: every module the reference builds, computed
    or not) -> tests/golden/deform_state_dict_layout.json."""
    import json
    out = {}
    for name, args in (("hypernerf", VARIANTS["hypernerf"]["args"]),
                       ("neu3d", dict(multires=[1, 2], defor_depth=0, no_do=False, no_dshs=False, no_dlang=1))):
        os.environ["language_feature_hiddendim"] = "3"
        base = dict(net_width=128, timebase_pe=4, defor_depth=0, posebase_pe=10, scale_rotation_pe=2, opacity_pe=2,
                    timenet_width=64, timenet_output=32, bounds=1.6,
                    kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                                    "resolution": [64, 64, 64, 150]},
                    multires=[1, 2], no_dx=False, no_grid=False, no_ds=False, no_dr=False, no_do=True, no_dshs=True,
                    no_dlang=1, empty_voxel=False, grid_pe=0, static_mlp=False, apply_rotation=False)
        base.update(args)
        net = deform_network(Namespace(**base))
        out[name] = {k: list(v.shape) for k, v in net.state_dict().items()}
    path = os.path.join(os.path.dirname(OUT), "deform_state_dict_layout.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path)


def main():
    deform_network = _import_reference()
    if "--layout" in sys.argv:
        state_dict_layout(deform_network)
        return
    out = {}
    for i, (name, spec) in enumerate(VARIANTS.items()):
        d, used = make_variant(deform_network, name, spec, seed=10 * i)
        out.update(d)
        print(f"{name}: {used} parameter tensors on the path")
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
