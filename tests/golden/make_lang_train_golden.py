"""Generate tests/golden/lang_train_golden.npz: one 'lang'-stage training iteration of the REFERENCE
(train.py:242-339) on a tiny scene, run in the build container only (/root/reference does not exist
on the GPU box).  The fixture is data: seeded inputs, the loss and the gradients.

What runs is the reference's own code, unchanged, on the CPU in float64:
  * gaussian_renderer.render (gaussian_renderer/__init__.py:19-248): stage logic, the language
    pre-normalisation, the deform_network call with no_dlang from args, the activations;
  * scene.deformation.deform_network with lang_deform (no_dlang 0, the residual mode, env
    language_feature_hiddendim 6; scripts/train_eval.sh:27-31);
  * utils.loss_utils.l1_loss / cos_loss combined as train.py:283-296 combines them (lam, beta,
    addcosloss, joint_train);
  * loss.backward() into the GaussianModel parameters and the field.
The rasterizer the reference imports (diff_gaussian_rasterization, an un-vendored CUDA submodule,
SURVEY.md 8(c)) is absent: a module of that name is registered whose GaussianRasterizer runs this
repository's C oracle (oracle/lsr_oracle.c, double build) forward and backward inside autograd --
the same oracle every rasterizer parity test is checked against.  Absent imports that the used code
never calls (lpips, open3d, plyfile, simple_knn, tkinter) are registered as empty modules; the
renderer module's torch.zeros_like drops device="cuda" and Tensor.cuda() is the identity (CPU run).

Variants: "lang" (fine-lang, lam 0.2), "cos_joint" (fine-lang with addcosloss, beta 0.01, and
joint_train: the RGB L1 too, every parameter trainable).  Each stores the GaussianModel parameters
and field parameters (float32 values), the camera, gt image / language / mask, the loss, the
rendered language image and the float64 gradients of every trainable tensor; `ambiguous` marks the
Gaussians with a field pre-activation within 1e-4 of a ReLU kink (their gradients may legitimately
differ between float32 and float64 evaluations; the test compares their rows loosely).

    python tests/golden/make_lang_train_golden.py
"""
import math
import os
import sys
import types
from argparse import Namespace
from typing import NamedTuple

import numpy as np
import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
OUT = os.path.join(HERE, "lang_train_golden.npz")
P, W, H, C = 500, 64, 48, 6
RES = [10, 9, 8, 7]


def _oracle_rasterizer_module():
    """A `diff_gaussian_rasterization` whose GaussianRasterizer is the C oracle (float64) in autograd."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    class GaussianRasterizationSettings(NamedTuple):
        image_height: int
        image_width: int
        tanfovx: float
        tanfovy: float
        bg: torch.Tensor
        scale_modifier: float
        viewmatrix: torch.Tensor
        projmatrix: torch.Tensor
        sh_degree: int
        campos: torch.Tensor
        prefiltered: bool
        debug: bool
        include_feature: bool = True

    npy = lambda t: t.detach().cpu().numpy().astype(np.float64)   # noqa: E731

    class _Raster(torch.autograd.Function):
        @staticmethod
        def forward(ctx, rs, means3D, means2D, shs, lang, opacities, scales, rotations):
            s = oracle.OracleSettings(rs.image_height, rs.image_width, rs.tanfovx, rs.tanfovy, npy(rs.bg),
                                      rs.scale_modifier, npy(rs.viewmatrix), npy(rs.projmatrix), rs.sh_degree,
                                      npy(rs.campos), rs.include_feature)
            r = oracle.forward(s, npy(means3D), npy(opacities), shs=npy(shs),
                               lang=npy(lang) if rs.include_feature else None, scales=npy(scales),
                               rotations=npy(rotations), double=True)
            ctx.r, ctx.include = r, rs.include_feature
            ctx.shapes = (shs.shape, opacities.shape)
            color, lang_img, depth, radii = r.color, r.lang, r.depth, r.radii
            if not rs.include_feature:
                lang_img = np.zeros((lang.shape[-1], rs.image_height, rs.image_width))
            t = lambda a: torch.tensor(a, dtype=torch.float64)   # noqa: E731
            ctx.mark_non_differentiable(t(radii))
            return t(color), t(lang_img), torch.tensor(radii), t(depth)

        @staticmethod
        def backward(ctx, g_color, g_lang, g_radii, g_depth):
            g = ctx.r.backward(npy(g_color), npy(g_lang) if ctx.include else None, npy(g_depth))
            t = lambda a: torch.tensor(a, dtype=torch.float64)   # noqa: E731
            sh_shape, op_shape = ctx.shapes
            return (None, t(g["means3D"]), t(g["means2D"]), t(g["sh"]).reshape(sh_shape),
                    t(g["lang"]) if ctx.include else None, t(g["opacity"]).reshape(op_shape), t(g["scales"]),
                    t(g["rotations"]))

    class GaussianRasterizer(nn.Module):
        def __init__(self, raster_settings):
            super().__init__()
            self.raster_settings = raster_settings

        def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, language_feature_precomp=None,
                    scales=None, rotations=None, cov3D_precomp=None):
            assert shs is not None and colors_precomp is None and cov3D_precomp is None
            return _Raster.apply(self.raster_settings, means3D, means2D, shs, language_feature_precomp, opacities,
                                 scales, rotations)

    mod = types.ModuleType("diff_gaussian_rasterization")
    mod.GaussianRasterizationSettings = GaussianRasterizationSettings
    mod.GaussianRasterizer = GaussianRasterizer
    return mod


def _import_reference():
    sys.path.insert(0, REF)
    tk = types.ModuleType("tkinter")
    tk.W = "w"
    sys.modules.setdefault("tkinter", tk)
    for name in ("open3d", "plyfile", "simple_knn", "simple_knn._C", "lpips"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["plyfile"].PlyData = sys.modules["plyfile"].PlyElement = None
    sys.modules["simple_knn._C"].distCUDA2 = None
    sys.modules["diff_gaussian_rasterization"] = _oracle_rasterizer_module()
    pkg = types.ModuleType("scene")
    pkg.__path__ = [os.path.join(REF, "scene")]
    sys.modules.setdefault("scene", pkg)
    import gaussian_renderer as gr
    import scene.gaussian_model as gmod
    from scene.deformation import deform_network
    from utils.loss_utils import cos_loss, l1_loss

    class _TorchCPU(types.ModuleType):
        def __getattr__(self, name):
            return getattr(torch, name)

        @staticmethod
        def zeros_like(*a, **k):
            k.pop("device", None)
            return torch.zeros_like(*a, **k)

    gr.torch = _TorchCPU("torch")
    torch.Tensor.cuda = lambda self, *a, **k: self
    return gr.render, gmod.GaussianModel, deform_network, l1_loss, cos_loss


def make_variant(ref, name, lam, beta, addcosloss, joint_train, seed):
    render, GaussianModel, deform_network, l1_loss, cos_loss = ref
    sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))
    import synthetic
    os.environ["language_feature_hiddendim"] = str(C)
    for k in ("use_discrete_lang_f", "no_resnet", "nonormalized", "centers_num"):
        os.environ.pop(k, None)
    g = torch.Generator().manual_seed(seed)
    f32 = lambda t: t.float().double()   # noqa: E731  (float32 values: the GPU run sees exactly these)
    torch.set_default_dtype(torch.float32)           # the synthetic generators are float32
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W, seed=seed, logscale_mean=-3.0)
    cam = synthetic.camera_batch(1, W, H, tanfovx=0.6, seed=seed + 3, max_yaw=8.0)[0]
    cam.time = 0.35
    torch.set_default_dtype(torch.float64)           # the reference's code runs in float64
    xyz = f32(sc.means3D)
    params = dict(xyz=xyz, f_dc=f32(sc.shs[:, :1]), f_rest=f32(sc.shs[:, 1:]),
                  opacity=f32(torch.logit(sc.opacities.reshape(P, 1).double())),
                  scaling=f32(torch.log(sc.scales.double())),
                  rotation=f32(sc.rotations.double() * (0.5 + torch.rand(P, 1, generator=g, dtype=torch.float64))),
                  language_feature=f32(torch.randn(P, C, generator=g, dtype=torch.float64)))
    gm = GaussianModel.__new__(GaussianModel)
    gm.setup_functions()
    attr = dict(xyz="_xyz", f_dc="_features_dc", f_rest="_features_rest", opacity="_opacity", scaling="_scaling",
                rotation="_rotation", language_feature="_language_feature")
    for k, a in attr.items():
        # training_setup's lang branch: requires_grad_(joint_train) on every group but the language
        setattr(gm, a, nn.Parameter(params[k].clone(), requires_grad=(k == "language_feature" or joint_train)))
    gm.active_sh_degree = gm.max_sh_degree = 3
    gm._deformation_table = torch.ones(P, dtype=torch.bool)
    hidden = dict(net_width=128, timebase_pe=4, defor_depth=0, posebase_pe=10, scale_rotation_pe=2, opacity_pe=2,
                  timenet_width=64, timenet_output=32, bounds=1.6,
                  kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                                  "resolution": list(RES)},
                  multires=[1, 2], no_dx=False, no_grid=False, no_ds=False, no_dr=False, no_do=False, no_dshs=False,
                  no_dlang=0, empty_voxel=False, grid_pe=0, static_mlp=False, apply_rotation=False)
    torch.manual_seed(seed + 1)
    net = deform_network(Namespace(**hidden)).double()
    lo, hi = xyz.min(0).values, xyz.max(0).values
    net.deformation_net.set_aabb(list(hi.numpy() + 0.1), list(lo.numpy() - 0.1))
    with torch.no_grad():
        net.deformation_net.grid.aabb.copy_(net.deformation_net.grid.aabb.float().double())
        for p in net.deformation_net.grid.grids.parameters():
            p.copy_(torch.rand(p.shape, generator=g, dtype=torch.float64) * 1.4 + 0.1)
        for pname, p in net.named_parameters():
            if "bias" in pname:
                p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float64) * 0.05)
            p.copy_(p.float().double())
    # training_setup's lang branch (gaussian_model.py:258-270)
    net.requires_grad_(joint_train)
    net.deformation_net.lang_deform.requires_grad_(True)
    gm._deformation = net
    # pre-activations of every Linear: Gaussians near a ReLU kink
    pre = []
    hooks = [m.register_forward_hook(lambda m, i, o: pre.append(o.detach()))
             for m in net.deformation_net.modules() if isinstance(m, nn.Linear)]

    camd = Namespace(FoVx=cam.FoVx, FoVy=cam.FoVy, image_width=W, image_height=H, time=cam.time,
                     world_view_transform=cam.world_view_transform.double(),
                     full_proj_transform=cam.full_proj_transform.double(), camera_center=cam.camera_center.double())
    bg = torch.ones(3, dtype=torch.float64)
    pipe = Namespace(debug=False, compute_cov3D_python=False, convert_SHs_python=False)
    args = Namespace(no_dlang=0)
    pkg = render(camd, gm, pipe, bg, None, stage="fine-lang", cam_type=None, args=args)
    for h in hooks:
        h.remove()
    image, lang_img = pkg["render"], pkg["language_feature_image"]
    gt_lang = f32(torch.randn(1, C, H, W, generator=g, dtype=torch.float64) * 0.5)
    mask = (torch.rand(1, 1, H, W, generator=g, dtype=torch.float64) > 0.3).double()
    gt_img = f32((image.detach() + (torch.randint(0, 2, image.shape, generator=g) * 2 - 1) * 0.1).unsqueeze(0))
    # train.py:272-296 with batch_size 1: the cat over views is the one view
    lf, lm, gl = lang_img.unsqueeze(0), mask, gt_lang
    loss = lam * l1_loss(lf * lm, gl * lm)
    if addcosloss:
        loss = loss + beta * cos_loss(lf * lm, gl * lm)
    if joint_train:
        loss = loss + l1_loss(image.unsqueeze(0), gt_img[:, :3])
    loss.backward()
    out = {}
    for k, a in attr.items():
        out["param/" + k] = params[k].float().numpy()
        p = getattr(gm, a)
        if p.grad is not None:
            out["grad/" + k] = p.grad.numpy().astype(np.float64)
    for k, v in net.deformation_net.named_parameters():
        out["field/" + k] = v.detach().float().numpy()
        if v.grad is not None:
            out["fieldgrad/" + k] = v.grad.numpy().astype(np.float64)
    out["field_aabb"] = net.deformation_net.grid.aabb.detach().float().numpy()
    amb = np.zeros(P, bool)
    for z in pre:
        if z.shape[0] == P:
            amb |= (z.abs() < 1e-4).any(dim=1).numpy()
    out.update(dict(loss=np.float64(loss.item()), lang_img=lang_img.detach().numpy(), image=image.detach().numpy(),
                    gt_lang=gt_lang.float().numpy(), mask=mask.float().numpy(), gt_img=gt_img.float().numpy(),
                    viewmatrix=cam.world_view_transform.numpy(), projmatrix=cam.full_proj_transform.numpy(),
                    campos=cam.camera_center.numpy(), fov=np.array([cam.FoVx, cam.FoVy]), time=np.float64(cam.time),
                    ambiguous=amb, hp=np.array([lam, beta, float(addcosloss), float(joint_train)]),
                    config=np.array(repr(dict(res=RES, multires=[1, 2], lang_dim=C, W=W, H=H)))))
    print(f"{name}: loss {loss.item():.6f}, {amb.sum()} kink-ambiguous Gaussians, "
          f"{sum(1 for k in out if k.startswith('fieldgrad/'))} field gradients")
    return {f"{name}/{k}": v for k, v in out.items()}


def main():
    if not os.path.isdir(REF):
        raise SystemExit("reference tree not present; the fixture is committed, nothing to do")
    ref = _import_reference()
    out = {}
    out.update(make_variant(ref, "lang", 0.2, 0.01, False, False, seed=3))
    out.update(make_variant(ref, "cos_joint", 0.2, 0.01, True, True, seed=4))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
