"""The 4D deformation field on MI355X: HexPlane sampling + MLP heads, fused in one HIP kernel
(csrc/deform.hip, C-ABI include/lsr_deform.h).  SURVEY.md 8(a) rows a2-a3, 8(f) row 1.

Mirrors the reference's `deform_network.forward_dynamic` (scene/deformation.py:232-248) in the
Neu3D structure (arguments/neu3d/default.py): per Gaussian, HexPlane features at (xyz, t) ->
feature_out Linear -> five residual heads (position, scales, rotations, opacity, SH); the
language feature passes through (no_dlang, the reference default).  Parameters keep the
reference's names (`from_reference_state_dict` accepts `deform_network.state_dict()`), so a
trained `deformation.pth` loads as is.

This round provides the forward (the render path, e.g. render.py); gradients are not produced,
so training keeps the reference module for now.  There is no CPU fallback.
"""
import ctypes
from typing import Dict, Sequence

import torch

from diff_gaussian_rasterization import _lib

HEADS = ("pos_deform", "scales_deform", "rotations_deform", "opacity_deform", "shs_deform")
HEAD_OUT = (3, 3, 4, 1, 48)


class DeformationField:
    """params: name -> tensor, names as in the reference `Deformation` module
    (grid.grids.{s}.{ci}, grid.aabb, feature_out.0.*, {head}.1.*, {head}.3.*).
    resolution / multires: the kplanes_config resolution [x, y, z, t] and multires list."""

    def __init__(self, params: Dict[str, torch.Tensor], resolution: Sequence[int], multires: Sequence[int],
                 device=None):
        device = device or params["feature_out.0.weight"].device
        if torch.device(device).type != "cuda":
            raise RuntimeError("the deformation field runs on the GPU only (no CPU fallback)")
        self.device = torch.device(device)
        self.p = {k: v.detach().to(self.device, torch.float32).contiguous() for k, v in params.items()}
        self.resolution, self.multires = list(resolution), list(multires)
        L = _lib.load()
        n = _lib.DeformNet()
        n.n_scales, n.channels, n.width = len(self.multires), self.p["grid.grids.0.0"].shape[1], \
            self.p["feature_out.0.weight"].shape[0]
        for i in range(4):
            n.res[i] = int(self.resolution[i])
            n.multires[i] = int(self.multires[i]) if i < len(self.multires) else 1
        n.aabb = self.p["grid.aabb"].data_ptr()
        for s in range(len(self.multires)):
            for ci in range(6):
                n.planes[s][ci] = self.p[f"grid.grids.{s}.{ci}"].data_ptr()
        n.w_feat, n.b_feat = self.p["feature_out.0.weight"].data_ptr(), self.p["feature_out.0.bias"].data_ptr()
        for h, name in enumerate(HEADS):
            n.w1[h], n.b1[h] = self.p[name + ".1.weight"].data_ptr(), self.p[name + ".1.bias"].data_ptr()
            n.w2[h], n.b2[h] = self.p[name + ".3.weight"].data_ptr(), self.p[name + ".3.bias"].data_ptr()
        self.net = n
        nbytes = int(L.lsr_deform_workspace_bytes(ctypes.byref(n)))
        if nbytes < 0:
            _lib.check(1, "lsr_deform_workspace_bytes")
        self.workspace = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self.prepare()

    @classmethod
    def from_reference_state_dict(cls, state_dict, resolution, multires, prefix="deformation_net.", device="cuda"):
        """Load `deform_network.state_dict()` (or a Deformation state dict with prefix="")."""
        params = {k[len(prefix):]: v for k, v in state_dict.items() if k.startswith(prefix)}
        return cls(params, resolution, multires, device=device)

    def prepare(self):
        """Repack planes and weights (call after every parameter update)."""
        L = _lib.load()
        _lib.check(L.lsr_deform_prepare(ctypes.byref(self.net), ctypes.c_void_p(self.workspace.data_ptr()),
                                        ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "lsr_deform_prepare")

    @torch.no_grad()
    def forward(self, means3D, scales, rotations, opacity, shs, lang, time):
        """Returns (means3D, scales, rotations, opacity, shs, lang, coff=None) like
        deform_network.forward (raw values, before activation)."""
        L = _lib.load()
        P = means3D.shape[0]
        f = lambda t, shape: t.detach().to(self.device, torch.float32).reshape(shape).contiguous()   # noqa: E731
        ins = (f(means3D, (P, 3)), f(scales, (P, 3)), f(rotations, (P, 4)), f(opacity, (P, 1)), f(shs, (P, 16, 3)))
        t = f(time, (P,)) if torch.is_tensor(time) and time.numel() == P else \
            torch.full((P,), float(time), device=self.device)
        outs = tuple(torch.empty_like(x) for x in ins)
        _lib.check(L.lsr_deform_forward(ctypes.byref(self.net), ctypes.c_void_p(self.workspace.data_ptr()), P,
                                        *[ctypes.c_void_p(x.data_ptr()) for x in ins], ctypes.c_void_p(t.data_ptr()),
                                        *[ctypes.c_void_p(x.data_ptr()) for x in outs],
                                        ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "lsr_deform_forward")
        return outs + (lang, None)

    __call__ = forward
