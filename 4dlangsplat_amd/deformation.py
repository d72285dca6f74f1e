"""The 4D deformation field on MI355X: HexPlane sampling + MLP heads, fused in one HIP kernel
(csrc/deform.hip, C-ABI include/lsr_deform.h).  SURVEY.md 8(a) rows a2-a3, 8(f) row 1.

Mirrors the reference's `deform_network.forward_dynamic` (scene/deformation.py:232-248) in the
Neu3D structure (arguments/neu3d/default.py): per Gaussian, HexPlane features at (xyz, t) ->
feature_out Linear -> five residual heads (position, scales, rotations, opacity, SH); the
language feature passes through (no_dlang, the reference default).  Parameters keep the
reference's names (`from_reference_state_dict` accepts `deform_network.state_dict()`), so a
trained `deformation.pth` loads as is.

Forward (the render path) and backward (lsr_deform_backward: input gradients, and the gradients
of every plane and Linear parameter, accumulated into `grads`); `apply` runs the forward inside
autograd.  There is no CPU fallback.
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

    @staticmethod
    def init_params(resolution: Sequence[int], multires: Sequence[int], aabb, channels: int = 16, width: int = 128,
                    seed: int = 0) -> Dict[str, torch.Tensor]:
        """A freshly initialised field, as the reference builds one (CPU tensors): spatial planes
        U(0.1, 0.5) and time planes ones (scene/hexplane.py:48-70), Linear weights Xavier-uniform
        (scene/deformation.py:254-260) and biases torch's default U(+-1/sqrt(fan_in)).
        aabb: [[x, y, z]_max, [x, y, z]_min]."""
        g = torch.Generator().manual_seed(seed)
        p = {"grid.aabb": torch.as_tensor(aabb, dtype=torch.float32)}
        for s, m in enumerate(multires):
            reso = [r * m for r in resolution[:3]] + [resolution[3]]
            for ci, (c0, c1) in enumerate([(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]):
                shape = (1, channels, reso[c1], reso[c0])
                p[f"grid.grids.{s}.{ci}"] = torch.ones(shape) if c1 == 3 else torch.rand(shape, generator=g) * 0.4 + 0.1

        def linear(name, n_out, n_in):
            bound = (6.0 / (n_in + n_out)) ** 0.5
            p[name + ".weight"] = (torch.rand(n_out, n_in, generator=g) * 2 - 1) * bound
            p[name + ".bias"] = (torch.rand(n_out, generator=g) * 2 - 1) / n_in ** 0.5
        linear("feature_out.0", width, channels * len(multires))
        for name, n in zip(HEADS, HEAD_OUT):
            linear(name + ".1", width, width)
            linear(name + ".3", n, width)
        return p

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

    # ---- backward (lsr_deform_backward) -------------------------------------------------------
    def zero_grad(self):
        """Parameter gradients (torch layouts, names as the parameters) set to zero."""
        self.grads = {k: torch.zeros_like(v) for k, v in self.p.items() if k != "grid.aabb"}

    def backward(self, means3D, time, d_means3D, d_scales, d_rotations, d_opacity, d_shs):
        """Gradients of forward() given the gradients of its five outputs: returns the input
        gradients (means3D, scales, rotations, opacity, shs) and ADDS the parameter gradients to
        self.grads (as torch accumulates .grad).  Call prepare() after parameter updates first."""
        L = _lib.load()
        if not hasattr(self, "grads"):
            self.zero_grad()
        P = means3D.shape[0]
        f = lambda t, shape: t.detach().to(self.device, torch.float32).reshape(shape).contiguous()   # noqa: E731
        m = f(means3D, (P, 3))
        t = f(time, (P,)) if torch.is_tensor(time) and time.numel() == P else \
            torch.full((P,), float(time), device=self.device)
        ups = (f(d_means3D, (P, 3)), f(d_scales, (P, 3)), f(d_rotations, (P, 4)), f(d_opacity, (P, 1)),
               f(d_shs, (P, 16, 3)))
        dm = torch.empty_like(m)
        g = _lib.DeformGrads()
        for s in range(len(self.multires)):
            for ci in range(6):
                g.planes[s][ci] = self.grads[f"grid.grids.{s}.{ci}"].data_ptr()
        g.w_feat, g.b_feat = self.grads["feature_out.0.weight"].data_ptr(), self.grads["feature_out.0.bias"].data_ptr()
        for h, name in enumerate(HEADS):
            g.w1[h], g.b1[h] = self.grads[name + ".1.weight"].data_ptr(), self.grads[name + ".1.bias"].data_ptr()
            g.w2[h], g.b2[h] = self.grads[name + ".3.weight"].data_ptr(), self.grads[name + ".3.bias"].data_ptr()
        nbytes = int(L.lsr_deform_backward_scratch_bytes(ctypes.byref(self.net), P))
        if nbytes < 0:
            _lib.check(1, "lsr_deform_backward_scratch_bytes")
        if getattr(self, "_scratch", None) is None or self._scratch.numel() < nbytes:
            self._scratch = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        vp = ctypes.c_void_p
        _lib.check(L.lsr_deform_backward(ctypes.byref(self.net), vp(self.workspace.data_ptr()), P, vp(m.data_ptr()),
                                         vp(t.data_ptr()), *[vp(u.data_ptr()) for u in ups], vp(dm.data_ptr()),
                                         ctypes.byref(g), vp(self._scratch.data_ptr()),
                                         vp(torch.cuda.current_stream(self.device).cuda_stream)),
                   "lsr_deform_backward")
        return (dm,) + ups[1:]

    def apply(self, means3D, scales, rotations, opacity, shs, lang, time):
        """forward() inside autograd: the input gradients flow back through lsr_deform_backward and
        the parameter gradients accumulate into self.grads."""
        outs = _DeformFunction.apply(self, time, means3D, scales, rotations, opacity, shs)
        return tuple(outs) + (lang, None)


class _DeformFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, field, time, means3D, scales, rotations, opacity, shs):
        ctx.field, ctx.time = field, time
        ctx.save_for_backward(means3D)
        return field.forward(means3D, scales, rotations, opacity, shs, None, time)[:5]

    @staticmethod
    def backward(ctx, dm, ds, dr, do, dsh):
        (means3D,) = ctx.saved_tensors
        P = means3D.shape[0]
        z = lambda g, n: g if g is not None else torch.zeros(P, n, device=means3D.device)   # noqa: E731
        grads = ctx.field.backward(means3D, ctx.time, z(dm, 3), z(ds, 3), z(dr, 4), z(do, 1), z(dsh, 48))
        return (None, None) + tuple(grads)
