"""The 4D deformation field on MI355X: HexPlane sampling + MLP heads, fused in HIP kernels
(csrc/deform.hip, C-ABI include/lsr_deform.h).  SURVEY.md 8(a) rows a2-a3, 8(f) row 1.

Mirrors the reference's `deform_network.forward_dynamic` (scene/deformation.py:232-248) with every
switch its configs and scripts use: per Gaussian, HexPlane features at (xyz, t) -> feature_out
(max(defor_depth, 1) Linear layers) -> the residual heads that are on (position, scales,
rotations -- added, or multiplied as quaternions with apply_rotation -- opacity, SH), and the
language feature: passed through (no_dlang), deformed by lang_deform over [lang ++ poc_fre(t)]
with the residual (or without: env no_resnet) and re-normalised, or combined from discrete centres
with the discrete_coff_generator head (env use_discrete_lang_f).  Parameters keep the reference's
names; `from_reference` takes `deform_network.state_dict()` plus the ModelHiddenParams and env the
reference was built with, and refuses any key that configuration does not explain.

Forward (the render path) and backward (lsr_deform_backward: input gradients, and the gradients
of every plane and Linear parameter, accumulated into `grads`); `apply` runs the forward inside
autograd.  There is no CPU fallback.
"""
import ctypes
import os
import re
from typing import Dict, Mapping, Optional, Sequence

import torch

from diff_gaussian_rasterization import _lib

HEADS = ("pos_deform", "scales_deform", "rotations_deform", "opacity_deform", "shs_deform")
HEAD_OUT = (3, 3, 4, 1, 48)
COFF = "discrete_coff_generator"
LANG_PASS, LANG_RESIDUAL, LANG_NORESNET, LANG_DISCRETE = 0, 1, 2, 3   # include/lsr_deform.h
MAX_DEPTH = 4
# modules the reference always builds (scene/deformation.py:45-69, :208-215) whether or not the
# configuration computes them
_ALWAYS_BUILT = re.compile(r"^(timenet\.|time_poc$|pos_poc$|rotation_scaling_poc$|opacity_poc$|"
                           r"(pos|scales|rotations|opacity|shs)_deform\.[13]\.|lang_deform\.[135]\.|"
                           r"discrete_coff_generator\.[13]\.)")


class DeformationField:
    """params: name -> tensor, names as in the reference `Deformation` module (grid.grids.{s}.{ci},
    grid.aabb, feature_out.{2k}.*, {head}.1.* / .3.*, discrete_coff_generator.*, lang_deform.*) --
    exactly the ones the configuration computes (anything else raises).
    resolution / multires: the kplanes_config resolution [x, y, z, t] and the multires list;
    depth: defor_depth; no_dx .. no_dshs, apply_rotation: ModelHiddenParams; lang_mode: LANG_*
    (no_dlang / use_discrete_lang_f / no_resnet), lang_dim: language_feature_hiddendim, centers:
    centers_num (discrete), time_pe: timebase_pe."""

    def __init__(self, params: Dict[str, torch.Tensor], resolution: Sequence[int], multires: Sequence[int],
                 device=None, depth: int = 0, no_dx: bool = False, no_ds: bool = False, no_dr: bool = False,
                 no_do: bool = False, no_dshs: bool = False, apply_rotation: bool = False, lang_mode: int = LANG_PASS,
                 lang_dim: int = 3, centers: int = 0, time_pe: int = 4):
        device = device or params["feature_out.0.weight"].device
        if torch.device(device).type != "cuda":
            raise RuntimeError("the deformation field runs on the GPU only (no CPU fallback)")
        self.device = torch.device(device)
        self.resolution, self.multires = list(resolution), list(multires)
        self.depth, self.apply_rotation, self.lang_mode = int(depth), bool(apply_rotation), int(lang_mode)
        self.lang_dim, self.centers, self.time_pe = int(lang_dim), int(centers), int(time_pe)
        self.head_on = tuple(not f for f in (no_dx, no_ds, no_dr, no_do, no_dshs))
        self.discrete = self.lang_mode == LANG_DISCRETE
        if self.discrete and self.centers < 1:
            raise ValueError("the discrete language mode needs centers >= 1")
        if not 0 <= self.depth <= MAX_DEPTH:
            raise ValueError(f"defor_depth {depth}: supported 0..{MAX_DEPTH}")
        want = self.param_names()
        extra, missing = sorted(set(params) - want), sorted(want - set(params))
        if extra or missing:
            raise ValueError(f"deformation parameters do not match the configuration: unexpected {extra}, "
                             f"missing {missing}")
        self.p = {k: v.detach().to(self.device, torch.float32).contiguous() for k, v in params.items()}
        self._check_shapes()
        self.net = self._net(self.lang_mode)
        L = _lib.load()
        nbytes = int(L.lsr_deform_workspace_bytes(ctypes.byref(self.net)))
        if nbytes < 0:
            _lib.check(1, "lsr_deform_workspace_bytes")
        self.workspace = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self.prepare()

    # ---- configuration --------------------------------------------------------------------------
    @property
    def n_layers(self) -> int:
        return max(self.depth, 1)

    def heads_computed(self):
        names = [h for h, on in zip(HEADS, self.head_on) if on]
        return names + ([COFF] if self.discrete else [])

    @property
    def lang_in(self) -> int:
        """Language channels of the input (the centres in discrete mode)."""
        return self.lang_dim * self.centers if self.discrete else self.lang_dim

    def param_names(self):
        n = {"grid.aabb"} | {f"grid.grids.{s}.{ci}" for s in range(len(self.multires)) for ci in range(6)}
        for k in range(self.n_layers):
            n |= {f"feature_out.{2 * k}.weight", f"feature_out.{2 * k}.bias"}
        for h in self.heads_computed():
            n |= {f"{h}.{i}.{w}" for i in (1, 3) for w in ("weight", "bias")}
        if self.lang_mode in (LANG_RESIDUAL, LANG_NORESNET):
            n |= {f"lang_deform.{i}.{w}" for i in (1, 3, 5) for w in ("weight", "bias")}
        return n

    def _check_shapes(self):
        S, W = len(self.multires), 128
        exp = {}
        for s, m in enumerate(self.multires):
            reso = [r * m for r in self.resolution[:3]] + [self.resolution[3]]
            for ci, (c0, c1) in enumerate([(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]):
                exp[f"grid.grids.{s}.{ci}"] = (1, 16, reso[c1], reso[c0])
        exp["grid.aabb"] = (2, 3)
        for k in range(self.n_layers):
            exp[f"feature_out.{2 * k}.weight"] = (W, 16 * S if k == 0 else W)
            exp[f"feature_out.{2 * k}.bias"] = (W,)
        outs = dict(zip(HEADS, HEAD_OUT), **{COFF: self.centers})
        for h in self.heads_computed():
            exp.update({f"{h}.1.weight": (W, W), f"{h}.1.bias": (W,), f"{h}.3.weight": (outs[h], W),
                        f"{h}.3.bias": (outs[h],)})
        if self.lang_mode in (LANG_RESIDUAL, LANG_NORESNET):
            kin = 2 * self.time_pe + 1 + self.lang_dim
            exp.update({"lang_deform.1.weight": (W, kin), "lang_deform.1.bias": (W,), "lang_deform.3.weight": (W, W),
                        "lang_deform.3.bias": (W,), "lang_deform.5.weight": (self.lang_dim, W),
                        "lang_deform.5.bias": (self.lang_dim,)})
        for k, shape in exp.items():
            if tuple(self.p[k].shape) != shape:
                raise ValueError(f"{k}: shape {tuple(self.p[k].shape)}, the configuration needs {shape}")

    def _net(self, lang_mode, coff_head: Optional[bool] = None):
        coff_head = self.discrete if coff_head is None else coff_head
        n = _lib.DeformNet()
        n.n_scales, n.channels, n.width = len(self.multires), 16, 128
        for i in range(4):
            n.res[i] = int(self.resolution[i])
            n.multires[i] = int(self.multires[i]) if i < len(self.multires) else 1
        n.depth = self.depth
        n.heads = sum(1 << h for h, on in enumerate(self.head_on) if on) | (32 if coff_head else 0)
        n.apply_rotation = int(self.apply_rotation)
        n.lang_mode, n.lang_dim, n.centers, n.time_pe = lang_mode, self.lang_dim, self.centers, self.time_pe
        n.aabb = self.p["grid.aabb"].data_ptr()
        for s in range(len(self.multires)):
            for ci in range(6):
                n.planes[s][ci] = self.p[f"grid.grids.{s}.{ci}"].data_ptr()
        for k in range(self.n_layers):
            n.w_feat[k], n.b_feat[k] = self.p[f"feature_out.{2 * k}.weight"].data_ptr(), \
                self.p[f"feature_out.{2 * k}.bias"].data_ptr()
        for h, name in enumerate(HEADS + (COFF,)):
            if name in self.heads_computed():
                n.w1[h], n.b1[h] = self.p[name + ".1.weight"].data_ptr(), self.p[name + ".1.bias"].data_ptr()
                n.w2[h], n.b2[h] = self.p[name + ".3.weight"].data_ptr(), self.p[name + ".3.bias"].data_ptr()
        if self.lang_mode in (LANG_RESIDUAL, LANG_NORESNET):
            for i, k in enumerate((1, 3, 5)):
                n.w_lang[i], n.b_lang[i] = self.p[f"lang_deform.{k}.weight"].data_ptr(), \
                    self.p[f"lang_deform.{k}.bias"].data_ptr()
        return n

    def _call_net(self, no_dlang: Optional[bool]):
        """The net of one call: the reference's render() forces no_dlang = 1 in the 'base' stages
        (gaussian_renderer/__init__.py:121-124).  The reference's discrete branch
        (scene/deformation.py:156) runs regardless, on the zeros [P, language_feature_hiddendim] that
        render() passes there: it slices and views them as centres and normalises zero vectors
        (0/0, NaN language) and computes a coff that train.py collects but never uses (train.py:240-247).
        Here a discrete field in a 'base' call runs without its coff head and passes the language
        through, as the PASS mode does: coff is None and the (unused) language is the input."""
        if no_dlang and self.lang_mode in (LANG_RESIDUAL, LANG_NORESNET):
            return self._net(LANG_PASS)
        if no_dlang and self.discrete:
            return self._net(LANG_PASS, coff_head=False)
        return self.net

    # ---- construction from the reference ----------------------------------------------------------
    @staticmethod
    def init_params(resolution: Sequence[int], multires: Sequence[int], aabb, channels: int = 16, width: int = 128,
                    seed: int = 0, depth: int = 0, heads=HEADS, lang_mode: int = LANG_PASS, lang_dim: int = 3,
                    centers: int = 0, time_pe: int = 4) -> Dict[str, torch.Tensor]:
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
        for k in range(max(depth, 1)):
            linear(f"feature_out.{2 * k}", width, channels * len(multires) if k == 0 else width)
        for name, n in zip(HEADS, HEAD_OUT):
            if name in heads:
                linear(name + ".1", width, width)
                linear(name + ".3", n, width)
        if lang_mode == LANG_DISCRETE:
            linear(COFF + ".1", width, width)
            linear(COFF + ".3", centers, width)
        if lang_mode in (LANG_RESIDUAL, LANG_NORESNET):
            linear("lang_deform.1", width, 2 * time_pe + 1 + lang_dim)
            linear("lang_deform.3", width, width)
            linear("lang_deform.5", lang_dim, width)
        return p

    @staticmethod
    def config_from_reference(state_dict: Mapping[str, torch.Tensor], hidden, env: Optional[Mapping[str, str]] = None,
                              prefix="deformation_net."):
        """(params, config kwargs) of a trained `deform_network` (`deformation.pth`,
        scene/gaussian_model.py:352-364): its state dict, the ModelHiddenParams it was built with (a
        dict or an object with the attributes: kplanes_config, multires, defor_depth, no_dx ..
        no_dshs, no_dlang, apply_rotation, timebase_pe, net_width, static_mlp, empty_voxel,
        no_grid, grid_pe; the reference's defaults where absent, arguments/__init__.py:84-113) and
        the environment (language_feature_hiddendim, use_discrete_lang_f, centers_num, no_resnet,
        use_tribute_dlang; default os.environ).  Modules the reference always builds but this
        configuration does not compute are skipped; any other key raises.  CPU only (no device)."""
        env = os.environ if env is None else env
        h = hidden if isinstance(hidden, Mapping) else vars(hidden)
        get = lambda k, d=None: h.get(k, d)   # noqa: E731
        for flag in ("static_mlp", "empty_voxel", "no_grid"):
            if get(flag, False):
                raise ValueError(f"{flag} is not supported (off in every reference config)")
        if get("grid_pe", 0):
            raise ValueError("grid_pe > 0 is not supported (0 in every reference config)")
        if env.get("use_tribute_dlang", "f") == "t":
            raise ValueError("use_tribute_dlang is not supported (the reference's lang_deform input width "
                             "does not admit it)")
        kp = get("kplanes_config")
        if get("net_width", 64) != 128 or kp.get("output_coordinate_dim", 32) != 16:
            raise ValueError("supported: net_width 128, output_coordinate_dim 16 (every HyperNeRF / Neu3D config)")
        lang_dim = int(env.get("language_feature_hiddendim", 3))
        if env.get("use_discrete_lang_f", "f") == "t":
            mode = LANG_DISCRETE
        elif get("no_dlang", 1):
            mode = LANG_PASS
        else:
            mode = LANG_NORESNET if env.get("no_resnet", "f") == "t" else LANG_RESIDUAL
        cfg = dict(resolution=list(kp["resolution"]), multires=list(get("multires", [1, 2, 4, 8])),
                   depth=int(get("defor_depth", 1)), no_dx=bool(get("no_dx", False)), no_ds=bool(get("no_ds", False)),
                   no_dr=bool(get("no_dr", False)), no_do=bool(get("no_do", True)), no_dshs=bool(get("no_dshs", True)),
                   apply_rotation=bool(get("apply_rotation", False)), lang_mode=mode, lang_dim=lang_dim,
                   centers=int(env.get("centers_num", 3)) if mode == LANG_DISCRETE else 0,
                   time_pe=int(get("timebase_pe", 4)))
        probe = DeformationField.__new__(DeformationField)   # the parameter set the configuration computes
        probe.multires, probe.depth, probe.lang_mode = cfg["multires"], cfg["depth"], mode
        probe.head_on = tuple(not cfg[f] for f in ("no_dx", "no_ds", "no_dr", "no_do", "no_dshs"))
        probe.discrete = mode == LANG_DISCRETE
        want = probe.param_names()
        params = {}
        for k, v in state_dict.items():
            if not k.startswith(prefix):
                if _ALWAYS_BUILT.match(k):   # deform_network-level buffers and the time net
                    continue
                raise ValueError(f"unexpected key {k!r} outside {prefix!r}")
            name = k[len(prefix):]
            if name in want:
                params[name] = v
            elif not _ALWAYS_BUILT.match(name):
                raise ValueError(f"state-dict key {k!r} is not computed by this configuration "
                                 f"(defor_depth {cfg['depth']}, multires {cfg['multires']})")
        return params, cfg

    @classmethod
    def from_reference(cls, state_dict: Mapping[str, torch.Tensor], hidden, env: Optional[Mapping[str, str]] = None,
                       device="cuda", prefix="deformation_net."):
        """The field of a trained `deform_network` (config_from_reference), on `device`."""
        params, cfg = cls.config_from_reference(state_dict, hidden, env, prefix)
        return cls(params, device=device, **cfg)

    def state_dict(self, prefix="deformation_net.") -> Dict[str, torch.Tensor]:
        """The parameters under the reference's names (deform_network.state_dict() keys; the
        modules this configuration does not compute are absent -- the reference loads with
        strict=False, scene/gaussian_model.py:355)."""
        return {prefix + k: v.detach().clone() for k, v in self.p.items()}

    def hidden_params(self) -> dict:
        """The ModelHiddenParams entries this field was built from (config_from_reference's input)."""
        return dict(kplanes_config={"resolution": list(self.resolution), "output_coordinate_dim": 16,
                                    "grid_dimensions": 2, "input_coordinate_dim": 4},
                    multires=list(self.multires), defor_depth=self.depth, net_width=128,
                    no_dx=not self.head_on[0], no_ds=not self.head_on[1], no_dr=not self.head_on[2],
                    no_do=not self.head_on[3], no_dshs=not self.head_on[4], apply_rotation=self.apply_rotation,
                    no_dlang=int(self.lang_mode == LANG_PASS), timebase_pe=self.time_pe)

    def env_params(self) -> Dict[str, str]:
        """The environment switches that select this field's language mode (config_from_reference's
        `env`): language_feature_hiddendim, use_discrete_lang_f, centers_num, no_resnet."""
        env = {"language_feature_hiddendim": str(self.lang_dim),
               "use_discrete_lang_f": "t" if self.lang_mode == LANG_DISCRETE else "f",
               "no_resnet": "t" if self.lang_mode == LANG_NORESNET else "f"}
        if self.lang_mode == LANG_DISCRETE:
            env["centers_num"] = str(self.centers)
        return env

    @classmethod
    def from_reference_state_dict(cls, state_dict, resolution, multires, prefix="deformation_net.", device="cuda"):
        """The Neu3D structure (arguments/neu3d/default.py): defor_depth 0, every head, language
        pass-through."""
        hidden = dict(kplanes_config={"resolution": list(resolution), "output_coordinate_dim": 16},
                      multires=list(multires), defor_depth=0, no_do=False, no_dshs=False, no_dlang=1, net_width=128)
        return cls.from_reference(state_dict, hidden, env={}, device=device, prefix=prefix)

    def prepare(self):
        """Repack planes and weights (call after every parameter update)."""
        L = _lib.load()
        _lib.check(L.lsr_deform_prepare(ctypes.byref(self.net), ctypes.c_void_p(self.workspace.data_ptr()),
                                        ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "lsr_deform_prepare")

    # ---- forward -----------------------------------------------------------------------------------
    def _time(self, time, P):
        if torch.is_tensor(time) and time.numel() == P:
            return time.detach().to(self.device, torch.float32).reshape(P).contiguous()
        return torch.full((P,), float(time), device=self.device)

    @torch.no_grad()
    def forward(self, means3D, scales, rotations, opacity, shs, lang, time, no_dlang: Optional[bool] = None):
        """Returns (means3D, scales, rotations, opacity, shs, lang, coff) like
        deform_network.forward (raw values, before activation; an output whose head is off is its
        input, coff is None unless the language is discrete).  no_dlang: the per-call override
        render() applies in the 'base' stages."""
        L = _lib.load()
        P = means3D.shape[0]
        net = self._call_net(no_dlang)
        f = lambda t, shape: t.detach().to(self.device, torch.float32).reshape(shape).contiguous()   # noqa: E731
        ins = [f(means3D, (P, 3)), f(scales, (P, 3)), f(rotations, (P, 4)), f(opacity, (P, 1)), f(shs, (P, 16, 3))]
        t = self._time(time, P)
        outs = [torch.empty_like(x) if on else None for x, on in zip(ins, self.head_on)]
        if self.apply_rotation:
            outs[2] = torch.empty_like(ins[2])
        lang_in = f(lang, (P, self.lang_in)) if lang is not None and net.lang_mode != LANG_PASS else None
        out_lang = torch.empty(P, self.lang_dim, device=self.device) if net.lang_mode != LANG_PASS else None
        out_coff = torch.empty(P, self.centers, device=self.device) if net.lang_mode == LANG_DISCRETE else None
        if net.lang_mode != LANG_PASS and lang_in is None:
            raise ValueError("this field deforms the language feature: lang is required")
        vp = lambda x: ctypes.c_void_p(x.data_ptr() if x is not None else 0)   # noqa: E731
        _lib.check(L.lsr_deform_forward(ctypes.byref(net), vp(self.workspace), P, *[vp(x) for x in ins], vp(lang_in),
                                        vp(t), *[vp(x) for x in outs], vp(out_lang), vp(out_coff),
                                        ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "lsr_deform_forward")
        res = [o if o is not None else x for o, x in zip(outs, ins)]
        if net.lang_mode == LANG_PASS:
            out_lang = lang[:, :self.lang_dim] if lang is not None else None
        return tuple(res) + (out_lang, out_coff)

    __call__ = forward

    # ---- backward (lsr_deform_backward) -------------------------------------------------------
    #: whether backward() also produces the HexPlane box's gradient grads["grid.aabb"].  The reference
    #: trains the box whenever the whole field has requires_grad -- the base stages and joint_train
    #: (scene/gaussian_model.py:258,291: requires_grad_(True) reaches the aabb Parameter that set_aabb
    #: made with requires_grad=False, and get_grid_parameters gives "grid.aabb" to Adam); TrainStep
    #: turns this on.  Off, the box is a constant (what a freshly built deform_network has).
    train_aabb = False

    def zero_grad(self):
        """Parameter gradients (torch layouts, names as the parameters) set to zero.  They are views
        of one flat buffer (256-byte aligned), zeroed with one fill instead of ~40 (one per tensor, a
        measurable share of a configs[4] iteration's launches); a caller keeping gradients across
        zero_grad() clones them, as with torch's .grad under zero_grad(set_to_none=False)."""
        keys = [k for k in self.p if k != "grid.aabb" or self.train_aabb]
        sig = tuple((k, tuple(self.p[k].shape)) for k in keys)
        if getattr(self, "_grad_sig", None) != sig:
            offs, o = {}, 0
            for k in keys:
                offs[k] = o
                o += (self.p[k].numel() + 63) // 64 * 64
            self._grad_flat = torch.empty(max(o, 1), device=self.device)
            self._grad_views = {k: self._grad_flat[offs[k]:offs[k] + self.p[k].numel()].view(self.p[k].shape)
                                for k in keys}
            self._grad_sig = sig
        self._grad_flat.zero_()
        self.grads = dict(self._grad_views)

    def backward(self, means3D, time, d_means3D, d_scales, d_rotations, d_opacity, d_shs, rotations=None, lang=None,
                 d_lang=None, d_coff=None, no_dlang: Optional[bool] = None):
        """Gradients of forward() given the gradients of its outputs: returns the input gradients
        (means3D, scales, rotations, opacity, shs, lang) and ADDS the parameter gradients to
        self.grads (as torch accumulates .grad).  rotations / lang: the forward's inputs (needed with
        apply_rotation / a deformed language).  Call prepare() after parameter updates first."""
        L = _lib.load()
        if not hasattr(self, "grads"):
            self.zero_grad()
        net = self._call_net(no_dlang)
        P = means3D.shape[0]
        f = lambda t, shape: None if t is None else t.detach().to(self.device, torch.float32).reshape(shape).contiguous()   # noqa: E731,E501
        m = f(means3D, (P, 3))
        t = self._time(time, P)
        ups = [f(d_means3D, (P, 3)), f(d_scales, (P, 3)), f(d_rotations, (P, 4)), f(d_opacity, (P, 1)),
               f(d_shs, (P, 16, 3))]
        for i, on in enumerate(self.head_on):
            if ups[i] is None and (on or i == 0):
                ups[i] = torch.zeros((P,) + ((16, 3) if i == 4 else (HEAD_OUT[i],)), device=self.device)
        dl_up = f(d_lang, (P, self.lang_dim))
        rot = f(rotations, (P, 4)) if self.apply_rotation else None
        lang_in = f(lang, (P, self.lang_in)) if net.lang_mode != LANG_PASS else None
        if self.apply_rotation and rot is None:
            raise ValueError("apply_rotation: the forward's rotations are required")
        if net.lang_mode != LANG_PASS and lang_in is None:
            raise ValueError("a deformed language feature needs the forward's lang")
        dm = torch.empty_like(m)
        drot = torch.empty(P, 4, device=self.device) if self.apply_rotation else None
        dlang = torch.empty(P, self.lang_in, device=self.device) if net.lang_mode != LANG_PASS else None
        g = _lib.DeformGrads()
        for s in range(len(self.multires)):
            for ci in range(6):
                g.planes[s][ci] = self.grads[f"grid.grids.{s}.{ci}"].data_ptr()
        for k in range(self.n_layers):
            g.w_feat[k] = self.grads[f"feature_out.{2 * k}.weight"].data_ptr()
            g.b_feat[k] = self.grads[f"feature_out.{2 * k}.bias"].data_ptr()
        for h, name in enumerate(HEADS + (COFF,)):
            if name in self.heads_computed():
                g.w1[h], g.b1[h] = self.grads[name + ".1.weight"].data_ptr(), self.grads[name + ".1.bias"].data_ptr()
                g.w2[h], g.b2[h] = self.grads[name + ".3.weight"].data_ptr(), self.grads[name + ".3.bias"].data_ptr()
        if self.lang_mode in (LANG_RESIDUAL, LANG_NORESNET):
            for i, k in enumerate((1, 3, 5)):
                g.w_lang[i] = self.grads[f"lang_deform.{k}.weight"].data_ptr()
                g.b_lang[i] = self.grads[f"lang_deform.{k}.bias"].data_ptr()
        if "grid.aabb" in self.grads:
            g.aabb = self.grads["grid.aabb"].data_ptr()
        nbytes = int(L.lsr_deform_backward_scratch_bytes(ctypes.byref(net), P))
        if nbytes < 0:
            _lib.check(1, "lsr_deform_backward_scratch_bytes")
        if getattr(self, "_scratch", None) is None or self._scratch.numel() < nbytes:
            self._scratch = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        vp = lambda x: ctypes.c_void_p(x.data_ptr() if x is not None else 0)   # noqa: E731
        _lib.check(L.lsr_deform_backward(ctypes.byref(net), vp(self.workspace), P, vp(m), vp(rot), vp(lang_in), vp(t),
                                         *[vp(u) for u in ups], vp(dl_up), vp(f(d_coff, (P, self.centers)) if net.lang_mode == LANG_DISCRETE else None), vp(dm),
                                         vp(drot), vp(dlang), ctypes.byref(g), vp(self._scratch),
                                         ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "lsr_deform_backward")
        # identity residuals (and heads that are off) pass their output gradient to the input
        d_in = [dm, ups[1] if ups[1] is not None else f(d_scales, (P, 3)),
                drot if drot is not None else (ups[2] if ups[2] is not None else f(d_rotations, (P, 4))),
                ups[3] if ups[3] is not None else f(d_opacity, (P, 1)),
                ups[4] if ups[4] is not None else f(d_shs, (P, 16, 3))]
        if net.lang_mode == LANG_PASS:
            if dl_up is None:
                dlang = None
            else:   # the input's width: lang_in, or lang_dim when a 'base' call passes zeros [P, lang_dim]
                width = lang.reshape(P, -1).shape[1] if lang is not None else self.lang_in
                dlang = torch.zeros(P, width, device=self.device)
                dlang[:, :self.lang_dim] = dl_up
        return tuple(d_in) + (dlang,)

    def apply(self, means3D, scales, rotations, opacity, shs, lang, time, no_dlang: Optional[bool] = None):
        """forward() inside autograd: the input gradients flow back through lsr_deform_backward and
        the parameter gradients accumulate into self.grads."""
        if lang is None:
            lang = torch.zeros(means3D.shape[0], self.lang_in, device=self.device)
        outs = _DeformFunction.apply(self, time, no_dlang, means3D, scales, rotations, opacity, shs, lang)
        coff = outs[6] if (self.discrete and outs[6].numel() > 0) else None
        return tuple(outs[:6]) + (coff,)


class _DeformFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, field, time, no_dlang, means3D, scales, rotations, opacity, shs, lang):
        ctx.field, ctx.time, ctx.no_dlang = field, time, no_dlang
        ctx.save_for_backward(means3D, rotations, lang)
        outs = field.forward(means3D, scales, rotations, opacity, shs, lang, time, no_dlang=no_dlang)
        ins = (means3D, scales, rotations, opacity, shs, lang)
        # outputs never alias inputs (a head that is off, the passed-through language)
        res = tuple(o.clone() if o.data_ptr() == x.data_ptr() else o for o, x in zip(outs[:6], ins))
        coff = outs[6] if outs[6] is not None else torch.zeros(0, device=means3D.device)
        return res + (coff,)

    @staticmethod
    def backward(ctx, dm, ds, dr, do, dsh, dl, dc):
        means3D, rotations, lang = ctx.saved_tensors
        f = ctx.field
        if torch.are_deterministic_algorithms_enabled():
            # the plane gradients are float-atomic scatters: no fixed-order variant
            if not torch.is_deterministic_algorithms_warn_only_enabled():
                raise RuntimeError("lsr_deform_backward does not have a deterministic implementation "
                                   "(torch.use_deterministic_algorithms(True, warn_only=True) to run it anyway)")
            import warnings
            warnings.warn("lsr_deform_backward does not have a deterministic implementation")
        grads = f.backward(means3D, ctx.time, dm, ds, dr, do, dsh, rotations=rotations, lang=lang, d_lang=dl,
                           d_coff=dc if (f.discrete and dc is not None and dc.numel() > 0) else None,
                           no_dlang=ctx.no_dlang)
        return (None, None, None) + tuple(grads)
