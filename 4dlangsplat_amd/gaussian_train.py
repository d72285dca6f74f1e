"""Training-step glue on the MI355X: the optimizer and densification state of
the reference's GaussianModel, with every per-Gaussian pass in liblsr.so (include/lsr_train.h).

Mirrors, with the reference's names, argument meaning and order of effects:
  training_setup's parameter groups and Adam(lr=0.0, eps=1e-15)   scene/gaussian_model.py:220-313
  update_learning_rate (xyz exponential schedule)                 scene/gaussian_model.py:315-329,
                                                                  utils/general_utils.py:35-66
  optimizer.step() / zero_grad(set_to_none=True)                  train.py:420-421
  max_radii2D update + add_densification_stats                    train.py:388-389, gaussian_model.py:746-748
  densify (clone, then split into N = 2, the split originals pruned)
                                                                  gaussian_model.py:726-731,575-627,541-573
  prune                                                           gaussian_model.py:714-723,487-508
  reset_opacity                                                   gaussian_model.py:391-394

Each of step / densification stats / reset_opacity is one kernel launch over all tensors; densify
and prune are a row-map kernel (device scan), one host read of the row counts (the reference's
boolean indexing synchronises the same way), one multi-tensor gather launch for parameters, both
Adam moments, the statistics and the deformation table, and for the split one launch for the new
positions and scales.  There is no CPU fallback: liblsr.so and a GPU are required.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, Optional

import numpy as np
import torch

from diff_gaussian_rasterization import _lib

# parameter groups of gaussian_model.py:273-288 and the GaussianScene attribute holding each
GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation", "language_feature")
SCENE_ATTR = {"xyz": "xyz", "f_dc": "features_dc", "f_rest": "features_rest", "opacity": "opacity",
              "scaling": "scaling", "rotation": "rotation", "language_feature": "language_feature"}


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:35-66: log-linear decay from lr_init (step 0) to lr_final (max_steps),
    optionally eased in over lr_delay_steps; 0 for step < 0 or an all-zero schedule."""
    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        return delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
    return helper


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class GaussianTrainer:
    """Optimizer + densification state over raw Gaussian tensors (a GaussianScene's, or a dict).

    params[name] are leaf float32 CUDA tensors (requires_grad) that autograd fills; lrs gives each
    trainable group's learning rate (groups absent from lrs, or whose .grad is None, are not
    stepped, as torch skips them).  exp_avg / exp_avg_sq are allocated at setup (zeros; the same
    arithmetic as torch's lazily created state)."""

    def __init__(self, params: Dict[str, torch.Tensor], lrs: Dict[str, float], percent_dense: float = 0.01,
                 betas=(0.9, 0.999), eps: float = 1e-15, deformation_table: Optional[torch.Tensor] = None):
        if not params:
            raise ValueError("no parameters")
        self._L = _lib.load()
        self.params: Dict[str, torch.Tensor] = {}
        dev = None
        for n in GROUPS:
            if n not in params or params[n] is None:
                continue
            t = params[n]
            if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
                raise ValueError(f"{n}: contiguous float32 CUDA tensor required")
            dev = t.device if dev is None else dev
            self.params[n] = t.detach().requires_grad_(True)
        self.device = dev
        P = self.P
        for n, t in self.params.items():
            if t.shape[0] != P:
                raise ValueError(f"{n}: {t.shape[0]} rows, expected {P}")
        self.lrs = dict(lrs)
        self.betas, self.eps = betas, eps
        self.percent_dense = percent_dense
        self.exp_avg = {n: torch.zeros_like(t) for n, t in self.params.items()}
        self.exp_avg_sq = {n: torch.zeros_like(t) for n, t in self.params.items()}
        self.steps = {n: 0 for n in self.params}
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)
        self._deformation_accum = torch.zeros((P, 3), device=dev)
        self._deformation_table = (deformation_table.to(dev, torch.bool).contiguous() if deformation_table is not None
                                   else torch.ones(P, dtype=torch.bool, device=dev))
        self.xyz_scheduler_args = None

    @classmethod
    def from_scene(cls, scene, lrs, **kw):
        return cls({n: getattr(scene, SCENE_ATTR[n]) for n in GROUPS}, lrs, **kw)

    @property
    def P(self) -> int:
        return next(iter(self.params.values())).shape[0]

    def __getitem__(self, name):
        return self.params[name]

    # ---- learning rate (gaussian_model.py:302-329) -------------------------------------------
    def set_xyz_schedule(self, lr_init, lr_final, lr_delay_mult=0.01, max_steps=30000):
        self.xyz_scheduler_args = get_expon_lr_func(lr_init=lr_init, lr_final=lr_final, lr_delay_mult=lr_delay_mult,
                                                    max_steps=max_steps)

    def update_learning_rate(self, iteration):
        if self.xyz_scheduler_args is not None and "xyz" in self.lrs:
            self.lrs["xyz"] = self.xyz_scheduler_args(iteration)
        return self.lrs.get("xyz")

    # ---- optimizer (train.py:420-421) -------------------------------------------------------
    def step(self):
        """One torch.optim.Adam step over every group with a gradient: one kernel launch."""
        groups = []
        for n, p in self.params.items():
            if n not in self.lrs or p.grad is None:
                continue
            g = p.grad
            if not g.is_contiguous() or g.dtype != torch.float32 or g.shape != p.shape:
                raise ValueError(f"{n}: gradient must be a contiguous float32 tensor of the parameter's shape")
            self.steps[n] += 1
            ag = _lib.AdamGroup()
            ag.param, ag.grad = p.data_ptr(), g.data_ptr()
            ag.exp_avg, ag.exp_avg_sq = self.exp_avg[n].data_ptr(), self.exp_avg_sq[n].data_ptr()
            ag.n, ag.lr, ag.step = p.numel(), float(self.lrs[n]), self.steps[n]
            groups.append(ag)
        if not groups:
            return
        arr = (_lib.AdamGroup * len(groups))(*groups)
        _lib.check(self._L.lsr_adam_step(arr, len(groups), self.betas[0], self.betas[1], self.eps,
                                         _stream(self.device)), "lsr_adam_step")

    def zero_grad(self, set_to_none=True):
        for p in self.params.values():
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    # ---- densification statistics (train.py:388-389, gaussian_model.py:746-748) ---------------
    def add_densification_stats(self, viewspace_point_grad: torch.Tensor, radii: torch.Tensor):
        """radii: int32 [P], the max over the iteration's views (train.py:266); visibility = radii > 0.
        Updates max_radii2D, xyz_gradient_accum (|grad[:, :2]|) and denom for the visible rows."""
        P = self.P
        g = viewspace_point_grad.detach()
        if g.dim() != 2 or g.shape[0] != P or g.shape[1] < 2 or g.stride(1) != 1 or g.dtype != torch.float32:
            raise ValueError("viewspace_point_grad must be float32 [P, >=2] with unit column stride")
        r = radii.to(torch.int32).contiguous()
        if r.shape != (P,):
            raise ValueError("radii must be [P]")
        _lib.check(self._L.lsr_densify_stats(P, _ptr(r), _ptr(g), g.stride(0), _ptr(self.max_radii2D),
                                             _ptr(self.xyz_gradient_accum), _ptr(self.denom), _stream(self.device)),
                   "lsr_densify_stats")

    # ---- row surgery -------------------------------------------------------------------------
    def _workspace(self, P):
        return torch.empty(int(self._L.lsr_train_workspace_bytes(P)), dtype=torch.uint8, device=self.device)

    def _gather(self, index: torch.Tensor, n_rows: int, zero_from: int, stats_keep: bool):
        """Every row tensor through `index`: parameters (copied), Adam moments (rows >= zero_from
        zeroed), statistics (copied if stats_keep, else zeroed), the deformation table (copied)."""
        jobs, new = [], {}

        def job(key, src, zf):
            shape = (n_rows,) + tuple(src.shape[1:])
            dst = torch.empty(shape, dtype=src.dtype, device=self.device)
            rt = _lib.RowTensor()
            rt.src, rt.dst = src.data_ptr(), dst.data_ptr()
            rt.row_bytes = int(np.prod(shape[1:], dtype=np.int64)) * src.element_size()
            rt.zero_from = zf
            jobs.append(rt)
            new[key] = dst

        for n, p in self.params.items():
            job(("p", n), p.detach(), n_rows)
            job(("m", n), self.exp_avg[n], zero_from)
            job(("v", n), self.exp_avg_sq[n], zero_from)
        stat_zf = n_rows if stats_keep else 0
        job(("s", "xyz_gradient_accum"), self.xyz_gradient_accum, stat_zf)
        job(("s", "denom"), self.denom, stat_zf)
        job(("s", "max_radii2D"), self.max_radii2D, stat_zf)
        job(("s", "_deformation_accum"), self._deformation_accum, stat_zf)
        job(("s", "_deformation_table"), self._deformation_table, n_rows)
        if len(jobs) > _lib.GATHER_MAX_TENSORS:
            raise ValueError("too many row tensors for one gather launch")
        arr = (_lib.RowTensor * len(jobs))(*jobs)
        _lib.check(self._L.lsr_gather_rows(len(jobs), arr, _ptr(index), n_rows, _stream(self.device)),
                   "lsr_gather_rows")
        return new

    def _install(self, new):
        for (kind, n), t in new.items():
            if kind == "p":
                self.params[n] = t.requires_grad_(True)
            elif kind == "m":
                self.exp_avg[n] = t
            elif kind == "v":
                self.exp_avg_sq[n] = t
            else:
                setattr(self, n, t)

    @torch.no_grad()
    def densify(self, max_grad, min_opacity, extent, max_screen_size=None, N: int = 2,
                samples: Optional[torch.Tensor] = None):
        """gaussian_model.py:726-731 (min_opacity / max_screen_size are unused there too).
        samples: optional standard-normal [N * n_split, 3] draws for the split (default torch.randn
        on the device).  Returns (n_clone, n_split)."""
        P = self.P
        for n in ("xyz", "scaling", "rotation"):
            if n not in self.params:
                raise ValueError(f"densify needs the {n} group")
        index = torch.empty((N + 1) * max(P, 1), dtype=torch.int32, device=self.device)
        counts = torch.zeros(3, dtype=torch.int64, device=self.device)
        ws = self._workspace(P)
        _lib.check(self._L.lsr_densify_plan(P, _ptr(self.xyz_gradient_accum), _ptr(self.denom),
                                            _ptr(self.params["scaling"]), float(max_grad), float(self.percent_dense),
                                            float(extent), N, _ptr(index), _ptr(counts), _ptr(ws),
                                            _stream(self.device)), "lsr_densify_plan")
        kept, n_clone, n_split = (int(x) for x in counts.cpu())
        n_rows = kept + n_clone + N * n_split
        old = {n: self.params[n].detach() for n in ("xyz", "scaling", "rotation")}
        new = self._gather(index, n_rows, zero_from=kept, stats_keep=False)
        if n_split:
            if samples is None:
                samples = torch.randn(N * n_split, 3, device=self.device)
            samples = samples.to(self.device, torch.float32).contiguous()
            if samples.shape != (N * n_split, 3):
                raise ValueError(f"samples must be [{N * n_split}, 3]")
            _lib.check(self._L.lsr_split_fixup(N * n_split, kept + n_clone, N, _ptr(index), _ptr(old["xyz"]),
                                               _ptr(old["scaling"]), _ptr(old["rotation"]), _ptr(samples),
                                               _ptr(new[("p", "xyz")]), _ptr(new[("p", "scaling")]),
                                               _stream(self.device)), "lsr_split_fixup")
        self._install(new)
        return n_clone, n_split

    @torch.no_grad()
    def prune(self, max_grad, min_opacity, extent, max_screen_size):
        """gaussian_model.py:714-723.  Returns the number of rows removed."""
        P = self.P
        index = torch.empty(max(P, 1), dtype=torch.int32, device=self.device)
        counts = torch.zeros(1, dtype=torch.int64, device=self.device)
        ws = self._workspace(P)
        _lib.check(self._L.lsr_prune_plan(P, _ptr(self.params["opacity"]), _ptr(self.max_radii2D),
                                          _ptr(self.params["scaling"]), float(min_opacity),
                                          float(max_screen_size or 0.0), float(extent), _ptr(index), _ptr(counts),
                                          _ptr(ws), _stream(self.device)), "lsr_prune_plan")
        kept = int(counts.cpu()[0])
        self._install(self._gather(index, kept, zero_from=kept, stats_keep=True))
        return P - kept

    @torch.no_grad()
    def reset_opacity(self):
        """gaussian_model.py:391-394: opacity <- inverse_sigmoid(min(sigmoid(opacity), 0.01)), its
        Adam moments zeroed (replace_tensor_to_optimizer, :446-459).  Like the fresh nn.Parameter
        the reference installs there, the group has no gradient afterwards (a following step()
        skips it)."""
        n = "opacity"
        self.params[n].grad = None
        _lib.check(self._L.lsr_reset_opacity(self.P, _ptr(self.params[n]), _ptr(self.exp_avg[n]),
                                             _ptr(self.exp_avg_sq[n]), _stream(self.device)), "lsr_reset_opacity")

    def state_rows(self) -> Iterable[str]:
        return tuple(self.params)

    # ---- checkpoint state (capture / restore, scene/gaussian_model.py:71-154) ------------------
    def adam_entry(self, n: str) -> Optional[dict]:
        """torch.optim.Adam's per-parameter state for group n ({"step", "exp_avg", "exp_avg_sq"}),
        None before its first step (torch creates the state lazily)."""
        if self.steps.get(n, 0) == 0:
            return None
        return {"step": torch.tensor(float(self.steps[n])), "exp_avg": self.exp_avg[n].detach().clone(),
                "exp_avg_sq": self.exp_avg_sq[n].detach().clone()}

    def load_adam_entry(self, n: str, entry: Optional[dict]) -> None:
        p = self.params[n]
        if entry is None:
            self.exp_avg[n], self.exp_avg_sq[n], self.steps[n] = torch.zeros_like(p), torch.zeros_like(p), 0
            return
        for k in ("exp_avg", "exp_avg_sq"):
            if tuple(entry[k].shape) != tuple(p.shape):
                raise ValueError(f"{n}: optimizer {k} of shape {tuple(entry[k].shape)}, parameter {tuple(p.shape)}")
        self.exp_avg[n] = entry["exp_avg"].to(self.device, torch.float32).contiguous().clone()
        self.exp_avg_sq[n] = entry["exp_avg_sq"].to(self.device, torch.float32).contiguous().clone()
        self.steps[n] = int(float(entry["step"]))

    @torch.no_grad()
    def load_rows(self, params: Dict[str, torch.Tensor], max_radii2D: torch.Tensor, xyz_gradient_accum: torch.Tensor,
                  denom: torch.Tensor, deformation_table: Optional[torch.Tensor] = None) -> None:
        """Installs restored per-Gaussian tensors (the row count may differ from the current one):
        parameters, densification statistics, deformation table; moments are reset (load_adam_entry
        sets them).  The statistics the reference does not checkpoint (_deformation_accum) start at
        zero, as its training_setup makes them (gaussian_model.py:224)."""
        P = None
        for n, t in params.items():
            if n not in GROUPS:
                raise ValueError(f"unknown parameter group {n}")
            t = t.detach().to(self.device, torch.float32).contiguous().clone()
            if P is not None and t.shape[0] != P:
                raise ValueError(f"{n}: {t.shape[0]} rows, expected {P}")
            P = t.shape[0]
            self.params[n] = t.requires_grad_(True)
            self.exp_avg[n], self.exp_avg_sq[n], self.steps[n] = torch.zeros_like(t), torch.zeros_like(t), 0
        for n in list(self.params):
            if n not in params:
                raise ValueError(f"the checkpoint has no {n} group")
        dev = self.device
        self.max_radii2D = max_radii2D.detach().to(dev, torch.float32).reshape(P).contiguous().clone()
        self.xyz_gradient_accum = xyz_gradient_accum.detach().to(dev, torch.float32).reshape(P, 1).contiguous().clone()
        self.denom = denom.detach().to(dev, torch.float32).reshape(P, 1).contiguous().clone()
        self._deformation_accum = torch.zeros((P, 3), device=dev)
        self._deformation_table = (deformation_table.detach().to(dev, torch.bool).reshape(P).contiguous().clone()
                                   if deformation_table is not None and deformation_table.numel() == P
                                   else torch.ones(P, dtype=torch.bool, device=dev))


class TensorAdam:
    """torch.optim.Adam over named tensors whose gradients arrive in a separate dict (the
    deformation field's planes and MLP weights, DeformationField.grads; gaussian_model.py:250-253,
    275-276 give them their own groups): lsr_adam_step, up to 16 tensors per launch."""

    def __init__(self, params: Dict[str, torch.Tensor], lr, betas=(0.9, 0.999), eps: float = 1e-15):
        self._L = _lib.load()
        self.params = params
        self.lr = lr if isinstance(lr, dict) else {n: float(lr) for n in params}
        self.betas, self.eps = betas, eps
        self.exp_avg = {n: torch.zeros_like(t) for n, t in params.items()}
        self.exp_avg_sq = {n: torch.zeros_like(t) for n, t in params.items()}
        self.steps = {n: 0 for n in params}

    def adam_entry(self, n: str) -> Optional[dict]:
        """torch.optim.Adam's state for tensor n, None before its first step."""
        if self.steps.get(n, 0) == 0:
            return None
        return {"step": torch.tensor(float(self.steps[n])), "exp_avg": self.exp_avg[n].detach().clone(),
                "exp_avg_sq": self.exp_avg_sq[n].detach().clone()}

    def load_adam_entry(self, n: str, entry: Optional[dict]) -> None:
        p = self.params[n]
        if entry is None:
            self.exp_avg[n].zero_()
            self.exp_avg_sq[n].zero_()
            self.steps[n] = 0
            return
        for k, dst in (("exp_avg", self.exp_avg[n]), ("exp_avg_sq", self.exp_avg_sq[n])):
            if tuple(entry[k].shape) != tuple(p.shape):
                raise ValueError(f"{n}: optimizer {k} of shape {tuple(entry[k].shape)}, parameter {tuple(p.shape)}")
            dst.copy_(entry[k])
        self.steps[n] = int(float(entry["step"]))

    def step(self, grads: Dict[str, torch.Tensor]):
        groups = []
        for n, p in self.params.items():
            g = grads.get(n)
            if g is None or n not in self.lr:
                continue
            if g.shape != p.shape or not g.is_contiguous() or not p.is_contiguous():
                raise ValueError(f"{n}: gradient and parameter must be contiguous and of one shape")
            self.steps[n] += 1
            ag = _lib.AdamGroup()
            ag.param, ag.grad = p.data_ptr(), g.data_ptr()
            ag.exp_avg, ag.exp_avg_sq = self.exp_avg[n].data_ptr(), self.exp_avg_sq[n].data_ptr()
            ag.n, ag.lr, ag.step = p.numel(), float(self.lr[n]), self.steps[n]
            groups.append(ag)
        dev = next(iter(self.params.values())).device
        for i in range(0, len(groups), _lib.ADAM_MAX_GROUPS):
            chunk = groups[i:i + _lib.ADAM_MAX_GROUPS]
            arr = (_lib.AdamGroup * len(chunk))(*chunk)
            _lib.check(self._L.lsr_adam_step(arr, len(chunk), self.betas[0], self.betas[1], self.eps, _stream(dev)),
                       "lsr_adam_step")
