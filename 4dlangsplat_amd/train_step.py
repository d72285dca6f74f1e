"""One training iteration of the reference's loop on the MI355X pieces (the
config-5 loop): deformation field -> rasterizer for every view of the batch -> L1 loss ->
backward through both -> densification statistics -> Adam on the Gaussians and on the field.

Follows train.py:224-421 for the 'base' stages (image loss):
  per view render(), stacked images, Ll1 = l1_loss(images, gts)            train.py:242-287
  loss.backward()                                                          :339
  viewspace gradient summed over views, radii max, visibility any         :265-271,350-352
  max_radii2D / add_densification_stats                                    :388-391
  densify / prune / reset_opacity (the caller's `densify` callback)        :393-414
  optimizer.step(); zero_grad(set_to_none=True)                            :420-421
The callback runs where the reference runs its densification, BEFORE the optimizer step.  Rows it
rebuilds (densify, prune: new parameter tensors) and the opacity it resets have no gradient
afterwards, so that iteration's Adam update skips those groups exactly as the reference's
optimizer.step() skips its freshly built nn.Parameters; the deformation field still steps.
The deformation field's parameters get their own Adam (their groups in training_setup,
scene/gaussian_model.py:273-276) and are repacked after every update.  Regularisers the reference
adds nothing here: its TV / time-smoothness term is gated on `stage == "fine"` (train.py:331), which
never equals the stage names it runs ('fine-base', 'fine-lang'), and lambda_dssim defaults to 0
(arguments/__init__.py:146), so the base-stage loss is the L1 alone.
set_reference_lr() installs the per-iteration learning-rate schedules of
gaussian_model.py:302-330 (xyz, deformation MLPs, grid planes; OptimizationParams defaults).

The 'lang' stages (coarse-lang, fine-lang, fine-lang-discrete) follow train.py:272-296 and
training_setup's lang branch (scene/gaussian_model.py:226-270):
  loss = lam * l1_loss(lang * mask, gt_lang * mask)                         train.py:287
         (+ beta * cos_loss(lang * mask, gt_lang * mask) with addcosloss)   :289-292, utils/loss_utils.py:26-27
         (+ l1_loss(images, gts[:, :3]) with joint_train)                   :293-296
  trainable: the language features; the deformation field's lang_deform when it deforms the
  language (no_dlang 0) and its discrete_coff_generator in a 'discrete' stage; with joint_train
  every Gaussian group and the whole field as well.  Frozen groups get no gradient and Adam skips
  them, as the reference's requires_grad_(False) parameters.  The renders' coff (discrete fields)
  is collected as train.py:245-247 collects it; the reference computes no loss from it.
  Densification statistics are gathered in the 'base' stages only (train.py:388).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import ctypes

import torch

from gaussian_scene import GaussianScene, render, render_views
from gaussian_train import GaussianTrainer, TensorAdam, get_expon_lr_func


class _L1Views(torch.autograd.Function):
    """l1_loss(stack(images), gts[:, :3]) (train.py:272-276) over the views' renders without stacking
    them: two launches forward, one backward (lsr_l1_loss_views / _backward, include/lsr_train.h); the
    gradient PyTorch's bit for bit, the loss's partial sums added in a fixed order."""

    @staticmethod
    def forward(ctx, gts3, *images):
        from diff_gaussian_rasterization import _lib
        L = _lib.load()
        V = len(images)
        imgs = [x.contiguous() for x in images]
        n = imgs[0].numel()
        if gts3.shape[0] != V or any(x.shape != imgs[0].shape or x.dtype != torch.float32 for x in imgs) \
                or tuple(gts3.shape[1:]) != tuple(imgs[0].shape) or gts3[0].stride() != imgs[0].stride():
            raise ValueError("l1 loss: V float32 images of one shape and gts[:, :3] of that shape")
        ptrs = (ctypes.c_void_p * V)(*[x.data_ptr() for x in imgs])
        ws = torch.empty(int(L.lsr_l1_workspace_bytes(V)), dtype=torch.uint8, device=imgs[0].device)
        loss = torch.empty((), device=imgs[0].device)
        st = torch.cuda.current_stream(imgs[0].device).cuda_stream
        _lib.check(L.lsr_l1_loss_views(V, n, ptrs, gts3.data_ptr(), gts3.stride(0), loss.data_ptr(), ws.data_ptr(), st),
                   "lsr_l1_loss_views")
        ctx.save_for_backward(gts3, *imgs)
        return loss

    @staticmethod
    def backward(ctx, g):
        from diff_gaussian_rasterization import _lib
        gts3, *imgs = ctx.saved_tensors
        V = len(imgs)
        grads = [torch.empty_like(x) for x in imgs]
        g = g.contiguous()
        st = torch.cuda.current_stream(g.device).cuda_stream
        _lib.check(_lib.load().lsr_l1_loss_views_backward(
            V, imgs[0].numel(), (ctypes.c_void_p * V)(*[x.data_ptr() for x in imgs]), gts3.data_ptr(), gts3.stride(0),
            g.data_ptr(), (ctypes.c_void_p * V)(*[x.data_ptr() for x in grads]), st), "lsr_l1_loss_views_backward")
        return (None,) + tuple(grads)


def l1_loss_views(images, gts):
    """mean |stack(images) - gts[:, :3]| with its gradient (the base stages' loss); native on the GPU
    for up to 8 views, PyTorch otherwise."""
    gts3 = gts[:, :3]
    if images[0].is_cuda and 1 <= len(images) <= 8 and gts3[0].is_contiguous():
        return _L1Views.apply(gts3, *images)
    return (torch.stack(images) - gts3).abs().mean()


class ReferenceSchedule:
    """The densification schedule of train.py:388-414 in the 'base' stages, as a TrainStep
    `densify` callback.  Defaults: OptimizationParams (arguments/__init__.py:149-166) with the
    Neu3D overrides (arguments/neu3d/default.py:24-33: densify_until_iter 10000,
    opacity_reset_interval 60000, opacity thresholds 0.005).  extent: scene.cameras_extent.
    Statistics are collected while iteration < densify_until_iter (collect_stats); densify every
    densification_interval after densify_from_iter while P < 360000, prune every pruning_interval
    after pruning_from_iter while P > 200000 (size threshold 20 once past opacity_reset_interval),
    reset opacity every opacity_reset_interval.  The reference's `stage == "coarse"` never matches its
    stage names, so the fine thresholds apply (interpolated over densify_until_iter)."""

    def __init__(self, extent: float, stage: str = "fine-base", densify_from_iter: int = 500,
                 densify_until_iter: int = 10_000, densification_interval: int = 100, pruning_from_iter: int = 500,
                 pruning_interval: int = 100, opacity_reset_interval: int = 60_000,
                 densify_grad_threshold_fine_init: float = 2e-4, densify_grad_threshold_after: float = 2e-4,
                 opacity_threshold_fine_init: float = 0.005, opacity_threshold_fine_after: float = 0.005,
                 max_points: int = 360_000, min_points: int = 200_000):
        self.extent, self.stage = extent, stage
        self.__dict__.update(densify_from_iter=densify_from_iter, densify_until_iter=densify_until_iter,
                             densification_interval=densification_interval, pruning_from_iter=pruning_from_iter,
                             pruning_interval=pruning_interval, opacity_reset_interval=opacity_reset_interval,
                             g_init=densify_grad_threshold_fine_init, g_after=densify_grad_threshold_after,
                             o_init=opacity_threshold_fine_init, o_after=opacity_threshold_fine_after,
                             max_points=max_points, min_points=min_points)
        self.events = []          # (iteration, what, P before, P after)

    def collect_stats(self, iteration: int) -> bool:
        return iteration < self.densify_until_iter and "base" in self.stage

    def __call__(self, tr: GaussianTrainer, iteration: int) -> None:
        if not self.collect_stats(iteration):
            return
        frac = iteration / self.densify_until_iter
        opacity_threshold = self.o_init - frac * (self.o_init - self.o_after)
        densify_threshold = self.g_init - frac * (self.g_init - self.g_after)
        size_threshold = 20 if iteration > self.opacity_reset_interval else None
        if iteration > self.densify_from_iter and iteration % self.densification_interval == 0 \
                and tr.P < self.max_points:
            p0 = tr.P
            tr.densify(densify_threshold, opacity_threshold, self.extent, size_threshold)
            self.events.append((iteration, "densify", p0, tr.P))
        if iteration > self.pruning_from_iter and iteration % self.pruning_interval == 0 and tr.P > self.min_points:
            p0 = tr.P
            tr.prune(densify_threshold, opacity_threshold, self.extent, size_threshold)
            self.events.append((iteration, "prune", p0, tr.P))
        if iteration % self.opacity_reset_interval == 0:
            tr.reset_opacity()
            self.events.append((iteration, "reset_opacity", tr.P, tr.P))


class TrainStep:
    """trainer: GaussianTrainer over the raw Gaussian tensors (xyz, f_dc, f_rest, opacity, scaling,
    rotation[, language_feature]); field: deformation.DeformationField for the 'fine' stages."""

    def __init__(self, trainer: GaussianTrainer, field=None, deform_lr: float = 1.6e-4, grid_lr: float = 1.6e-3,
                 bg: Optional[torch.Tensor] = None, stage: str = "fine-base", sh_degree: int = 3,
                 densify: Optional[Callable[[GaussianTrainer, int], None]] = None, batch_views: bool = True,
                 joint_train: bool = False, lam: float = 0.2, beta: float = 0.01, addcosloss: bool = False):
        """densify(trainer, iteration): optional densify / prune / reset_opacity schedule, run
        between the densification statistics and the optimizer step (train.py:388-421).
        batch_views: the batch's views share one deformation-field launch (render_views)
        instead of one per view (render); same values.  On by default since round 4: with the
        field's box-gradient atomics spread over partial rows the one launch fills the GPU better
        than two half-size ones (configs[4] stand-in 187-188 vs 184-185 iterations/s, the field's
        backward 1.45 vs 1.74 ms per iteration); round 3 had measured the opposite
        (127.8 vs 140.5) while those atomics serialised.
        joint_train, lam, beta, addcosloss: the 'lang' stages' switches (train.py --joint_coarse /
        --joint_fine, --lam 0.2, --beta 0.01, env addcosloss)."""
        if joint_train and "lang" not in stage:
            raise ValueError("joint_train needs a 'lang' stage (train.py:103-104)")
        if "lang" in stage and "language_feature" not in trainer.params:
            raise ValueError("a 'lang' stage trains the language features: the trainer needs a language_feature group")
        self.trainer, self.field, self.stage = trainer, field, stage
        self.joint_train, self.lam, self.beta, self.addcosloss = joint_train, lam, beta, addcosloss
        self.coff = []              # the last iteration's renders' coff (train.py:240-247)
        self.batch_views = batch_views
        self.densify = densify
        self.iteration = 0
        self.sh_degree = sh_degree
        self.bg = bg if bg is not None else torch.ones(3, device=trainer.device)
        self.field_opt = None
        self.spatial_lr_scale = 0.0
        if field is not None:
            # the box trains too (gaussian_model.py:250-253,258,291: "grid.aabb" is among
            # get_grid_parameters and has requires_grad once the whole module does)
            field.train_aabb = True
            params = dict(field.p)
            lrs = {k: (grid_lr if k.startswith("grid.") else deform_lr) for k in params}
            self.field_opt = TensorAdam(params, lrs)

    def set_reference_lr(self, spatial_lr_scale: float, position_lr_init=1.6e-4, position_lr_final=1.6e-6,
                         position_lr_delay_mult=0.01, position_lr_max_steps=20_000, deformation_lr_init=1.6e-4,
                         deformation_lr_final=1.6e-5, deformation_lr_delay_mult=0.01, grid_lr_init=1.6e-3,
                         grid_lr_final=1.6e-4):
        """training_setup's schedules (gaussian_model.py:239-253, 302-313), all scaled by
        spatial_lr_scale (the scene's cameras_extent); applied at the start of every iteration as
        train.py:233 calls gaussians.update_learning_rate(iteration)."""
        s = spatial_lr_scale
        self.spatial_lr_scale = float(s)
        self.trainer.set_xyz_schedule(position_lr_init * s, position_lr_final * s, position_lr_delay_mult,
                                      position_lr_max_steps)
        self._deform_sched = get_expon_lr_func(deformation_lr_init * s, deformation_lr_final * s,
                                               lr_delay_mult=deformation_lr_delay_mult, max_steps=position_lr_max_steps)
        self._grid_sched = get_expon_lr_func(grid_lr_init * s, grid_lr_final * s,
                                             lr_delay_mult=deformation_lr_delay_mult, max_steps=position_lr_max_steps)

    def update_learning_rate(self, iteration: int) -> None:
        """gaussian_model.py:315-330."""
        self.trainer.update_learning_rate(iteration)
        if self.field_opt is not None and getattr(self, "_grid_sched", None) is not None:
            lg, ld = float(self._grid_sched(iteration)), float(self._deform_sched(iteration))
            for k in self.field_opt.lr:
                self.field_opt.lr[k] = lg if k.startswith("grid.") else ld

    @property
    def lang_stage(self) -> bool:
        return "lang" in self.stage

    def field_trainable(self, name: str) -> bool:
        """Whether the field parameter `name` trains in this stage (training_setup,
        scene/gaussian_model.py:248-262: _deformation.requires_grad_(joint_train), then
        lang_deform.requires_grad_(no_dlang == 0), discrete_coff_generator on in 'discrete' stages)."""
        if not self.lang_stage:
            return True
        if name.startswith("lang_deform."):
            return True           # present only when the field deforms the language (no_dlang 0)
        if name.startswith("discrete_coff_generator."):
            return self.joint_train or "discrete" in self.stage
        return self.joint_train

    def scene(self) -> GaussianScene:
        tr = self.trainer
        lang = tr.params.get("language_feature")
        if lang is None:
            lang = torch.zeros(tr.P, 3, device=tr.device)
        # a 'lang' stage without joint_train freezes the geometry and colours (requires_grad_(False))
        g = (lambda t: t) if (not self.lang_stage or self.joint_train) else (lambda t: t.detach())   # noqa: E731
        return GaussianScene(g(tr["xyz"]), g(tr["f_dc"]), g(tr["f_rest"]), lang, g(tr["opacity"]), g(tr["scaling"]),
                             g(tr["rotation"]), max_sh_degree=self.sh_degree, active_sh_degree=self.sh_degree,
                             deformation=self.field)

    def loss(self, outs, gts: Optional[torch.Tensor], gt_lang: Optional[torch.Tensor] = None,
             lang_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The stage's loss over the views' render outputs (train.py:272-296).  Base stages: L1 of the
        images against gts [V, 3(+), H, W].  'lang' stages: gt_lang [V, C, H, W], lang_mask [V, 1, H, W]
        (the reference trains them one view at a time, batch_size 1, where its cat over views is this
        stack)."""
        if not self.lang_stage:
            return l1_loss_views([o["render"] for o in outs], gts)
        if gt_lang is None or lang_mask is None:
            raise ValueError("a 'lang' stage needs gt_lang and lang_mask")
        lang = torch.stack([o["language_feature_image"] for o in outs])
        a, b = lang * lang_mask, gt_lang * lang_mask
        loss = self.lam * (a - b).abs().mean()
        if self.addcosloss:
            loss = loss + self.beta * (1 - torch.nn.functional.cosine_similarity(a, b, dim=-1).mean())
        if self.joint_train:
            images = torch.stack([o["render"] for o in outs])
            loss = loss + (images - gts[:, :3]).abs().mean()
        return loss

    def forward_backward(self, cams: Sequence, gts: Optional[torch.Tensor], gt_lang: Optional[torch.Tensor] = None,
                         lang_mask: Optional[torch.Tensor] = None):
        """Render every view, the stage's loss, loss.backward() (train.py:242-339).  Leaves the
        gradients in the trainer's parameters' .grad and the field's grads; returns (loss, outs)."""
        if self.field is not None:
            self.field.zero_grad()
        sc = self.scene()
        if self.batch_views:
            outs = render_views(cams, sc, self.bg, stage=self.stage)
        else:
            outs = [render(cam, sc, self.bg, stage=self.stage) for cam in cams]
        self.coff = [o["coff"] for o in outs if o.get("coff") is not None]
        loss = self.loss(outs, gts, gt_lang, lang_mask)
        loss.backward()
        return loss, outs

    def __call__(self, cams: Sequence, gts: Optional[torch.Tensor], iteration: Optional[int] = None,
                 gt_lang: Optional[torch.Tensor] = None, lang_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One iteration over the views `cams` with ground-truth images gts [V, 3, H, W] (and, in
        the 'lang' stages, language features gt_lang [V, C, H, W] with masks lang_mask [V, 1, H, W]).
        Returns the loss (a device scalar; no host synchronisation here unless `densify` makes one)."""
        tr = self.trainer
        self.iteration = self.iteration + 1 if iteration is None else iteration
        self.update_learning_rate(self.iteration)
        loss, outs = self.forward_backward(cams, gts, gt_lang, lang_mask)
        collect = getattr(self.densify, "collect_stats", None)
        # train.py:388: while iteration < densify_until_iter, in the 'base' stages
        if "base" in self.stage and (collect is None or collect(self.iteration)):
            rl = [o["radii"] for o in outs]
            if rl[0].is_cuda and rl[0].dtype == torch.int32:   # train.py:266's max over the views, one launch
                from diff_gaussian_rasterization import radii_max_native
                radii = radii_max_native(rl, torch.empty_like(rl[0]))
            else:
                radii = torch.stack(rl).max(dim=0).values
            vgrad = outs[0]["viewspace_points"].grad
            for o in outs[1:]:
                vgrad = vgrad + o["viewspace_points"].grad
            tr.add_densification_stats(vgrad, radii)
        if self.densify is not None:
            self.densify(tr, self.iteration)
        tr.step()
        tr.zero_grad(set_to_none=True)
        if self.field is not None:
            grads = self.field.grads if not self.lang_stage else \
                {k: v for k, v in self.field.grads.items() if self.field_trainable(k)}
            if grads:
                self.field_opt.step(grads)
                self.field.prepare()
        return loss.detach()

    # ---- checkpoints (scene/gaussian_model.py:71-154, train.py:104-109,424-426,579) ---------------
    def _group_layout(self):
        """[(group name, [(owner, key, reference parameter name)])] in training_setup's order
        (gaussian_model.py:273-288 base stages; :236-255 lang stages with joint_train)."""
        tr, f = self.trainer, self.field
        gauss = lambda n: [("g", n, "_" + n if n not in ("f_dc", "f_rest") else "_features_" + n[2:])]  # noqa: E731
        mlp = [("f", k, "deformation_net." + k) for k in (f.p if f is not None else ()) if "grid" not in k]
        grid = [("f", k, "deformation_net." + k) for k in (f.p if f is not None else ()) if "grid" in k]
        if self.lang_stage and not self.joint_train:
            order = ["deformation", "grid", "language_feature"]
        else:
            order = ["xyz", "deformation", "grid", "f_dc", "f_rest", "opacity", "scaling", "rotation",
                     "language_feature"]
        out = []
        for name in order:
            if name == "deformation":
                if mlp:
                    out.append((name, mlp))
            elif name == "grid":
                if grid:
                    out.append((name, grid))
            elif name in tr.params:
                out.append((name, gauss(name)))
        return out

    def optimizer_state_dict(self) -> dict:
        """The Gaussians' and the field's Adam state in torch.optim.Adam.state_dict()'s layout (one
        optimizer over training_setup's groups, parameters numbered in group order, state only for
        parameters that have stepped), with each group's reference parameter names (param_names)."""
        tr, fo = self.trainer, self.field_opt
        state, groups, i = {}, [], 0
        for name, members in self._group_layout():
            ids, names = [], []
            for owner, key, ref in members:
                e = tr.adam_entry(key) if owner == "g" else (fo.adam_entry(key) if fo is not None else None)
                if e is not None:
                    state[i] = e
                ids.append(i)
                names.append(ref)
                i += 1
            owner, key, _ = members[0]
            lr = tr.lrs.get(key, 0.0) if owner == "g" else (fo.lr.get(key, 0.0) if fo is not None else 0.0)
            groups.append({"params": ids, "lr": float(lr), "name": name, "betas": tuple(tr.betas), "eps": tr.eps,
                           "weight_decay": 0, "amsgrad": False, "maximize": False, "foreach": None,
                           "capturable": False, "differentiable": False, "fused": None, "param_names": names})
        return {"state": state, "param_groups": groups}

    def load_optimizer_state_dict(self, opt: dict) -> None:
        """Inverse of optimizer_state_dict: by param_names when the groups carry them, else by the
        group order of training_setup."""
        tr, fo = self.trainer, self.field_opt
        ref_to_key = {}
        for _, members in self._group_layout():
            for owner, key, ref in members:
                ref_to_key[ref] = (owner, key)
        layout = [m for _, ms in self._group_layout() for m in ms]
        seen = set()
        for gi, g in enumerate(opt["param_groups"]):
            names = g.get("param_names")
            for j, pid in enumerate(g["params"]):
                if names is not None:
                    if names[j] not in ref_to_key:
                        raise ValueError(f"checkpoint parameter {names[j]} is not in this model")
                    owner, key = ref_to_key[names[j]]
                else:
                    if pid >= len(layout):
                        raise ValueError("checkpoint optimizer has more parameters than this model")
                    owner, key, _ = layout[pid]
                entry = opt["state"].get(pid)
                if owner == "g":
                    tr.load_adam_entry(key, entry)
                    tr.lrs[key] = float(g["lr"])
                elif fo is not None:
                    fo.load_adam_entry(key, entry)
                    fo.lr[key] = float(g["lr"])
                seen.add((owner, key))
        for owner, key, ref in layout:
            if (owner, key) not in seen:
                raise ValueError(f"the checkpoint's optimizer has no state for {ref}")

    def capture(self, include_feature: Optional[bool] = None) -> tuple:
        """GaussianModel.capture (gaussian_model.py:71-105): (active_sh_degree, _xyz, the field's
        state_dict, _deformation_table, _features_dc, _features_rest, _scaling, _rotation, _opacity,
        [_language_feature,] max_radii2D, xyz_gradient_accum, denom, optimizer.state_dict(),
        spatial_lr_scale); 15 entries with include_feature (default: whether the trainer has a
        language group), else 14.  Tensors are cloned: training on does not change a capture."""
        tr = self.trainer
        if include_feature is None:
            include_feature = "language_feature" in tr.params
        if include_feature and "language_feature" not in tr.params:
            raise ValueError("include_feature needs a language_feature group")
        c = lambda t: t.detach().clone()  # noqa: E731
        head = (self.sh_degree, c(tr["xyz"]), self.field.state_dict() if self.field is not None else {},
                c(tr._deformation_table), c(tr["f_dc"]), c(tr["f_rest"]), c(tr["scaling"]), c(tr["rotation"]),
                c(tr["opacity"]))
        lang = (c(tr["language_feature"]),) if include_feature else ()
        return head + lang + (c(tr.max_radii2D), c(tr.xyz_gradient_accum), c(tr.denom), self.optimizer_state_dict(),
                              float(self.spatial_lr_scale))

    def restore(self, model_args: tuple, fresh_optimizer: bool = False, reference: bool = False) -> None:
        """GaussianModel.restore (gaussian_model.py:107-154) of a capture(): parameters, field,
        deformation table, statistics and the optimizer state.  The reference re-runs training_setup
        after loading, which builds a fresh Adam (its moments and step counts are not resumed);
        fresh_optimizer=True does the same, the default resumes them (training N iterations equals
        training k, capture, restore, N - k more).

        A 14-entry capture (no language features) restored into a trainer with a language group
        starts that group from zeros, as training_setup does for a language stage initialised from
        an RGB model (gaussian_model.py:232-234), with a fresh optimizer (the reference loads no
        optimizer state when include_feature is on: :146-147).

        reference=True reproduces the reference's restore exactly: a fresh optimizer, and the
        deformation field's state loaded only from a 14-entry capture (its 15-entry branch never
        calls _deformation.load_state_dict: :111-129 vs :130-150)."""
        if len(model_args) == 15:
            (sh, xyz, deform, table, f_dc, f_rest, scaling, rotation, opacity, lang, max_r, accum, denom, opt,
             slr) = model_args
        elif len(model_args) == 14:
            (sh, xyz, deform, table, f_dc, f_rest, scaling, rotation, opacity, max_r, accum, denom, opt,
             slr) = model_args
            lang = None
        else:
            raise ValueError(f"a capture has 14 or 15 entries, got {len(model_args)}")
        tr = self.trainer
        params = dict(xyz=xyz, f_dc=f_dc, f_rest=f_rest, opacity=opacity, scaling=scaling, rotation=rotation)
        if lang is not None:
            params["language_feature"] = lang
        elif "language_feature" in tr.params:    # language stage from an RGB capture: zeros, fresh Adam
            width = int(tr["language_feature"].shape[1])   # the trainer's language_feature_hiddendim
            params["language_feature"] = torch.zeros(xyz.shape[0], width, dtype=torch.float32, device=xyz.device)
            fresh_optimizer = True
        tr.load_rows(params, max_r, accum, denom, table)
        self.sh_degree = int(sh)
        self.spatial_lr_scale = float(slr)
        if self.field is not None and not (reference and len(model_args) == 15):
            pre = "deformation_net."
            sd = {k[len(pre):]: v for k, v in deform.items() if k.startswith(pre)}
            missing = sorted(set(self.field.p) - set(sd))
            if missing:
                raise ValueError(f"the capture's field lacks {missing}")
            with torch.no_grad():
                for k, t in self.field.p.items():
                    if tuple(sd[k].shape) != tuple(t.shape):
                        raise ValueError(f"{k}: shape {tuple(sd[k].shape)} vs {tuple(t.shape)}")
                    t.copy_(sd[k])
            self.field.prepare()
        if fresh_optimizer or reference:
            for n in tr.params:
                tr.load_adam_entry(n, None)
            if self.field_opt is not None:
                for n in self.field_opt.params:
                    self.field_opt.load_adam_entry(n, None)
        else:
            self.load_optimizer_state_dict(opt)

    def save_checkpoint(self, model_path: str, iteration: int, include_feature: Optional[bool] = None) -> str:
        """train.py:424-426: torch.save((capture(include_feature), iteration)) as
        <model_path>/chkpnt_<stage>_<iteration>.pth.  Everything in it loads with weights_only=True."""
        import os
        path = os.path.join(model_path, f"chkpnt_{self.stage}_{iteration}.pth")
        torch.save((self.capture(include_feature), int(iteration)), path)
        return path

    def load_checkpoint(self, path: str, fresh_optimizer: bool = False, reference: bool = False) -> int:
        """train.py:104-109 (--start_checkpoint): restore a save_checkpoint file; returns its
        iteration (the loop's first_iter), which also becomes self.iteration.  fresh_optimizer /
        reference: as restore()."""
        model_args, first_iter = torch.load(path, map_location=self.trainer.device, weights_only=True)
        self.restore(model_args, fresh_optimizer=fresh_optimizer, reference=reference)
        self.iteration = int(first_iter)
        return self.iteration
