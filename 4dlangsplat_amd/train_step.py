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
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch

from gaussian_scene import GaussianScene, render, render_views
from gaussian_train import GaussianTrainer, TensorAdam, get_expon_lr_func


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
                 densify: Optional[Callable[[GaussianTrainer, int], None]] = None, batch_views: bool = False):
        """densify(trainer, iteration): optional densify / prune / reset_opacity schedule, run
        between the densification statistics and the optimizer step (train.py:388-421).
        batch_views: the batch's views share one deformation-field launch (render_views)
        instead of one per view (render); same values.  Off by default: at configs[4] size
        the repeat / split copies around the one launch cost more than the per-call fixed work
        saved (127.8 vs 140.5 iterations/s)."""
        self.trainer, self.field, self.stage = trainer, field, stage
        self.batch_views = batch_views
        self.densify = densify
        self.iteration = 0
        self.sh_degree = sh_degree
        self.bg = bg if bg is not None else torch.ones(3, device=trainer.device)
        self.field_opt = None
        if field is not None:
            params = {k: v for k, v in field.p.items() if k != "grid.aabb"}
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

    def scene(self) -> GaussianScene:
        tr = self.trainer
        lang = tr.params.get("language_feature")
        if lang is None:
            lang = torch.zeros(tr.P, 3, device=tr.device)
        return GaussianScene(tr["xyz"], tr["f_dc"], tr["f_rest"], lang, tr["opacity"], tr["scaling"], tr["rotation"],
                             max_sh_degree=self.sh_degree, active_sh_degree=self.sh_degree, deformation=self.field)

    def __call__(self, cams: Sequence, gts: torch.Tensor, iteration: Optional[int] = None) -> torch.Tensor:
        """One iteration over the views `cams` with ground-truth images gts [V, 3, H, W].
        Returns the loss (a device scalar; no host synchronisation here unless `densify` makes one)."""
        tr = self.trainer
        self.iteration = self.iteration + 1 if iteration is None else iteration
        self.update_learning_rate(self.iteration)
        if self.field is not None:
            self.field.zero_grad()
        sc = self.scene()
        if self.batch_views:
            outs = render_views(cams, sc, self.bg, stage=self.stage)
        else:
            outs = [render(cam, sc, self.bg, stage=self.stage) for cam in cams]
        images = torch.stack([o["render"] for o in outs])
        loss = (images - gts).abs().mean()
        loss.backward()
        collect = getattr(self.densify, "collect_stats", None)
        if collect is None or collect(self.iteration):   # train.py:388: while iteration < densify_until_iter
            radii = torch.stack([o["radii"] for o in outs]).max(dim=0).values
            vgrad = outs[0]["viewspace_points"].grad
            for o in outs[1:]:
                vgrad = vgrad + o["viewspace_points"].grad
            tr.add_densification_stats(vgrad, radii)
        if self.densify is not None:
            self.densify(tr, self.iteration)
        tr.step()
        tr.zero_grad(set_to_none=True)
        if self.field is not None:
            self.field_opt.step(self.field.grads)
            self.field.prepare()
        return loss.detach()
