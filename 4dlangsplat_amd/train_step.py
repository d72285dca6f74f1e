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
adds in the fine stages (plane TV / time smoothness, lambda_dssim) are not included.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch

from gaussian_scene import GaussianScene, render
from gaussian_train import GaussianTrainer, TensorAdam


class TrainStep:
    """trainer: GaussianTrainer over the raw Gaussian tensors (xyz, f_dc, f_rest, opacity, scaling,
    rotation[, language_feature]); field: deformation.DeformationField for the 'fine' stages."""

    def __init__(self, trainer: GaussianTrainer, field=None, deform_lr: float = 1.6e-4, grid_lr: float = 1.6e-3,
                 bg: Optional[torch.Tensor] = None, stage: str = "fine-base", sh_degree: int = 3,
                 densify: Optional[Callable[[GaussianTrainer, int], None]] = None):
        """densify(trainer, iteration): optional densify / prune / reset_opacity schedule, run
        between the densification statistics and the optimizer step (train.py:388-421)."""
        self.trainer, self.field, self.stage = trainer, field, stage
        self.densify = densify
        self.iteration = 0
        self.sh_degree = sh_degree
        self.bg = bg if bg is not None else torch.ones(3, device=trainer.device)
        self.field_opt = None
        if field is not None:
            params = {k: v for k, v in field.p.items() if k != "grid.aabb"}
            lrs = {k: (grid_lr if k.startswith("grid.") else deform_lr) for k in params}
            self.field_opt = TensorAdam(params, lrs)

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
        if self.field is not None:
            self.field.zero_grad()
        sc = self.scene()
        outs = [render(cam, sc, self.bg, stage=self.stage) for cam in cams]
        images = torch.stack([o["render"] for o in outs])
        loss = (images - gts).abs().mean()
        loss.backward()
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
