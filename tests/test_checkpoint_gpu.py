"""Optimizer-state checkpoints of the training loop (TrainStep.capture / restore / save_checkpoint /
load_checkpoint): the reference's GaussianModel.capture / restore (scene/gaussian_model.py:71-154),
train.py:424-426 (torch.save((capture, iteration), chkpnt_{stage}_{iter}.pth)) and --start_checkpoint
(train.py:104-109,579).  Files load with torch.load(weights_only=True).

The exact-resume check runs with torch.use_deterministic_algorithms(True): the rasterizer's autograd
backward then takes lsr_backward's fixed-order reduction, so training 20 iterations equals training
10, checkpointing, restoring into fresh objects and training 10 more, bit for bit (a densify and a
prune inside the second half prove the densification statistics and Adam moments came back).  The
deformation field's backward has float-atomic plane gradients (no deterministic variant), so the
field case checks that the restored state equals the captured one exactly and that training goes
on from it as from the original."""
import os
import tempfile

import pytest
import torch

import synthetic
from deformation import DeformationField
from gaussian_scene import render
from gaussian_train import GaussianTrainer
from train_step import ReferenceSchedule, TrainStep

pytestmark = pytest.mark.gpu
P, W, H = 4000, 160, 120
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-2, "f_rest": 2.5e-2 / 20, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3}
AABB = [[7.0, 5.5, 10.5], [-7.0, -5.5, 1.5]]
RES, MULTIRES = [16, 16, 16, 10], [1, 2]


def _raw(sc):
    shs = sc.shs
    return {"xyz": sc.means3D.contiguous(), "f_dc": shs[:, :1].contiguous(), "f_rest": shs[:, 1:].contiguous(),
            "opacity": torch.logit(sc.opacities.reshape(P, 1)).contiguous(),
            "scaling": torch.log(sc.scales).contiguous(), "rotation": sc.rotations.contiguous()}


def _problem(stage, field_p=None):
    dev = torch.device("cuda")
    sc = synthetic.make_scene(P, C=3, tanfovx=0.6, tanfovy=0.6 * H / W, seed=3, logscale_mean=-3.0).to(dev)
    cams = synthetic.camera_batch(2, W, H, tanfovx=0.6, seed=2)
    mk = (lambda: DeformationField({k: v.to(dev) for k, v in field_p.items()}, RES, MULTIRES)) if field_p else \
        (lambda: None)
    with torch.no_grad():
        teacher = TrainStep(GaussianTrainer(_raw(sc), LRS), mk(), stage=stage)
        gts = torch.stack([render(c, teacher.scene(), torch.ones(3, device=dev), stage=stage)["render"] for c in cams])
    g = torch.Generator(device="cpu").manual_seed(9)
    noise = {"f_dc": torch.randn(P, 1, 3, generator=g) * 0.5, "xyz": torch.randn(P, 3, generator=g) * 0.01}

    def student():
        raw = {k: v.clone() for k, v in _raw(sc).items()}   # fresh storage: training steps in place
        for k, v in noise.items():
            raw[k] = (raw[k] + v.to(dev)).contiguous()
        sched = ReferenceSchedule(8.0, stage=stage, densify_from_iter=12, densification_interval=5,
                                  pruning_from_iter=12, pruning_interval=5, densify_grad_threshold_fine_init=2e-6,
                                  densify_grad_threshold_after=2e-6, min_points=0, max_points=10 ** 9)
        st = TrainStep(GaussianTrainer(raw, LRS), mk(), stage=stage, densify=sched)
        st.set_reference_lr(8.0)
        return st, sched

    return cams, gts, student


def _state(st):
    tr = st.trainer
    out = {}
    for n in tr.params:
        out["p." + n] = tr.params[n].detach().clone()
        out["m." + n] = tr.exp_avg[n].clone()
        out["v." + n] = tr.exp_avg_sq[n].clone()
    for n in ("max_radii2D", "xyz_gradient_accum", "denom", "_deformation_table"):
        out[n] = getattr(tr, n).clone()
    if st.field is not None:
        for k, t in st.field.p.items():
            out["f." + k] = t.clone()
            out["fm." + k] = st.field_opt.exp_avg[k].clone()
            out["fv." + k] = st.field_opt.exp_avg_sq[k].clone()
    return out


def _assert_equal_states(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert a[k].shape == b[k].shape and torch.equal(a[k], b[k]), k


def test_resume_is_bit_exact():
    cams, gts, student = _problem("coarse-base")
    prev = (torch.are_deterministic_algorithms_enabled(), torch.is_deterministic_algorithms_warn_only_enabled())
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        torch.cuda.manual_seed(11)
        a, sched_a = student()
        for it in range(1, 21):
            a(cams, gts, iteration=it)
        torch.cuda.manual_seed(11)
        b, _ = student()
        for it in range(1, 11):
            b(cams, gts, iteration=it)
        with tempfile.TemporaryDirectory() as d:
            path = b.save_checkpoint(d, 10)
            assert os.path.basename(path) == "chkpnt_coarse-base_10.pth"
            del b
            c, _ = student()                                 # fresh objects, initial parameters
            assert c.load_checkpoint(path) == 10 and c.iteration == 10
        for it in range(11, 21):
            c(cams, gts, iteration=it)
        torch.cuda.synchronize()
    finally:
        torch.use_deterministic_algorithms(prev[0], warn_only=prev[1])
    kinds = [e[1] for e in sched_a.events]
    assert "densify" in kinds and "prune" in kinds and a.trainer.P != P, sched_a.events
    _assert_equal_states(_state(a), _state(c))
    assert a.trainer.steps == c.trainer.steps and a.trainer.lrs == c.trainer.lrs


def test_capture_layout_and_restore_with_field():
    field_p = DeformationField.init_params(RES, MULTIRES, AABB, seed=1)
    cams, gts, student = _problem("fine-base", field_p)
    a, _ = student()
    for it in range(1, 6):
        a(cams, gts, iteration=it)
    cap = a.capture()
    assert len(cap) == 14 and cap[0] == 3 and cap[-1] == 8.0
    opt = cap[12]
    names = [g["name"] for g in opt["param_groups"]]
    assert names == ["xyz", "deformation", "grid", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    assert all(k.startswith("deformation_net.") for k in cap[2])
    nparams = sum(len(g["params"]) for g in opt["param_groups"])
    assert sorted(opt["state"]) == list(range(nparams))          # every parameter has stepped
    assert float(opt["state"][0]["step"]) == 5.0
    with tempfile.TemporaryDirectory() as d:
        path = a.save_checkpoint(d, 5)
        loaded, it0 = torch.load(path, weights_only=True)            # nothing but tensors and plain data
        assert it0 == 5 and len(loaded) == 14
        b, _ = student()
        b.load_checkpoint(path)
    _assert_equal_states(_state(a), _state(b))
    la = [float(a(cams, gts, iteration=it)) for it in range(6, 9)]
    lb = [float(b(cams, gts, iteration=it)) for it in range(6, 9)]
    for x, y in zip(la, lb):
        assert abs(x - y) <= 1e-4 * abs(x), (la, lb)
    # the reference's restore re-runs training_setup: a fresh optimizer
    c, _ = student()
    c.restore(cap, fresh_optimizer=True)
    assert all(s == 0 for s in c.trainer.steps.values())
    assert torch.equal(c.trainer["xyz"], cap[1])


def test_reference_restore_semantics():
    """restore(reference=True) is the reference's GaussianModel.restore + training_setup
    (gaussian_model.py:111-154): a fresh optimizer; the field's state loaded from a 14-entry capture
    only (its 15-entry branch never calls _deformation.load_state_dict).  A 14-entry (RGB) capture
    restored into a trainer with a language group starts that group from zeros with a fresh optimizer
    (training_setup, :232-234), in either mode, instead of raising."""
    field_p = DeformationField.init_params(RES, MULTIRES, AABB, seed=1)
    cams, gts, student = _problem("fine-base", field_p)
    a, _ = student()
    for it in range(1, 4):
        a(cams, gts, iteration=it)
    cap14 = a.capture()
    assert len(cap14) == 14
    b, _ = student()
    f0 = {k: t.clone() for k, t in b.field.p.items()}
    b.restore(cap14, reference=True)                  # 14 entries: the field comes back
    assert all(torch.equal(b.field.p[k], a.field.p[k]) for k in f0)
    assert all(s == 0 for s in b.trainer.steps.values())
    assert all(float(b.field_opt.exp_avg[k].abs().max()) == 0 for k in b.field_opt.exp_avg)
    # a 15-entry capture (a language stage's): the reference keeps the field it has
    dev = torch.device("cuda")
    lang_lrs = dict(LRS, language_feature=2.5e-3)
    g = torch.Generator(device="cpu").manual_seed(4)

    def lang_step(lang):
        raw = {k: v.clone() for k, v in _raw(synthetic.make_scene(P, C=3, tanfovx=0.6, tanfovy=0.6 * H / W, seed=3,
                                                                   logscale_mean=-3.0).to(dev)).items()}
        raw["language_feature"] = lang.to(dev)
        return TrainStep(GaussianTrainer(raw, lang_lrs),
                         DeformationField({k: v.to(dev) for k, v in field_p.items()}, RES, MULTIRES), stage="fine-base")

    c = lang_step(torch.randn(P, 3, generator=g))
    cap15 = c.capture()
    assert len(cap15) == 15
    d = lang_step(torch.randn(P, 3, generator=g))
    with torch.no_grad():
        for t in d.field.p.values():
            t.add_(0.5)                                # a field that differs from the capture's
    fd = {k: t.clone() for k, t in d.field.p.items()}
    d.restore(cap15, reference=True)
    assert all(torch.equal(d.field.p[k], fd[k]) for k in fd)       # not loaded, as the reference
    assert torch.equal(d.trainer["language_feature"], cap15[9])
    d.restore(cap15)                                               # the resume mode loads it
    assert all(torch.equal(d.field.p[k], c.field.p[k]) for k in fd)
    # RGB capture into the language trainer: zeros, fresh Adam (both modes)
    for ref in (False, True):
        e = lang_step(torch.randn(P, 3, generator=g))
        e.restore(cap14, reference=ref)
        assert e.trainer["language_feature"].shape == (P, 3)
        assert float(e.trainer["language_feature"].abs().max()) == 0
        assert torch.equal(e.trainer["xyz"], cap14[1])
        assert all(s == 0 for s in e.trainer.steps.values())
