"""The 'lang' training stages (train.py:272-296, gaussian_model.py:226-270) through TrainStep on the
GPU, against tests/golden/lang_train_golden.npz: one iteration of the REFERENCE's own render(),
deform_network (lang_deform, residual mode), loss functions and autograd, in float64, with the C
oracle as the rasterizer (tests/golden/make_lang_train_golden.py).

  lang       fine-lang, lam 0.2: the loss, the rendered language image, dL/d language features and
             the lang_deform weight gradients; the geometry and the rest of the field stay frozen
  cos_joint  fine-lang with addcosloss (beta 0.01) and joint_train: the RGB L1 joins the loss and
             every Gaussian group and field tensor trains -- the HexPlane box (grid.aabb) included,
             as the reference's requires_grad_(True) + get_grid_parameters make it

Tolerances (float32 here against a float64 golden): loss 1e-5 relative; images 1e-4
absolute at all but 0.1 % of the values and 1e-2 everywhere (a contributor decision alpha >= 1/255 or
T (1 - alpha) >= 1e-4 that lands on the other side in float32 moves its pixel by up to alpha T |c|,
as in tests/test_oracle_drift.py); gradients 1e-4 of each tensor's largest magnitude per row on 99 %
of the rows and 2e-2 on every row (the same flips reach the Gaussians of the flipped pixels, and the
rows the golden marks kink-ambiguous -- a field pre-activation within 1e-4 of a ReLU kink, where
float32 and float64 may take different sides -- are held to 2e-2 only); the field's summed weight
gradients within 2e-3."""
import ast
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "lang_train_golden.npz")
GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation", "language_feature")
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3,
       "language_feature": 2.5e-3}


def _load(name):
    z = np.load(GOLDEN)
    pre = name + "/"
    return {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}


def _setup(d):
    import synthetic
    from deformation import DeformationField
    from gaussian_train import GaussianTrainer
    from train_step import TrainStep
    cfg = ast.literal_eval(str(d["config"]))
    dev = torch.device("cuda")
    params = {k: torch.tensor(d["param/" + k], device=dev).contiguous() for k in GROUPS}
    tr = GaussianTrainer(params, LRS)
    state = {"deformation_net." + k[len("field/"):]: torch.tensor(v) for k, v in d.items() if k.startswith("field/")}
    state["deformation_net.grid.aabb"] = torch.tensor(d["field_aabb"])
    hidden = dict(kplanes_config={"resolution": cfg["res"], "output_coordinate_dim": 16}, multires=cfg["multires"],
                  defor_depth=0, net_width=128, no_do=False, no_dshs=False, no_dlang=0)
    field = DeformationField.from_reference(state, hidden, env={"language_feature_hiddendim": str(cfg["lang_dim"])},
                                            device=dev)
    lam, beta, cos, joint = (float(x) for x in d["hp"])
    step = TrainStep(tr, field, stage="fine-lang", joint_train=bool(joint), lam=lam, beta=beta, addcosloss=bool(cos))
    W, H = cfg["W"], cfg["H"]
    cam = synthetic.Camera(W, H, float(d["fov"][0]), float(d["fov"][1]), torch.tensor(d["viewmatrix"]).to(dev),
                           torch.zeros(4, 4, device=dev), torch.tensor(d["projmatrix"]).to(dev),
                           torch.tensor(d["campos"]).to(dev), float(d["time"]))
    t = lambda k: torch.tensor(d[k], device=dev)   # noqa: E731
    return step, tr, field, cam, t("gt_img"), t("gt_lang"), t("mask")


def _rowwise(got, ref, amb, tight=1e-4, loose=2e-2, share=0.99):
    got, ref = got.reshape(ref.shape[0], -1).astype(np.float64), ref.reshape(ref.shape[0], -1)
    scale = max(float(np.abs(ref).max()), 1e-30)
    err = np.abs(got - ref).max(axis=1) / scale
    clear = err[~amb]
    within = float((clear <= tight).mean()) if clear.size else 1.0
    return within >= share and float(err.max(initial=0.0)) <= loose, \
        dict(within_tight=within, worst_clear=float(clear.max(initial=0.0)), worst=float(err.max(initial=0.0)))


def _image_ok(got, ref, tight=1e-4, loose=1e-2, share=1e-3):
    err = np.abs(np.asarray(got, np.float64) - ref)
    above = float((err > tight).mean())
    return above <= share and float(err.max()) <= loose, dict(above_share=above, max=float(err.max()))


@pytest.mark.parametrize("name", ("lang", "cos_joint"))
def test_lang_stage_iteration_matches_reference(name):
    d = _load(name)
    step, tr, field, cam, gt_img, gt_lang, mask = _setup(d)
    loss, outs = step.forward_backward([cam], gt_img, gt_lang=gt_lang, lang_mask=mask)
    torch.cuda.synchronize()
    assert abs(float(loss) - float(d["loss"])) <= 1e-5 * abs(float(d["loss"])), (float(loss), float(d["loss"]))
    lang_img = outs[0]["language_feature_image"].detach().cpu().numpy()
    ok, e = _image_ok(lang_img, d["lang_img"])
    assert ok, ("language image", e)
    ok, e = _image_ok(outs[0]["render"].detach().cpu().numpy(), d["image"])
    assert ok, ("image", e)
    amb = d["ambiguous"].astype(bool)
    joint = bool(d["hp"][3])
    # the trainable set is the reference's: the Gaussian groups with a gradient, the field tensors
    # whose requires_grad training_setup leaves on
    want_g = {k[len("grad/"):] for k in d if k.startswith("grad/")}
    have_g = {k for k, p in tr.params.items() if p.grad is not None}
    assert have_g == want_g, (have_g, want_g)
    want_f = {k[len("fieldgrad/"):] for k in d if k.startswith("fieldgrad/")}
    have_f = {k for k in field.grads if step.field_trainable(k)}
    assert have_f == want_f, (sorted(have_f ^ want_f))
    assert ("grid.aabb" in want_f) == joint
    for k in sorted(want_g):
        ok, e = _rowwise(tr.params[k].grad.cpu().numpy(), d["grad/" + k], amb)
        assert ok, (k, e)
    for k in sorted(want_f):
        ref = d["fieldgrad/" + k]
        got = field.grads[k].cpu().numpy().reshape(ref.shape).astype(np.float64)
        err = float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))
        assert err <= 2e-3, (k, err)


def test_lang_stage_step_updates_only_trainable():
    """A full lang-stage iteration (Adam included): the language features and lang_deform move, the
    geometry, colours and the rest of the field (the box included) do not."""
    d = _load("lang")
    step, tr, field, cam, gt_img, gt_lang, mask = _setup(d)
    before = {k: v.detach().clone() for k, v in tr.params.items()}
    fbefore = {k: v.clone() for k, v in field.p.items()}
    step([cam], gt_img, iteration=1, gt_lang=gt_lang, lang_mask=mask)
    torch.cuda.synchronize()
    for k, v in tr.params.items():
        assert torch.equal(v.detach(), before[k]) == (k != "language_feature"), k
    for k, v in field.p.items():
        assert torch.equal(v, fbefore[k]) == (not k.startswith("lang_deform.")), k
    assert tr.steps["language_feature"] == 1 and tr.steps["xyz"] == 0
