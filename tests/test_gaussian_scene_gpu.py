"""render() and render_set() of gaussian_scene.py (the reference's gaussian_renderer.render and
render.py loop) on the GPU: the stage logic, activations and
option paths reproduce direct rasterizer calls; render_set writes the files eval/eval.py reads."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # CPU container: the driver only runs these on the MI355X box
    pytest.skip("needs a GPU", allow_module_level=True)

import diff_gaussian_rasterization as dgr  # noqa: E402
import gaussian_scene as gs  # noqa: E402
import synthetic  # noqa: E402
from deformation import DeformationField  # noqa: E402

W, H = 96, 72


def _scene(P=3000, C=6, seed=0):
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W, seed=seed, logscale_mean=-4.0)
    g = torch.Generator().manual_seed(seed)
    # raw parameters whose activations are the synthetic scene's values
    q = sc.rotations * (0.5 + torch.rand(P, 1, generator=g))
    s = gs.GaussianScene(xyz=sc.means3D, features_dc=sc.shs[:, :1].clone(), features_rest=sc.shs[:, 1:].clone(),
                         language_feature=sc.lang * 3.0, opacity=torch.logit(sc.opacities),
                         scaling=torch.log(sc.scales), rotation=q)
    return s.to("cuda")


def _cam(t=0.25):
    cam = synthetic.origin_camera(W, H, 0.6)
    cam.time = t
    return cam


def _direct(s, cam, **kw):
    rs = dgr.GaussianRasterizationSettings(H, W, cam.tanfovx, cam.tanfovy, torch.ones(3, device="cuda"), 1.0,
                                           cam.world_view_transform.cuda(), cam.full_proj_transform.cuda(), 3,
                                           cam.camera_center.cuda(), False, False, kw.pop("include_feature", True))
    return dgr.forward_native(rs, kw.pop("means3D", s.xyz), torch.sigmoid(kw.pop("opacity", s.opacity)), **kw)


def test_coarse_stage_is_the_activated_rasterizer_call():
    s, cam = _scene(), _cam()
    out = gs.render(cam, s, torch.ones(3, device="cuda"), stage="coarse-lang")
    lang = s.language_feature / (s.language_feature.norm(dim=-1, keepdim=True) + 1e-9)
    color, lang_img, radii, depth, _ = _direct(s, cam, shs=s.get_features, language_feature=lang,
                                               scales=torch.exp(s.scaling),
                                               rotations=torch.nn.functional.normalize(s.rotation))
    assert torch.equal(out["render"], color) and torch.equal(out["language_feature_image"], lang_img)
    assert torch.equal(out["radii"], radii) and torch.equal(out["visibility_filter"], radii > 0)
    assert out["viewspace_points"].requires_grad


def test_base_stage_drops_language():
    s, cam = _scene(), _cam()
    out = gs.render(cam, s, torch.ones(3, device="cuda"), stage="coarse-base", language_feature_hiddendim=6)
    assert out["language_feature_image"] is None
    ref = gs.render(cam, s, torch.ones(3, device="cuda"), stage="coarse-lang")
    assert torch.equal(out["render"], ref["render"])


def test_python_sh_and_covariance_paths():
    s, cam = _scene(), _cam()
    bg = torch.ones(3, device="cuda")
    ref = gs.render(cam, s, bg, stage="coarse-lang")["render"]
    a = gs.render(cam, s, bg, stage="coarse-lang", convert_SHs_python=True)["render"]
    b = gs.render(cam, s, bg, stage="coarse-lang", compute_cov3D_python=True)["render"]
    assert float((a - ref).abs().max()) < 1e-5
    assert float((b - ref).abs().max()) < 1e-4


def test_fine_stage_applies_the_deformation_field():
    import test_deform_gpu as td
    P = 2000
    params, res, multires, _ = td._neu3d_case(P)
    field = DeformationField({k: torch.tensor(v, dtype=torch.float32) for k, v in params.items()}, res, multires,
                             device="cuda")
    s, cam = _scene(P=P), _cam(0.4)
    s.deformation = field
    out = gs.render(cam, s, torch.ones(3, device="cuda"), stage="fine-lang")
    t = torch.full((P, 1), 0.4, device="cuda")
    lang = s.language_feature / (s.language_feature.norm(dim=-1, keepdim=True) + 1e-9)
    m, sc, r, o, sh, l, _ = field(s.xyz, s.scaling, s.rotation, s.opacity, s.get_features, lang, t)
    color, lang_img, *_ = _direct(s, cam, means3D=m, opacity=o, shs=sh, language_feature=l, scales=torch.exp(sc),
                                  rotations=torch.nn.functional.normalize(r))
    assert torch.equal(out["render"], color) and torch.equal(out["language_feature_image"], lang_img)
    assert not torch.equal(out["render"], gs.render(cam, s, torch.ones(3, device="cuda"), stage="coarse-lang")["render"])



def test_panoptic_dict_camera():
    """cam_type == "PanopticSports" (gaussian_renderer/__init__.py:46, 74-76): the dict camera's
    prebuilt settings (dataset_readers.py:491-516 setup_camera) are used as they are and its time
    drives the deformation field."""
    import test_deform_gpu as td
    P = 2000
    params, res, multires, _ = td._neu3d_case(P)
    field = DeformationField({k: torch.tensor(v, dtype=torch.float32) for k, v in params.items()}, res, multires,
                             device="cuda")
    s = _scene(P=P)
    s.deformation = field
    fx = W / (2 * 0.6)
    k = [[fx, 0.0, W / 2], [0.0, fx, H / 2], [0.0, 0.0, 1.0]]
    w2c = np.eye(4, dtype=np.float32)
    w2c[:3, 3] = [0.1, -0.05, 0.3]
    cam = gs.panoptic_camera(W, H, k, w2c, 0.7)
    rs = cam["camera"]
    assert rs.sh_degree == 0 and rs.include_feature and float(rs.bg.abs().sum()) == 0.0
    out = gs.render(cam, s, torch.ones(3, device="cuda"), stage="fine-lang", cam_type="PanopticSports")
    t = torch.full((P, 1), 0.7, device="cuda")
    lang = s.language_feature / (s.language_feature.norm(dim=-1, keepdim=True) + 1e-9)
    m, sc, r, o, sh, l, _ = field(s.xyz, s.scaling, s.rotation, s.opacity, s.get_features, lang, t)
    color, lang_img, radii, *_ = dgr.forward_native(rs, m, torch.sigmoid(o), shs=sh, language_feature=l,
                                                    scales=torch.exp(sc), rotations=torch.nn.functional.normalize(r))
    assert int((radii > 0).sum()) > 100
    assert torch.equal(out["render"], color) and torch.equal(out["language_feature_image"], lang_img)
    assert torch.equal(out["radii"], radii)
    # the dict's time, not a camera attribute, reaches the field
    cam2 = dict(cam, time=0.1)
    assert not torch.equal(gs.render(cam2, s, torch.ones(3, device="cuda"), stage="fine-lang",
                                     cam_type="PanopticSports")["render"], out["render"])

def test_render_set_writes_eval_inputs(tmp_path):
    s = _scene(C=6)
    views = [_cam(t) for t in (0.0, 0.5, 1.0)]
    fps = gs.render_set(str(tmp_path), "test", 7, views, s, torch.ones(3, device="cuda"), output_channel="lang",
                        stage="coarse-lang")
    base = tmp_path / "test_lang" / "ours_7"
    for i in range(3):
        a = np.load(base / "renders_npy" / f"{i:05d}.npy")
        assert a.shape == (H, W, 6) and a.dtype == np.float32
        assert (base / "renders" / f"{i:05d}.png").stat().st_size > 0
    assert fps > 0


def test_model_directory_load_and_render(tmp_path):
    """A model directory in the reference's layout (save_model_dir: point_cloud.ply, deformation.pth
    with the reference's keys, deformation_table / accum) loads back through load_model_dir (the
    HyperNeRF field from the ModelHiddenParams, render.py's Scene(load_iteration=-1)) and renders
    exactly what the in-memory model renders, in the fine-lang and fine-base stages."""
    P = 2500
    s = _scene(P=P, C=3)
    hidden = dict(kplanes_config={"output_coordinate_dim": 16, "resolution": [12, 10, 9, 7]}, multires=[1, 2, 4],
                  defor_depth=1, net_width=128, no_dlang=1)
    params, cfg = DeformationField.config_from_reference(
        {"deformation_net." + k: v for k, v in DeformationField.init_params(
            [12, 10, 9, 7], [1, 2, 4], torch.stack([s.xyz.max(0).values, s.xyz.min(0).values]).cpu(), depth=1,
            heads=("pos_deform", "scales_deform", "rotations_deform"), seed=5).items()}, hidden, env={})
    s.deformation = DeformationField(params, device="cuda", **cfg)
    s.extra["deformation_table"] = torch.ones(P, dtype=torch.bool)
    for it in (3000, 9000):
        gs.save_model_dir(s, str(tmp_path), it, "fine-lang")
    m, it = gs.load_model_dir(str(tmp_path), hidden, env={"language_feature_hiddendim": "3"})
    assert it == 9000 and m.deformation.heads_computed() == ["pos_deform", "scales_deform", "rotations_deform"]
    bg = torch.ones(3, device="cuda")
    for stage in ("fine-lang", "fine-base"):
        a, b = gs.render(_cam(0.6), s, bg, stage=stage), gs.render(_cam(0.6), m, bg, stage=stage)
        assert torch.equal(a["render"], b["render"]), stage
        assert torch.equal(a["radii"], b["radii"]), stage
    assert not torch.equal(gs.render(_cam(0.6), m, bg, stage="fine-lang")["render"],
                           gs.render(_cam(0.6), m, bg, stage="coarse-lang")["render"])


def test_model_directory_records_the_language_mode(tmp_path):
    """The reference selects lang_deform's residual / no_resnet / discrete modes by environment
    variables that deformation.pth does not record; save_model_dir writes them next to it
    (deformation_config.json) and load_model_dir restores the same mode without env, and refuses an
    env that contradicts it (a NORESNET field must not reload as RESIDUAL with the same weights)."""
    from deformation import LANG_NORESNET, LANG_RESIDUAL
    P = 1500
    s = _scene(P=P, C=3)
    aabb = torch.stack([s.xyz.max(0).values, s.xyz.min(0).values]).cpu()
    params = DeformationField.init_params([12, 10, 9, 7], [1, 2], aabb, seed=3, lang_mode=LANG_NORESNET, lang_dim=3)
    s.deformation = DeformationField(params, [12, 10, 9, 7], [1, 2], lang_mode=LANG_NORESNET, lang_dim=3,
                                     device="cuda")
    gs.save_model_dir(s, str(tmp_path), 100, "fine-lang")
    m, it = gs.load_model_dir(str(tmp_path))
    assert it == 100 and m.deformation.lang_mode == LANG_NORESNET
    bg = torch.ones(3, device="cuda")
    a, b = gs.render(_cam(0.3), s, bg, stage="fine-lang"), gs.render(_cam(0.3), m, bg, stage="fine-lang")
    assert torch.equal(a["language_feature_image"], b["language_feature_image"])
    with pytest.raises(ValueError, match="no_resnet"):
        gs.load_model_dir(str(tmp_path), env={})
    assert LANG_RESIDUAL != LANG_NORESNET


def test_native_activations_match_torch():
    """lsr_activate / lsr_activate_backward (the render path's exp / normalize / sigmoid) against the
    PyTorch ops and their autograd: the forward bit for bit, the gradients within float rounding;
    including a zero quaternion (the normalize clamp) and a call where only one input needs a gradient."""
    g = torch.Generator(device="cpu").manual_seed(3)
    N = 100_003
    s = (torch.randn(N, 3, generator=g) * 2).cuda()
    r = torch.randn(N, 4, generator=g).cuda()
    r[7] = 0.0
    r[8] = 1e-14
    o = (torch.randn(N, 1, generator=g) * 3).cuda()
    ds, dr, do = (torch.randn(N, k, generator=g).cuda() for k in (3, 4, 1))
    leaves = [t.clone().requires_grad_(True) for t in (s, r, o)]
    got = gs._Activate.apply(*leaves)
    torch.autograd.backward(got, (ds, dr, do))
    refl = [t.clone().requires_grad_(True) for t in (s, r, o)]
    ref = (torch.exp(refl[0]), torch.nn.functional.normalize(refl[1]), torch.sigmoid(refl[2]))
    torch.autograd.backward(ref, (ds, dr, do))
    for a, b in zip(got, ref):   # the forward in PyTorch's order of operations: bit for bit
        assert torch.equal(a, b)
    for a, b, name in zip(leaves, refl, ("scales", "rotations", "opacity")):
        if name == "rotations":   # the zero rows: 1 / clamp(1e-12), huge in both; compare the rest
            keep = torch.ones(N, dtype=torch.bool, device="cuda")
            keep[7:9] = False
            torch.testing.assert_close(a.grad[keep], b.grad[keep], rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(a.grad[7:9], b.grad[7:9], rtol=1e-5, atol=0.0)
        else:
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-7)
    # only the opacity needs a gradient: the others are not computed
    o2 = o.clone().requires_grad_(True)
    _, _, oo = gs._Activate.apply(s, r, o2)
    oo.sum().backward()
    torch.testing.assert_close(o2.grad, (torch.sigmoid(o) * (1 - torch.sigmoid(o))), rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("V", [2, 3])
def test_repeat_views_matches_torch(V):
    """lsr_repeat_rows / lsr_sum_row_blocks (render_views' inputs repeated once per view) against
    Tensor.repeat and its autograd: the copies bit for bit, the folded gradients bit for bit at two
    views (one addition either way) and within rounding at three; an input without a gradient and
    a gradient that does not reach one output."""
    g = torch.Generator(device="cpu").manual_seed(V)
    P = 50_001
    xs = [torch.randn(P, *shape, generator=g).cuda() for shape in ((3,), (4,), (1,), (16, 3))]
    a = [x.clone().requires_grad_(k != 2) for k, x in enumerate(xs)]
    b = [x.clone().requires_grad_(k != 2) for k, x in enumerate(xs)]
    got = gs.repeat_views(V, *a)
    ref = [x.repeat(V, *([1] * (x.dim() - 1))) for x in b]
    for u, w in zip(got, ref):
        assert torch.equal(u, w)
    ups = [torch.randn(u.shape, generator=g).cuda() for u in got]
    torch.autograd.backward([got[0], got[1], got[3]], [ups[0], ups[1], ups[3]])
    torch.autograd.backward([ref[0], ref[1], ref[3]], [ups[0], ups[1], ups[3]])
    assert a[2].grad is None
    for k in (0, 1, 3):
        if V == 2:
            assert torch.equal(a[k].grad, b[k].grad)
        else:
            torch.testing.assert_close(a[k].grad, b[k].grad, rtol=1e-6, atol=1e-6)


def test_split_views_matches_torch():
    """split_views (render_views' per-view blocks of the field's outputs) against Tensor.split: the
    same views, and the assembled gradients bit for bit, with a view whose gradient never arrives
    (zeros) and an output no view's gradient reaches (None)."""
    g = torch.Generator(device="cpu").manual_seed(11)
    V, P = 3, 20_011
    xs = [torch.randn(V * P, *shape, generator=g).cuda() for shape in ((3,), (16, 3), (1,))]
    a = [x.clone().requires_grad_(True) for x in xs]
    b = [x.clone().requires_grad_(True) for x in xs]
    pa = gs.split_views(V, *a, None)
    pb = [x.split(P) for x in b]
    assert pa[3] == (None,) * V
    for u, w in zip(pa[:3], pb):
        for x, y in zip(u, w):
            assert torch.equal(x, y)
    ups = {(k, v): torch.randn(pa[k][v].shape, generator=g).cuda() for k in (0, 1) for v in range(V) if (k, v) != (1, 1)}
    torch.autograd.backward([pa[k][v] for k, v in ups], list(ups.values()))
    torch.autograd.backward([pb[k][v] for k, v in ups], list(ups.values()))
    assert torch.equal(a[0].grad, b[0].grad) and torch.equal(a[1].grad, b[1].grad)
    assert a[2].grad is None and b[2].grad is None
