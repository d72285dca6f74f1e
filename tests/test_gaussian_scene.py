"""Scene I/O and render-path helpers (4dlangsplat_amd/gaussian_scene.py) on
the CPU: the reference's PLY attribute list and round trip, foreign PLY encodings, eval_sh and
the Python covariance against golden vectors from the reference's own code, PNG output."""
import os

import numpy as np
import pytest
import torch

import gaussian_scene as gs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scene(P=300, C=3, deg=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    n = (deg + 1) ** 2
    return gs.GaussianScene(xyz=torch.randn(P, 3, generator=g), features_dc=torch.randn(P, 1, 3, generator=g),
                            features_rest=torch.randn(P, n - 1, 3, generator=g),
                            language_feature=torch.randn(P, C, generator=g), opacity=torch.randn(P, 1, generator=g),
                            scaling=torch.randn(P, 3, generator=g) - 4, rotation=torch.randn(P, 4, generator=g),
                            max_sh_degree=deg, active_sh_degree=deg)


def test_attribute_list_is_the_references():
    # gaussian_model.py:331-345 for SH degree 3 and 3 language channels
    want = (["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"] + [f"f_rest_{i}" for i in range(45)]
            + ["f_lang_0", "f_lang_1", "f_lang_2", "opacity", "scale_0", "scale_1", "scale_2",
               "rot_0", "rot_1", "rot_2", "rot_3"])
    assert _scene().attribute_names() == want


@pytest.mark.parametrize("C,deg", [(3, 3), (6, 3), (32, 3), (3, 1)])
def test_ply_round_trip(tmp_path, C, deg):
    s = _scene(C=C, deg=deg)
    p = str(tmp_path / "point_cloud.ply")
    s.save_ply(p)
    t = gs.GaussianScene.load_ply(p, max_sh_degree=deg)
    for name in ("xyz", "features_dc", "features_rest", "language_feature", "opacity", "scaling", "rotation"):
        assert torch.equal(getattr(s, name), getattr(t, name)), name
    with open(p, "rb") as f:
        head = f.read(200)
    assert head.startswith(b"ply\nformat binary_little_endian 1.0\nelement vertex 300\n")
    with pytest.raises(ValueError, match="f_rest"):
        gs.GaussianScene.load_ply(p, max_sh_degree=deg + 1 if deg < 3 else 2)


def test_reads_ascii_and_big_endian(tmp_path):
    names = ["x", "y", "z", "opacity"]
    cols = np.arange(12, dtype=np.float32).reshape(3, 4) / 7
    a = tmp_path / "a.ply"
    a.write_text("ply\nformat ascii 1.0\ncomment x\nelement vertex 3\n" + "".join(f"property float {n}\n" for n in names)
                 + "end_header\n" + "".join(" ".join(repr(float(v)) for v in r) + "\n" for r in cols))
    b = tmp_path / "b.ply"
    with open(b, "wb") as f:
        f.write(("ply\nformat binary_big_endian 1.0\nelement vertex 3\n" + "".join(f"property float {n}\n" for n in names)
                 + "end_header\n").encode())
        f.write(cols.astype(">f4").tobytes())
    for p in (a, b):
        v = gs.read_ply_vertices(str(p))
        for i, n in enumerate(names):
            np.testing.assert_array_equal(v[n].astype(np.float32), cols[:, i])


def test_eval_sh_matches_reference_golden():
    d = np.load(os.path.join(ROOT, "tests", "golden", "sh_golden.npz"))
    for deg in range(4):
        sh = torch.tensor(d[f"sh_{deg}"]).transpose(1, 2)           # [P, 3, 16] as render() views it
        dirs = torch.tensor(d[f"pos_{deg}"] - d[f"campos_{deg}"])
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(gs.eval_sh(deg, sh, dirs) + 0.5, 0.0)
        np.testing.assert_allclose(rgb.numpy(), d[f"rgb_{deg}"], rtol=0, atol=2e-6)


def test_covariance_matches_reference_golden():
    d = np.load(os.path.join(ROOT, "tests", "golden", "cov3d.npz"))
    cov = gs._covariance(torch.tensor(d["scales"]), float(d["mod"]), torch.tensor(d["rotations"]))
    np.testing.assert_allclose(cov.numpy(), d["cov"], rtol=1e-5, atol=2e-8)


def test_png_writer(tmp_path):
    from PIL import Image
    img = (np.random.default_rng(0).uniform(0, 1, (13, 17, 3)))
    p = str(tmp_path / "x.png")
    gs.write_png(p, gs.to8b(img))
    np.testing.assert_array_equal(np.asarray(Image.open(p)), gs.to8b(img))


# ---- trained model directories (scene/__init__.py:35-37,85-101; gaussian_model.py:352-370) ------
def _reference_state_dict(config, seed=0):
    """A deform_network state dict with the keys and shapes the reference builds
    (tests/golden/deform_state_dict_layout.json, from the reference module), random values."""
    import json
    layout = json.load(open(os.path.join(ROOT, "tests", "golden", "deform_state_dict_layout.json")))[config]
    g = torch.Generator().manual_seed(seed)
    return {k: torch.randn(*shape, generator=g) for k, shape in layout.items()}


HYPERNERF = dict(kplanes_config={"grid_dimensions": 2, "input_coordinate_dim": 4, "output_coordinate_dim": 16,
                                 "resolution": [64, 64, 64, 150]},
                 multires=[1, 2, 4], defor_depth=1, net_width=128, no_dlang=1)   # arguments/hypernerf/default.py


def test_model_directory_round_trip(tmp_path):
    """A directory in the reference's layout (several stages and iterations): the largest iteration of
    the requested stage is found, the PLY, deformation.pth (weights_only), deformation_table.pth and
    deformation_accum.pth are read, and the HyperNeRF field's parameters are exactly the state
    dict's computed modules (the unused ones the reference always builds are skipped)."""
    from deformation import DeformationField
    root = tmp_path / "model"
    sd = _reference_state_dict("hypernerf")
    for stage, it in (("coarse-base", 3000), ("fine-lang", 7000), ("fine-lang", 10000), ("fine-base", 14000)):
        d = root / "point_cloud" / f"{stage}_iteration_{it}"
        d.mkdir(parents=True)
        _scene(P=257, seed=it).save_ply(str(d / "point_cloud.ply"))
        torch.save(sd, str(d / "deformation.pth"))
        if it == 10000:
            torch.save(torch.arange(257) % 3 > 0, str(d / "deformation_table.pth"))
            torch.save(torch.full((257, 3), 0.5), str(d / "deformation_accum.pth"))
    assert gs.search_for_max_iteration(str(root / "point_cloud"), "fine-lang") == 10000
    assert gs.search_for_max_iteration(str(root / "point_cloud"), "fine-base") == 14000
    scene, state, it = gs.read_model_dir(str(root))
    assert it == 10000 and scene.P == 257
    assert torch.equal(scene.xyz, _scene(P=257, seed=10000).xyz)
    assert torch.equal(scene.extra["deformation_table"], torch.arange(257) % 3 > 0)
    assert float(scene.extra["deformation_accum"].sum()) == 257 * 3 * 0.5
    scene7, _, it7 = gs.read_model_dir(str(root), load_iteration=7000)
    assert it7 == 7000 and bool(scene7.extra["deformation_table"].all())   # defaults without the files
    params, cfg = DeformationField.config_from_reference(state, HYPERNERF, env={"language_feature_hiddendim": "3"})
    assert cfg["multires"] == [1, 2, 4] and cfg["depth"] == 1 and cfg["lang_mode"] == 0
    heads = sorted({k.split(".")[0] for k in params if not k.startswith(("grid", "feature_out"))})
    assert heads == ["pos_deform", "rotations_deform", "scales_deform"]    # no_do, no_dshs: the defaults
    assert len([k for k in params if k.startswith("grid.grids")]) == 18 and "grid.aabb" in params
    for k, v in params.items():
        assert torch.equal(v, sd["deformation_net." + k])


def test_reference_config_is_strict():
    from deformation import DeformationField
    sd = _reference_state_dict("neu3d")
    neu3d = dict(kplanes_config={"output_coordinate_dim": 16, "resolution": [64, 64, 64, 150]}, multires=[1, 2],
                 defor_depth=0, net_width=128, no_do=False, no_dshs=False, no_dlang=1)
    params, cfg = DeformationField.config_from_reference(sd, neu3d, env={})
    assert sum(k.endswith(".3.weight") for k in params) == 5
    # the language modes come from no_dlang and the environment, as the reference reads them
    _, c = DeformationField.config_from_reference(sd, dict(neu3d, no_dlang=0), env={"language_feature_hiddendim": "3"})
    assert c["lang_mode"] == 1
    _, c = DeformationField.config_from_reference(sd, dict(neu3d, no_dlang=0), env={"no_resnet": "t"})
    assert c["lang_mode"] == 2
    _, c = DeformationField.config_from_reference(sd, neu3d, env={"use_discrete_lang_f": "t", "centers_num": "3"})
    assert c["lang_mode"] == 3 and c["centers"] == 3
    with pytest.raises(ValueError, match="feature_out.2"):    # a deeper network than the config says
        DeformationField.config_from_reference(dict(sd, **{"deformation_net.feature_out.2.weight": torch.zeros(1)}),
                                               neu3d, env={})
    with pytest.raises(ValueError, match="outside"):
        DeformationField.config_from_reference(dict(sd, stray=torch.zeros(1)), neu3d, env={})
    for bad in (dict(static_mlp=True), dict(empty_voxel=True), dict(grid_pe=2), dict(net_width=64)):
        with pytest.raises(ValueError):
            DeformationField.config_from_reference(sd, dict(neu3d, **bad), env={})
    with pytest.raises(ValueError, match="use_tribute_dlang"):
        DeformationField.config_from_reference(sd, neu3d, env={"use_tribute_dlang": "t"})
