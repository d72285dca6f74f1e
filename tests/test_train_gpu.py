"""Training-step glue on the GPU (gaussian_train.GaussianTrainer -> include/lsr_train.h) against the
reference's own GaussianModel outputs (tests/golden/train_golden.npz) and the oracle
(oracle/train_oracle.py).  Row surgery is compared bit-exactly; float updates within the stated
tolerances (Adam: 1e-6 relative, as the oracle against torch.optim.Adam)."""
import os

import numpy as np
import pytest
import torch

import train_oracle as to

pytestmark = pytest.mark.gpu

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation", "language_feature")


@pytest.fixture(scope="module")
def gold(golden_dir):
    with np.load(os.path.join(golden_dir, "train_golden.npz")) as z:
        return {k: z[k] for k in z.files}


def _cuda(a):
    return torch.tensor(np.ascontiguousarray(a)).cuda()


def _trainer(gold, prefix, moments=None, table="init_deformation_table"):
    from gaussian_train import GaussianTrainer
    tr = GaussianTrainer({n: _cuda(gold[f"{prefix}{n}"]) for n in NAMES}, dict(zip(NAMES, gold["lrs"])),
                         deformation_table=_cuda(gold[table]))
    if moments:
        for n in NAMES:
            tr.exp_avg[n].copy_(_cuda(gold[f"{moments}_m_{n}"]))
            tr.exp_avg_sq[n].copy_(_cuda(gold[f"{moments}_v_{n}"]))
            tr.steps[n] = 3
    return tr


def _close(got, ref, what):
    ref = np.asarray(ref)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6 * float(np.abs(ref).max() or 1.0), err_msg=what)


def test_adam_three_steps_match_reference(gold):
    tr = _trainer(gold, "init_")
    for s in range(3):
        for n in NAMES:
            tr[n].grad = _cuda(gold[f"grad{s}_{n}"])
        tr.step()
        tr.zero_grad()
    torch.cuda.synchronize()
    for n in NAMES:
        _close(tr[n].detach().cpu().numpy(), gold[f"adam_{n}"], n)
        _close(tr.exp_avg[n].cpu().numpy(), gold[f"adam_m_{n}"], "m " + n)
        _close(tr.exp_avg_sq[n].cpu().numpy(), gold[f"adam_v_{n}"], "v " + n)
        assert tr.steps[n] == 3


def test_adam_skips_groups_without_grad(gold):
    tr = _trainer(gold, "init_")
    tr["xyz"].grad = _cuda(gold["grad0_xyz"])
    tr.step()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tr["opacity"].detach().cpu().numpy(), gold["init_opacity"])
    assert tr.steps["xyz"] == 1 and tr.steps["opacity"] == 0


@pytest.mark.parametrize("n,offset", [(2_000_003, 0), (65_537, 1), (4096, 0), (5, 3)])
def test_adam_kernel_vs_oracle_sizes(n, offset):
    """Vector (16-byte aligned, full chunks) and scalar (unaligned / tail) paths, several steps."""
    from gaussian_train import GaussianTrainer
    rng = np.random.default_rng(n)
    base = rng.normal(size=n + offset).astype(np.float32)
    buf = _cuda(base)
    p = buf[offset:]                       # offset 1 or 3 floats: not 16-byte aligned
    tr = GaussianTrainer({"opacity": buf[:n + offset]}, {"opacity": 1e-2})
    tr.params["opacity"] = p.detach().requires_grad_(True)
    tr.exp_avg["opacity"] = torch.zeros_like(p)
    tr.exp_avg_sq["opacity"] = torch.zeros_like(p)
    pr, m, v = base[offset:].copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for s in range(3):
        g = rng.normal(size=n).astype(np.float32) * np.float32(0.1)
        tr["opacity"].grad = _cuda(g)
        tr.step()
        to.adam_step(pr, g, m, v, 1e-2, s + 1)
    torch.cuda.synchronize()
    _close(tr["opacity"].detach().cpu().numpy(), pr, "p")
    _close(tr.exp_avg["opacity"].cpu().numpy(), m, "m")
    _close(tr.exp_avg_sq["opacity"].cpu().numpy(), v, "v")


def test_densification_stats_match_reference(gold):
    tr = _trainer(gold, "init_")
    for it in range(2):
        tr.add_densification_stats(_cuda(gold[f"stats{it}_grad"]), _cuda(gold[f"stats{it}_radii"]))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tr.max_radii2D.cpu().numpy(), gold["stats_max_radii2D"])
    np.testing.assert_array_equal(tr.denom.cpu().numpy(), gold["stats_denom"])
    np.testing.assert_allclose(tr.xyz_gradient_accum.cpu().numpy(), gold["stats_accum"], rtol=1e-6, atol=0)


def test_densify_matches_reference(gold):
    tr = _trainer(gold, "adam_", moments="adam")
    tr.xyz_gradient_accum.copy_(_cuda(gold["stats_accum"]))
    tr.denom.copy_(_cuda(gold["stats_denom"]))
    tr.max_radii2D.copy_(_cuda(gold["stats_max_radii2D"]))
    maxg, pd, ext = (float(x) for x in gold["densify_args"])
    tr.percent_dense = pd
    n_clone, n_split = tr.densify(maxg, 0.005, ext, None, samples=_cuda(gold["densify_z"]))
    torch.cuda.synchronize()
    P2 = gold["dens_xyz"].shape[0]
    assert tr.P == P2 and 2 * n_split == gold["densify_z"].shape[0] and n_clone > 0
    base = P2 - 2 * n_split
    for n in NAMES:
        got = tr[n].detach().cpu().numpy()
        if n in ("xyz", "scaling"):
            np.testing.assert_array_equal(got[:base], gold[f"dens_{n}"][:base], err_msg=n)
        else:
            np.testing.assert_array_equal(got, gold[f"dens_{n}"], err_msg=n)
        np.testing.assert_array_equal(tr.exp_avg[n].cpu().numpy(), gold[f"dens_m_{n}"], err_msg="m " + n)
        np.testing.assert_array_equal(tr.exp_avg_sq[n].cpu().numpy(), gold[f"dens_v_{n}"], err_msg="v " + n)
    np.testing.assert_allclose(tr["xyz"].detach().cpu().numpy()[base:], gold["dens_xyz"][base:], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(tr["scaling"].detach().cpu().numpy()[base:], gold["dens_scaling"][base:],
                               rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(tr._deformation_table.cpu().numpy(), gold["dens_deformation_table"])
    for s in (tr.xyz_gradient_accum, tr.denom, tr.max_radii2D, tr._deformation_accum):   # postfix resets
        assert s.shape[0] == P2 and not s.any()


def test_prune_matches_reference(gold):
    tr = _trainer(gold, "dens_", moments="dens", table="dens_deformation_table")
    tr.max_radii2D.copy_(_cuda(gold["prune_in_max_radii2D"]))
    tr.xyz_gradient_accum.copy_(_cuda(gold["prune_in_accum"]))
    tr.denom.copy_(_cuda(gold["prune_in_denom"]))
    min_op, max_screen, ext = (float(x) for x in gold["prune_args"])
    removed = tr.prune(4e-4, min_op, ext, max_screen)
    torch.cuda.synchronize()
    assert removed == gold["dens_xyz"].shape[0] - gold["prune_xyz"].shape[0]
    for n in NAMES:
        np.testing.assert_array_equal(tr[n].detach().cpu().numpy(), gold[f"prune_{n}"], err_msg=n)
        np.testing.assert_array_equal(tr.exp_avg[n].cpu().numpy(), gold[f"prune_m_{n}"])
        np.testing.assert_array_equal(tr.exp_avg_sq[n].cpu().numpy(), gold[f"prune_v_{n}"])
    np.testing.assert_array_equal(tr.max_radii2D.cpu().numpy(), gold["prune_max_radii2D"])
    np.testing.assert_array_equal(tr.xyz_gradient_accum.cpu().numpy(), gold["prune_accum"])
    np.testing.assert_array_equal(tr.denom.cpu().numpy(), gold["prune_denom"])
    np.testing.assert_array_equal(tr._deformation_table.cpu().numpy(), gold["prune_deformation_table"])
    tr.reset_opacity()
    torch.cuda.synchronize()
    np.testing.assert_allclose(tr["opacity"].detach().cpu().numpy(), gold["reset_opacity"], rtol=1e-5, atol=1e-5)
    assert not tr.exp_avg["opacity"].any() and not tr.exp_avg_sq["opacity"].any()


def test_prune_without_screen_size_and_edge_cases(gold):
    tr = _trainer(gold, "dens_", table="dens_deformation_table")
    keep = to.prune_plan(gold["dens_opacity"], None, gold["dens_scaling"], 0.08, None, 3.0)
    tr.prune(4e-4, 0.08, 3.0, None)
    np.testing.assert_array_equal(tr["rotation"].detach().cpu().numpy(), gold["dens_rotation"][keep])
    # nothing selected: densify keeps every row and still resets the statistics (the clone's postfix)
    tr.xyz_gradient_accum.fill_(1.0)
    tr.denom.fill_(1.0)
    P = tr.P
    assert tr.densify(1e9, 0.0, 3.0) == (0, 0)
    assert tr.P == P and not tr.xyz_gradient_accum.any()
    # everything pruned, then the empty model
    assert tr.prune(0, 2.0, 3.0, None) == P and tr.P == 0
    assert tr.prune(0, 2.0, 3.0, None) == 0
    assert tr.densify(0.0, 0.0, 3.0) == (0, 0)


@pytest.mark.parametrize("dtype,cols,offset", [(torch.uint8, 1, 0), (torch.float32, 3, 0), (torch.float32, 4, 0),
                                               (torch.float32, 45, 0), (torch.float32, 3, 1), (torch.int16, 3, 0)])
def test_gather_rows_bit_exact(dtype, cols, offset):
    import ctypes
    from diff_gaussian_rasterization import _lib
    L = _lib.load()
    rng = np.random.default_rng(cols)
    P, n_out, zf = 10_007, 14_000, 12_500
    src_all = torch.randint(0, 100, (P * cols + offset,), dtype=torch.int32).to(dtype).cuda()
    src = src_all[offset:].view(P, cols)
    idx = rng.integers(0, P, size=n_out).astype(np.int32)
    dst = torch.full((n_out, cols), 7, dtype=dtype).cuda()
    rt = _lib.RowTensor()
    rt.src, rt.dst, rt.row_bytes, rt.zero_from = src.data_ptr(), dst.data_ptr(), cols * src.element_size(), zf
    idx_t = _cuda(idx)
    _lib.check(L.lsr_gather_rows(1, ctypes.byref(rt), ctypes.c_void_p(idx_t.data_ptr()), n_out, None), "gather")
    torch.cuda.synchronize()
    ref = src.cpu().numpy()[idx]
    ref[zf:] = 0
    np.testing.assert_array_equal(dst.cpu().numpy(), ref)
