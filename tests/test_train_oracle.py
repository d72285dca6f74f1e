"""The training-glue oracle (oracle/train_oracle.py) against the reference's own GaussianModel
outputs (tests/golden/train_golden.npz, made by tests/golden/make_train_golden.py) and
torch.optim.Adam; plus the host module's learning-rate schedule (CPU)."""
import os

import numpy as np
import pytest
import torch

import train_oracle as to

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation", "language_feature")


@pytest.fixture(scope="module")
def gold(golden_dir):
    with np.load(os.path.join(golden_dir, "train_golden.npz")) as z:
        return {k: z[k] for k in z.files}


def oracle_adam(gold):
    lrs = dict(zip(NAMES, gold["lrs"]))
    st = {}
    for n in NAMES:
        p = gold[f"init_{n}"].copy()
        m, v = np.zeros_like(p), np.zeros_like(p)
        for s in range(3):
            to.adam_step(p, gold[f"grad{s}_{n}"], m, v, lrs[n], s + 1)
        st[n] = (p, m, v)
    return st


def test_adam_matches_reference_torch_adam(gold):
    for n, (p, m, v) in oracle_adam(gold).items():
        # element rounding differs by an ulp where m nearly cancels: atol relative to the tensor's scale
        for got, key in ((m, "adam_m_"), (v, "adam_v_"), (p, "adam_")):
            ref = gold[key + n]
            np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6 * float(np.abs(ref).max()), err_msg=key + n)


def test_adam_matches_torch_adam_single_group():
    """Also against torch.optim.Adam directly, 20 steps, a learning-rate change midway."""
    rng = np.random.default_rng(0)
    p0 = rng.normal(size=(257, 5)).astype(np.float32)
    t = torch.nn.Parameter(torch.tensor(p0))
    opt = torch.optim.Adam([{"params": [t], "lr": 1e-3}], lr=0.0, eps=1e-15)
    p, m, v = p0.copy(), np.zeros_like(p0), np.zeros_like(p0)
    for s in range(20):
        lr = 1e-3 if s < 10 else 3e-4
        opt.param_groups[0]["lr"] = lr
        g = rng.normal(size=p0.shape).astype(np.float32) * np.float32(0.01)
        t.grad = torch.tensor(g)
        opt.step()
        to.adam_step(p, g, m, v, lr, s + 1)
    np.testing.assert_allclose(p, t.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_densify_stats(gold):
    P = gold["init_xyz"].shape[0]
    mr, acc, den = np.zeros(P, np.float32), np.zeros((P, 1), np.float32), np.zeros((P, 1), np.float32)
    for it in range(2):
        to.densify_stats(gold[f"stats{it}_radii"], gold[f"stats{it}_grad"], mr, acc[:, 0], den[:, 0])
    np.testing.assert_array_equal(mr, gold["stats_max_radii2D"])
    np.testing.assert_array_equal(den, gold["stats_denom"])
    np.testing.assert_allclose(acc, gold["stats_accum"], rtol=1e-6, atol=0)


def test_densify_plan_and_split(gold):
    """Row map of clone + split == the reference's cat-then-prune; split rows from the same draws."""
    maxg, pd, ext = (float(x) for x in gold["densify_args"])
    st = oracle_adam(gold)
    idx, kept, ncl, nsp = to.densify_plan(gold["stats_accum"][:, 0], gold["stats_denom"][:, 0],
                                          gold["adam_scaling"], maxg, pd, ext)
    assert len(idx) == gold["dens_xyz"].shape[0] and nsp * 2 == gold["densify_z"].shape[0] and ncl > 0 and nsp > 0
    base = kept + ncl
    for n in NAMES:
        src = gold[f"adam_{n}"]
        got = src[idx]
        if n in ("xyz", "scaling"):
            np.testing.assert_array_equal(got[:base], gold[f"dens_{n}"][:base], err_msg=n)
        else:
            np.testing.assert_array_equal(got, gold[f"dens_{n}"], err_msg=n)
        # moments: copied for rows kept, zero for appended rows
        for k in ("m", "v"):
            ref = gold[f"dens_{k}_{n}"]
            np.testing.assert_array_equal(gold[f"adam_{k}_{n}"][idx[:kept]], ref[:kept])
            assert not ref[kept:].any()
    np.testing.assert_array_equal(gold["init_deformation_table"][idx], gold["dens_deformation_table"])
    nx, ns = to.split_rows(gold["adam_xyz"], gold["adam_scaling"], gold["adam_rotation"], idx[base:],
                           gold["densify_z"])
    np.testing.assert_allclose(nx, gold["dens_xyz"][base:], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ns, gold["dens_scaling"][base:], rtol=1e-6, atol=1e-6)
    del st


def test_prune_plan(gold):
    min_op, max_screen, ext = (float(x) for x in gold["prune_args"])
    keep = to.prune_plan(gold["dens_opacity"], gold["prune_in_max_radii2D"], gold["dens_scaling"], min_op, max_screen,
                         ext)
    for n in NAMES:
        np.testing.assert_array_equal(gold[f"dens_{n}"][keep], gold[f"prune_{n}"], err_msg=n)
        np.testing.assert_array_equal(gold[f"dens_m_{n}"][keep], gold[f"prune_m_{n}"])
    np.testing.assert_array_equal(gold["prune_in_max_radii2D"][keep], gold["prune_max_radii2D"])
    np.testing.assert_array_equal(gold["prune_in_accum"][keep], gold["prune_accum"])
    np.testing.assert_array_equal(gold["dens_deformation_table"][keep], gold["prune_deformation_table"])


def test_reset_opacity(gold):
    np.testing.assert_allclose(to.reset_opacity(gold["prune_opacity"]), gold["reset_opacity"], rtol=1e-5, atol=1e-5)
    assert not gold["reset_m"].any() and not gold["reset_v"].any()


def test_expon_lr_schedule(gold):
    """oracle and the product module's get_expon_lr_func against the reference's values."""
    from gaussian_train import get_expon_lr_func
    for cfg, row in zip(gold["lr_cfgs"], gold["lr_values"]):
        a, b, c, d, e = cfg
        f = get_expon_lr_func(lr_init=a, lr_final=b, lr_delay_steps=int(c), lr_delay_mult=d, max_steps=int(e))
        for s, ref in zip(gold["lr_steps"], row):
            assert to.expon_lr(int(s), a, b, int(c), d, int(e)) == pytest.approx(ref, rel=1e-12, abs=0)
            assert f(int(s)) == pytest.approx(ref, rel=1e-12, abs=0)
