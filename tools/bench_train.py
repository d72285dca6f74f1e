"""Training-glue timing (gaussian_train.GaussianTrainer -> train.hip) at the headline size: 2M
Gaussians with every group of gaussian_model.py:273-288 plus 32 language channels (91 floats per
Gaussian).  Timed with HIP events on the launch stream; beside each, torch.optim.Adam (foreach, the
reference's optimizer) on the same GPU tensors.  Prints one JSON line.

Algorithmic bytes: Adam 28 B per float (read p, g, m, v; write p, m, v); densify / prune: the
row gather reads and writes each surviving row of params + both moments + statistics once."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import torch  # noqa: E402

from gaussian_train import GaussianTrainer  # noqa: E402

SHAPES = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,),
          "language_feature": (32,)}
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3,
       "language_feature": 2.5e-3}


def timed(fn, reps=10):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    P = int(os.environ.get("BENCH_P", 2_000_000))
    g = torch.Generator(device="cuda").manual_seed(0)
    params = {n: (torch.randn((P,) + s, device="cuda", generator=g) * 0.1) for n, s in SHAPES.items()}
    params["scaling"] -= 4.0
    tr = GaussianTrainer(params, LRS)
    for n, p in tr.params.items():
        p.grad = torch.randn(p.shape, device="cuda", generator=g) * 1e-3
    floats = sum(p.numel() for p in tr.params.values())
    adam_ms = timed(tr.step)
    ref = [t.detach().clone().requires_grad_(True) for t in tr.params.values()]
    for r, p in zip(ref, tr.params.values()):
        r.grad = p.grad.clone()
    opt = torch.optim.Adam([{"params": [r], "lr": LRS[n]} for r, n in zip(ref, tr.params)], lr=0.0, eps=1e-15)
    torch_ms = timed(opt.step)

    # densification statistics, densify (about 5% cloned, 5% split) and prune (about 10% removed)
    radii = torch.randint(0, 20, (P,), device="cuda", dtype=torch.int32, generator=g)
    vgrad = torch.randn(P, 3, device="cuda", generator=g) * 2e-4
    stats_ms = timed(lambda: tr.add_densification_stats(vgrad, radii))
    tr.xyz_gradient_accum.copy_(torch.rand(P, 1, device="cuda", generator=g))
    tr.denom.fill_(1.0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ncl, nsp = tr.densify(0.9, 0.005, 1.8)       # percent_dense * 1.8 = 0.018: about half of the selected rows split
    b.record()
    torch.cuda.synchronize()
    dens_ms = a.elapsed_time(b)
    P2 = tr.P
    tr.max_radii2D.copy_(torch.randint(0, 30, (P2,), device="cuda", generator=g).float())
    a.record()
    removed = tr.prune(0.9, 0.05, 1.8, 25)
    b.record()
    torch.cuda.synchronize()
    prune_ms = a.elapsed_time(b)
    row_bytes = 4 * (3 * 91 + 1 + 1 + 1 + 3) + 1       # params + m + v, 4 stat columns, table
    print(json.dumps(dict(
        metric="training glue (train.hip) @ 2M Gaussians, 91 floats/G", gaussians=P, floats=floats,
        adam_ms=round(adam_ms, 4), adam_gbs=round(28 * floats / adam_ms / 1e6, 1),
        adam_frac_of_8tbs=round(28 * floats / adam_ms / 1e6 / 8000, 3), torch_adam_foreach_ms=round(torch_ms, 4),
        densify_stats_ms=round(stats_ms, 4), densify_ms=round(dens_ms, 3), cloned=ncl, split=nsp,
        densify_rows=P2, densify_gbs=round(row_bytes * (P + P2) / dens_ms / 1e6, 1),
        prune_ms=round(prune_ms, 3), pruned=removed, prune_gbs=round(row_bytes * (P2 + P2 - removed) / prune_ms / 1e6, 1))))


if __name__ == "__main__":
    main()
