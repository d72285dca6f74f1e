"""Worker for tests/test_multirank_gpu.py (not a test module): one view-parallel step of the HIP
rasterizer on `world` ranks that share the box's one GPU over gloo (the RCCL product path needs one
GPU per rank; the code path above the collectives -- rank spawn, device binding, view slicing, the
bucket's SUM / radii MAX, ShardedAdam's reduce-scatter / all-gather -- is the same).

    python tests/mp_view_parallel_gpu.py --out DIR --world 2 --mode allreduce|sharded [--steps S]
                                         [--chunks C] [--views V]

world > 1: the parent starts the ranks with view_parallel.launch_ranks before it touches the GPU
(fresh interpreters) and never initialises HIP itself; every rank writes DIR/rank{r}.pt.
world == 1 runs the same function in-process (the serial reference: every view, every row).
Reference semantics: the sequential multi-view loop of train.py:242-271 with loss.backward() at
:339 and optimizer.step() at :420-421."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "4dlangsplat_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

N_VIEWS, P, W, H, C = 16, 20000, 160, 120, 32
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3,
       "language_feature": 2.5e-3}


def raw_scene(seed=5):
    """Raw parameters and the scene of their activations (render()'s exp, normalize, sigmoid, SH
    cat, language / (|language| + 1e-9)), on the CPU."""
    import torch
    import synthetic
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W, seed=seed, logscale_mean=-4.0)
    g = torch.Generator().manual_seed(seed)
    raw = dict(xyz=sc.means3D.clone(), f_dc=sc.shs[:, :1].clone(), f_rest=sc.shs[:, 1:].clone(),
               opacity=torch.logit(sc.opacities.reshape(P, 1)).clone(), scaling=torch.log(sc.scales).clone(),
               rotation=sc.rotations * (0.5 + torch.rand(P, 1, generator=g)),
               language_feature=sc.lang * (1 + 2 * torch.rand(P, 1, generator=g)))
    sc.rotations = torch.nn.functional.normalize(raw["rotation"])
    sc.lang = raw["language_feature"] / (raw["language_feature"].norm(dim=-1, keepdim=True) + 1e-9)
    return sc, raw


def run_rank(rank, world, out, mode, steps, chunks=1, n_views=N_VIEWS):
    import torch
    import torch.distributed as dist

    import diff_gaussian_rasterization as dgr
    import synthetic
    from view_parallel import GradBucket, ShardedAdam, ViewParallelStep, native_view_renderer

    torch.cuda.set_device(0)                      # every rank on the box's one card
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world and dist.get_rank() == rank
    try:
        sc_cpu, raw = raw_scene()
        sc = sc_cpu.to("cuda")
        cams = synthetic.camera_batch(n_views, W, H, tanfovx=0.6, seed=2)
        bg = torch.ones(3, device="cuda")
        settings = [dgr.GaussianRasterizationSettings(H, W, c.tanfovx, c.tanfovy, bg, 1.0,
                                                      c.world_view_transform.cuda(), c.full_proj_transform.cuda(),
                                                      3, c.camera_center.cuda(), False, False, True) for c in cams]
        g = torch.Generator(device="cpu").manual_seed(7)
        grads = [((torch.randn(3, H, W, generator=g) * 1e-2).cuda(), (torch.randn(C, H, W, generator=g) * 1e-2).cuda())
                 for _ in range(n_views)]
        up = None
        rm = 1
        rec = {}                          # step -> group -> [(global row ids, reduced gradient rows)]
        if mode == "sharded":
            up = ShardedAdam(sc, {k: v.cuda() for k, v in raw.items()}, LRS, chunks=chunks)
            rm = ShardedAdam.row_multiple(P, world, chunks=chunks)

            def hook(st, g0, valid, gr):
                for k, x in gr.items():
                    rec.setdefault(st, {}).setdefault(k, []).append(
                        (torch.arange(g0, g0 + valid), x[:valid].detach().cpu().clone()))
            up.grad_hook = hook
        b = GradBucket(P, sc.shs.shape[1], C, "cuda", densify_stats=True, row_multiple=rm)
        # chunks > 1: the chunk pipeline, the next step's preprocess waiting per row chunk
        step = ViewParallelStep(b, n_views, update=up, defer_gather=chunks > 1)
        render = native_view_renderer(sc, settings, lambda v, c, l, d: (grads[v][0], grads[v][1], None),
                                      overlap="batched", early_views=3)
        for _ in range(steps):
            step.run(render)
        step.finish()                     # the last step's all-gathers (deferred with chunks > 1)
        torch.cuda.synchronize()
        res = dict(world=world, views=list(step.views), radii=b.radii.cpu())
        if mode == "allreduce":
            res["grads"] = {k: (v.cpu().clone() if v is not None else None) for k, v in b.views.items()}
        else:
            res["rows"] = (up.r0, up.r1)
            res["grads_rec"] = {st: {k: (torch.cat([i for i, _ in v]), torch.cat([x for _, x in v]))
                                     for k, v in d.items()} for st, d in rec.items()}
            res["full"] = {k: tuple(x.cpu().clone() for x in up.full_rows(k)) for k in up.raw}
            res["act"] = {k: getattr(sc, k).cpu().clone() for k in ("means3D", "scales", "rotations", "opacities",
                                                                      "shs", "lang")}
        if out:
            torch.save(res, os.path.join(out, f"rank{rank}.pt"))
        return res
    finally:
        if world > 1:
            dist.destroy_process_group()


def _child(rank, world, out, mode, steps, chunks, n_views):
    run_rank(rank, world, out, mode, steps, chunks, n_views)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mode", choices=("allreduce", "sharded"), default="allreduce")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--views", type=int, default=N_VIEWS)
    a = ap.parse_args()
    if a.world > 1:
        from view_parallel import launch_ranks   # spawns before this process touches the GPU
        launch_ranks(a.world, _child, (a.out, a.mode, a.steps, a.chunks, a.views))
    else:
        run_rank(0, 1, a.out, a.mode, a.steps, a.chunks, a.views)


if __name__ == "__main__":
    main()
