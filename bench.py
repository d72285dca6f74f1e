#!/usr/bin/env python3
"""bench.py -- rasterizer fwd+bwd frames/s at 2M Gaussians, 1352x1014, 32 language channels.

Workload (BASELINE.json configs[2] per GPU, configs[3] across GPUs): the synthetic S2M scene of
SURVEY.md 8(d) (seeded; the Neu3D checkpoints are not available offline), replicated on every
rank; each rank renders V views per step (default 8 = the 64-view batch of configs[3] over 8
GPUs), forward + full backward of the rasterizer for each view, accumulating all Gaussian
gradients in one flat fp32 buffer (means3D, scales, rotations, opacities, SH, language
features and the means2D gradient train.py:352-354 feeds to densification = 62 + C floats per
Gaussian) and the per-Gaussian radii MAX; with N > 1 ranks the buffer is SUM all-reduced (RCCL)
and the radii MAX all-reduced once per step.  `--gpus N` without torchrun starts the N ranks
itself (view_parallel.launch_ranks).  Upstream gradients dL/dcolor, dL/dlanguage are fixed seeded tensors, so the
step is the rasterizer alone.  Inputs are resident in HBM before the timed region.

value = frames (views) rendered fwd+bwd by all ranks / max over ranks of the timed wall time.
roofline: the dominant kernel (largest event-timed phase of one untimed all-phase step),
algorithmic bytes per launch (the per-phase formulas below) / its mean launch time
(hipEvents on the launch stream, recorded live over the timed region; only that phase carries
events there, the per-phase breakdown comes from the untimed step).
cpu_baseline: the C oracle (oracle/, OpenMP) on 3 headline frames fwd+bwd, rank 0 only; its
configs0 entry: the oracle on BASELINE configs[0] at full size (50k, 400x400, RGB only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "4dlangsplat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def phase_bytes(phase, P, Pvis, K, npix, ntiles, C, M=16, accumulate=True, V=1, Pvis_sum=None, Pany=None,
                means2D=False):
    """Algorithmic HBM bytes of one launch of each phase (each byte counted once).
    preprocess_bwd_views covers V views: Pvis_sum = visible Gaussians summed over them, Pany =
    Gaussians visible in at least one; means2D: the screen-space gradient rows are written too."""
    rec = 4 + 8 + 16 + 16 + 4 * C          # id + xy + conic/opacity + rgb/depth + language row
    if phase == "preprocess":              # inputs; radii, radius, tiles, key, rect, sort ids; screen
        return (P * (12 + 12 + 16 + 4 + 4 * 3 * M) + P * (4 + 4 + 4 + 4 + 8 + 4)   # records; zeroed
                + Pvis * (8 + 16 + 16 + 1 + 64))                                   # accumulator rows
    if phase == "depth_sort":              # pass 1 over all keys, passes 2-4 over the visible (culled
        n = [P, Pvis, Pvis, Pvis]           # dropped); the last pass writes ids + the rect gather
        return (sum(ni * (4 + 16) for ni in n) - Pvis * 4 + Pvis * (8 + 8 + 4)   # (rect, rect_sorted,
                + P * 4)                    # counts) instead of keys; the culled ranks' zero counts
    if phase == "instance_scan":           # exclusive scan of the depth-ranked counts
        return P * (4 + 4)
    if phase == "emit":                    # order, offsets, counts, rect (depth order) -> keys, values
        return P * (4 + 4 + 4 + 8) + K * 8
    if phase == "tile_sort":               # two passes; the last one also makes the tile ranges
        return 2 * K * (4 + 16) + ntiles * 8
    if phase == "tile_ranges":
        return K * 4 + ntiles * 8
    if phase == "render_fwd":
        return K * rec + ntiles * 12 + npix * (4 * (3 + C + 1) + 8)
    if phase == "render_bwd":
        return K * rec + ntiles * 12 + npix * (4 * (3 + C + 1) + 8) + Pvis * (8 + 16 + 12 + 4 + 4 * C)
    if phase == "preprocess_bwd":          # visible rows: inputs + screen grads; gradient rows (RMW if accumulating)
        grads = 4 * (3 + 3 + 4 + 1 + 3 * M)
        return P * 4 + Pvis * (12 + 12 + 16 + 4 * 3 * M + 1 + 48) + (2 * Pvis * grads if accumulate else P * grads)
    if phase == "preprocess_bwd_views":    # per view: tiles, and for its visible rows clamped + screen sums;
        grads = 4 * (3 + 3 + 4 + 1 + 3 * M + (3 if means2D else 0))  # once: rows of the visible-anywhere set; grads
        return (V * P * 4 + Pvis_sum * (1 + 48) + Pany * (12 + 12 + 16 + 4 * 3 * M)   # RMW, or all P written
                + (2 * Pany * grads if accumulate else P * grads))
    return 0


def cpu_baseline(scene, cams, C, threads):
    """The C oracle (oracle/lsr_oracle.c) on the headline workload: fwd + full bwd of each camera."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    tf = tb = 0.0
    for cam in cams:
        s = oracle.OracleSettings(cam.image_height, cam.image_width, cam.tanfovx, cam.tanfovy, np.ones(3, np.float32),
                                  1.0, cam.world_view_transform.numpy(), cam.full_proj_transform.numpy(), 3,
                                  cam.camera_center.numpy(), True)
        H, W = cam.image_height, cam.image_width
        rng = np.random.default_rng(0)
        gc = (rng.normal(size=(3, H, W)) * 1e-3).astype(np.float32)
        gl = (rng.normal(size=(C, H, W)) * 1e-3).astype(np.float32)
        args = dict(shs=scene.shs.numpy(), lang=scene.lang.numpy(), scales=scene.scales.numpy(),
                    rotations=scene.rotations.numpy(), nthreads=threads)
        t0 = time.perf_counter()
        r = oracle.forward(s, scene.means3D.numpy(), scene.opacities.numpy(), **args)
        t1 = time.perf_counter()
        r.backward(gc, gl, None, nthreads=threads)
        t2 = time.perf_counter()
        r.close()
        tf += t1 - t0
        tb += t2 - t1
    return tf + tb, tf, tb


def configs0_leg(threads, dev, reps=20):
    """BASELINE configs[0] at full size: 50k random Gaussians, one 400x400 camera,
    RGB only (include_feature=False, a zeros language tensor as gaussian_renderer/__init__.py:96-99
    passes), fwd + full bwd.  The C oracle on the host cores, and the same frame through liblsr.so on
    the GPU for reference (device-resident inputs, per-call workspaces, as forward_native /
    backward_native allocate them).  Returns (cpu dict, gpu frames/s)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import synthetic
    import diff_gaussian_rasterization as dgr
    W = H = 400
    sc = synthetic.make_scene(50_000, C=3, tanfovx=0.6, tanfovy=0.6, seed=0)
    sc.lang = torch.zeros_like(sc.lang)
    cam = synthetic.origin_camera(W, H, tanfovx=0.6, tanfovy=0.6)
    s = oracle.OracleSettings(H, W, cam.tanfovx, cam.tanfovy, np.ones(3, np.float32), 1.0,
                              cam.world_view_transform.numpy(), cam.full_proj_transform.numpy(), 3,
                              cam.camera_center.numpy(), False)
    gc = (np.random.default_rng(7).normal(size=(3, H, W)) * 1e-3).astype(np.float32)
    args = dict(shs=sc.shs.numpy(), lang=sc.lang.numpy(), scales=sc.scales.numpy(), rotations=sc.rotations.numpy(),
                nthreads=threads)
    tf = tb = 0.0
    n = 0
    t_start = time.perf_counter()
    while n < reps or time.perf_counter() - t_start < 2.0:
        t0 = time.perf_counter()
        r = oracle.forward(s, sc.means3D.numpy(), sc.opacities.numpy(), **args)
        t1 = time.perf_counter()
        r.backward(gc, None, None, nthreads=threads)
        t2 = time.perf_counter()
        r.close()
        tf += t1 - t0
        tb += t2 - t1
        n += 1
        if n >= 200:
            break
    cpu = dict(value=round(n / (tf + tb), 3), unit="frames/s", cores=threads, kind="port",
               sample=f"BASELINE configs[0]: 50k Gaussians, 400x400, 3-ch RGB, include_feature=False, {n} frames "
                      f"fwd {tf / n * 1e3:.1f} ms + bwd {tb / n * 1e3:.1f} ms per frame, C oracle, OpenMP {threads} threads")
    gs = sc.to(dev)
    rs = dgr.GaussianRasterizationSettings(H, W, cam.tanfovx, cam.tanfovy, torch.ones(3, device=dev), 1.0,
                                           cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), 3,
                                           cam.camera_center.to(dev), False, False, False)
    gcd = torch.tensor(gc, device=dev)

    def frame():
        *_, st = dgr.forward_native(rs, gs.means3D, gs.opacities, shs=gs.shs, language_feature=gs.lang,
                                    scales=gs.scales, rotations=gs.rotations)
        dgr.backward_native(st, gcd, None, None)

    for _ in range(3):
        frame()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(50):
        frame()
    torch.cuda.synchronize(dev)
    return cpu, round(50 / (time.perf_counter() - t0), 1)


def host_cpu():
    """Host cores the CPU baseline may use (the process's affinity, capped by a cgroup CPU quota)
    and the host's description: os.cpu_count(), lscpu model, threads per core."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except Exception:
        pass
    info = dict(os_cpu_count=os.cpu_count(), affinity=n, cgroup_quota=quota)
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Thread(s) per core", "Socket(s)", "Core(s) per socket"):
                info[k.strip().lower().replace("(s)", "s").replace(" ", "_")] = v.strip()
    except Exception:
        pass
    return min(n, quota) if quota else n, info


def _early_views(text):
    parts = [int(x) for x in str(text).split(",") if x.strip()]
    if not parts or any(x < 0 for x in parts):
        raise argparse.ArgumentTypeError("--early-views: e or e,s1,s2,... (non-negative)")
    return parts[0] if len(parts) == 1 else tuple(parts)


def _n_binning_batches(early, V):
    """Binning batches (= compositor launch pairs) of a V-view step under --early-views."""
    sizes = tuple(early) if isinstance(early, tuple) else (early,)
    if not 0 < sizes[0] < V:
        return 1
    cuts = [sizes[0]]
    for n in sizes[1:]:
        if cuts[-1] + n < V:
            cuts.append(cuts[-1] + n)
    return len(cuts) + 1


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--views", type=int, default=8, help="views per GPU per step")
    ap.add_argument("--gaussians", type=int, default=2_000_000)
    ap.add_argument("--channels", type=int, default=32)
    ap.add_argument("--width", type=int, default=1352)
    ap.add_argument("--height", type=int, default=1014)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads (0 = every core available to the process)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=3, help="headline frames timed on the CPU oracle")
    ap.add_argument("--no-configs0", action="store_true",
                    help="skip cpu_baseline.configs0 (BASELINE configs[0]: 50k, 400x400, RGB only, on the oracle)")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-densify-stats", action="store_true",
                    help="diagnostic: no means2D gradient / radii MAX in the step (train.py:350-352 needs them)")
    ap.add_argument("--early-views", type=_early_views, default=2,
                    help="batched pipeline: views binned before compositing starts (2: same-box 985 vs 976 "
                         "frames/s for 3 over 8 alternating runs, profiles/r05_g/ab_early_views.txt); the rest bin on a side stream "
                         "while they composite (0: all binned first); 'e,s1,...': side binning batches of s1, ... "
                         "views and one of the rest, each composited as soon as it is binned")
    ap.add_argument("--no-overlap", action="store_true", help="diagnostic: no side stream (uncontended phase times)")
    ap.add_argument("--main-priority", type=int, default=0,
                    help="run the step on a stream of this torch priority (negative = higher than the side stream's "
                         "binning; 0: the current stream)")
    ap.add_argument("--side-priority", type=int, default=0,
                    help="torch stream priority of the side-stream binning (negative = higher)")
    ap.add_argument("--side-after-binning", action="store_true",
                    help="diagnostic: the side-stream binning waits for the early views' binning too")
    ap.add_argument("--no-wait-fill", action="store_true",
                    help="diagnostic: zero the bucket and split the language rows before the preprocess "
                         "instead of while the host waits for the instance counts")
    ap.add_argument("--fill-on-side", action="store_true",
                    help="the language split, bucket zeroing and radii MAX on the side stream beside the early "
                         "views' binning instead of on the main stream before it")
    ap.add_argument("--no-order-on-side", dest="order_on_side", action="store_false",
                    help="depth-sort every view before the early views' binning (default: the views past "
                         "--early-views are depth-sorted on the side stream, so the early views' binning waits "
                         "for their own depth order only: 0.43 ms shorter head, profiles/r05_early)")
    ap.add_argument("--order-on-side", dest="order_on_side", action="store_true", help="the default (kept for scripts)")
    ap.add_argument("--binning", choices=("sort", "bucket"), default="sort",
                    help="per-tile lists by a depth sort of the Gaussians + a stable 13-bit tile sort of the "
                         "instances (sort), or by bucketing the instances by tile and sorting each bucket in LDS "
                         "(bucket); same lists")
    ap.add_argument("--per-view-composite", action="store_true",
                    help="one compositor launch per view instead of one per binning batch of views")
    ap.add_argument("--pipeline", choices=("batched", "lookahead", "side"), default=None,
                    help="view pipelining: the step's forward phase 1 + binning of all views as one batch (batched, "
                         "default), next view's preprocess queued ahead on one stream with a deferred count "
                         "(lookahead), or run on a side stream (side)")
    ap.add_argument("--single-view-steps", type=int, default=10,
                    help="secondary figure: single-view forward_native + backward_native frames timed (0: skip)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun: start one rank per GPU here, before this process touches the GPU
        from view_parallel import launch_ranks
        launch_ranks(args.gpus, _rank_main, (args,))
        return
    run(args)


def _rank_main(rank, world, args):
    run(args)


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # LSR_BENCH_BACKEND=gloo with LSR_BENCH_SHARE_DEVICE=1 rehearses the N > 1 path on a one-GPU box
    # (ranks share the card, the bucket all-reduce goes through gloo); the product path is RCCL
    backend = os.environ.get("LSR_BENCH_BACKEND", "nccl")
    dev_index = local_rank % max(1, torch.cuda.device_count()) if os.environ.get("LSR_BENCH_SHARE_DEVICE") else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    pg_ranks = 1
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        pg_ranks = dist.get_world_size()

    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _lib
    import synthetic
    if args.pipeline is None:
        args.pipeline = "batched"

    P, C, W, H, V = args.gaussians, args.channels, args.width, args.height, args.views
    tanfovx = 0.6
    scene_cpu = synthetic.make_scene(P, C=C, tanfovx=tanfovx, tanfovy=tanfovx * H / W)
    scene = scene_cpu.to(dev)
    from view_parallel import GradBucket, ViewParallelStep, native_view_renderer
    M = scene.shs.shape[1]
    bucket = GradBucket(P, M, C, dev, densify_stats=not args.no_densify_stats)  # flat grads, 62 + C floats (means2D
                                                           # for the densification statistics), radii MAX
    dp = ViewParallelStep(bucket, world * V)               # this rank's slice of the world*V batch
    all_cams = synthetic.camera_batch(world * V, W, H, tanfovx=tanfovx, seed=1)
    bg = torch.ones(3, device=dev)
    settings = {v: dgr.GaussianRasterizationSettings(H, W, c.tanfovx, c.tanfovy, bg, 1.0,
                                                     c.world_view_transform.to(dev), c.full_proj_transform.to(dev),
                                                     3, c.camera_center.to(dev), False, False, True)
                for v, c in enumerate(all_cams) if v in dp.views}
    g = torch.Generator(device="cpu").manual_seed(123)
    gcol = (torch.randn(3, H, W, generator=g) * 1e-3).to(dev)
    glang = (torch.randn(C, H, W, generator=g) * 1e-3).to(dev)
    render = native_view_renderer(scene, settings, lambda v, color, lang, depth: (gcol, glang, None),
                                  overlap=False if args.no_overlap else (True if args.pipeline == "side"
                                                                         else args.pipeline),
                                  early_views=args.early_views, composite_batch=not args.per_view_composite,
                                  side_priority=args.side_priority, side_from_preprocess=not args.side_after_binning,
                                  split_behind_counts=not args.no_wait_fill, fill_on_side=args.fill_on_side,
                                  order_on_side=args.order_on_side, tile_bucket=args.binning == "bucket")
    Ks = []

    def render_view(v, b):
        r = render(v, b)
        Ks.append(render.last_num_rendered)
        return r

    if hasattr(render, "render_batch"):                    # one compositor launch per binning batch

        def render_batch(views, b, before_wait=None):
            r = render.render_batch(views, b, before_wait=before_wait)
            Ks.extend(render.render_batch.last_num_rendered)
            render_batch.radii_reduced = render.render_batch.radii_reduced
            return r
        render_batch.before_wait = not args.no_wait_fill
        render_view.render_batch = render_batch
    if hasattr(render, "flush"):                           # batched backward of the step's views
        render_view.flush = render.flush
    render_view.begin_step, render_view.end_step = render.begin_step, render.end_step   # the step's views

    main_stream = torch.cuda.Stream(device=dev, priority=args.main_priority) if args.main_priority else None

    def step():
        if main_stream is None:
            dp.run(render_view)                            # fwd+bwd per view, SUM all-reduce (RCCL) if world > 1
        else:                                              # the step's own stream, at a higher priority than the side
            with torch.cuda.stream(main_stream):           # stream's binning
                dp.run(render_view)

    for _ in range(args.warmup):
        step()
    # per-phase breakdown: one untimed step with every phase event-timed; it also picks the
    # dominant kernel (the single-kernel phase with the most time; multi-kernel phases such as the
    # sorts cannot be matched to one rocprof kernel line)
    prof_all, dom = {}, None
    if not args.no_profile:
        torch.cuda.synchronize(dev)
        _lib.profile_enable(True)
        step()
        torch.cuda.synchronize(dev)
        prof_all = _lib.profile_read()
        single = [k for k in ("render_bwd", "render_fwd", "preprocess", "preprocess_bwd_views", "preprocess_bwd",
                              "emit", "tile_ranges") if prof_all.get(k, (0, 0))[1]]
        dom = max(single, key=lambda k: prof_all[k][0])
        # timed region: only the dominant kernel carries events (two records per launch)
        _lib.profile_enable(True, phases=[dom])
    Ks.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = _lib.profile_read() if not args.no_profile else {}
    _lib.profile_enable(False)
    # every view's backward ran, timed (a batched launch serves a binning batch of views)
    if hasattr(render, "render_batch"):
        want = _n_binning_batches(args.early_views, V)
    else:
        want = V
    if dom == "render_bwd" and prof["render_bwd"][1] != want * args.steps:
        raise RuntimeError(f"expected {want * args.steps} backward launches, profiled {prof['render_bwd'][1]}")
    el = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    frames = world * V * args.steps
    value = frames / elapsed

    single = None
    if args.single_view_steps > 0 and world == 1:   # configs[2] literally: one GPU
        # secondary figure: BASELINE configs[2] literally, one view at a time through the per-view
        # entry points (forward_native + backward_native, workspaces allocated per call), no batching
        v0 = dp.views[0]
        kw = dict(shs=scene.shs, language_feature=scene.lang, scales=scene.scales, rotations=scene.rotations)

        def one_view():
            *_, st = dgr.forward_native(settings[v0], scene.means3D, scene.opacities, **kw)
            dgr.backward_native(st, gcol, glang, None, out=bucket.views, accumulate=True, need=bucket.need())

        one_view()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.single_view_steps):
            one_view()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t1) / args.single_view_steps
        single = dict(value=round(1.0 / dt, 3), unit="frames/s", ms_per_frame=round(dt * 1e3, 3),
                      frames=args.single_view_steps,
                      path="forward_native + backward_native per view (configs[2]: one view fwd+bwd, no batching)")

    if rank == 0:
        Kmean = float(np.mean(Ks)) if Ks else 0.0
        with torch.no_grad():
            vis_sum, any_vis = 0, torch.zeros(P, dtype=torch.bool, device=dev)
            for v in dp.views:
                _, _, radii, _, _ = dgr.forward_native(settings[v], scene.means3D, scene.opacities, shs=scene.shs,
                                                       language_feature=scene.lang, scales=scene.scales,
                                                       rotations=scene.rotations)
                vis_sum += int((radii > 0).sum())
                any_vis |= radii > 0
                if v == dp.views[0]:
                    Pvis = int((radii > 0).sum())
            Pany = int(any_vis.sum())
        pb = dict(V=len(dp.views), Pvis_sum=vis_sum, Pany=Pany, means2D=bucket.densify_stats,
                  accumulate=not getattr(getattr(render, "flush", None), "overwrites", False))
        ntiles = ((W + 15) // 16) * ((H + 15) // 16)
        roof = None
        phases = {}
        pmc_all = {}
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                pmc_all = json.load(open(pmc))
            except Exception:
                pmc_all = {}
        if prof:
            for k, (ms, n) in prof_all.items():   # the untimed all-phase step
                if n:   # per view (a batched launch serves several); preprocess_bwd_views: per launch
                    per = ms / n if k == "preprocess_bwd_views" else ms / len(dp.views)
                    rec = pmc_all.get(k, {}) if isinstance(pmc_all.get(k), dict) else {}
                    # alg_gbs: the per-VIEW algorithmic bytes (phase_bytes) over the per-view time.  A
                    # batched launch (preprocess, the compositors) reads a Gaussian's inputs once per
                    # launch, not once per view, so for those this overstates what the chip moved;
                    # pmc_gbs: the PMC bytes of one launch (profiles/pmc_traffic.json, the same step
                    # structure) over the mean launch time -- the bandwidth really drawn
                    phases[k] = dict(mean_ms=per, launches=n,
                                     alg_gbs=phase_bytes(k, P, Pvis, Kmean, W * H, ntiles, C, M, **pb)
                                     / (per * 1e-3) / 1e9,
                                     pmc_gbs=(rec["hbm_bytes_per_launch"] / (ms / n * 1e-3) / 1e9)
                                     if rec.get("hbm_bytes_per_launch") else None)
            ms, n = prof[dom]                      # live, over the timed region
            byts = phase_bytes(dom, P, Pvis, Kmean, W * H, ntiles, C, M, **pb)
            if dom.startswith("render"):           # per view; a batched launch composites several views
                byts *= V * args.steps / n
            ach = byts / (ms / n * 1e-3) / 1e9
            pmc_rec = pmc_all.get(dom, {}) if isinstance(pmc_all.get(dom), dict) else {}
            # the HBM roofline is the contract's; the compositors are bound by VALU issue and atomics
            # (DESIGN.md 4), so the PMC VALU-issue share and matrix-core busy fraction ride along
            # the compositors' VALU side: wave64 VALU instructions per launch (PMC SQ_INSTS_VALU) at
            # the SIMD's peak rate of one per 2 cycles (MI355X_MICROARCH.md), 1024 SIMDs at 2.4 GHz
            vi = pmc_rec.get("valu_insts_per_launch")
            valu_frac = round(vi * 2 / (1024 * 2.4e9 * ms / n * 1e-3), 4) if vi else None
            roof = dict(kernel=dom, bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(ach / HBM_PEAK_GBS, 4), traffic=pmc_rec.get("hbm_bytes_per_launch"),
                        traffic_source="profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes)",
                        algorithmic_bytes=int(byts), mean_launch_ms=round(ms / n, 4),
                        limiter=("latency+atomics (2 waves/SIMD; VALU instructions below the issue peak: "
                                 "valu_issue_frac)") if dom == "render_bwd" else ("issue+latency" if dom == "render_fwd"
                                                                                   else "hbm"),
                        valu_issue_per_wave=pmc_rec.get("valu_issue_per_wave"), valu_issue_frac=valu_frac,
                        mfma_busy_frac=pmc_rec.get("mfma_busy_frac"))
        # whole-frame algorithmic bytes (SURVEY.md 8(d) formula with the measured K): every phase of a
        # frame's fwd + bwd, each byte counted once, over the measured time per frame
        fwd_b = P * 339 + Kmean * 216 + W * H * (4 * (3 + C + 1) + 8)
        bwd_b = Kmean * 176 + W * H * (4 * (3 + C) + 8) + P * (44 + 4 * C) + P * 316 + P * 256
        fb = fwd_b + bwd_b
        frame_roof = dict(algorithmic_bytes_per_frame=int(fb), achieved=round(fb * value / 1e9, 1), peak=HBM_PEAK_GBS,
                          unit="GB/s", frac=round(fb * value / 1e9 / HBM_PEAK_GBS, 4),
                          formula="SURVEY.md 8(d): fwd P*339 + K*216 + Npix*(4(3+C+1)+8); bwd K*176 + "
                                  "Npix*(4(3+C)+8) + P*(44+4C) + P*316 + P*256, K measured",
                          note="charges every frame the per-view preprocess (P-proportional) bytes; the batched "
                               "step reads a Gaussian's inputs and writes its gradient rows once per launch of "
                               "up to 8 views, so it moves less than this: see pmc_step (measured traffic) and "
                               "single_view.frame_roofline (the per-frame path this formula describes)")
        step_rec = pmc_all.get("_step") if isinstance(pmc_all.get("_step"), dict) else None
        if step_rec and step_rec.get("hbm_bytes_per_step"):
            # the step's measured HBM traffic: PMC bytes of EVERY dispatch of one 8-view step (the
            # sorts, scans and fills included; tools/pmc_summary.py step_bytes), per frame
            per_frame = step_rec["hbm_bytes_per_step"] / len(dp.views)
            frame_roof["pmc_step"] = dict(hbm_bytes_per_frame=int(per_frame), achieved=round(per_frame * value / 1e9, 1),
                                          frac=round(per_frame * value / 1e9 / HBM_PEAK_GBS, 4),
                                          source="profiles/pmc_traffic.json _step: (2 FETCH_SIZE + WRITE_SIZE) over "
                                                 "every dispatch of a step")
        elif prof and pmc_all:
            # older records: PMC bytes per launch of every profiled phase x its launches in one
            # step, per frame (kernels without a PMC record, the sorts and scans, left out: a lower bound)
            step_b = sum(pmc_all[k]["hbm_bytes_per_launch"] * n for k, (ms, n) in prof_all.items()
                         if n and isinstance(pmc_all.get(k), dict) and pmc_all[k].get("hbm_bytes_per_launch"))
            per_frame = step_b / len(dp.views)
            frame_roof["pmc_step"] = dict(hbm_bytes_per_frame=int(per_frame), achieved=round(per_frame * value / 1e9, 1),
                                          frac=round(per_frame * value / 1e9 / HBM_PEAK_GBS, 4),
                                          phases=sorted(k for k in prof_all if isinstance(pmc_all.get(k), dict)),
                                          source="profiles/pmc_traffic.json (sorts/scans not included)")
        if single is not None:
            single["frame_roofline"] = dict(algorithmic_bytes_per_frame=int(fb),
                                            achieved=round(fb * single["value"] / 1e9, 1), peak=HBM_PEAK_GBS,
                                            unit="GB/s", frac=round(fb * single["value"] / 1e9 / HBM_PEAK_GBS, 4))
        cpu = None
        if not args.no_cpu_baseline and world == 1:   # the contract's CPU leg: rank 0 at N = 1 only
            avail, host = host_cpu()
            threads = args.cpu_threads or avail
            nf = args.cpu_frames
            tot, tf, tb = cpu_baseline(scene_cpu, all_cams[:nf], C, threads)
            cpu = dict(value=round(nf / tot, 5), unit="frames/s", cores=threads, kind="port",
                       sample=f"{nf} headline frames (P={P}, {W}x{H}, C={C}, the first cameras of the batch) "
                              f"fwd {tf:.2f}s + bwd {tb:.2f}s, C oracle oracle/lsr_oracle.c, OpenMP {threads} threads",
                       host=host)
            if not args.no_configs0:
                cpu["configs0"], gpu0 = configs0_leg(threads, dev)
                cpu["configs0"]["gpu_frames_per_s"] = gpu0
        line = dict(
            metric="rasterizer fwd+bwd frames/sec @ 2M Gaussians, 1352x1014, 32-ch features",
            value=round(value, 3), unit="frames/s", n_gpus=world, ranks=pg_ranks, steps=args.steps, warmup=args.warmup,
            ms_per_step=round(elapsed / args.steps * 1e3, 3), higher_is_better=True, scaling="weak",
            vs_baseline=None, dtype="f32", data="synthetic",
            precision=("fp32 per-pixel arithmetic (T, alpha, RGB, depth, the recurrences); the language "
                       "channel sums and the backward's per-Gaussian pixel sums on MFMA as bf16 hi/lo "
                       "splits, three products, fp32 accumulation (~2^-17 relative)"),
            config=dict(workload="S2M synthetic (BASELINE configs[2] per GPU; configs[3] batch split)",
                        gaussians=P, width=W, height=H, channels=C, views_per_gpu_per_step=V,
                        global_batch=world * V, parallelism=f"dp{world}", pipeline="none" if args.no_overlap else args.pipeline, binning=args.binning, early_views=args.early_views, order_on_side=args.order_on_side, num_rendered_mean=int(Kmean),
                        visible=Pvis, visible_any_view=Pany, grad_bucket_mb=round(bucket.nbytes / 2**20, 1)),
            roofline=roof, frame_roofline=frame_roof, cpu_baseline=cpu, single_view=single,
            phases={k: dict(mean_ms=round(v["mean_ms"], 4), alg_gbs=round(v["alg_gbs"], 1),
                            pmc_gbs=None if v["pmc_gbs"] is None else round(v["pmc_gbs"], 1)) for k, v in phases.items()},
            phases_note=("mean_ms per view (a batched launch's time / its views; preprocess_bwd_views per launch); "
                         "alg_gbs = per-view algorithmic bytes / per-view time (overstates batched launches, which "
                         "read the Gaussians once per launch); pmc_gbs = PMC HBM bytes per launch / launch time"),
        )
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
