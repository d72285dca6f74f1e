"""Per-view data parallelism on CPU: view partitioning, the flat gradient
bucket, and a world_size-2 gloo step whose SUM / MAX reductions must equal one process
rendering the whole batch (the reference's sequential multi-view loop, train.py:242-271,350-352).
The per-view renderer here is the CPU oracle (test infrastructure); on the GPU the same
ViewParallelStep runs native_view_renderer (bench.py)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import synthetic
from helpers import oracle_settings
from view_parallel import GradBucket, ViewParallelStep, view_slice

N_VIEWS, P, W, H, C = 5, 1500, 64, 48, 4


@pytest.mark.parametrize("n,world", [(64, 8), (5, 2), (3, 4), (0, 3), (7, 1), (9, 4)])
def test_view_slice_partitions_batch(n, world):
    seen = []
    sizes = []
    for r in range(world):
        a, b = view_slice(n, world, r)
        seen.extend(range(a, b))
        sizes.append(b - a)
    assert seen == list(range(n))
    assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        view_slice(n, world, world)


@pytest.mark.parametrize("densify", [False, True])
def test_bucket_layout(densify):
    b = GradBucket(10, 16, 32, "cpu", densify_stats=densify)
    assert b.floats_per_gaussian == 3 + 3 + 4 + 1 + 48 + 32 + (3 if densify else 0)
    assert b.views["sh"].shape == (10, 16, 3) and b.views["language_feature"].shape == (10, 32)
    # every view aliases the flat buffer, fields do not overlap and cover it exactly
    ptrs = sorted((v.data_ptr(), v.numel()) for v in b.views.values() if v is not None)
    o = b.flat.data_ptr()
    for p, n in ptrs:
        assert p == o
        o += 4 * n
    assert o == b.flat.data_ptr() + b.nbytes
    assert b.need()["means2D"] == densify and not b.need()["colors"]
    b.views["opacities"].fill_(1)
    b.zero_()
    assert float(b.flat.abs().sum()) == 0


def _scene_and_cams():
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W, seed=3, logscale_mean=-4.0)
    cams = synthetic.camera_batch(N_VIEWS, W, H, tanfovx=0.6, seed=1)
    return sc, cams


def _view_grads(v):
    g = np.random.default_rng(100 + v)
    return g.normal(size=(3, H, W)).astype(np.float32), g.normal(size=(C, H, W)).astype(np.float32)


def oracle_renderer(sc, cams, batched=False, chunked=False):
    """batched: like native_view_renderer(batch_backward=True), the language gradient goes into
    the bucket per view and every other field only at flush (the batched preprocess backward);
    chunked: the flush writes row chunks and reports each (flush(bucket, row_chunks, on_rows))."""
    names = dict(means3D="means3D", scales="scales", rotations="rotations", opacity="opacities", sh="sh",
                 lang="language_feature", means2D="means2D")
    held = []

    def render_view(v, bucket):
        r = oracle.forward(oracle_settings(cams[v]), sc.means3D.numpy(), sc.opacities.numpy(), shs=sc.shs.numpy(),
                           lang=sc.lang.numpy(), scales=sc.scales.numpy(), rotations=sc.rotations.numpy())
        gc, gl = _view_grads(v)
        g = r.backward(gc, gl, None, nthreads=1)
        for k, name in names.items():
            if bucket.views.get(name) is not None:
                if batched and name != "language_feature":
                    held.append((name, torch.from_numpy(g[k].copy())))
                else:
                    bucket.views[name] += torch.from_numpy(g[k])
        radii = torch.from_numpy(r.radii.copy())
        r.close()
        return radii

    def flush(bucket, row_chunks=None, on_rows=None):
        for r0, r1 in (row_chunks or [(0, bucket.P)]):
            for name, t in held:
                bucket.views[name][r0:r1] += t[r0:r1]
            if on_rows is not None:
                on_rows(r0, r1)
        held.clear()

    if batched:
        render_view.flush = flush
        flush.chunked = chunked
    return render_view


def _serial_reference(densify):
    sc, cams = _scene_and_cams()
    b = GradBucket(P, sc.shs.shape[1], C, "cpu", densify_stats=densify)
    step = ViewParallelStep(b, N_VIEWS)
    assert list(step.views) == list(range(N_VIEWS))
    step.run(oracle_renderer(sc, cams))
    return b


def _worker(rank, world, port, outdir, densify, batched=False, chunked=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc, cams = _scene_and_cams()
        b = GradBucket(P, sc.shs.shape[1], C, "cpu", densify_stats=densify)
        step = ViewParallelStep(b, N_VIEWS, flush_chunks=3)
        assert step.world == world and step.rank == rank
        calls = []
        render = oracle_renderer(sc, cams, batched, chunked)

        def counted(v, bucket):
            calls.append(v)
            return render(v, bucket)

        if batched:
            counted.flush = render.flush

        step.run(counted)
        assert calls == list(range(*view_slice(N_VIEWS, world, rank)))
        torch.save(dict(flat=b.flat.clone(), radii=None if b.radii is None else b.radii.clone(),
                        vis=step.visibility() if densify else None, calls=calls),
                   os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("densify,batched,chunked", [(False, False, False), (True, False, False),
                                                     (True, True, False), (True, True, True)])
def test_two_rank_step_equals_serial_batch(densify, batched, chunked):
    """batched: the language field's SUM is issued before the flush and overlaps it; chunked: the
    flush runs in row chunks (P = 1500 -> 512-row chunks) and each chunk's rows of every other
    field are SUMmed asynchronously as the chunk ends."""
    ref = _serial_reference(densify)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d, densify, batched, chunked), nprocs=2, join=True)
        outs = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    assert sorted(outs[0]["calls"] + outs[1]["calls"]) == list(range(N_VIEWS))
    # both ranks hold the same reduced bucket, equal to the serial sum up to fp32 reassociation
    assert torch.equal(outs[0]["flat"], outs[1]["flat"])
    scale = float(ref.flat.abs().max())
    assert scale > 0
    err = float((outs[0]["flat"] - ref.flat).abs().max())
    assert err <= 1e-5 * scale, err
    if densify:
        assert torch.equal(outs[0]["radii"], ref.radii) and torch.equal(outs[1]["radii"], ref.radii)
        assert torch.equal(outs[0]["vis"], ref.radii > 0)
        assert int(ref.radii.gt(0).sum()) > 0


class _FakePending:
    def __init__(self, v, log):
        self.v, self.log, self.num_rendered = v, log, 0
        self.ready = None                        # one binning batch

    def resolve(self, binning=False):
        self.log.append(("resolve", self.v))
        return self


def _lookahead_worker(rank, world, port, outdir, mode="lookahead"):
    """native_view_renderer's one-stream lookahead (or the batched forward) with LIST settings
    (every view of the batch visible to every rank): each rank must preprocess exactly its own
    views, never the next rank's first view, and leave nothing pending after the step; batched:
    in ONE preprocess + binning batch per step.  The native calls are replaced by recorders (no
    GPU here); the control flow is the product's."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import diff_gaussian_rasterization as dgr
        from view_parallel import native_view_renderer
        log = []
        Pn = 16

        def preprocess_native(settings, *a, **k):
            log.append(("preprocess", settings))
            return _FakePending(settings, log)

        def render_native(pf):
            log.append(("render", pf.v))
            z = torch.zeros(3, 4, 4)
            return z, torch.zeros(2, 4, 4), torch.full((Pn,), pf.v + 1, dtype=torch.int32), z[:1], pf

        def backward_composite_native(st, gc, gl, gd, dL_dlanguage=None):
            log.append(("composite_bwd", st.v))
            return st

        def preprocess_views_native(settings_list, *a, **k):
            log.append(("preprocess_views", list(settings_list)))
            return [_FakePending(v, log) for v in settings_list]

        def binning_views_native(pfs):
            log.append(("binning_views", [pf.v for pf in pfs]))

        def backward_preprocess_views_native(held, out=None, accumulate=False, need=None, row_chunks=None,
                                             on_rows=None):
            log.append(("flush", [h.v for h in held]))
            for t in out.values():
                if t is not None:
                    t.zero_()
            for r0, r1 in (row_chunks or []):
                on_rows(r0, r1)

        def render_views_native(pfs):
            return [render_native(pf) for pf in pfs]

        def backward_composite_views_native(sts, gcs, gls, gds, dL_dlanguage=None):
            return [backward_composite_native(st, gc, gl, gd) for st, gc, gl, gd in zip(sts, gcs, gls, gds)]

        dgr.render_views_native, dgr.backward_composite_views_native = render_views_native, \
            backward_composite_views_native
        dgr.preprocess_native, dgr.render_native = preprocess_native, render_native
        dgr.backward_composite_native = backward_composite_native
        dgr.backward_preprocess_views_native = backward_preprocess_views_native
        dgr.preprocess_views_native, dgr.binning_views_native = preprocess_views_native, binning_views_native

        class S:
            means3D = opacities = shs = lang = scales = rotations = torch.zeros(Pn, 3)

        n_views = 5
        settings = list(range(n_views))          # "settings" of view v is just v here
        render = native_view_renderer(S(), settings, lambda v, c, l, d: (c, l, d), overlap=mode)
        b = GradBucket(Pn, 1, 2, "cpu", densify_stats=True)
        step = ViewParallelStep(b, n_views)
        for _ in range(2):                       # two steps: nothing carried over
            step.run(render)
            assert not render.pending
        mine = list(step.views)
        if mode == "batched":
            assert [s for k, s in log if k == "preprocess_views"] == [mine] * 2, (rank, log)
            assert [s for k, s in log if k == "binning_views"] == [mine] * 2, (rank, log)
            assert not [s for k, s in log if k == "preprocess"]
        else:
            pre = [s for k, s in log if k == "preprocess"]
            assert pre == mine * 2, (rank, pre, mine)
        assert [s for k, s in log if k == "render"] == mine * 2
        assert [s for k, s in log if k == "flush"] == [mine] * 2
        torch.save(dict(radii=b.radii.clone()), os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["lookahead", "batched"])
def test_two_rank_lookahead_stays_in_rank_slice(mode):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_lookahead_worker, args=(2, _free_port(), d, mode), nprocs=2, join=True)
        outs = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    # radii MAX over all 5 views (the fake radius of view v is v + 1)
    assert torch.equal(outs[0]["radii"], torch.full((16,), 5, dtype=torch.int32))
    assert torch.equal(outs[1]["radii"], outs[0]["radii"])


def test_row_chunks_tile_rows():
    from view_parallel import row_chunks
    for P, n in ((1500, 3), (2_000_000, 4), (100, 8), (256, 1), (0, 4), (257, 2)):
        ch = row_chunks(P, n)
        assert ch[0][0] == 0 and ch[-1][1] == P and len(ch) <= max(n, 1)
        assert all(a % 256 == 0 for a, _ in ch)
        assert all(ch[i][1] == ch[i + 1][0] for i in range(len(ch) - 1))


def _launched(rank, world, outdir):
    """A rank started by view_parallel.launch_ranks: the torchrun environment is set, the gloo
    group forms from it, and a step with a stub renderer (view v adds v + 1 to every gradient,
    radius v + 1) reduces over all ranks."""
    assert os.environ["RANK"] == str(rank) and os.environ["WORLD_SIZE"] == str(world)
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo")
    try:
        b = GradBucket(8, 1, 2, "cpu", densify_stats=True)
        step = ViewParallelStep(b, 6)

        def stub(v, bucket):
            bucket.flat += float(v + 1)
            return torch.full((8,), v + 1, dtype=torch.int32)

        step.run(stub)
        torch.save(dict(world=dist.get_world_size(), flat=b.flat.clone(), radii=b.radii.clone(),
                        views=list(step.views)), os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_launch_ranks_starts_world_ranks(world, monkeypatch):
    """bench.py --gpus N without torchrun: launch_ranks starts N ranks that form one group."""
    from view_parallel import launch_ranks
    monkeypatch.delenv("MASTER_PORT", raising=False)
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    with tempfile.TemporaryDirectory() as d:
        launch_ranks(world, _launched, (d,))
        outs = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    assert all(o["world"] == world for o in outs)
    assert sorted(v for o in outs for v in o["views"]) == list(range(6))
    for o in outs:
        assert torch.equal(o["flat"], torch.full_like(o["flat"], 21.0))   # 1 + 2 + ... + 6
        assert torch.equal(o["radii"], torch.full((8,), 6, dtype=torch.int32))


# ---- the sharded optimizer step (ShardedAdam: reduce-scatter, Adam on row shards, all-gather) --------
LRS_SH = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20, "opacity": 0.05, "scaling": 5e-3, "rotation": 1e-3,
          "language_feature": 2.5e-3}


def _np_adam(p, g, m, v, lr, step):
    """the numpy restatement of torch.optim.Adam (oracle/train_oracle.py, pinned by train_golden.npz)."""
    import train_oracle
    pn, mn, vn = p.numpy(), m.numpy(), v.numpy()
    train_oracle.adam_step(pn, g.numpy(), mn, vn, lr, step)


def _raw_scene(seed=3):
    """raw parameters and the scene of their activations (render()'s: exp, normalize, sigmoid, SH cat,
    language / (|language| + 1e-9))."""
    sc = synthetic.make_scene(P, C=C, tanfovx=0.6, tanfovy=0.6 * H / W, seed=seed, logscale_mean=-4.0)
    g = torch.Generator().manual_seed(seed)
    raw = dict(xyz=sc.means3D.clone(), f_dc=sc.shs[:, :1].clone(), f_rest=sc.shs[:, 1:].clone(),
               opacity=torch.logit(sc.opacities.reshape(P, 1)).clone(), scaling=torch.log(sc.scales).clone(),
               rotation=sc.rotations * (0.5 + torch.rand(P, 1, generator=g)),
               language_feature=sc.lang * (1 + 2 * torch.rand(P, 1, generator=g)))
    sc.rotations = torch.nn.functional.normalize(raw["rotation"])
    sc.lang = raw["language_feature"] / (raw["language_feature"].norm(dim=-1, keepdim=True) + 1e-9)
    return sc, raw


def test_sharded_adam_single_rank_equals_autograd_and_torch_adam():
    """world 1: the activations' backward and the Adam step of ShardedAdam against torch autograd
    through the same activations and torch.optim.Adam(eps=1e-15) (gaussian_model.py:301)."""
    from view_parallel import ShardedAdam
    sc, raw = _raw_scene()
    up = ShardedAdam(sc, raw, LRS_SH, adam=_np_adam)
    b = GradBucket(P, 16, C, "cpu", row_multiple=ShardedAdam.row_multiple(P, 1))
    gen = torch.Generator().manual_seed(5)
    for name in ("means3D", "scales", "rotations", "opacities", "sh", "language_feature"):
        b.views[name].copy_(torch.randn(b.views[name].shape, generator=gen) * 1e-3)
    leaves = {k: v.clone().requires_grad_(True) for k, v in raw.items()}
    act = dict(means3D=leaves["xyz"], scales=torch.exp(leaves["scaling"]),
               rotations=torch.nn.functional.normalize(leaves["rotation"]),
               opacities=torch.sigmoid(leaves["opacity"]), sh=torch.cat([leaves["f_dc"], leaves["f_rest"]], 1),
               language_feature=leaves["language_feature"] / (leaves["language_feature"].norm(dim=-1, keepdim=True)
                                                              + 1e-9))
    sum((act[k] * b.views[k].reshape(act[k].shape)).sum() for k in act).backward()
    opt = torch.optim.Adam([{"params": [leaves[k]], "lr": LRS_SH[k]} for k in leaves], lr=0.0, eps=1e-15)
    opt.step()
    up.step(b)
    for k in raw:
        ref = leaves[k].detach()
        got = up.full_rows(k)[1]          # world 1: the shard is every row (padding past P dropped)
        assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6), (k, float((got - ref).abs().max()))
    # the scene now renders the updated parameters' activations
    assert torch.allclose(sc.scales, torch.exp(leaves["scaling"].detach()), rtol=1e-5)
    assert torch.allclose(sc.opacities, torch.sigmoid(leaves["opacity"].detach()), rtol=1e-5, atol=1e-7)


def _sharded_worker(rank, world, port, outdir, steps, chunks=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from view_parallel import ShardedAdam
        sc, raw = _raw_scene()
        _, cams = _scene_and_cams()
        up = ShardedAdam(sc, raw, LRS_SH, adam=_np_adam, chunks=chunks)
        b = GradBucket(P, 16, C, "cpu", densify_stats=True,
                       row_multiple=ShardedAdam.row_multiple(P, world, chunks=chunks))
        step = ViewParallelStep(b, N_VIEWS, update=up)
        render = oracle_renderer(sc, cams, batched=True, chunked=chunks > 1)
        issued = []
        if chunks > 1:   # record the flush's chunk reports: each chunk's reduce-scatter starts behind it
            on_rows = up.on_rows
            up.on_rows = lambda bucket, r0, r1: (issued.append((r0, r1, len(up._rs))), on_rows(bucket, r0, r1))
        for _ in range(steps):
            step.run(render)
        full = {k: up.full_rows(k) for k in up.raw}
        torch.save(dict(raw={k: v.clone() for k, v in up.raw.items()}, rows=(up.r0, up.r1), issued=issued,
                        full={k: (i.clone(), r.clone()) for k, (i, r) in full.items()},
                        act={k: getattr(sc, k).clone() for k in ("means3D", "scales", "rotations", "opacities", "shs",
                                                                  "lang")},
                        radii=b.radii.clone()), os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        if world > 1:
            dist.destroy_process_group()


def _assemble(outs, k):
    """The full [P, ...] rows of raw group k from the ranks' shards (ShardedAdam.full_rows)."""
    idx0, rows0 = outs[0]["full"][k]
    got = torch.zeros((P,) + tuple(rows0.shape[1:]), dtype=rows0.dtype)
    seen = torch.zeros(P, dtype=torch.bool)
    for o in outs:
        idx, rows = o["full"][k]
        assert not seen[idx].any()
        got[idx] = rows
        seen[idx] = True
    assert bool(seen.all()), k                                          # the shards partition the rows
    return got


def test_sharded_step_two_ranks_equals_serial():
    """Two optimizer steps of the view batch: world 2 (reduce-scatter, Adam on each rank's half of the
    rows, all-gather) against one process doing every view and every row.  The parameters and the
    activated inputs agree up to the fp32 reassociation of the view sums."""
    with tempfile.TemporaryDirectory() as d:
        _sharded_worker(0, 1, 0, d, 2)
        ser = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_sharded_worker, args=(2, _free_port(), d, 2), nprocs=2, join=True)
        outs = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    assert outs[0]["rows"][1] == outs[1]["rows"][0] and outs[1]["rows"][1] == P and outs[0]["rows"][0] == 0
    for k in ser["raw"]:
        v = _assemble([ser], k)
        got = _assemble(outs, k)
        moved = (v - _raw_scene()[1][k]).abs().max()
        assert float(moved) > 0, k
        assert torch.allclose(got, v, rtol=1e-5, atol=1e-6), (k, float((got - v).abs().max()))
    for k, v in ser["act"].items():
        assert torch.equal(outs[0]["act"][k], outs[1]["act"][k]), k      # every rank renders the same scene
        assert torch.allclose(outs[0]["act"][k], v, rtol=1e-5, atol=1e-6), k
    assert torch.equal(outs[0]["radii"], ser["radii"])


def test_sharded_adam_schedule_and_field_guard():
    """ShardedAdam follows GaussianTrainer's xyz schedule (gaussian_model.py:315-329) and refuses a
    scene with a deformation field (its bucket's means3D gradient is not the xyz gradient there)."""
    from gaussian_train import get_expon_lr_func
    from view_parallel import ShardedAdam
    sc, raw = _raw_scene()
    up = ShardedAdam(sc, raw, LRS_SH, adam=_np_adam)
    assert up.update_learning_rate(100) == LRS_SH["xyz"]          # no schedule: the constant lr
    up.set_xyz_schedule(1.6e-4 * 5, 1.6e-6 * 5, 0.01, 20_000)
    ref = get_expon_lr_func(1.6e-4 * 5, 1.6e-6 * 5, lr_delay_mult=0.01, max_steps=20_000)
    for it in (0, 1, 500, 19_999, 40_000):
        assert up.update_learning_rate(it) == float(ref(it)) and up.lrs["xyz"] == float(ref(it))
    sc2, raw2 = _raw_scene()
    sc2.deformation = object()
    with pytest.raises(ValueError, match="deformation field"):
        ShardedAdam(sc2, raw2, LRS_SH, adam=_np_adam)


def test_sharded_chunked_pipeline_two_ranks_equals_serial():
    """ShardedAdam(chunks=4): the shard is one piece per row chunk, the flush reports each chunk and that
    chunk's reduce-scatter starts behind it, Adam runs chunk by chunk and each chunk's all-gather is
    issued as soon as its rows are updated.  Two steps at world size 2 against the serial step
    (world 1, one chunk): parameters and activated inputs agree up to the view sums' fp32
    reassociation; every rank renders the same scene."""
    with tempfile.TemporaryDirectory() as d:
        _sharded_worker(0, 1, 0, d, 2)
        ser = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_sharded_worker, args=(2, _free_port(), d, 2, 4), nprocs=2, join=True)
        outs = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for o in outs:   # 3 chunks hold rows (P = 1500 of 2048 padded rows), reported in order, each issued once
        assert [(r0, r1) for r0, r1, _ in o["issued"][:3]] == [(0, 512), (512, 1024), (1024, 1500)]
    for k in ser["raw"]:
        v, got = _assemble([ser], k), _assemble(outs, k)
        assert torch.allclose(got, v, rtol=1e-5, atol=1e-6), (k, float((got - v).abs().max()))
    for k, v in ser["act"].items():
        assert torch.equal(outs[0]["act"][k], outs[1]["act"][k]), k
        assert torch.allclose(outs[0]["act"][k], v, rtol=1e-5, atol=1e-6), k
    assert torch.equal(outs[0]["radii"], ser["radii"])
