"""Per-view data parallelism for the rasterizer step.

The reference renders the views of one training batch sequentially on one GPU and lets
autograd sum their gradients (train.py:242-268, loss.backward() at :339).  Three per-view
statistics are reduced alongside the gradients:
  * radii      -> MAX over views           (train.py:270)
  * visibility -> ANY over views = radii>0  (train.py:271)
  * viewspace (means2D) gradient -> SUM over views (train.py:350-352), later consumed by
    add_densification_stats (scene/gaussian_model.py:744-746).

Here the Gaussians are replicated on every rank, the view batch is split into contiguous
per-rank slices (view_slice), each rank accumulates its views' gradients into ONE flat fp32
bucket (GradBucket; the rasterizer backward accumulates in place, no per-view copies), and a
step ends with one SUM all-reduce of that bucket plus, when densification statistics are
requested, one MAX all-reduce of the int32 radii.  On MI355X the process group is "nccl"
(= RCCL over xGMI); the CPU tests drive the same code over "gloo".  There is no other
data-path collective: views are independent (SURVEY.md 8(e) "Shards naturally? Yes").

The per-view work is a callback so that the same step runs the native HIP rasterizer
(native_view_renderer, the product path) or, in tests only, the CPU oracle.
"""
import os
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist

# gradient fields of the flat bucket, in order; None = width depends on M (SH) or C (language)
GRAD_FIELDS = (("means3D", 3), ("scales", 3), ("rotations", 4), ("opacities", 1), ("sh", None),
               ("language_feature", None))


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_child(rank: int, fn: Callable, world: int, fn_args: tuple):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world))
    fn(rank, world, *fn_args)


def launch_ranks(world: int, fn: Callable, fn_args: tuple = ()) -> None:
    """One process per rank on this node without torchrun: spawns `world` children (fresh
    interpreters, so call this before the parent touches the GPU) with the torchrun environment
    (RANK, LOCAL_RANK, WORLD_SIZE; MASTER_ADDR 127.0.0.1 and a free MASTER_PORT unless set) and
    runs fn(rank, world, *fn_args) in each; raises if any rank fails.  The children initialise
    their own process group ("nccl" = RCCL on the GPU, "gloo" in the CPU tests)."""
    import torch.multiprocessing as mp
    if world < 1:
        raise ValueError(f"world size {world}")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver
    mp.spawn(_rank_child, args=(fn, world, tuple(fn_args)), nprocs=world, join=True)


def view_slice(n_views: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) of the batch's views owned by `rank` (the first
    n_views % world ranks take one extra view)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n_views, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class GradBucket:
    """One flat fp32 buffer holding every per-Gaussian gradient of a step, field-major
    ([P,3] means3D | [P,3] scales | [P,4] rotations | [P,1] opacities | [P,M,3] SH | [P,C]
    language | optional [P,3] means2D), so one collective moves all of it.  `views` maps the
    rasterizer's gradient names onto slices of `flat` (pass it as backward_native(out=...))."""

    def __init__(self, P: int, M: int, C: int, device, densify_stats: bool = False):
        self.P, self.M, self.C = P, M, C
        self.densify_stats = densify_stats
        fields = [(n, w if w is not None else (3 * M if n == "sh" else C)) for n, w in GRAD_FIELDS]
        if densify_stats:
            fields.append(("means2D", 3))
        self.floats_per_gaussian = sum(w for _, w in fields)
        self.flat = torch.zeros(P * self.floats_per_gaussian, dtype=torch.float32, device=device)
        self.views: Dict[str, Optional[torch.Tensor]] = {}
        self.ranges: Dict[str, Tuple[int, int]] = {}     # field -> [start, end) in flat
        o = 0
        for name, w in fields:
            seg = self.flat[o * P:(o + w) * P]
            self.ranges[name] = (o * P, (o + w) * P)
            if w == 0:
                self.views[name] = None
            elif name == "sh":
                self.views[name] = seg.view(P, M, 3)
            else:
                self.views[name] = seg.view(P, w)
            o += w
        self.radii = torch.zeros(P, dtype=torch.int32, device=device) if densify_stats else None

    def zero_(self):
        self.flat.zero_()
        if self.radii is not None:
            self.radii.zero_()

    def zero_accumulated_(self):
        """Zero only what the views accumulate into (language gradients, radii): for a batched
        flush that overwrites every other field."""
        lo, hi = self.ranges["language_feature"]
        if hi > lo:
            self.flat[lo:hi].zero_()
        if self.radii is not None:
            self.radii.zero_()

    def need(self) -> Dict[str, bool]:
        """The `need` mask for backward_native: only the bucket's fields are produced."""
        return dict(means3D=True, scales=True, rotations=True, opacities=True, sh=self.M > 0,
                    language_feature=self.C > 0, means2D=self.densify_stats, colors=False, cov3D=False)

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * 4


def row_chunks(P: int, n: int, align: int = 256):
    """[(r0, r1), ...]: [0, P) in at most n contiguous chunks, every r0 a multiple of `align`."""
    if P <= 0:
        return [(0, 0)]
    step = -(-P // max(1, n))
    step = -(-step // align) * align
    return [(r0, min(P, r0 + step)) for r0 in range(0, P, step)]


class ViewParallelStep:
    """One data-parallel step over a batch of `n_views` views.

    run(render_view) calls render_view(v, bucket) for every view v this rank owns; the callback
    adds view v's gradients into bucket.views (and returns view v's int32 radii [P], or None).
    A callback with a `render_batch(views, bucket)` attribute is called once with all of them
    instead (and returns their radii).
    Afterwards the bucket holds the SUM over ALL views of the batch on every rank, and
    bucket.radii the MAX over all views (when densify_stats)."""

    def __init__(self, bucket: GradBucket, n_views: int, group=None, flush_chunks: int = 4):
        self.bucket = bucket
        self.n_views = n_views
        self.group = group
        self.flush_chunks = flush_chunks   # world > 1: the flush in row chunks, each all-reduced as it ends
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.views = range(*view_slice(n_views, self.world, self.rank))

    def run(self, render_view: Callable[[int, GradBucket], Optional[torch.Tensor]]) -> GradBucket:
        b = self.bucket
        begin = getattr(render_view, "begin_step", None)
        if begin is not None:             # the renderer may look ahead only within this rank's views
            begin(self.views)
        flush = getattr(render_view, "flush", None)
        zero = b.zero_accumulated_ if getattr(flush, "overwrites", False) else b.zero_
        # (the flush writes every other field: HBM write saved)
        batch = getattr(render_view, "render_batch", None)
        if batch is not None:             # every view of the rank at once (batched compositor launches)
            if getattr(batch, "before_wait", False):
                radii_views = [r for r in batch(self.views, b, before_wait=zero) if r is not None]
            else:
                zero()
                radii_views = [r for r in batch(self.views, b) if r is not None]
            if b.radii is None:
                radii_views = []
        else:
            zero()
            radii_views = []
            for v in self.views:
                radii = render_view(v, b)
                if b.radii is not None and radii is not None:
                    radii_views.append(radii)
        # radii MAX over the views (train.py:270) after the views' launches, not between them
        # (a batch renderer may have reduced them itself, in one launch)
        if not (batch is not None and getattr(batch, "radii_reduced", False)):
            for radii in radii_views:
                torch.maximum(b.radii, radii.to(torch.int32), out=b.radii)
        pending = []
        lo, hi = b.ranges["language_feature"]
        if self.world > 1 and b.radii is not None:   # final once the last view's forward ran
            pending.append(dist.all_reduce(b.radii, op=dist.ReduceOp.MAX, group=self.group, async_op=True))
        if self.world > 1 and flush is not None and hi > lo:
            # with the batched backward the language gradients are final once the last view's
            # compositor backward ran; their SUM runs during the flush (the preprocess backward,
            # which writes every other field) instead of after it
            pending.append(dist.all_reduce(b.flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        chunked = self.world > 1 and getattr(flush, "chunked", False) and self.flush_chunks > 1
        if chunked:
            # the flush in Gaussian-row chunks: each chunk's rows of every other field are SUMmed
            # (asynchronously, behind that chunk's launch) while the next chunk is computed
            def on_rows(r0, r1):
                for name, (f0, f1) in b.ranges.items():
                    w = (f1 - f0) // b.P if b.P else 0
                    if name == "language_feature" or w == 0 or r1 <= r0:
                        continue
                    pending.append(dist.all_reduce(b.flat[f0 + r0 * w:f0 + r1 * w], op=dist.ReduceOp.SUM,
                                                   group=self.group, async_op=True))
            flush(b, row_chunks=row_chunks(b.P, self.flush_chunks), on_rows=on_rows)
        elif flush is not None:      # renderers that batch the backward over the rank's views
            flush(b)
        end = getattr(render_view, "end_step", None)
        if end is not None:
            end()
        if self.world > 1:
            if not chunked:
                if flush is not None and hi > lo:
                    segs = (b.flat[:lo], b.flat[hi:])
                else:
                    segs = (b.flat,)
                for seg in segs:
                    if seg.numel():
                        dist.all_reduce(seg, op=dist.ReduceOp.SUM, group=self.group)
            for h in pending:
                h.wait()
        return b

    def visibility(self) -> torch.Tensor:
        """ANY over the batch's views (train.py:271): a Gaussian is visible if some view gave it
        a positive radius."""
        if self.bucket.radii is None:
            raise RuntimeError("visibility needs GradBucket(densify_stats=True)")
        return self.bucket.radii > 0


def native_view_renderer(scene, settings, grad_fn: Callable, deterministic: bool = False, overlap: bool = True,
                         batch_backward: bool = True, early_views: int = 3, composite_batch: bool = True,
                         side_priority: int = 0, side_from_preprocess: bool = True, split_behind_counts: bool = True):
    """render_view callback for ViewParallelStep on the HIP rasterizer (the product path).

    scene    : object with means3D, opacities, shs, lang, scales, rotations device tensors
    settings : dict (or list) of GaussianRasterizationSettings, indexed by view
    grad_fn  : grad_fn(v, color, lang, depth) -> (dL_dcolor, dL_dlang, dL_ddepth) for view v
    Forward + backward of view v with the gradients accumulated straight into the bucket.

    batch_backward=True (atomic mode only) runs each view's compositor backward right after its
    forward (lsr_backward_composite, language gradients straight into the bucket) and the
    preprocess backward of all the rank's views once at the end of the step
    (lsr_backward_preprocess_views): the Gaussian rows are read and the bucket's gradient rows
    written once per step instead of once per view.

    overlap=True pipelines the views: once view v's render and backward are enqueued, view v+1's
    preprocess (its depth order and instance count, the one host synchronisation of a forward)
    and its tile binning run on a side stream, concurrently with them, so the device never waits
    for the host between views and the main stream only composites.  Results are identical to
    the sequential order (preprocess and binning only read the Gaussians and write their own
    workspaces).

    overlap="batched" runs the forward phase 1 and the binning of ALL of the step's views (from
    the first one rendered) as one batch when the step starts (lsr_forward_preprocess_views_async,
    lsr_forward_binning_views: a Gaussian's inputs read once per 8 views, one set of sort launches
    for all views, one host wait for their counts); each view then only composites.  Needs the
    step's views (begin_step, as ViewParallelStep.run calls it); without them, views batch alone.

    With more than `early_views` views in the batch, only the first `early_views` are binned on
    the current stream; the others' binning (emission, tile sort, tile ranges: chains of short,
    dependent launches that leave most of the GPU idle) runs on a side stream while those first
    views composite, and each later view's compositing waits for it (an event); the side binning
    starts right behind the preprocess batch, beside the early views' binning
    (side_from_preprocess; behind it: 925 vs 941 frames/s same-box).  With
    composite_batch (batched only) the step runs through render_batch: one compositor forward and
    one compositor backward launch per binning batch instead of per view.

    overlap="lookahead" keeps ONE stream: view v+1's preprocess is enqueued ahead of view v's
    compositing with its instance count copied to pinned memory (lsr_forward_preprocess_async);
    the host waits for that count only (an event), while view v's compositing is still queued,
    then enqueues view v+1's binning behind it.  No host gap between views and no contention
    between the side chain and the compositors."""
    import diff_gaussian_rasterization as dgr

    lookahead = overlap == "lookahead"
    batch_fwd = overlap == "batched"
    side = (torch.cuda.Stream(device=scene.means3D.device) if (overlap and not lookahead and not batch_fwd)
            else None)
    bin_side = [None]                     # created at the first split batch (CUDA tensors only)
    pending = {}
    params_ready = torch.cuda.Event() if side is not None else None
    step_views = [None]                   # this rank's views of the current step (begin_step)

    def has_view(v):
        """v+1 is prefetched only if THIS rank renders it in this step: with list settings and
        world > 1 the next index may be the next rank's first view."""
        if step_views[0] is not None and v not in step_views[0]:
            return False
        return v in settings if isinstance(settings, dict) else 0 <= v < len(settings)

    def preprocess(v, stream=None, defer=False):
        return dgr.preprocess_native(settings[v], scene.means3D, scene.opacities, shs=scene.shs,
                                     language_feature=scene.lang, scales=scene.scales, rotations=scene.rotations,
                                     stream=stream, binning=stream is not None, defer_count=defer)

    batched = batch_backward and not deterministic
    held = []                             # (state, dL_dcolor, dL_dlang, dL_ddepth) awaiting flush

    def batch_preprocess(v, before_wait=None, radii_out=None):
        """The step's views from v on, as one batch: preprocess + depth sorts + instance scans, one
        host wait for their counts, then their binning (lsr_forward_*_views).  before_wait() is
        enqueued behind the batch's launches, ahead of that wait (work that fills the device's
        idle stretch while the host reads the counts)."""
        views = [w for w in step_views[0] if w >= v] if step_views[0] is not None else [v]
        views = [w for w in views if has_view(w)] or [v]
        pfs = dgr.preprocess_views_native([settings[w] for w in views], scene.means3D, scene.opacities,
                                          shs=scene.shs, language_feature=scene.lang, scales=scene.scales,
                                          rotations=scene.rotations, split_behind_counts=split_behind_counts)
        if before_wait is not None:
            before_wait()
        if radii_out is not None:     # the views' radii MAX, also while the host waits for the counts
            dgr.radii_max_native([pf.radii for pf in pfs], radii_out)
        if 0 < early_views < len(pfs) and scene.means3D.is_cuda:
            dev = scene.means3D.device
            if bin_side[0] is None:
                bin_side[0] = torch.cuda.Stream(device=dev, priority=side_priority)
            side_b = bin_side[0]
            if side_from_preprocess:      # the side binning starts beside the early views' binning
                side_b.wait_stream(torch.cuda.current_stream(dev))   # after the preprocess batch
            dgr.binning_views_native(pfs[:early_views])      # waits for the batch's counts
            if not side_from_preprocess:  # ... or behind it
                side_b.wait_stream(torch.cuda.current_stream(dev))
            for pf in pfs[early_views:]:
                pf.geom.record_stream(side_b)
            dgr.binning_views_native(pfs[early_views:], stream=side_b)
        else:
            dgr.binning_views_native(pfs)
        pending.update(zip(views, pfs))

    def render_view(v: int, bucket: GradBucket):
        if batch_fwd and v not in pending:
            batch_preprocess(v)
        pf = pending.pop(v, None)
        if pf is None:                    # first view of a step: the Gaussians are final here
            pf = preprocess(v)
            if params_ready is not None:
                params_ready.record(torch.cuda.current_stream())
        if lookahead:
            pf.resolve(binning=True)      # count of view v (enqueued a view earlier), then its binning
            if has_view(v + 1):           # view v+1's preprocess ahead of view v's compositing
                pending[v + 1] = preprocess(v + 1, defer=True)
        color, lang, radii, depth, st = dgr.render_native(pf)
        gc, gl, gd = grad_fn(v, color, lang, depth)
        if batched:                   # compositor backward now, preprocess backward at flush
            held.append(dgr.backward_composite_native(st, gc, gl, gd, dL_dlanguage=bucket.views["language_feature"]))
        else:
            dgr.backward_native(st, gc, gl, gd, out=bucket.views, accumulate=True, need=bucket.need(),
                                deterministic=deterministic)
        render_view.last_num_rendered = st.num_rendered
        if side is not None and has_view(v + 1):
            side.wait_event(params_ready)     # orders after the parameters, not after view v's work
            pending[v + 1] = preprocess(v + 1, stream=side)
        return radii

    def render_batch(views, bucket: GradBucket, before_wait=None):
        """Every view of the step at once (ViewParallelStep.run prefers this to per-view calls):
        forward phase 1 and binning as one batch, then per binning batch (the early views binned
        on this stream, the rest on the side stream) ONE compositor forward launch for its views,
        their upstream gradients (grad_fn, as train.py computes the loss on the stacked renders
        before backward), and ONE compositor backward launch.  Two launches per group instead of
        two per view: the chip no longer drains at every view's last waves.  before_wait() (the
        step's bucket zeroing) runs behind the preprocess launches, while the host waits for the
        instance counts.  Returns the radii."""
        views = list(views)
        if not views:
            if before_wait is not None:
                before_wait()
            return []
        reduce_radii = bucket.radii is not None and scene.means3D.is_cuda
        fresh = views[0] not in pending
        if fresh:
            batch_preprocess(views[0], before_wait, radii_out=bucket.radii if reduce_radii else None)
        elif before_wait is not None:
            before_wait()
        pfs = [pending.pop(v) for v in views]
        groups = []                        # consecutive views binned by one launch set (one event)
        for v, pf in zip(views, pfs):
            if groups and groups[-1][0][1].ready is pf.ready:
                groups[-1].append((v, pf))
            else:
                groups.append([(v, pf)])
        radii, ks = [], []
        for grp in groups:
            res = dgr.render_views_native([pf for _, pf in grp])
            gcs, gls, gds = [], [], []
            for (v, _), (color, lang, r, depth, st) in zip(grp, res):
                gc, gl, gd = grad_fn(v, color, lang, depth)
                gcs.append(gc)
                gls.append(gl)
                gds.append(gd)
                radii.append(r)
                ks.append(st.num_rendered)
            held.extend(dgr.backward_composite_views_native([x[4] for x in res], gcs, gls, gds,
                                                            dL_dlanguage=bucket.views["language_feature"]))
        if reduce_radii and not fresh:
            dgr.radii_max_native(radii, bucket.radii)
        render_batch.last_num_rendered = ks
        render_batch.radii_reduced = reduce_radii   # bucket.radii already holds this rank's MAX
        return radii

    def flush(bucket: GradBucket, row_chunks=None, on_rows=None):
        # overwrites every field but the language gradients (all P rows, culled ones with zeros), so
        # ViewParallelStep zeroes only the accumulated fields before the views
        if held:
            dgr.backward_preprocess_views_native(held, out=bucket.views, accumulate=False, need=bucket.need(),
                                                 row_chunks=row_chunks, on_rows=on_rows)
            held.clear()
        else:                             # no views on this rank this step
            lo, hi = bucket.ranges["language_feature"]
            bucket.flat[:lo].zero_()
            bucket.flat[hi:].zero_()
            for r0, r1 in (row_chunks or []):
                if on_rows is not None:
                    on_rows(r0, r1)

    flush.overwrites = True
    flush.chunked = True

    def begin_step(views):
        pending.clear()
        step_views[0] = range(views.start, views.stop) if isinstance(views, range) else list(views)

    def end_step():
        pending.clear()                   # nothing is carried across steps (the Gaussians change)
        step_views[0] = None

    render_view.begin_step = begin_step
    render_view.end_step = end_step
    render_view.pending = pending         # inspection (tests)
    render_view.last_num_rendered = 0
    if batched:
        render_view.flush = flush
        if batch_fwd and composite_batch:
            render_batch.last_num_rendered = []
            render_batch.before_wait = True   # takes the step's zeroing into its host-wait stretch
            render_view.render_batch = render_batch
    return render_view
