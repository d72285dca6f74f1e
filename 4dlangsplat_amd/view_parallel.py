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

    def __init__(self, P: int, M: int, C: int, device, densify_stats: bool = False, row_multiple: int = 1):
        """row_multiple: every field is allocated with Pa >= P rows, a multiple of row_multiple (the
        rows past P stay zero), so that a reduce-scatter can split each field into equal row shards
        (ShardedAdam); the views cover the first P rows."""
        self.P, self.M, self.C = P, M, C
        self.Pa = -(-P // row_multiple) * row_multiple if P > 0 else 0
        self.densify_stats = densify_stats
        fields = [(n, w if w is not None else (3 * M if n == "sh" else C)) for n, w in GRAD_FIELDS]
        if densify_stats:
            fields.append(("means2D", 3))
        self.widths = dict(fields)
        self.floats_per_gaussian = sum(w for _, w in fields)
        Pa = self.Pa
        self.flat = torch.zeros(Pa * self.floats_per_gaussian, dtype=torch.float32, device=device)
        self.views: Dict[str, Optional[torch.Tensor]] = {}
        self.ranges: Dict[str, Tuple[int, int]] = {}     # field -> [start, end) in flat (Pa rows)
        o = 0
        for name, w in fields:
            seg = self.flat[o * Pa:o * Pa + w * P]
            self.ranges[name] = (o * Pa, (o + w) * Pa)
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

    def __init__(self, bucket: GradBucket, n_views: int, group=None, flush_chunks: int = 4, update=None,
                 defer_gather: bool = False):
        """update: a ShardedAdam.  Without it the step ends with the bucket SUM all-reduced on every
        rank; with it the bucket is reduce-scattered by Gaussian rows, each rank runs Adam on its row
        shard and the updated rasterizer inputs are all-gathered (update.step).

        defer_gather (opt-in, needs a renderer with set_row_waits): run() returns with the
        all-gathers into the scene's tensors still in flight, and the next run()'s preprocess waits
        for each row chunk as it lands.  Between such steps the scene's rows may be old or
        half-written: call finish() before anything else reads the scene (evaluation,
        densification, capture).  By default run() returns with the scene final."""
        self.update = update
        self.defer_gather = bool(defer_gather)
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
        upd = self.update
        defer = False
        if upd is not None and hasattr(upd, "gather_waits"):
            # the previous step's all-gathers may still be in flight: a renderer that preprocesses by
            # row chunks waits for each chunk's rows itself, any other waits for all of them now
            waits = upd.gather_waits()
            setter = getattr(render_view, "set_row_waits", None) if self.defer_gather else None
            if waits and setter is not None:
                setter(waits)
                upd._ag = []
            else:
                upd.wait_all()
            defer = setter is not None
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
        sharded = self.update is not None
        if self.world > 1 and flush is not None and hi > lo and not sharded:
            # with the batched backward the language gradients are final once the last view's
            # compositor backward ran; their SUM runs during the flush (the preprocess backward,
            # which writes every other field) instead of after it
            pending.append(dist.all_reduce(b.flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        chunked = self.world > 1 and getattr(flush, "chunked", False) and self.flush_chunks > 1 and not sharded
        sharded_chunks = sharded and getattr(flush, "chunked", False) and getattr(self.update, "chunks", 1) > 1
        if sharded_chunks:
            # the flush in the optimizer's row chunks: each chunk's reduce-scatters start behind it
            flush(b, row_chunks=self.update.chunk_rows(), on_rows=lambda r0, r1: self.update.on_rows(b, r0, r1))
        elif chunked:
            # the flush in Gaussian-row chunks: each chunk's rows of every other field are SUMmed
            # (asynchronously, behind that chunk's launch) while the next chunk is computed
            def on_rows(r0, r1):
                for name, (f0, f1) in b.ranges.items():
                    w = b.widths[name]
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
        if sharded:
            if defer:
                self.update.step(b, wait_gather=False)   # the next step's preprocess waits per row chunk
            else:
                self.update.step(b)
            for h in pending:
                h.wait()
        elif self.world > 1:
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

    def finish(self) -> None:
        """Wait for the all-gathers a defer_gather step left in flight: the scene is final after it."""
        if self.update is not None and hasattr(self.update, "wait_all"):
            self.update.wait_all()

    def visibility(self) -> torch.Tensor:
        """ANY over the batch's views (train.py:271): a Gaussian is visible if some view gave it
        a positive radius."""
        if self.bucket.radii is None:
            raise RuntimeError("visibility needs GradBucket(densify_stats=True)")
        return self.bucket.radii > 0


def native_view_renderer(scene, settings, grad_fn: Callable, deterministic: bool = False, overlap: bool = True,
                         batch_backward: bool = True, early_views=3, composite_batch: bool = True,
                         side_priority: int = 0, side_from_preprocess: bool = True, split_behind_counts: bool = True,
                         fill_on_side: bool = False, order_on_side: bool = False, tile_bucket: bool = False):
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

    early_views may also be a tuple (e, s1, s2, ...): the first e views binned on the current stream,
    then side-stream binning batches of s1, s2, ... views and one of the rest, in that order, each
    with its own event, so render_batch composites each batch as soon as its own binning is done
    (the first compositor launch waits only for e views' binning).
    With more than `early_views` views in the batch, only the first `early_views` are binned on
    the current stream; the others' binning (emission, tile sort, tile ranges: chains of short,
    dependent launches that leave most of the GPU idle) runs on a side stream while those first
    views composite, and each later view's compositing waits for it (an event); the side binning
    starts right behind the preprocess batch, beside the early views' binning
    (side_from_preprocess; behind it: 925 vs 941 frames/s same-box).  fill_on_side: the language
    split, the step's bucket zeroing and the radii MAX run on that side stream ahead of its
    binning instead of on the main stream between the instance scan and the early views' emission
    (the first compositor launch waits for them).  order_on_side: the later views' depth sorts and
    instance scans run on that side stream too (the preprocess stays one launch for all views): the
    early views' binning no longer waits for every view's depth order, and the later views are
    binned once the early views' compositing is enqueued.  tile_bucket (batched only): the
    tile-bucket binning (no depth sort; instances bucketed by tile, each bucket sorted in LDS:
    preprocess_views_native(tile_bucket=True)); same lists, same results.  With
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
    fill_ready = [None]                   # fill_on_side: the side stream's fills (the compositors wait)
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
    row_waits = [None]                    # [(r0, r1, wait)]: the scene's rows still arriving (ShardedAdam)

    def take_row_waits(chunked_ok):
        """The pending row waits: returned for a row-chunked preprocess, else all waited for here."""
        w, row_waits[0] = row_waits[0], None
        if not w or chunked_ok:
            return w
        for _, _, fn in w:
            fn()
        return None

    def batch_preprocess(v, before_wait=None, radii_out=None):
        """The step's views from v on, as one batch: preprocess + depth sorts + instance scans, one
        host wait for their counts, then their binning (lsr_forward_*_views).  before_wait() is
        enqueued behind the batch's launches, ahead of that wait (work that fills the device's
        idle stretch while the host reads the counts)."""
        views = [w for w in step_views[0] if w >= v] if step_views[0] is not None else [v]
        views = [w for w in views if has_view(w)] or [v]
        sizes = tuple(early_views) if isinstance(early_views, (tuple, list)) else (early_views,)
        e0 = int(sizes[0])
        split_side = 0 < e0 < len(views) and scene.means3D.is_cuda
        if split_side and bin_side[0] is None:
            bin_side[0] = torch.cuda.Stream(device=scene.means3D.device, priority=side_priority)
        to_side = fill_on_side and split_side
        late_order = order_on_side and split_side and not to_side
        waits = take_row_waits(scene.means3D.is_cuda)
        pfs = dgr.preprocess_views_native([settings[w] for w in views], scene.means3D, scene.opacities,
                                          shs=scene.shs, language_feature=scene.lang, scales=scene.scales,
                                          rotations=scene.rotations, split_behind_counts=split_behind_counts,
                                          split_stream=bin_side[0] if to_side else None,
                                          order_first=e0 if late_order else None,
                                          order_stream=bin_side[0] if late_order else None,
                                          row_chunks=waits, tile_bucket=tile_bucket)
        fill_ready[0] = None
        if to_side:                   # the fills beside the early views' binning, ahead of the side binning
            bin_side[0].wait_stream(torch.cuda.current_stream(scene.means3D.device))   # after the preprocess batch
            with torch.cuda.stream(bin_side[0]):
                if before_wait is not None:
                    before_wait()
                if radii_out is not None:
                    for pf in pfs:
                        pf.radii.record_stream(bin_side[0])
                    dgr.radii_max_native([pf.radii for pf in pfs], radii_out, stream=bin_side[0])
            fill_ready[0] = torch.cuda.Event()
            fill_ready[0].record(bin_side[0])
        else:
            if before_wait is not None:
                before_wait()
            if radii_out is not None:     # the views' radii MAX, also while the host waits for the counts
                dgr.radii_max_native([pf.radii for pf in pfs], radii_out)
        if late_order:   # the later views are binned by render_batch, after the early views' compositing
            dgr.binning_views_native(pfs[:e0])
        elif split_side:
            dev = scene.means3D.device
            side_b = bin_side[0]
            if side_from_preprocess and not to_side:   # the side binning starts beside the early views' binning
                side_b.wait_stream(torch.cuda.current_stream(dev))   # after the preprocess batch
            dgr.binning_views_native(pfs[:e0])      # waits for the batch's counts
            if not side_from_preprocess:  # ... or behind it
                side_b.wait_stream(torch.cuda.current_stream(dev))
            for pf in pfs[e0:]:
                pf.geom.record_stream(side_b)
            cuts = [e0]
            for n in sizes[1:]:
                if cuts[-1] + int(n) < len(views):
                    cuts.append(cuts[-1] + int(n))
            cuts.append(len(views))
            for a0, a1 in zip(cuts, cuts[1:]):   # each side batch with its own event
                dgr.binning_views_native(pfs[a0:a1], stream=side_b)
        else:
            dgr.binning_views_native(pfs)
        pending.update(zip(views, pfs))

    def render_view(v: int, bucket: GradBucket):
        if batch_fwd and v not in pending:
            batch_preprocess(v)
        take_row_waits(False)             # per-view preprocess: every row first
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
        if fill_ready[0] is not None:      # the language split and the bucket zeroing ran on the side stream
            torch.cuda.current_stream(scene.means3D.device).wait_event(fill_ready[0])
            fill_ready[0] = None
        groups = []                        # consecutive views binned by one launch set (one event)
        for v, pf in zip(views, pfs):
            if groups and groups[-1][0][1].ready is pf.ready:
                groups[-1].append((v, pf))
            else:
                groups.append([(v, pf)])
        radii, ks = [], []
        sizes = tuple(early_views) if isinstance(early_views, (tuple, list)) else (early_views,)
        split_groups = []
        for grp in groups:
            unbinned = [pf for _, pf in grp if getattr(pf, "binning", True) is None]
            if unbinned and unbinned[0].stream is not None and unbinned[0].stream != torch.cuda.current_stream(
                    scene.means3D.device):   # depth-ordered on the side stream (order_on_side): binned there too,
                # in the batches early_views[1:] names (each with its own event, so each composites as soon
                # as it is binned), all enqueued before any of them composites
                cuts = [0]
                for n in sizes[1:]:
                    if cuts[-1] + int(n) < len(grp):
                        cuts.append(cuts[-1] + int(n))
                cuts.append(len(grp))
                for a0, a1 in zip(cuts, cuts[1:]):
                    dgr.binning_views_native([pf for _, pf in grp[a0:a1]], stream=unbinned[0].stream)
                    split_groups.append(grp[a0:a1])
            else:
                split_groups.append(grp)
        for grp in split_groups:
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

    def set_row_waits(waits):
        row_waits[0] = list(waits) if waits else None

    render_view.begin_step = begin_step
    render_view.end_step = end_step
    render_view.set_row_waits = set_row_waits
    render_view.pending = pending         # inspection (tests)
    render_view.last_num_rendered = 0
    if batched:
        render_view.flush = flush
        if batch_fwd and composite_batch:
            render_batch.last_num_rendered = []
            render_batch.before_wait = True   # takes the step's zeroing into its host-wait stretch
            render_view.render_batch = render_batch
    return render_view


class ShardedAdam:
    """The optimizer step of a view-parallel training step, sharded by Gaussian rows (ZeRO-1 style;
    the reference runs one process: loss.backward(), then optimizer.step(), train.py:339,420-421).

    Every rank holds the ACTIVATED rasterizer inputs of all P Gaussians (what the views render: the
    scene's means3D, scales, rotations, opacities, shs, lang); the raw parameters and both Adam moments
    exist only for the rank's row shard.  step(bucket), once the views' gradients are in the bucket:
      1. reduce-scatter each gradient field by rows: the rank receives the SUM over every rank's views
         of its own rows only;
      2. back through the activations (gaussian_renderer/__init__.py:95-97,191-193 and the model's
         activations, scene/gaussian_model.py:38-47): scaling exp, opacity sigmoid, rotation and
         language L2 normalisations; SH split into f_dc / f_rest;
      3. Adam on the shard (lsr_adam_step; `adam` overrides it for the CPU tests), torch.optim.Adam's
         arithmetic with eps 1e-15;
      4. the activations again, on the shard, and an all-gather of each activated field back into the
         scene's tensors, which the next step renders.
    The traffic per rank is (N-1)/N of the bucket (reduce-scatter) plus (N-1)/N of the activated
    inputs (all-gather) -- the volume of the all-reduce it replaces -- while the activation math and
    Adam run on 1/N of the rows and the parameters' optimizer state shrinks N-fold.

    chunks = C > 1 pipelines it by row chunks.  The row space [0, Pa) is cut into C chunks of
    Pa / C rows and each chunk into one piece per rank (the rank's shard is its C pieces), so every
    chunk is reduce-scattered and all-gathered as a contiguous row range of its own:
      * the flush (the batched preprocess backward, which writes every non-language gradient row)
        runs in these chunks and reports each (on_rows): the chunk's reduce-scatters start right behind
        its launch while the next chunk is computed;
      * step() takes the chunks in order: wait for the chunk's reduce-scatters, activations' backward +
        Adam + activations on the rank's piece, start the chunk's all-gathers -- and returns without
        waiting for them;
      * the next step's renderer preprocesses each row chunk once its all-gather is in
        (gather_waits(), native_view_renderer's row waits: lsr_forward_preprocess_views_rows_async per
        chunk), so the all-gather overlaps the last chunks' Adam and the first chunks' preprocess.
        A renderer that cannot wait per chunk gets wait_all() before the step.
    Shard boundaries are multiples of `align` rows (256 with chunks > 1, the preprocess's row-chunk
    granularity); the bucket must be built with GradBucket(row_multiple=ShardedAdam.row_multiple(...))."""

    GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation", "language_feature")
    BUCKET_FIELDS = ("means3D", "scales", "rotations", "opacities", "sh", "language_feature")
    ACT_FIELDS = ("means3D", "scales", "rotations", "opacities", "shs", "lang")

    @staticmethod
    def row_multiple(P: int, world: int, align: int = 64, chunks: int = 1) -> int:
        """Pa: a multiple of world * chunks * piece alignment covering P rows."""
        align = max(align, 256) if chunks > 1 else align
        unit = world * max(1, chunks) * align
        return -(-max(P, 1) // unit) * unit

    def __init__(self, scene, raw: Dict[str, torch.Tensor], lrs: Dict[str, float], group=None, align: int = 64,
                 betas=(0.9, 0.999), eps: float = 1e-15, adam: Optional[Callable] = None, nonormalized: bool = False,
                 chunks: int = 1):
        """scene: object with the activated tensors (means3D, scales, rotations, opacities, shs, lang);
        they are re-bound to row-padded storage.  raw: the full raw parameters (xyz, f_dc, f_rest,
        opacity, scaling, rotation, language_feature), of which this rank keeps its shard.
        adam(p, g, m, v, lr, step): in place on one group's rows (default: lsr_adam_step)."""
        if getattr(scene, "deformation", None) is not None:
            # the bucket's means3D gradient is the xyz gradient and the gathered rows are the
            # rasterizer's inputs only without a field between the parameters and the rasterizer
            raise ValueError("ShardedAdam steps the rasterizer inputs directly: a scene with a deformation "
                             "field needs the field's backward between the bucket and the parameters")
        self.distributed = dist.is_available() and dist.is_initialized()
        self.group = group
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.xyz_scheduler_args = None
        self.chunks = max(1, int(chunks))
        self.P = P = scene.means3D.shape[0]
        self.Pa = self.row_multiple(P, self.world, align, self.chunks) if P > 0 else 0
        self.Pc = self.Pa // self.chunks                # rows per chunk
        self.piece = self.Pc // self.world              # rows per rank per chunk
        self.rows = self.chunks * self.piece            # the shard (padding rows past P included)
        # the rank's pieces: shard rows [c piece, (c + 1) piece) are global rows [g0, g0 + piece)
        self.pieces = [(c * self.Pc + self.rank * self.piece, c * self.Pc + (self.rank + 1) * self.piece)
                       for c in range(self.chunks)]
        # chunks = 1: the shard is one contiguous row range [r0, r1) (clipped to P)
        self.r0 = min(P, self.pieces[0][0]) if self.pieces else 0
        self.r1 = min(P, self.pieces[0][1]) if self.pieces else 0
        self.lrs, self.betas, self.eps, self.nonormalized = dict(lrs), betas, eps, nonormalized
        self._adam = adam
        self.scene = scene
        dev = scene.means3D.device
        # activated inputs in row-padded storage (all-gather target); the scene's tensors view it
        self.act = {}
        for name in self.ACT_FIELDS:
            t = getattr(scene, name)
            buf = torch.zeros((self.Pa,) + tuple(t.shape[1:]), dtype=torch.float32, device=dev)
            buf[:P] = t
            self.act[name] = buf
            setattr(scene, name, buf[:P])
        self.raw = {}
        for n in self.GROUPS:
            if n not in raw:
                continue
            src = raw[n].detach().to(dev, torch.float32)
            t = torch.zeros((self.rows,) + tuple(src.shape[1:]), dtype=torch.float32, device=dev)
            for c, (g0, g1) in enumerate(self.pieces):
                hi = min(g1, P)
                if hi > g0:
                    t[c * self.piece:c * self.piece + hi - g0] = src[g0:hi]
            self.raw[n] = t.contiguous()
        self.exp_avg = {n: torch.zeros_like(t) for n, t in self.raw.items()}
        self.exp_avg_sq = {n: torch.zeros_like(t) for n, t in self.raw.items()}
        self.steps = {n: 0 for n in self.raw}
        self._rs = {}            # chunk -> (shard gradient rows per field, handles): reduce-scatters in flight
        self._ag = []            # [(r0, r1, handles)]: the last step's all-gathers, not yet waited for
        # inspection (tests): grad_hook(step, g0, valid, grads) sees each piece's reduced gradients of
        # the raw groups (after the activations' backward, before Adam): global rows [g0, g0 + valid)
        self.grad_hook: Optional[Callable] = None

    # ---- learning rate (gaussian_model.py:302-329; GaussianTrainer's schedule) ----------------------
    def set_xyz_schedule(self, lr_init, lr_final, lr_delay_mult=0.01, max_steps=30000):
        from gaussian_train import get_expon_lr_func
        self.xyz_scheduler_args = get_expon_lr_func(lr_init=lr_init, lr_final=lr_final, lr_delay_mult=lr_delay_mult,
                                                    max_steps=max_steps)

    def update_learning_rate(self, iteration):
        """train.py:233 calls gaussians.update_learning_rate(iteration) at every iteration: the xyz
        group follows its exponential schedule (every rank computes the same value)."""
        if self.xyz_scheduler_args is not None and "xyz" in self.lrs:
            self.lrs["xyz"] = float(self.xyz_scheduler_args(iteration))
        return self.lrs.get("xyz")

    # ---- row chunks ----------------------------------------------------------------------------------
    def chunk_rows(self):
        """The chunks' global row ranges clipped to [0, P) (empty ones dropped): the flush's row_chunks."""
        out = []
        for c in range(self.chunks):
            r0, r1 = c * self.Pc, min((c + 1) * self.Pc, self.P)
            if r1 > r0:
                out.append((r0, r1))
        return out

    def gather_waits(self):
        """[(r0, r1, wait)] over [0, P) for the all-gathers still in flight (wait() makes the current
        stream, or with gloo the host, wait for that chunk's rows); [] when none are."""
        out = []
        for r0, r1, hs in self._ag:
            r1 = min(r1, self.P)
            if r1 > r0:
                out.append((r0, r1, (lambda hs=hs: [h.wait() for h in hs])))
        return out

    def wait_all(self):
        for _, _, hs in self._ag:
            for h in hs:
                h.wait()
        self._ag = []

    # ---- 1. reduce-scatter ------------------------------------------------------------------------
    def _issue_rs(self, bucket, c):
        if c in self._rs:
            return
        if bucket.Pa != self.Pa:
            raise ValueError(f"bucket rows {bucket.Pa} != {self.Pa}: build it with GradBucket(row_multiple=...)")
        out, handles = {}, []
        for name in self.BUCKET_FIELDS:
            f0, _ = bucket.ranges[name]
            w = bucket.widths[name]
            if w == 0:
                continue
            full = bucket.flat[f0 + c * self.Pc * w:f0 + (c + 1) * self.Pc * w]
            if self.world > 1:
                shard = torch.empty(self.piece * w, dtype=torch.float32, device=full.device)
                handles.append(dist.reduce_scatter_tensor(shard, full, group=self.group, async_op=True))
            else:
                shard = full
            out[name] = shard.view(self.piece, w)
        self._rs[c] = (out, handles)

    def on_rows(self, bucket, r0, r1):
        """The flush finished rows [r0, r1) of every gradient field: reduce-scatter the chunks they complete."""
        for c in range(self.chunks):
            if r0 <= c * self.Pc and min((c + 1) * self.Pc, self.P) <= r1:
                self._issue_rs(bucket, c)

    # ---- 2. activations' backward, 3. Adam, 4. activations + all-gather ----------------------------------
    def _lang_act(self, x):
        return x if self.nonormalized else x / (x.norm(dim=-1, keepdim=True) + 1e-9)

    def step(self, bucket, wait_gather: bool = True) -> None:
        """wait_gather=False returns with the all-gathers in flight (gather_waits / wait_all)."""
        self.wait_all()   # a previous step's gathers (nothing may overwrite the scene rows under them)
        for n in self.raw:
            self.steps[n] += 1
        for c in range(self.chunks):
            self._issue_rs(bucket, c)
        for c in range(self.chunks):
            g, handles = self._rs.pop(c)
            for h in handles:
                h.wait()
            self._step_chunk(c, g)
        if wait_gather:
            self.wait_all()

    def _step_chunk(self, c, g):
        sl = slice(c * self.piece, (c + 1) * self.piece)
        raw = {n: t[sl] for n, t in self.raw.items()}
        n_rows = self.piece
        grads = {}
        if "means3D" in g:
            grads["xyz"] = g["means3D"]
        if "sh" in g:
            sh = g["sh"].reshape(n_rows, -1, 3)
            grads["f_dc"], grads["f_rest"] = sh[:, :1], sh[:, 1:]
        if "opacities" in g and "opacity" in raw:
            o = torch.sigmoid(raw["opacity"])
            grads["opacity"] = g["opacities"].reshape(o.shape) * o * (1 - o)
        if "scales" in g and "scaling" in raw:
            grads["scaling"] = g["scales"] * torch.exp(raw["scaling"])
        if "rotations" in g and "rotation" in raw:
            q = raw["rotation"]
            nq = q.norm(dim=-1, keepdim=True).clamp_min(1e-12)      # F.normalize's eps
            r = q / nq
            gr = g["rotations"]
            grads["rotation"] = (gr - r * (r * gr).sum(-1, keepdim=True)) / nq
        if "language_feature" in g and "language_feature" in raw:
            x, gl = raw["language_feature"], g["language_feature"]
            if self.nonormalized:
                grads["language_feature"] = gl
            else:
                nx = x.norm(dim=-1, keepdim=True)
                d = nx + 1e-9
                grads["language_feature"] = gl / d - x * (x * gl).sum(-1, keepdim=True) / (nx.clamp_min(1e-30) * d * d)
        if self.grad_hook is not None:
            g0 = self.pieces[c][0]
            self.grad_hook(max(self.steps.values(), default=0), g0, max(0, min(self.piece, self.P - g0)),
                           {n: gr for n, gr in grads.items() if n in raw and n in self.lrs})
        for name, gr in grads.items():
            if name not in raw or name not in self.lrs:
                continue
            gr = gr.reshape(raw[name].shape).contiguous()
            self._adam_group(raw[name], gr, self.exp_avg[name][sl], self.exp_avg_sq[name][sl], self.lrs[name],
                             self.steps[name])
        # 4. activated piece rows, gathered into every rank's scene tensors
        act_rows = dict(means3D=raw.get("xyz"), scales=torch.exp(raw["scaling"]) if "scaling" in raw else None,
                        rotations=torch.nn.functional.normalize(raw["rotation"]) if "rotation" in raw else None,
                        opacities=torch.sigmoid(raw["opacity"]) if "opacity" in raw else None,
                        shs=torch.cat([raw["f_dc"], raw["f_rest"]], dim=1) if "f_dc" in raw else None,
                        lang=self._lang_act(raw["language_feature"]) if "language_feature" in raw else None)
        g0 = self.pieces[c][0]
        valid = max(0, min(self.piece, self.P - g0))   # rows past P stay as they are (never rendered)
        handles = []
        for name, rows in act_rows.items():
            if rows is None:
                continue
            buf = self.act[name]
            w = buf[0].numel() if self.Pa else 0
            flat = buf.view(self.Pa, -1)
            mine = flat[g0:g0 + self.piece]
            if valid > 0:
                mine[:valid] = rows.reshape(self.piece, w)[:valid]
            if self.world > 1:
                chunk = flat[c * self.Pc:(c + 1) * self.Pc]
                handles.append(dist.all_gather_into_tensor(chunk.reshape(-1), mine.reshape(-1).clone(), group=self.group,
                                                           async_op=True))
        self._ag.append((c * self.Pc, (c + 1) * self.Pc, handles))

    def full_rows(self, name: str) -> torch.Tensor:
        """This rank's shard of raw group `name` as (global row index tensor, rows) clipped to P (tests)."""
        idx, parts = [], []
        for c, (g0, g1) in enumerate(self.pieces):
            hi = min(g1, self.P)
            if hi > g0:
                idx.append(torch.arange(g0, hi))
                parts.append(self.raw[name][c * self.piece:c * self.piece + hi - g0])
        if not idx:
            return torch.zeros(0, dtype=torch.long), self.raw[name][:0]
        return torch.cat(idx), torch.cat(parts)

    def _adam_group(self, p, g, m, v, lr, step):
        if self._adam is not None:
            self._adam(p, g, m, v, lr, step)
            return
        import ctypes

        from diff_gaussian_rasterization import _lib
        L = _lib.load()
        ag = _lib.AdamGroup()
        ag.param, ag.grad, ag.exp_avg, ag.exp_avg_sq = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
        ag.n, ag.lr, ag.step = p.numel(), float(lr), int(step)
        arr = (_lib.AdamGroup * 1)(ag)
        _lib.check(L.lsr_adam_step(arr, 1, self.betas[0], self.betas[1], self.eps,
                                   ctypes.c_void_p(torch.cuda.current_stream(p.device).cuda_stream)), "lsr_adam_step")
