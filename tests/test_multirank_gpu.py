"""configs[3]'s code path on the one-GPU box (BASELINE.json: 64-view batch, per-view data parallel,
8 x MI355X over RCCL).  The box has one GPU, so the ranks share it and the collectives run over
gloo (LSR_BENCH_BACKEND=gloo, LSR_BENCH_SHARE_DEVICE=1); everything above the collectives is the
product path: bench.py's rank spawn (view_parallel.launch_ranks), the device binding, the barrier
and MAX-over-ranks timing, the view slicing, the batched renderer, the bucket's SUM and the radii
MAX, and ShardedAdam's reduce-scatter / Adam on the row shard / all-gather.  The scaling curve
itself (RCCL over xGMI, one GPU per rank) stays unmeasured here: the driver runs it on an 8-GPU
node.  Every multi-rank run is a fresh child process (subprocess.run), never an exec of this one.
Reference semantics: train.py:242-271 (views rendered in a loop, radii MAX, visibility ANY),
:339 (one backward over the batch), :420-421 (optimizer step)."""
import json
import os
import subprocess
import sys
import tempfile

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import mp_view_parallel_gpu as mpv  # noqa: E402

pytestmark = pytest.mark.gpu


def _env():
    env = dict(os.environ)
    env.update(LSR_BENCH_BACKEND="gloo", LSR_BENCH_SHARE_DEVICE="1", MASTER_ADDR="127.0.0.1",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("MASTER_PORT", None)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


@pytest.mark.timeout(420)
def test_bench_two_ranks_prints_one_line():
    """bench.py --gpus 2 at the headline size (2M, 1352x1014, C = 32, 8 views per rank): one JSON
    line from rank 0 with both ranks' 16 views counted and the process group's rank count."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--single-view-steps", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks"] == 2
    assert line["config"]["global_batch"] == 16 and line["config"]["parallelism"] == "dp2"
    assert line["steps"] == 2 and line["value"] > 0
    assert abs(line["value"] - 16 * 2 / (line["ms_per_step"] * 2e-3)) <= 1e-3 * line["value"]
    # the dominant kernel is picked by event time; with both ranks on one device an event pair of one
    # rank also spans the other rank's kernels, so which phase comes out ahead here is arbitrary (the
    # one-GPU line, where it is render_bwd, is bench.py's own run)
    assert line["roofline"]["kernel"] in ("render_bwd", "render_fwd", "preprocess", "preprocess_bwd_views",
                                          "preprocess_bwd", "emit", "tile_ranges")
    assert line["roofline"]["frac"] > 0 and line["cpu_baseline"] is None


def _spawn(mode, steps, chunks=1):
    d = tempfile.mkdtemp(prefix="lsr_mp_")
    cmd = [sys.executable, os.path.join(HERE, "mp_view_parallel_gpu.py"), "--out", d, "--world", "2",
           "--mode", mode, "--steps", str(steps), "--chunks", str(chunks)]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    outs = [torch.load(os.path.join(d, f"rank{k}.pt"), weights_only=True) for k in range(2)]
    for k in range(2):
        os.remove(os.path.join(d, f"rank{k}.pt"))
    os.rmdir(d)
    return outs


@pytest.mark.timeout(300)
def test_two_rank_bucket_equals_one_rank_sum():
    """Two ranks (views 0-7 and 8-15, the batched renderer with 3 early views each) end the step
    with the same bucket on both ranks, equal to one rank rendering all 16 views up to the fp32
    reassociation of the float-atomic view sums; radii MAX exactly."""
    ser = mpv.run_rank(0, 1, None, "allreduce", 1)
    outs = _spawn("allreduce", 1)
    assert outs[0]["views"] == list(range(8)) and outs[1]["views"] == list(range(8, 16))
    assert ser["views"] == list(range(16))
    for k, v in ser["grads"].items():
        if v is None:
            continue
        a, b = outs[0]["grads"][k], outs[1]["grads"][k]
        assert torch.equal(a, b), k                      # the all-reduce leaves every rank the same sum
        scale = float(v.abs().max())
        assert scale > 0, k
        assert float((a - v).abs().max()) <= 1e-5 * scale, (k, float((a - v).abs().max()), scale)
    assert torch.equal(outs[0]["radii"], ser["radii"]) and torch.equal(outs[1]["radii"], ser["radii"])


def _assemble(outs, k):
    """[P, ...] rows of raw group k from the ranks' shards (ShardedAdam.full_rows: global row ids, rows)."""
    rows0 = outs[0]["full"][k][1]
    got = torch.zeros((mpv.P,) + tuple(rows0.shape[1:]), dtype=rows0.dtype)
    seen = torch.zeros(mpv.P, dtype=torch.bool)
    for o in outs:
        idx, rows = o["full"][k]
        assert not seen[idx].any()
        got[idx], seen[idx] = rows, True
    assert bool(seen.all()), k
    return got


@pytest.mark.timeout(300)
@pytest.mark.parametrize("chunks", [1, 4])
def test_two_rank_sharded_adam_equals_serial(chunks):
    """Two optimizer steps with ShardedAdam (reduce-scatter by Gaussian rows, lsr_adam_step on each
    rank's shard, all-gather of the activated inputs) against one rank doing every view and row.
    chunks = 4: the chunk pipeline (each flush chunk's reduce-scatter behind its launch, Adam and the
    all-gather chunk by chunk, and the second step's batched preprocess launched per row chunk as
    each chunk's gather lands: lsr_forward_preprocess_views_rows_async).  Both ranks render the same
    scene afterwards; parameters agree up to the view sums' fp32 reassociation (Adam's first step
    moves a parameter by about lr * sign(g), so a gradient within rounding of zero may move either
    way: bounded by 2 lr per step)."""
    steps = 2
    ser = mpv.run_rank(0, 1, None, "sharded", steps)
    outs = _spawn("sharded", steps, chunks)
    if chunks == 1:
        r0, r1 = outs[0]["rows"], outs[1]["rows"]
        assert r0[0] == 0 and r0[1] == r1[0] and r1[1] == mpv.P
    init = mpv.raw_scene()[1]
    for k in ser["full"]:
        v = _assemble([ser], k)
        got = _assemble(outs, k)
        assert float((v - init[k]).abs().max()) > 0, k               # the step moved the parameters
        d = (got - v).abs()
        tight = d <= 1e-6 + 1e-5 * v.abs()
        # a few near-zero gradients may flip Adam's first-step sign (one opacity of the 10k rows did in
        # one run); a wrong reduction would move most rows
        assert float(tight.double().mean()) >= 0.999, (k, float(d.max()))
        assert float(d.max()) <= 2 * mpv.LRS[k] * steps, (k, float(d.max()))
    for k, v in ser["act"].items():
        assert torch.equal(outs[0]["act"][k], outs[1]["act"][k]), k   # every rank renders the same scene
        d = (outs[0]["act"][k] - v).abs()
        assert float((d <= 1e-5 + 1e-4 * v.abs()).double().mean()) >= 0.999, k
    assert torch.equal(outs[0]["radii"], ser["radii"])
