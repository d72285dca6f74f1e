#!/bin/bash
# deformation measurement set: tools/bench_deform.py at 2M (with the eager-PyTorch comparison), the
# configs[4] stand-in loop (tools/bench_train_loop.py), and a rocprofv3 kernel-stats pass of the 2M
# bench.  Output: gpurun_out/r5d/
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5d
timeout -k 10 300 python tools/bench_deform.py --iters 20 > gpurun_out/r5d/bench_deform.log 2>&1 || { tail -5 gpurun_out/r5d/bench_deform.log; exit 1; }
grep '^{' gpurun_out/r5d/bench_deform.log > gpurun_out/r5d/bench_deform.json; cat gpurun_out/r5d/bench_deform.json | cut -c1-300
timeout -k 10 400 python tools/bench_train_loop.py > gpurun_out/r5d/bench_train_loop.log 2>&1 || { tail -5 gpurun_out/r5d/bench_train_loop.log; exit 1; }
grep '^{' gpurun_out/r5d/bench_train_loop.log | tail -1 > gpurun_out/r5d/bench_train_loop.json; cut -c1-400 gpurun_out/r5d/bench_train_loop.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5d/prof -o run -- \
    python3 tools/bench_deform.py --no-torch --iters 10 > gpurun_out/r5d/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
f=$(find gpurun_out/r5d/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5d/deform_kernel_stats.csv
rm -rf gpurun_out/r5d/prof
