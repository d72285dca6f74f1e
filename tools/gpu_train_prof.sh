#!/bin/bash
# rocprofv3 kernel stats of the configs[4] stand-in loop (tools/bench_train_loop.py, $ITERS iterations)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/tlprof; mkdir -p gpurun_out/tlprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tlprof -o run -- \
    python3 tools/bench_train_loop.py --iters ${ITERS:-300} > gpurun_out/tlprof/b.log 2>&1 || { tail -5 gpurun_out/tlprof/b.log; exit 1; }
grep -h '^{' gpurun_out/tlprof/b.log | cut -c1-200
f=$(find gpurun_out/tlprof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -16
