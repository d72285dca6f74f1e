#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC here; counters go in separate passes).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -30 "$f"
exit $rc
