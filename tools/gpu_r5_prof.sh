#!/bin/bash
# round-5 measurement set: bench line (with cpu_baseline + configs0), rocprofv3 kernel trace + stats,
# the step timeline, and the PMC passes (whole-step traffic included).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r5p/bench.log 2>&1 || { tail -5 gpurun_out/r5p/bench.log; exit 1; }
grep '^{' gpurun_out/r5p/bench.log | tail -1 > gpurun_out/r5p/bench.json; head -c 600 gpurun_out/r5p/bench.json; echo
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5p/prof -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --single-view-steps 0 > gpurun_out/r5p/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r5p/prof_bench.log; exit 1; }
f=$(find gpurun_out/r5p/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5p/kernel_stats.csv; head -12 gpurun_out/r5p/kernel_stats.csv | cut -c1-150
t=$(find gpurun_out/r5p/prof -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5p/step_timeline.txt; tail -25 gpurun_out/r5p/step_timeline.txt
grep '^{' gpurun_out/r5p/prof_bench.log | tail -1 > gpurun_out/r5p/bench_under_rocprof.json
rm -rf gpurun_out/pmc
BENCH_ARGS="--single-view-steps 0" bash tools/gpu_pmc.sh > gpurun_out/r5p/pmc.log 2>&1; rc=$?
tail -4 gpurun_out/r5p/pmc.log
cp gpurun_out/pmc/summary.txt gpurun_out/r5p/pmc_summary.txt 2>/dev/null; cp gpurun_out/pmc/pmc_traffic.json gpurun_out/r5p/pmc_traffic.json 2>/dev/null
rm -rf gpurun_out/r5p/prof gpurun_out/pmc/p*/
exit $rc
