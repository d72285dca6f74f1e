#!/bin/bash
# Device idle gaps and host-side cost of the bench step: the view-parallel GPU tests, a bench line,
# a rocprofv3 kernel trace (tools/trace_gaps.py over one step) and a cProfile of the host loop.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
timeout -k 10 300 python -m pytest tests/test_view_parallel_gpu.py -q -x -p no:cacheprovider > gpurun_out/gaps/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/gaps/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/gaps/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/gaps/bench.log | tail -1 | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS:-} > gpurun_out/gaps/prof_bench.log 2>&1 || exit $?
python3 tools/trace_gaps.py "$(find gpurun_out/gaps/prof -name '*kernel_trace.csv' | head -1)" 8
timeout -k 10 300 python3 -m cProfile -s tottime bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile ${BENCH_ARGS:-} \
    > gpurun_out/gaps/cprof.log 2>&1 || exit $?
grep -A25 "Ordered by" gpurun_out/gaps/cprof.log
