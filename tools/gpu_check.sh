#!/bin/bash
# One GPU call: the GPU test suite (optionally filtered by PYTEST_ARGS), then the default bench line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/t.log 2>&1; rc=$?
grep -E "passed|failed|PASSED|FAILED|Error" gpurun_out/t.log | tail -${TAIL:-15}
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | tail -1
