#!/bin/bash
# Iteration loop: parity tests (PYTEST_ARGS filter), then REPS headline bench runs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/iter_tests.log 2>&1; rc=$?
tail -3 gpurun_out/iter_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" gpurun_out/iter_tests.log | head -20; exit $rc; fi
REPS=${REPS:-2} bash tools/gpu_bench_rep.sh
