#!/bin/bash
# round 5: the new multi-rank / checkpoint / 8-view headline tests, then the bench (with cpu_baseline).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_multirank_gpu.py tests/test_checkpoint_gpu.py tests/test_headline_gpu.py} \
    -m gpu -v -x --timeout 420 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5a_tests.log | tail -20
grep -E "^E " gpurun_out/r5a_tests.log | head -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/r5a_bench.log 2>&1; rc=$?
tail -c 3000 gpurun_out/r5a_bench.log
exit $rc
