#!/bin/bash
# round 5: packed-fp32 bisection (race tool per build), then the round's changed-path tests, then the bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-slp slp_pad1 slp_pad2 slp_wz}" RACE_R=${RACE_R:-6} bash tools/gpu_deform_race.sh; echo "race rc=$?"
if [ -f 4dlangsplat_amd/build/variants/liblsr_fcount.so ]; then
  LSR_LIBRARY=4dlangsplat_amd/build/variants/liblsr_fcount.so timeout -k 10 240 python tools/fwd_activity.py > gpurun_out/fwd_activity.json 2> gpurun_out/fwd_activity.err; echo "fwd_activity rc=$?"; tail -c 1200 gpurun_out/fwd_activity.json
fi
timeout -k 10 780 python -u -m pytest ${TESTS:-tests/test_multirank_gpu.py tests/test_checkpoint_gpu.py tests/test_deform_gpu.py tests/test_deform_lds_poison_gpu.py tests/test_train_step_gpu.py tests/test_view_parallel_gpu.py tests/test_abi.py} \
    -m "gpu or not gpu" -v --timeout 420 --timeout-method thread -p no:cacheprovider > gpurun_out/r5d_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5d_tests.log | tail -60
grep -E "^E " gpurun_out/r5d_tests.log | head -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --single-view-steps 0 > gpurun_out/r5d_bench.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r5d_bench.log
exit $rc
