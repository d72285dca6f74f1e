#!/bin/bash
# round 5: the packed-fp32 bisection builds under the race tool, then the deform / training / checkpoint tests
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-slp slp_pad1 slp_pad2 slp_wz}" RACE_R=${RACE_R:-6} bash tools/gpu_deform_race.sh; echo "race rc=$?"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_checkpoint_gpu.py tests/test_deform_gpu.py tests/test_deform_lds_poison_gpu.py tests/test_train_step_gpu.py tests/test_train_gpu.py} \
    -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5c_tests.log | tail -40
grep -E "^E " gpurun_out/r5c_tests.log | head -30
exit $rc
