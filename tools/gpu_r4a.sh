#!/bin/bash
# round 4: the new / touched GPU tests, then a baseline bench line
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_train_lang_gpu.py tests/test_train_step_gpu.py tests/test_gaussian_scene_gpu.py tests/test_deform_gpu.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_new.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_new.log | tail -40
grep -E "^E " gpurun_out/t_new.log | head -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b0.log 2>&1 || exit $?
tail -c 1500 gpurun_out/b0.log
