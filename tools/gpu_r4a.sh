#!/bin/bash
# round 4: the new / touched GPU tests, then a baseline bench line
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train_step_gpu.py tests/test_gaussian_scene_gpu.py tests/test_deform_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_new.log 2>&1; rc=$?
tail -25 gpurun_out/t_new.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b0.log 2>&1 || exit $?
tail -c 400 gpurun_out/b0.log
