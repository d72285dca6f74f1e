#!/bin/bash
# the whole -m gpu suite, then a bench line and the deformation bench (stops at a crash; a test
# failure still benches)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/t_all.log | tail -30
grep -E "^E " gpurun_out/t_all.log | head -40
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b0.log 2>&1 || exit $?
tail -c 2500 gpurun_out/b0.log
timeout -k 10 300 python tools/bench_deform.py --no-torch > gpurun_out/bd.log 2>&1 || exit $?
tail -c 1500 gpurun_out/bd.log
