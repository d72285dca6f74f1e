#!/bin/bash
# round 5: diagnostics + the changed paths' tests, then bench A/B of --order-on-side (same box).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -f tools/scratch/ckpt_diag.py ]; then
  timeout -k 10 300 python tools/scratch/ckpt_diag.py > gpurun_out/ckdiag.log 2>&1; echo "ckdiag rc=$?"; tail -25 gpurun_out/ckdiag.log
fi
timeout -k 10 1200 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_view_parallel_gpu.py tests/test_checkpoint_gpu.py tests/test_headline_gpu.py} \
    -m gpu -v -s --timeout 420 --timeout-method thread -p no:cacheprovider > gpurun_out/r5b_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|mode [0-9]|co-residency" gpurun_out/r5b_tests.log | tail -40
grep -E "^E " gpurun_out/r5b_tests.log | head -30
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
  for a in "" "--order-on-side"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --single-view-steps 0 $a > gpurun_out/r5b_bench.log 2>&1 || exit $?
    echo "bench [$a]: $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r5b_bench.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], {k: v['mean_ms'] for k, v in d['phases'].items()})")"
  done
done
exit $rc
