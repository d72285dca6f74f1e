#!/bin/bash
# Deformation: GPU tests, bench line, then rocprofv3 kernel-trace + stats of tools/bench_deform.py.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dprof
timeout -k 10 300 python -u -m pytest tests/test_deform_gpu.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/t_deform.log 2>&1
rc=$?; tail -3 gpurun_out/t_deform.log
[ $rc -ne 0 ] && { grep -E "^E " gpurun_out/t_deform.log | head -10; exit $rc; }
timeout -k 10 200 python tools/bench_deform.py > gpurun_out/bench_deform.json 2>&1 || exit $?
cat gpurun_out/bench_deform.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dprof -o run -- \
    python3 tools/bench_deform.py --iters ${ITERS:-6} > gpurun_out/dprof/b.log 2>&1
rc=$?
f=$(find gpurun_out/dprof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
exit $rc
