#!/bin/bash
# multi-batch early views: the renderer test, then same-box A/B of --early-views settings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/early
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    "tests/test_view_parallel_gpu.py::test_batched_composite_step_agrees" > gpurun_out/early/tests.txt 2>&1 \
    || { tail -30 gpurun_out/early/tests.txt; exit 1; }
tail -1 gpurun_out/early/tests.txt
for r in 1 2 3; do
  for e in ${SETTINGS:-3 1,2 2,2 1,3 2,3}; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --single-view-steps 0 \
        --early-views $e > gpurun_out/early/e${e}_$r.json 2> gpurun_out/early/e${e}_$r.err || { tail -20 gpurun_out/early/e${e}_$r.err; exit 1; }
    grep '^{' gpurun_out/early/e${e}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', d['value'], d['ms_per_step'])"
  done
done
