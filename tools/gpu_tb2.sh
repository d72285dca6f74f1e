#!/bin/bash
# tile-bucket round 2: tests, uncontended kernel profile of both paths, default-pipeline A/B, then the
# round-5 measurement set (tools/gpu_r5_prof.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tb
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tilebin_gpu.py \
    > gpurun_out/tb/tests2.txt 2>&1 || { tail -40 gpurun_out/tb/tests2.txt; exit 1; }
tail -3 gpurun_out/tb/tests2.txt
EXTRA="--early-views 8" bash tools/gpu_tb_prof.sh || exit 1
for r in 1 2; do
  for b in sort bucket; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --single-view-steps 0 --binning $b \
        > gpurun_out/tb/ab2_${b}_$r.json 2> gpurun_out/tb/ab2_${b}_$r.err || { tail -20 gpurun_out/tb/ab2_${b}_$r.err; exit 1; }
    grep '^{' gpurun_out/tb/ab2_${b}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b', d['value'], d['ms_per_step'])"
  done
done
bash tools/gpu_r5_prof.sh
