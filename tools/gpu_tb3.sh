#!/bin/bash
# tile-bucket words variant: its tests, then same-box A/B: sort | bucket | bucket with 4-byte bucket words
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tb3
V=$PWD/4dlangsplat_amd/build/variants/liblsr_tbw.so
LSR_LIBRARY=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tilebin_gpu.py \
    > gpurun_out/tb3/tests_tbw.txt 2>&1 || { tail -30 gpurun_out/tb3/tests_tbw.txt; exit 1; }
tail -1 gpurun_out/tb3/tests_tbw.txt
for r in 1 2 3; do
  for m in sort bucket tbw; do
    lib=$PWD/4dlangsplat_amd/build/liblsr.so; b=$m
    [ $m = tbw ] && { lib=$V; b=bucket; }
    LSR_LIBRARY=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --single-view-steps 0 \
        --binning $b > gpurun_out/tb3/${m}_$r.json 2> gpurun_out/tb3/${m}_$r.err || { tail -20 gpurun_out/tb3/${m}_$r.err; exit 1; }
    grep '^{' gpurun_out/tb3/${m}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'])"
  done
done
