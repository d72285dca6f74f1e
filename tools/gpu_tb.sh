#!/bin/bash
# Tile-bucket binning: its GPU tests, then a same-box A/B of bench.py --binning sort|bucket
# (alternating runs), then a rocprof kernel trace of the bucket path.
set -o pipefail
out=gpurun_out/tb
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tilebin_gpu.py \
    > $out/tests.txt 2>&1 || { tail -40 $out/tests.txt; exit 1; }
tail -8 $out/tests.txt
for r in 1 2; do
  for b in sort bucket; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --single-view-steps 0 \
        --binning $b > $out/bench_${b}_$r.json 2> $out/bench_${b}_$r.err || { tail -20 $out/bench_${b}_$r.err; exit 1; }
    python - "$out/bench_${b}_$r.json" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], d["value"], d["ms_per_step"], d["config"]["binning"])
PY
  done
done
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o tb -- python bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline --single-view-steps 0 --binning bucket > $out/prof_bench.json 2> $out/prof_bench.err \
    || { tail -20 $out/prof_bench.err; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -3
