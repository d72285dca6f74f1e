#!/bin/bash
# kernel-trace stats of bench.py with each binning path (5 timed steps)
set -o pipefail
out=gpurun_out/tbp
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for b in bucket sort; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$b -o run -- python bench.py \
      --steps 5 --warmup 2 --no-cpu-baseline --single-view-steps 0 --binning $b $EXTRA > $out/bench_$b.json 2> $out/bench_$b.err \
      || { tail -20 $out/bench_$b.err; exit 1; }
done
find $out -name "*kernel_stats.csv"
for b in bucket sort; do
  t=$(find $out/$b -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py "$t" > $out/timeline_$b.txt && head -40 $out/timeline_$b.txt
done
