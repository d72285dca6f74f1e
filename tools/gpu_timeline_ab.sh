#!/bin/bash
# kernel-trace step timelines of bench.py variants (VARIANTS="name:args;name:args")
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/tl; mkdir -p $out
IFS=';' read -ra VS <<< "${VARIANTS:-base:;side:--order-on-side}"
for spec in "${VS[@]}"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$n -o run -- python3 bench.py --steps 5 --warmup 2 \
      --no-cpu-baseline --single-view-steps 0 $a > $out/bench_$n.json 2> $out/bench_$n.err || { tail -20 $out/bench_$n.err; exit 1; }
  t=$(find $out/$n -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py "$t" > $out/timeline_$n.txt
  echo "== $n $a: $(grep '^{' $out/bench_$n.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  grep -n "render_fwd" $out/timeline_$n.txt | head -2
  grep "step span" $out/timeline_$n.txt
done
