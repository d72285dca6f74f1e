#!/bin/bash
# same-box A/B of bench.py under environment variants (VARIANTS="name:VAR=val[,VAR2=val2];..."; "base:" = none),
# REPS alternating rounds, STEPS timed steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/abe; mkdir -p $out
IFS=';' read -ra VS <<< "${VARIANTS}"
for r in $(seq 1 ${REPS:-3}); do
  for spec in "${VS[@]}"; do
    n=${spec%%:*}; e=${spec#*:}; e=${e//,/ }
    env $e timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --single-view-steps 0 ${ARGS:-} \
        > $out/${n}_$r.json 2> $out/${n}_$r.err || { tail -20 $out/${n}_$r.err; exit 1; }
    echo "$n $(grep '^{' $out/${n}_$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
