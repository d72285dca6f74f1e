#!/bin/bash
# Same-box A/B of the headline bench over environment settings: ENVS holds '|'-separated sets of
# VAR=value assignments ("-" = none), REPS alternating rounds.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/eab
IFS='|' read -ra SETS <<< "${ENVS:--}"
for i in $(seq 1 ${REPS:-2}); do
    k=0
    for set in "${SETS[@]}"; do
        k=$((k + 1)); vars=""; [ "$set" != "-" ] && vars="$set"
        env $vars timeout -k 10 300 python -u bench.py --no-cpu-baseline --single-view-steps 0 ${BENCH_ARGS:-} \
            > gpurun_out/eab/s${k}_$i.log 2>&1 || { tail -5 gpurun_out/eab/s${k}_$i.log; exit 1; }
        grep "^{" gpurun_out/eab/s${k}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases']; print('$set'.ljust(24), d['value'], d['ms_per_step'], 'depth', p['depth_sort']['mean_ms'], 'tile', p['tile_sort']['mean_ms'], 'bwd', p['render_bwd']['mean_ms'], 'flush', p['preprocess_bwd_views']['mean_ms'])"
    done
done
