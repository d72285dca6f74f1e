#!/bin/bash
# Same-box A/B of the configs[4] stand-in loop over environment settings of the working-tree build:
# ENVS holds '|'-separated sets of VAR=value assignments ("-" = none), REPS alternating rounds.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tenv
IFS='|' read -ra SETS <<< "${ENVS:--}"
for i in $(seq 1 ${REPS:-2}); do
    k=0
    for set in "${SETS[@]}"; do
        k=$((k + 1)); vars=""; [ "$set" != "-" ] && vars="$set"
        env $vars timeout -k 10 300 python tools/bench_train_loop.py --iters ${ITERS:-400} ${TRAIN_ARGS:-} \
            > gpurun_out/tenv/s${k}_$i.log 2>&1 || { tail -5 gpurun_out/tenv/s${k}_$i.log; exit 1; }
        python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2].ljust(40),d['value'],d['window_ms_per_iteration'],d['deformation']['backward_ms'])" gpurun_out/tenv/s${k}_$i.log "$set"
    done
done
