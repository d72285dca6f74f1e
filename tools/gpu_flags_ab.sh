#!/bin/bash
# Same-box A/B of bench flag sets (same library): GPU tests once, then REPS rounds alternating the
# flag sets in FLAGSETS (separated by '|'), one summary line per run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fab
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/fab/tests.log 2>&1; rc=$?
    tail -1 gpurun_out/fab/tests.log
    if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" gpurun_out/fab/tests.log | head -20; exit $rc; fi
fi
IFS='|' read -ra SETS <<< "${FLAGSETS:-}"
for i in $(seq 1 ${REPS:-2}); do
    for j in "${!SETS[@]}"; do
        f=${SETS[$j]}
        envs=(); flags=()   # leading VAR=value tokens go to the environment
        for t in $f; do if [[ ${#flags[@]} -eq 0 && $t == *=* && $t != -* ]]; then envs+=("$t"); else flags+=("$t"); fi; done
        env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline "${flags[@]}" > gpurun_out/fab/s${j}_$i.log 2>&1 || { tail -5 gpurun_out/fab/s${j}_$i.log; exit 1; }
        python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2].ljust(24),d['value'],' '.join(f'{k}={v[\"mean_ms\"]}' for k,v in d['phases'].items()))" gpurun_out/fab/s${j}_$i.log "[$f]"
    done
done
