#!/bin/bash
# Same-box A/B of bench.py argument sets, alternating: ARGS_A / ARGS_B (REPS rounds)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/aab
for i in $(seq 1 ${REPS:-3}); do
    for v in A B; do
        if [ $v = A ]; then args="$ARGS_A"; else args="$ARGS_B"; fi
        timeout -k 10 300 python -u bench.py --no-cpu-baseline --single-view-steps 0 --steps ${STEPS:-30} $args \
            > gpurun_out/aab/${v}_$i.log 2>&1 || { tail -5 gpurun_out/aab/${v}_$i.log; exit 1; }
        grep "^{" gpurun_out/aab/${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases']; print('$v', d['value'], d['ms_per_step'], 'fwd', p['render_fwd']['mean_ms'], 'bwd', p['render_bwd']['mean_ms'])"
    done
done
