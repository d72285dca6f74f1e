#!/bin/bash
# Same-box A/B of the headline bench: the working tree and each variant library, alternating.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bab
for i in $(seq 1 ${REPS:-2}); do
    for v in cur ${VARIANTS:-}; do
        lib=$PWD/4dlangsplat_amd/build/liblsr.so
        [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
        LSR_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --single-view-steps 0 ${BENCH_ARGS:-} \
            > gpurun_out/bab/${v}_$i.log 2>&1 || { tail -5 gpurun_out/bab/${v}_$i.log; exit 1; }
        grep "^{" gpurun_out/bab/${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases']; print('$v', d['value'], d['ms_per_step'], 'fwd', p['render_fwd']['mean_ms'], 'bwd', p['render_bwd']['mean_ms'])"
    done
done
