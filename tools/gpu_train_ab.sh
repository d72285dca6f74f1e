#!/bin/bash
# Same-box A/B of the configs[4] training-loop stand-in: the working tree and each variant
# library, alternating (ITERS iterations each; the JSON line's value and window times).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tab
for i in $(seq 1 ${REPS:-2}); do
    for v in cur ${VARIANTS:-}; do
        lib=$PWD/4dlangsplat_amd/build/liblsr.so
        [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
        LSR_LIBRARY=$lib timeout -k 10 400 python -u tools/bench_train_loop.py --iters ${ITERS:-300} ${TRAIN_ARGS:-} \
            > gpurun_out/tab/${v}_$i.log 2>&1 || { tail -5 gpurun_out/tab/${v}_$i.log; exit 1; }
        grep "^{" gpurun_out/tab/${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['window_ms_per_iteration'], d['window_loss'])"
    done
done
