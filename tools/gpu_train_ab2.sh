#!/bin/bash
# Same-box A/B of the configs[4] stand-in loop over library variants (VARIANTS: "cur" = the
# working-tree build, else build/variants/liblsr_<v>.so), REPS alternating rounds of ITERS iterations.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tab
for i in $(seq 1 ${REPS:-2}); do
    for v in ${VARIANTS:-cur}; do
        lib=$PWD/4dlangsplat_amd/build/liblsr.so
        [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
        LSR_LIBRARY=$lib timeout -k 10 300 python tools/bench_train_loop.py --iters ${ITERS:-400} ${TRAIN_ARGS:-} > gpurun_out/tab/${v}_$i.log 2>&1 || { tail -5 gpurun_out/tab/${v}_$i.log; exit 1; }
        python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2].ljust(8),d['value'],d['window_ms_per_iteration'])" gpurun_out/tab/${v}_$i.log $v
    done
done
