#!/bin/bash
# Same-box A/B over (library, bench flags) configurations: GPU tests once on the working-tree
# library, then REPS rounds alternating the configurations in CONFIGS ('|'-separated, each
# "<variant> <bench flags...>", variant "cur" = build/liblsr.so, else build/variants/liblsr_<v>.so).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/mix
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/mix/tests.log 2>&1; rc=$?
    tail -1 gpurun_out/mix/tests.log
    if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" gpurun_out/mix/tests.log | head -20; exit $rc; fi
fi
IFS='|' read -ra SETS <<< "${CONFIGS:-cur}"
for i in $(seq 1 ${REPS:-2}); do
    for j in "${!SETS[@]}"; do
        read -ra f <<< "${SETS[$j]}"
        v=${f[0]}; flags=("${f[@]:1}")
        lib=$PWD/4dlangsplat_amd/build/liblsr.so
        [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
        LSR_LIBRARY=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --single-view-steps 0 "${flags[@]}" > gpurun_out/mix/s${j}_$i.log 2>&1 || { tail -5 gpurun_out/mix/s${j}_$i.log; exit 1; }
        python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2].ljust(28),d['value'],' '.join(f'{k}={v[\"mean_ms\"]}' for k,v in d['phases'].items()))" gpurun_out/mix/s${j}_$i.log "[${SETS[$j]}]"
    done
done
