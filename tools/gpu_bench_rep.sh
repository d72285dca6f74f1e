#!/bin/bash
# Repeated headline bench runs (run-to-run spread): REPS x bench.py --steps STEPS.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
    timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/rep_$i.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/rep_$i.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],{k:v['mean_ms'] for k,v in d['phases'].items()})"
done
