#!/bin/bash
# Same-box A/B of the working-tree library against named variants (VARIANTS="base ..."), after the
# GPU tests named in $TESTS: alternating bench runs, one summary line per run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 700 python -u -m pytest $TESTS -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/tests.log 2>&1; rc=$?
    tail -1 gpurun_out/ab/tests.log
    if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" gpurun_out/ab/tests.log | head -20; exit $rc; fi
fi
for i in $(seq 1 ${REPS:-3}); do
    for v in cur ${VARIANTS:-base}; do
        lib=$PWD/4dlangsplat_amd/build/liblsr.so
        [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
        LSR_LIBRARY=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --single-view-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab/${v}_$i.log 2>&1 || { tail -5 gpurun_out/ab/${v}_$i.log; exit 1; }
        python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2].ljust(10),d['value'],' '.join(f'{k}={v[\"mean_ms\"]}' for k,v in d['phases'].items()))" gpurun_out/ab/${v}_$i.log $v
    done
done
