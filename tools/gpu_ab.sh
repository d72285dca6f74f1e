#!/bin/bash
# Same-box A/B: parity tests on the working-tree library, then alternating bench runs of the
# working tree and each variants/*.so (REPS rounds), one JSON summary line per run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/ab/tests.log 2>&1; rc=$?
    tail -1 gpurun_out/ab/tests.log
    if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" gpurun_out/ab/tests.log | head -20; exit $rc; fi
fi
shopt -s nullglob
for i in $(seq 1 ${REPS:-2}); do
    for lib in 4dlangsplat_amd/build/liblsr.so 4dlangsplat_amd/build/variants/*.so; do
        n=$(basename $lib .so)
        LSR_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/${n}_$i.log 2>&1 || { tail -5 gpurun_out/ab/${n}_$i.log; exit 1; }
        python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2].ljust(16),d['value'],' '.join(f'{k}={v[\"mean_ms\"]}' for k,v in d['phases'].items()))" gpurun_out/ab/${n}_$i.log $n
    done
done
