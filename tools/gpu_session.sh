#!/bin/bash
# One GPU session: unit kernels + parity tests, then a short bench with per-phase timings.
# Every GPU step has its own time limit; a crash/timeout (exit code other than 0/1) ends the session.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
    echo "== $name rc=$rc"; tail -${TAILN:-15} "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-}
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
step bench 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS---no-cpu-baseline}
