#!/bin/bash
# Bench each ablation variant (4dlangsplat_amd/build/variants/*.so) + the regular build; prints
# the per-phase times.  Each run has its own time limit; the first failure ends the script.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/var
shopt -s nullglob
for lib in 4dlangsplat_amd/build/liblsr.so 4dlangsplat_amd/build/variants/*.so; do
    n=$(basename $lib .so)
    LSR_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var/$n.log 2>&1
    rc=$?
    echo "== $n rc=$rc"
    python3 - gpurun_out/var/$n.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print("  value", d["value"], " ".join(f"{k}={v['mean_ms']}" for k, v in d["phases"].items()))
PY
    [ $rc -ne 0 ] && { tail -5 gpurun_out/var/$n.log; exit $rc; }
done
exit 0
