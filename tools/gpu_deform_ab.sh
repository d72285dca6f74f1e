#!/bin/bash
# Deformation bench for the working tree and each variant library (same box).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dab
for v in cur ${VARIANTS:-}; do
    lib=$PWD/4dlangsplat_amd/build/liblsr.so
    [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
    LSR_LIBRARY=$lib timeout -k 10 200 python -u tools/bench_deform.py --no-torch > gpurun_out/dab/$v.json 2>&1 || exit $?
    echo "== $v"; grep -o '"metric[^,]*\|"ms_per_call": [0-9.]*' gpurun_out/dab/$v.json
done
