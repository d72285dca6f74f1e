#!/bin/bash
# tools/bench_deform.py for the regular build and every ablation variant.
cd "$GRAFT_REPO_ROOT"
shopt -s nullglob
for lib in 4dlangsplat_amd/build/liblsr.so 4dlangsplat_amd/build/variants/*.so; do
    n=$(basename $lib .so)
    echo "== $n"
    LSR_LIBRARY=$PWD/$lib timeout -k 10 300 python tools/bench_deform.py --iters 10 || exit $?
done
