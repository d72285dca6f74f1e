#!/bin/bash
# Time the standalone radix sort (tests/kernels/t_sort.hip) under several -D configurations.
# Usage (on the GPU box): SORT_VARIANTS="base: nolb:-DLSR_ABL_NOLOOKBACK" bash tools/gpu_sort_variants.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sortv
for spec in ${SORT_VARIANTS:-base:}; do
    name=${spec%%:*}; defs=${spec#*:}; defs=${defs//,/ }
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off $defs -I 4dlangsplat_amd/csrc \
        -o gpurun_out/sortv/t_$name tests/kernels/t_sort.hip || exit 2
    timeout -k 10 120 gpurun_out/sortv/t_$name 20 > gpurun_out/sortv/$name.log 2>&1
    rc=$?; echo "== $name rc=$rc"; cat gpurun_out/sortv/$name.log
    [ $rc -gt 1 ] && exit $rc
done
exit 0
