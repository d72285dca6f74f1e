#!/bin/bash
# deformation backward timing ablations (wrong gradients; timing only): backward ms per variant
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dabl
for i in $(seq 1 ${REPS:-2}); do
for v in cur ${VARIANTS}; do
  lib=$PWD/4dlangsplat_amd/build/liblsr.so
  [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
  LSR_LIBRARY=$lib timeout -k 10 200 python tools/bench_deform.py --no-torch --iters 10 > gpurun_out/dabl/d_$v.log 2>&1 || { tail -5 gpurun_out/dabl/d_$v.log; exit 1; }
  echo "$v: $(grep -h backward gpurun_out/dabl/d_$v.log | grep -o '"ms_per_call": [0-9.]*')"
done
done
