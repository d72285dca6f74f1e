#!/bin/bash
# deformation bench (2M) + a short configs[4] loop per library variant ($VARIANTS; cur = in-tree)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dvar
for i in $(seq 1 ${REPS:-1}); do
for v in cur ${VARIANTS:-}; do
  lib=$PWD/4dlangsplat_amd/build/liblsr.so
  [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
  LSR_LIBRARY=$lib timeout -k 10 200 python tools/bench_deform.py --no-torch --iters 10 > gpurun_out/dvar/d_$v.log 2>&1 || exit 1
  LSR_LIBRARY=$lib timeout -k 10 300 python tools/bench_train_loop.py ${LOOP_ARGS:-} > gpurun_out/dvar/t_$v.log 2>&1 || exit 1
  echo "$v: fwd $(grep -h 'deformation forward' gpurun_out/dvar/d_$v.log | grep -o '"ms_per_call": [0-9.]*' | head -1) bwd $(grep -h backward gpurun_out/dvar/d_$v.log | grep -o '"ms_per_call": [0-9.]*') $(grep -h '^{' gpurun_out/dvar/t_$v.log | grep -o '"value": [0-9.]*' | head -1) $(grep -o '"backward_ms": [0-9.]*' gpurun_out/dvar/t_$v.log)"
done
done
