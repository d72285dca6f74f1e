#!/bin/bash
# deformation plane-gradient replica count A/B: bench_deform (2M) and a short configs[4] loop (100k)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rep
for r in ${REPLICAS:-16 4}; do
  LSR_DEFORM_REPLICAS=$r timeout -k 10 200 python tools/bench_deform.py --no-torch --iters 10 > gpurun_out/rep/d_$r.log 2>&1 || exit 1
  LSR_DEFORM_REPLICAS=$r timeout -k 10 300 python tools/bench_train_loop.py --iters 300 > gpurun_out/rep/t_$r.log 2>&1 || exit 1
  echo "replicas $r: $(grep -h backward gpurun_out/rep/d_$r.log | grep -o '"ms_per_call": [0-9.]*') $(grep -h '^{' gpurun_out/rep/t_$r.log | grep -o '"value": [0-9.]*' | head -1)"
done
