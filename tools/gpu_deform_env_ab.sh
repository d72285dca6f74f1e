#!/bin/bash
# deformation bench (2M) + a short configs[4] loop per environment variant of the in-tree library:
# VARIANTS="name:VAR=val[,VAR2=val2] ..." (cur = no extra environment), REPS alternations
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/denv
for i in $(seq 1 ${REPS:-1}); do
for spec in cur ${VARIANTS:-}; do
  name=${spec%%:*}; envs=""
  [ "$spec" != cur ] && envs=${spec#*:}; envs=${envs//,/ }
  env $envs timeout -k 10 200 python tools/bench_deform.py --no-torch --iters 10 > gpurun_out/denv/d_$name.log 2>&1 || exit 1
  env $envs timeout -k 10 300 python tools/bench_train_loop.py ${LOOP_ARGS:-} > gpurun_out/denv/t_$name.log 2>&1 || exit 1
  echo "$name: $(grep -h backward gpurun_out/denv/d_$name.log | grep -o '"ms_per_call": [0-9.]*') $(grep -h '^{' gpurun_out/denv/t_$name.log | grep -o '"value": [0-9.]*' | head -1) $(grep -o '"backward_ms": [0-9.]*' gpurun_out/denv/t_$name.log)"
done
done
