#!/bin/bash
# a subset of the -m gpu tests (arguments: test files / node ids), then optional side benches named
# in $BENCHES (deform, train_loop, render)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sub.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/t_sub.log | tail -30
grep -E "^E " gpurun_out/t_sub.log | head -30
[ $rc -gt 1 ] && exit $rc
for b in $BENCHES; do
  case $b in
    deform) timeout -k 10 300 python tools/bench_deform.py --no-torch > gpurun_out/bd.log 2>&1 || exit $?; tail -c 1500 gpurun_out/bd.log;;
    train_loop) timeout -k 10 400 python tools/bench_train_loop.py > gpurun_out/btl.log 2>&1 || exit $?; tail -c 2500 gpurun_out/btl.log;;
    render) timeout -k 10 300 python tools/bench_render.py > gpurun_out/br.log 2>&1 || exit $?; tail -c 1500 gpurun_out/br.log;;
  esac
done
exit $rc
