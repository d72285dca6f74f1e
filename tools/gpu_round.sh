#!/bin/bash
# Round artefacts in one GPU call: parity tests + headline bench (with cpu_baseline), then the
# rocprofv3 kernel-trace/stats summary, then the PMC traffic passes.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="${BENCH_ARGS_MAIN:-}" STEPS=${STEPS:-5} bash tools/gpu_session.sh || exit $?
bash tools/gpu_prof.sh || exit $?
bash tools/gpu_pmc.sh || exit $?
