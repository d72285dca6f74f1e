#!/bin/bash
# Stall breakdown passes (SQ wave-state counters) over a short bench run; summary per kernel.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${PMC_TAG:-stall}
mkdir -p gpurun_out/pmc_$tag
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS:-}"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" ${EXTRA_PMC:-}; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/p$i -o run -- \
        python3 bench.py $ARGS > gpurun_out/pmc_$tag/p$i.log 2>&1
    rc=$?; echo "pass $i ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$tag/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag/summary.txt 2>&1; grep -E "k_render|k_radix|k_preprocess" gpurun_out/pmc_$tag/summary.txt
