#!/bin/bash
# PMC passes (one counter group per pass, kernel trace only) over an arbitrary python command:
#   PMC_CMD="tools/bench_deform.py --iters 3" PMC_TAG=deform bash tools/gpu_pmc_cmd.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${PMC_TAG:-cmd}
mkdir -p gpurun_out/pmc_$tag
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" ${EXTRA_PMC:-}; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/p$i -o run -- \
        python3 $PMC_CMD > gpurun_out/pmc_$tag/p$i.log 2>&1
    rc=$?; echo "pass $i ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$tag/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag/summary.txt 2>&1; cat gpurun_out/pmc_$tag/summary.txt
