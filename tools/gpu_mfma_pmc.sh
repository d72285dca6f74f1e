#!/bin/bash
# One PMC pass (matrix-core busy cycles + GPU active cycles) over the headline bench and over the
# deformation bench; summaries with the MFMA busy fraction per kernel.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/mfma
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d gpurun_out/mfma/raster/p1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile \
    > gpurun_out/mfma/raster.log 2>&1 || { tail -5 gpurun_out/mfma/raster.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d gpurun_out/mfma/deform/p1 -o run -- python3 tools/bench_deform.py --iters 2 --no-torch \
    > gpurun_out/mfma/deform.log 2>&1 || { tail -5 gpurun_out/mfma/deform.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/mfma/raster > gpurun_out/mfma/raster_summary.txt
python3 tools/pmc_summary.py gpurun_out/mfma/deform > gpurun_out/mfma/deform_summary.txt
cat gpurun_out/mfma/raster_summary.txt gpurun_out/mfma/deform_summary.txt
