#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tbd
timeout -k 10 300 python tools/tb_lengths.py > gpurun_out/tbd/lengths.txt 2>&1 || { tail -20 gpurun_out/tbd/lengths.txt; exit 1; }
cat gpurun_out/tbd/lengths.txt
EXTRA="--early-views 8" bash tools/gpu_tb_prof.sh
