#!/bin/bash
# Copy one profiling call's results (tools/gpu.sh bench prof pmc mfma, OUT=<dir>) from
# gpurun_out/<dir>/ into profiles/<tag>/ and make its PMC traffic the one bench.py reports.
set -e
tag=$1; src=${2:-run}; [ -n "$tag" ] || { echo "usage: $0 <tag> [gpurun_out subdir]"; exit 1; }
root=$(cd "$(dirname "$0")/.." && pwd); o=$root/gpurun_out/$src; d=$root/profiles/$tag
mkdir -p "$d"
for f in bench.json bench_under_rocprof.json kernel_stats.csv step_timeline.txt pmc_summary.txt pmc_traffic.json \
         mfma_raster.txt mfma_deform.txt stall_summary.txt gpu_tests.txt ab.txt deform_ab.txt bench_deform.log; do
    [ -f "$o/$f" ] && cp "$o/$f" "$d/$f"
done
[ -f "$o/pmc_traffic.json" ] && cp "$o/pmc_traffic.json" "$root/profiles/pmc_traffic.json"
ls "$d"
