#!/bin/bash
# Copy one round-profiling call's results (tools/gpu_round.sh + tools/gpu_mfma_pmc.sh) from
# gpurun_out/ into profiles/<tag>/ and make its PMC traffic the one bench.py reports.
set -e
tag=$1; [ -n "$tag" ] || { echo "usage: $0 <tag>"; exit 1; }
root=$(cd "$(dirname "$0")/.." && pwd); o=$root/gpurun_out; d=$root/profiles/$tag
mkdir -p "$d"
grep '^{' "$o/bench.log" | tail -1 > "$d/bench.json"
grep '^{' "$o/prof_bench.log" | tail -1 > "$d/bench_under_rocprof.json" || true
cp "$(find "$o/prof" -name '*kernel_stats.csv' | head -1)" "$d/kernel_stats.csv"
cp "$o/pmc/summary.txt" "$d/pmc_summary.txt"
cp "$o/pmc/pmc_traffic.json" "$d/pmc_traffic.json"
cp "$o/pmc/pmc_traffic.json" "$root/profiles/pmc_traffic.json"
[ -f "$o/mfma/raster_summary.txt" ] && cp "$o/mfma/raster_summary.txt" "$d/mfma_raster.txt"
[ -f "$o/mfma/deform_summary.txt" ] && cp "$o/mfma/deform_summary.txt" "$d/mfma_deform.txt"
ls "$d"
