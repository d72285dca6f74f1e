#!/bin/bash
# rocprofv3 kernel stats of tools/bench_deform.py under each library variant in $VARIANTS
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then lib=4dlangsplat_amd/build/liblsr.so; else lib=4dlangsplat_amd/build/variants/liblsr_$v.so; fi
  mkdir -p gpurun_out/dstat_$v
  LSR_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dstat_$v -o run -- \
      python3 tools/bench_deform.py --iters ${ITERS:-6} --no-torch > gpurun_out/dstat_$v/b.log 2>&1 || { tail -5 gpurun_out/dstat_$v/b.log; exit 1; }
  echo "== $v"; grep -h '^{' gpurun_out/dstat_$v/b.log | cut -c1-160
  f=$(find gpurun_out/dstat_$v -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -6
done
