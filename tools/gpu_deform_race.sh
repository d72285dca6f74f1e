#!/bin/bash
# deformation backward repeatability (tools/deform_race.py) under each library variant named in
# $VARIANTS (default: the in-tree build), P = ${RACE_P:-60000}, ${RACE_R:-4} runs each
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then lib=4dlangsplat_amd/build/liblsr.so; else lib=4dlangsplat_amd/build/variants/liblsr_$v.so; fi
  echo "== $v"
  LSR_LIBRARY=$lib timeout -k 10 200 python tools/deform_race.py ${RACE_P:-60000} ${RACE_R:-4} > gpurun_out/race_$v.log 2>&1 || { tail -5 gpurun_out/race_$v.log; exit 1; }
  grep -E "^run" gpurun_out/race_$v.log | cut -c1-150
done
