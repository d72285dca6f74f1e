#!/bin/bash
# Deformation backward repeatability for each variant library (tools/deform_race.py).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/race
for v in cur ${VARIANTS:-}; do
    lib=$PWD/4dlangsplat_amd/build/liblsr.so
    [ "$v" != cur ] && lib=$PWD/4dlangsplat_amd/build/variants/liblsr_$v.so
    LSR_LIBRARY=$lib timeout -k 10 200 python -u tools/deform_race.py ${P:-20000} ${R:-6} > gpurun_out/race/$v.log 2>&1
    rc=$?
    echo "== $v rc=$rc: $(grep -c 'DIFFERS\|rel [0-9.]*e-0[0-3] (bad rows [1-9]' gpurun_out/race/$v.log) bad runs"
    grep run gpurun_out/race/$v.log | cut -c1-150
    [ $rc -ne 0 ] && exit $rc
done
exit 0
