#!/bin/bash
# rocprofv3 kernel stats for the regular build and every ablation variant (short bench each).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
shopt -s nullglob
for lib in 4dlangsplat_amd/build/liblsr.so 4dlangsplat_amd/build/variants/*.so; do
    n=$(basename $lib .so)
    LSR_LIBRARY=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv/$n -o run -- \
        python3 bench.py --steps 1 --warmup 1 --views 2 --no-cpu-baseline > gpurun_out/pv/$n.log 2>&1
    rc=$?; echo "== $n rc=$rc"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/pv/$n.log; exit $rc; }
done
exit 0
