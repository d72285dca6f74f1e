#!/bin/bash
# round-5 closing set: the whole -m gpu suite, then tools/gpu_r5_prof.sh (bench line with both CPU
# legs, rocprofv3 kernel trace + stats, step timeline, PMC passes incl. the whole-step record)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5f; rm -rf gpurun_out/r5p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r5f/gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r5f/gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR|E )" gpurun_out/r5f/gpu_tests.txt | head -20; exit $rc; }
bash tools/gpu_r5_prof.sh
