#!/bin/bash
# rocprofv3 kernel stats of the standalone radix sort (tests/kernels/t_sort.hip, 20 timed reps).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/sortp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off ${SORT_DEFS:-} -I 4dlangsplat_amd/csrc \
    -o gpurun_out/sortp/t_sort tests/kernels/t_sort.hip || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sortp/prof -o run -- \
    gpurun_out/sortp/t_sort 20 > gpurun_out/sortp/run.log 2>&1
rc=$?; echo "rc=$rc"; cat gpurun_out/sortp/run.log | grep -v "^W\|^E" | tail -8
f=$(find gpurun_out/sortp/prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0][-40:]
    g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
    by[(n, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:42s} grid={g:9d} calls={len(v):4d} mean={sum(v)/len(v):8.1f} us")
PY
exit $rc
