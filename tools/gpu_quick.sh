#!/bin/bash
# Quick iteration: parity tests (optionally filtered), then the bench without and with stream overlap.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/t.log 2>&1; rc=$?
tail -3 gpurun_out/t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -eq 1 ] && grep -E "^(FAILED|E )" gpurun_out/t.log | head -20
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-overlap > gpurun_out/b_noov.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_ov.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/b_noov.log", "gpurun_out/b_ov.log"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], {k: v["mean_ms"] for k, v in d["phases"].items()})
PY
