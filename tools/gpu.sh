#!/bin/bash
# One parameterised runner for the GPU box (run through gpurun, from the repository root):
#   bash tools/gpu.sh <task> [task ...]        tasks run in order; the first failure ends the call
# Every GPU step runs under its own time limit; a crash, abort or timeout ends the call there.
# Results go to gpurun_out/$OUT (default gpurun_out/run).
#
# tasks
#   tests      the -m gpu suite (PYTEST_ARGS: extra args / node ids, default the whole tests/ dir)
#   bench      bench.py --steps ${STEPS:-20} --warmup 5, the full line with both CPU legs ($BENCH_ARGS)
#   prof       rocprofv3 --kernel-trace --stats of a 5-step bench, kernel_stats.csv + step_timeline.txt
#   pmc        the PMC passes (one counter group each, kernel trace only) + pmc_summary / pmc_traffic.json
#   mfma       matrix-core busy cycles over the headline bench and the deformation bench
#   stall      SQ wave-state counters (stall breakdown per kernel)
#   ab         same-box A/B: REPS rounds alternating CONFIGS ('|'-separated "<variant> <bench flags...>";
#              variant cur = build/liblsr.so, else build/variants/liblsr_<variant>.so)
#   deform     tools/bench_deform.py at 2M (forward / backward per kernel)
#   deform_ab  deformation bench (DEFORM_ARGS) + a short configs[4] loop per VARIANTS ("cur name ..." library variants,
#              or "name:VAR=val[,VAR2=val2]" environment variants), REPS rounds
#   race       tools/deform_race.py (deformation backward repeatability) per library VARIANTS
#   side       the side benches: configs[1] stand-in (bench_render), configs[4] loop (bench_train_loop)
# Library variants are built on the CPU beforehand (tools/build_variants.sh, tools/ab_base.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-run}
mkdir -p "$O"

lib_of() { [ "$1" = cur ] && echo "$PWD/4dlangsplat_amd/build/liblsr.so" || echo "$PWD/4dlangsplat_amd/build/variants/liblsr_$1.so"; }
fail() { echo "FAILED: $*"; exit 1; }
summ() {  # one bench line: value and per-phase ms
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2].ljust(28),d['value'],' '.join(f'{k}={v[\"mean_ms\"]}' for k,v in d.get('phases',{}).items()))" "$1" "$2"
}
pmc_passes() {  # dir, per-pass timeout, bench args, counter groups...
    local d=$1 t=$2 args=$3; shift 3
    local i=0
    for grp in "$@"; do
        i=$((i + 1))
        timeout -k 10 "$t" rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$d/p$i" -o run -- \
            python3 bench.py $args > "$d/p$i.log" 2>&1 || { tail -5 "$d/p$i.log"; fail "pmc pass $i ($grp)"; }
        echo "pmc pass $i ($grp) ok"
    done
}

for task in "$@"; do
  echo "== $task"
  case $task in
    tests)
      timeout -k 10 ${TESTS_TIMEOUT:-1500} python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -v --timeout 600 \
          --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.txt" 2>&1; rc=$?
      tail -3 "$O/gpu_tests.txt"
      [ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR|E )" "$O/gpu_tests.txt" | head -30; exit $rc; } ;;
    bench)
      timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > "$O/bench.log" 2>&1 \
          || { tail -5 "$O/bench.log"; fail bench; }
      grep '^{' "$O/bench.log" | tail -1 > "$O/bench.json"; head -c 700 "$O/bench.json"; echo ;;
    prof)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
          python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --single-view-steps 0 ${BENCH_ARGS:-} \
          > "$O/prof_bench.log" 2>&1 || { tail -5 "$O/prof_bench.log"; fail rocprof; }
      cp "$(find "$O/prof" -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats.csv"
      python3 tools/step_timeline.py "$(find "$O/prof" -name '*kernel_trace.csv' | head -1)" > "$O/step_timeline.txt"
      grep '^{' "$O/prof_bench.log" | tail -1 > "$O/bench_under_rocprof.json"
      head -14 "$O/kernel_stats.csv" | cut -c1-150; tail -12 "$O/step_timeline.txt"
      rm -rf "$O/prof" ;;
    pmc)
      rm -rf "$O/pmc"; mkdir -p "$O/pmc"
      pmc_passes "$O/pmc" 300 "--steps 1 --warmup 1 --no-cpu-baseline --no-profile --single-view-steps 0 ${BENCH_ARGS:-}" \
          "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
          "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
          "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
          "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" ${EXTRA_PMC:-}
      python3 tools/pmc_summary.py "$O/pmc" --json "$O/pmc_traffic.json" > "$O/pmc_summary.txt" 2>&1
      head -30 "$O/pmc_summary.txt"; rm -rf "$O"/pmc/p*/ ;;
    mfma)
      for w in raster deform; do
        if [ $w = raster ]; then cmd="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --single-view-steps 0"
        else cmd="tools/bench_deform.py --iters 2 --no-torch"; fi
        timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
            --output-format csv -d "$O/mfma_$w/p1" -o run -- python3 $cmd > "$O/mfma_$w.log" 2>&1 \
            || { tail -5 "$O/mfma_$w.log"; fail "mfma $w"; }
        python3 tools/pmc_summary.py "$O/mfma_$w" > "$O/mfma_$w.txt"; head -20 "$O/mfma_$w.txt"; rm -rf "$O/mfma_$w/p1"
      done ;;
    stall)
      rm -rf "$O/stall"; mkdir -p "$O/stall"
      pmc_passes "$O/stall" 180 "--steps 1 --warmup 1 --no-cpu-baseline --no-profile --single-view-steps 0 ${BENCH_ARGS:-}" \
          "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
          "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
      python3 tools/pmc_summary.py "$O/stall" > "$O/stall_summary.txt" 2>&1
      grep -E "k_render|k_rts|k_preprocess|k_emit" "$O/stall_summary.txt"; rm -rf "$O"/stall/p*/ ;;
    ab)
      IFS='|' read -ra SETS <<< "${CONFIGS:-cur}"
      for i in $(seq 1 ${REPS:-2}); do
        for j in "${!SETS[@]}"; do
          read -ra f <<< "${SETS[$j]}"
          LSR_LIBRARY=$(lib_of "${f[0]}") timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 2 \
              --no-cpu-baseline --single-view-steps 0 "${f[@]:1}" > "$O/ab_s${j}_$i.log" 2>&1 \
              || { tail -5 "$O/ab_s${j}_$i.log"; fail "ab ${SETS[$j]}"; }
          summ "$O/ab_s${j}_$i.log" "[${SETS[$j]}]" | tee -a "$O/ab.txt"
        done
      done ;;
    deform)
      timeout -k 10 300 python tools/bench_deform.py --no-torch ${DEFORM_ARGS:-} > "$O/bench_deform.log" 2>&1 \
          || { tail -5 "$O/bench_deform.log"; fail deform; }
      tail -c 1500 "$O/bench_deform.log"; echo ;;
    deform_ab)
      for i in $(seq 1 ${REPS:-1}); do
        for spec in ${VARIANTS:-cur}; do
          name=${spec%%:*}; envs=""; lib=$(lib_of cur)
          if [[ $spec == *:* ]]; then envs=${spec#*:}; envs=${envs//,/ }; else lib=$(lib_of "$name"); fi
          env $envs LSR_LIBRARY=$lib timeout -k 10 200 python tools/bench_deform.py --no-torch --iters 10 ${DEFORM_ARGS:-} \
              > "$O/d_$name.log" 2>&1 || { tail -5 "$O/d_$name.log"; fail "deform $name"; }
          if [ "${NO_LOOP:-0}" != 1 ]; then
            env $envs LSR_LIBRARY=$lib timeout -k 10 300 python tools/bench_train_loop.py ${LOOP_ARGS:-} \
                > "$O/t_$name.log" 2>&1 || { tail -5 "$O/t_$name.log"; fail "loop $name"; }
          fi
          echo "$name: fwd/bwd $(grep -h -o '"ms_per_call": [0-9.]*' "$O/d_$name.log" | tr '\n' ' ')" \
               "$(grep -h '^{' "$O/t_$name.log" 2>/dev/null | grep -o '"value": [0-9.]*' | head -1)" | tee -a "$O/deform_ab.txt"
        done
      done ;;
    race)
      for v in ${VARIANTS:-cur}; do
        LSR_LIBRARY=$(lib_of "$v") timeout -k 10 200 python tools/deform_race.py ${RACE_P:-60000} ${RACE_R:-4} \
            > "$O/race_$v.log" 2>&1 || { tail -5 "$O/race_$v.log"; fail "race $v"; }
        echo "$v:"; grep -E "^run" "$O/race_$v.log" | cut -c1-150
      done ;;
    side)
      timeout -k 10 300 python tools/bench_render.py > "$O/bench_render.log" 2>&1 || { tail -5 "$O/bench_render.log"; fail render; }
      tail -c 800 "$O/bench_render.log"; echo
      timeout -k 10 400 python tools/bench_train_loop.py > "$O/bench_train_loop.log" 2>&1 || { tail -5 "$O/bench_train_loop.log"; fail loop; }
      tail -c 1500 "$O/bench_train_loop.log"; echo ;;
    *) fail "unknown task $task" ;;
  esac
done
