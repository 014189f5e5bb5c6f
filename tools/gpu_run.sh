#!/bin/bash
# The one parametrised GPU-box runner (round 5 folded the single-purpose
# gpu_*.sh scripts of rounds 1-4 into its steps; the provenance of a
# measurement lives in its profiles/ JSON, which records the tag, command and
# library sha).
#
#   gpurun -- 'TAG=r05a tools/gpu_run.sh tests smoke bench kt pmc'
#
# Steps run in the order given, each under its own time limit; the first
# failing step ends the call (no GPU step is started after a fault, abort,
# segfault or time-out).  Outputs: gpurun_out/<step>_<TAG>.*
#   tests    python -m pytest -m gpu (TEST_ARGS: files, default the whole GPU suite; TEST_K: a -k expression)
#   smoke    __graft_entry__.smoke()
#   bench    python bench.py $BENCH_ARGS                      -> bench_<TAG>.json
#   kt       rocprofv3 --kernel-trace --stats of bench.py --no-cpu-baseline $BENCH_ARGS
#            (+ tools/kt_summary.py)                          -> kt_<TAG>/
#   pmc      three separate --pmc passes (FETCH_SIZE; WRITE_SIZE;
#            TCC_EA0_RDREQ/HIT/MISS) on the same command, for
#            tools/pmc_summary.py                             -> pmc{1,2,3}_<TAG>/
#   counters one --pmc pass per group of PMC_GROUPS (groups separated by ';',
#            e.g. "SQ_WAVES SQ_WAIT_ANY SQ_INSTS_VALU;TCP_TCC_READ_REQ_sum") on
#            bench.py --no-cpu-baseline $BENCH_ARGS, kernels matching $KRE;
#            per-kernel means printed by tools/pmc_lines.py   -> cnt<i>_<TAG>/
#   ab       tools/ab_inproc.py $AB_ARGS (walk-kernel library / knob A/B in one
#            process)                                         -> ab_<TAG>.jsonl
#   tsab     tools/ts_lib_ab.py $TSAB_ARGS (TopSim library / knob A/B)
#                                                             -> tsab_<TAG>.jsonl
#   calib    tools/calib/calib_sweep $CALIB_ARGS (random-block read rates; built
#            in-tree beforehand) + its TCC request pass       -> calib_<TAG>/
#   py       python $PY_ARGS (any tools/ script)              -> py_<TAG>.{out,err}
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-run}
KRE=${KRE:-"k_walk|k_topsim"}
T_TESTS=${T_TESTS:-1100}
T_STEP=${T_STEP:-600}
O=gpurun_out

step_fail() {  # name rc log
  echo "STEP_FAIL $1 rc=$2"
  [ -f "$3" ] && tail -25 "$3"
  exit 1
}

for step in "$@"; do
  case "$step" in
    tests)
      log=$O/tests_$TAG.log
      timeout -k 10 "$T_TESTS" python -u -m pytest ${TEST_ARGS:-tests} ${TEST_K:+-k "$TEST_K"} -m gpu -x -q \
        --timeout 300 --timeout-method thread > "$log" 2>&1 || step_fail tests $? "$log"
      echo "STEP_OK tests: $(tail -1 "$log")" ;;
    smoke)
      log=$O/smoke_$TAG.log
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || step_fail smoke $? "$log"
      echo "STEP_OK smoke" ;;
    bench)
      timeout -k 10 "$T_STEP" python bench.py $BENCH_ARGS > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" ||
        step_fail bench $? "$O/bench_$TAG.err"
      echo "STEP_OK bench: $(python -c "import json;d=json.load(open('$O/bench_$TAG.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])")" ;;
    kt)
      timeout -k 10 "$T_STEP" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$TAG" -o kt -- \
        python bench.py --no-cpu-baseline $BENCH_ARGS > "$O/kt_$TAG.json" 2> "$O/kt_$TAG.err" ||
        step_fail kt $? "$O/kt_$TAG.err"
      python tools/kt_summary.py "$O/kt_$TAG/kt_kernel_trace.csv" "$O/kt_$TAG/kernel_dispatch_summary.json" > /dev/null || true
      python tools/kt_lines.py "$O/kt_$TAG/kt_kernel_trace.csv" "$O/kt_$TAG.json" "$O/kt_$TAG/kt_lines.json" > /dev/null || true
      echo "STEP_OK kt" ;;
    pmc)
      i=0
      for counters in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
        i=$((i + 1))
        timeout -k 10 "$T_STEP" rocprofv3 --pmc $counters --kernel-include-regex "$KRE" --output-format csv \
          -d "$O/pmc${i}_$TAG" -o pmc -- python bench.py --no-cpu-baseline $BENCH_ARGS \
          > "$O/pmc${i}_$TAG.json" 2> "$O/pmc${i}_$TAG.err" || step_fail "pmc$i" $? "$O/pmc${i}_$TAG.err"
        echo "STEP_OK pmc$i"
      done ;;
    counters)
      i=0
      IFS=';' read -ra groups <<< "${PMC_GROUPS:?set PMC_GROUPS}"
      for counters in "${groups[@]}"; do
        i=$((i + 1))
        timeout -k 10 "$T_STEP" rocprofv3 --pmc $counters --kernel-include-regex "$KRE" --output-format csv \
          -d "$O/cnt${i}_$TAG" -o pmc -- python bench.py --no-cpu-baseline $BENCH_ARGS \
          > "$O/cnt${i}_$TAG.json" 2> "$O/cnt${i}_$TAG.err" || step_fail "counters$i" $? "$O/cnt${i}_$TAG.err"
        python tools/pmc_lines.py "$O/cnt${i}_$TAG" "$O/cnt${i}_$TAG.json" || true
        echo "STEP_OK counters$i ($counters)"
      done ;;
    ab)
      timeout -k 10 "$T_STEP" python tools/ab_inproc.py $AB_ARGS > "$O/ab_$TAG.jsonl" 2> "$O/ab_$TAG.err" ||
        step_fail ab $? "$O/ab_$TAG.err"
      echo "STEP_OK ab"; cat "$O/ab_$TAG.jsonl" ;;
    tsab)
      timeout -k 10 "$T_STEP" python tools/ts_lib_ab.py $TSAB_ARGS > "$O/tsab_$TAG.jsonl" 2> "$O/tsab_$TAG.err" ||
        step_fail tsab $? "$O/tsab_$TAG.err"
      echo "STEP_OK tsab"; cut -c1-300 "$O/tsab_$TAG.jsonl" ;;
    calib)
      mkdir -p "$O/calib_$TAG"
      timeout -k 10 300 ./tools/calib/calib_sweep $CALIB_ARGS > "$O/calib_$TAG/sweep.jsonl" 2> "$O/calib_$TAG/sweep.err" ||
        step_fail calib $? "$O/calib_$TAG/sweep.err"
      timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv \
        -d "$O/calib_$TAG/pmc" -o pmc -- ./tools/calib/calib_sweep ${CALIB_PMC_ARGS:---sizes 256,2048,8192 --waves 5 --dep 1 --reps 1} \
        > "$O/calib_$TAG/pmc.jsonl" 2> "$O/calib_$TAG/pmc.err" || step_fail calib_pmc $? "$O/calib_$TAG/pmc.err"
      echo "STEP_OK calib (summarise: python3 tools/calib/calib_summary.py $O/calib_$TAG <tag>)" ;;
    py)
      timeout -k 10 "$T_STEP" python $PY_ARGS > "$O/py_$TAG.out" 2> "$O/py_$TAG.err" || step_fail py $? "$O/py_$TAG.err"
      echo "STEP_OK py"; tail -5 "$O/py_$TAG.out" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo ALL_OK
