#!/bin/bash
# round-3 check set d: the whole GPU suite, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_r03d.log 2>&1
echo TEST_RC=$?; tail -4 gpurun_out/t_r03d.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err
echo BENCH_RC=$?; cut -c1-300 gpurun_out/bench_d.json
timeout -k 10 300 python tools/ab_inproc.py 47ac162 main --reps 8 > gpurun_out/ab_dual_r20.json 2> gpurun_out/ab_dual_r20.err
echo AB20_RC=$?; cat gpurun_out/ab_dual_r20.json
timeout -k 10 400 python tools/ab_inproc.py 47ac162 main --scale 24 --ef 6 --walks 1 --reps 8 --rebuild 1 > gpurun_out/ab_dual_r24e6.json 2> gpurun_out/ab_dual_r24e6.err
echo AB24_RC=$?; cat gpurun_out/ab_dual_r24e6.json
