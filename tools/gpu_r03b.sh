#!/bin/bash
# round-3 check set b: the whole GPU suite, build timings under a kernel trace, the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 400 --timeout-method thread > gpurun_out/t_r03b.log 2>&1
echo TEST_RC=$?; tail -4 gpurun_out/t_r03b.log; grep "\[law\]" gpurun_out/t_r03b.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_build_b -o kt -- python tools/build_time.py --graphs r20,r24e6 --modes bitset,listed > gpurun_out/build_time_b.json 2> gpurun_out/build_time_b.err
echo BUILD_RC=$?; grep "\[build\]" gpurun_out/build_time_b.err
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err
echo BENCH_RC=$?; cut -c1-400 gpurun_out/bench_b.json
