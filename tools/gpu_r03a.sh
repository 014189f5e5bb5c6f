#!/bin/bash
# round-3 check set: full-size + TopSim tests, then build timings (kernel trace) and a config-4 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_fullsize_gpu.py tests/test_topsim_gpu.py tests/test_simrank_gpu.py tests/test_topsim_law_gpu.py tests/test_bench_gpu.py -x -q -s --timeout 400 --timeout-method thread > gpurun_out/t_r03a.log 2>&1
echo TEST_RC=$?; tail -4 gpurun_out/t_r03a.log; grep "\[law\]" gpurun_out/t_r03a.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_build -o kt -- python tools/build_time.py --graphs r20,r24e6,r22 > gpurun_out/build_time.json 2> gpurun_out/build_time.err
echo BUILD_RC=$?; cat gpurun_out/build_time.json; grep "\[build\]" gpurun_out/build_time.err
timeout -k 10 300 python bench.py --no-cpu-baseline --config 4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
echo BENCH_RC=$?; cut -c1-800 gpurun_out/bench_c4.json
