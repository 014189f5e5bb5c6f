#!/bin/bash
# round-3 check set c: the node2vec GPU tests, build timings under a kernel trace, the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_n2v_gpu.py tests/test_walk_law_gpu.py tests/test_fullsize_gpu.py tests/test_bench_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/t_r03c.log 2>&1
echo TEST_RC=$?; tail -4 gpurun_out/t_r03c.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_build_c -o kt -- python tools/build_time.py --graphs r20,r24e6 --modes bitset,listed,plain --walks 10 > gpurun_out/build_time_c.json 2> gpurun_out/build_time_c.err
echo BUILD_RC=$?; grep "\[build\]\|\[walk\]" gpurun_out/build_time_c.err
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err
echo BENCH_RC=$?; cut -c1-300 gpurun_out/bench_c.json
