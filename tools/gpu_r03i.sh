#!/bin/bash
# round-3 check set i: TopSim merged level scan (A/B against the round's base
# library), TopSim tests, build timing after the hoisted first-round load
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_topsim_gpu.py tests/test_topsim_law_gpu.py tests/test_n2v_gpu.py -x -q --timeout 300 --timeout-method thread -k "topsim or bitset" > gpurun_out/t_r03i.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03i.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ts_lib_ab.py main graph-embedding_amd/gwamd/ab/libgraphwalk_ccb0774.so --graphs p10m,blog --reps 4 > gpurun_out/ts_ab_i.json 2> gpurun_out/ts_ab_i.err
echo AB_RC=$?; cat gpurun_out/ts_ab_i.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_build_i -o bt -- python tools/build_time.py --graphs r20,r24e6 --modes bitset --reps 2 > gpurun_out/build_time_i.json 2> gpurun_out/build_time_i.err
echo BT_RC=$?; grep "\[build\]" gpurun_out/build_time_i.err
