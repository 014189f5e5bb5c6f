#!/bin/bash
# round-3 check set g: node2vec + TopSim GPU tests (build kernel scalarised, TopSim
# body templated on the workgroup size), build timing, TopSim hash-mode A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_n2v_gpu.py tests/test_fullsize_gpu.py tests/test_topsim_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r03g.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03g.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_build_g -o bt -- python tools/build_time.py --graphs r20,r24e6 --modes bitset --reps 2 > gpurun_out/build_time_g.json 2> gpurun_out/build_time_g.err
echo BT_RC=$?; cat gpurun_out/build_time_g.json; grep "\[build\]" gpurun_out/build_time_g.err
timeout -k 10 400 python tools/ts_mode_ab.py --modes 2,3 --graphs p10m,arxiv --reps 3 > gpurun_out/ts_mode_ab_g.json 2> gpurun_out/ts_mode_ab_g.err
echo AB_RC=$?; cat gpurun_out/ts_mode_ab_g.json
