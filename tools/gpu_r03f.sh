#!/bin/bash
# round-3 check set f: node2vec GPU tests after a build-kernel change, build timing + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_n2v_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r03f.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03f.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_build_f -o bt -- python tools/build_time.py --graphs r20,r24e6 --modes bitset --reps 2 > gpurun_out/build_time_f.json 2> gpurun_out/build_time_f.err
echo BT_RC=$?; cat gpurun_out/build_time_f.json; grep build gpurun_out/build_time_f.err
