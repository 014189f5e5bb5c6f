#!/bin/bash
# round-3 set s: naive SimRank with the row-padded stream — GPU tests, timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_simrank_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sr_tests_r03s.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -5 gpurun_out/sr_tests_r03s.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sr_time.py g333 moreno blog > gpurun_out/sr_time_r03s.log 2>&1
echo TIME_RC=$?; cat gpurun_out/sr_time_r03s.log
