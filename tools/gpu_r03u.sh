#!/bin/bash
# round-3 set u: degree-ordered bitset tables — bitset GPU parity tests, then the
# in-process A/B against the id-ordered library (abl/base_6f5939f5.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_n2v_gpu.py tests/test_walk_law_gpu.py tests/test_fullsize_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r03u.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -5 gpurun_out/t_r03u.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_inproc.py abl/base_6f5939f5.so main --reps 8 --rebuild 2 > gpurun_out/ab_r03u.json 2> gpurun_out/ab_r03u.err
rc=$?; echo AB_RC=$rc; cat gpurun_out/ab_r03u.json; grep prepare gpurun_out/ab_r03u.err | head -4
