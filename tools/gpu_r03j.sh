#!/bin/bash
# round-3 check set j: TopSim barrier cuts (empty levels, wave-level compaction,
# double-buffered radix passes): tests + in-process A/B against the round's base
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_topsim_gpu.py tests/test_topsim_law_gpu.py tests/test_topsim_m_gpu.py tests/test_topsim_double_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r03j.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03j.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/ts_lib_ab.py main graph-embedding_amd/gwamd/ab/libgraphwalk_ccb0774.so --graphs p10m,blog,arxiv --reps 4 > gpurun_out/ts_ab_j.json 2> gpurun_out/ts_ab_j.err
echo AB_RC=$?; cut -c1-200 gpurun_out/ts_ab_j.json
