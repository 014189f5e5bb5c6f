#!/bin/bash
# round-3 check set o: TopSim LDS hash reservation (A/B vs b782b8e)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_topsim_gpu.py tests/test_topsim_law_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r03o.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03o.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/ts_lib_ab.py main graph-embedding_amd/gwamd/ab/libgraphwalk_hcount.so graph-embedding_amd/gwamd/ab/libgraphwalk_b782b8e.so --graphs p10m,blog,arxiv --reps 4 > gpurun_out/ts_ab_o.json 2> gpurun_out/ts_ab_o.err
echo AB_RC=$?; cut -c1-160 gpurun_out/ts_ab_o.json
