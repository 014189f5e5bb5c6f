#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_topsim_m_gpu.py} -x -q ${PYTEST_ARGS} > gpurun_out/tm.log 2>&1
rc=$?; tail -30 gpurun_out/tm.log; exit $rc
