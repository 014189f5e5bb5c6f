#!/bin/bash
# round-3 full GPU suite (as the driver runs it) + smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r03_full.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03.log 2>&1
echo SMOKE_RC=$?; tail -2 gpurun_out/smoke_r03.log
