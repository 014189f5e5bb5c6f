#!/bin/bash
# round-3 set p: full GPU suite + smoke, then TopSim P10M A/Bs (diag library,
# in-process): 16 B vs packed 8 B slot entries; walker reads confined to
# 1 / 2 GB of the slot table (timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r03p_full.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03p_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03p.log 2>&1
rc=$?; echo SMOKE_RC=$rc; tail -2 gpurun_out/smoke_r03p.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ts_mode_ab.py --env GW_DIAG_TS_E16 --modes 1,0 --graphs p10m,arxiv --reps 4 > gpurun_out/ts_e8_ab.json 2> gpurun_out/ts_e8_ab.err
rc=$?; echo AB_RC=$rc; cut -c1-220 gpurun_out/ts_e8_ab.json
[ $rc -eq 0 ] || exit $rc
GW_DIAG_TS_E16=1 timeout -k 10 400 python tools/ts_mode_ab.py --env GW_DIAG_TS --modes 0,4,8 --graphs p10m --reps 3 > gpurun_out/ts_footprint_ab.json 2> gpurun_out/ts_footprint_ab.err
echo AB2_RC=$?; cut -c1-200 gpurun_out/ts_footprint_ab.json
