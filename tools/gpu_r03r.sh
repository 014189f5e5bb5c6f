#!/bin/bash
# round-3 set r: headline in-process A/B (main vs deferred flush vs walk index
# re-derived per iteration), walks compared bitwise; LDS random-gather calibration
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_inproc.py main abl/deferflush.so abl/wbase.so --reps 8 --rebuild 2 > gpurun_out/ab_r03r.json 2> gpurun_out/ab_r03r.err
rc=$?; echo AB_RC=$rc; cat gpurun_out/ab_r03r.json
[ $rc -eq 0 ] || { tail -5 gpurun_out/ab_r03r.err; exit $rc; }
timeout -k 10 120 ./tools/calib/calib_lds > gpurun_out/calib_lds.jsonl 2> gpurun_out/calib_lds.err
echo CALIB_RC=$?; cat gpurun_out/calib_lds.jsonl
