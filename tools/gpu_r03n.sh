#!/bin/bash
# round-3 check set n: config-4 graph (R-MAT-24 ef 16): lists-only build time with the
# edge-centric builder vs plain rejection prepare, one 1-walk/vertex launch each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/build_time.py --graphs r24 --modes listed,plain --reps 2 --walks 1 > gpurun_out/build_time_n.json 2> gpurun_out/build_time_n.err
echo BT_RC=$?; cat gpurun_out/build_time_n.json; grep -E "\[build\]|\[walk\]" gpurun_out/build_time_n.err
