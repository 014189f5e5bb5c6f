#!/bin/bash
# round-3 set t: naive SimRank kernel trace (pass 1 vs pass 2 durations)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sr_kt -o kt -- python tools/sr_time.py blog > gpurun_out/sr_kt.log 2>&1
echo KT_RC=$?; cat gpurun_out/sr_kt.log | grep blog; f=$(ls gpurun_out/sr_kt/*kernel_stats.csv gpurun_out/sr_kt/*/*kernel_stats.csv 2>/dev/null | head -1); cut -d, -f1-8 "$f" | head -12
