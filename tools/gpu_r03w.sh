#!/bin/bash
# round-3 set w: the default bench line on the shipped library (traffic and
# request-rate fields now keyed in profiles/pmc_summary.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/bench_r03w.json 2> gpurun_out/bench_r03w.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_r03w.err; exit 1; }
echo BENCH_OK
