#!/bin/bash
# round-end set, part A: the default bench line and a kernel trace of the same command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r03
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo BENCH_OK
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o kt -- python bench.py --no-cpu-baseline > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || { echo PROF_FAIL; tail -20 gpurun_out/prof_$TAG.err; exit 1; }
echo KT_OK
python tools/kt_summary.py gpurun_out/prof_$TAG/kt_kernel_trace.csv gpurun_out/prof_$TAG/kernel_dispatch_summary.json > /dev/null || true
echo ALL_OK
