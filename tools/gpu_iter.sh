#!/bin/bash
# quick iteration: GPU parity tests then one bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-iter}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
