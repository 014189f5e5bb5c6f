#!/bin/bash
# bitset walk: parity tests then bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-bs}
timeout -k 10 900 python -m pytest tests/test_n2v_gpu.py -x -q -k "bitset or scale" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-topsim ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
