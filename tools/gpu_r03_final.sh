#!/bin/bash
# round-3 final measurement set on the shipped library: the default bench line,
# a kernel trace of the same command, then three separate PMC passes
# (FETCH_SIZE; WRITE_SIZE; TCC_EA0_RDREQ/HIT/MISS) for tools/pmc_summary.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r03f
KRE="k_walk|k_topsim"
NOCPU="--no-cpu-baseline"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/t_$TAG.log; exit 1; }
echo TESTS_OK; tail -1 gpurun_out/t_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
echo SMOKE_OK
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo BENCH_OK
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o kt -- python bench.py $NOCPU > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || { echo PROF_FAIL; tail -20 gpurun_out/prof_$TAG.err; exit 1; }
echo KT_OK
python tools/kt_summary.py gpurun_out/prof_$TAG/kt_kernel_trace.csv gpurun_out/prof_$TAG/kernel_dispatch_summary.json > /dev/null || true
timeout -k 10 360 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d gpurun_out/pmc1_$TAG -o pmc -- python bench.py $NOCPU > gpurun_out/pmc1_$TAG.json 2> gpurun_out/pmc1_$TAG.err || { echo PMC1_FAIL; tail -20 gpurun_out/pmc1_$TAG.err; exit 1; }
echo PMC1_OK
timeout -k 10 360 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d gpurun_out/pmc2_$TAG -o pmc -- python bench.py $NOCPU > gpurun_out/pmc2_$TAG.json 2> gpurun_out/pmc2_$TAG.err || { echo PMC2_FAIL; tail -20 gpurun_out/pmc2_$TAG.err; exit 1; }
echo PMC2_OK
timeout -k 10 360 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE" --output-format csv -d gpurun_out/pmc3_$TAG -o pmc -- python bench.py $NOCPU > gpurun_out/pmc3_$TAG.json 2> gpurun_out/pmc3_$TAG.err || { echo PMC3_FAIL; tail -20 gpurun_out/pmc3_$TAG.err; exit 1; }
echo PMC3_OK
