#!/bin/bash
# bench + rocprofv3 kernel trace + PMC (FETCH_SIZE / WRITE_SIZE in separate passes).
# kernel_dispatch_summary.json splits each kernel by grid size: the headline launch
# (R-MAT-20, 6,463,230 walks) is the k_walk_bitset row with grid=6463232.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o kt -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_bench_$TAG.err || { echo PROF_FAIL; tail -20 gpurun_out/prof_bench_$TAG.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_walk_scale|k_walk_bitset|k_topsim" --output-format csv -d gpurun_out/pmc1_$TAG -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-simrank --no-walk10m --no-rmat24 > gpurun_out/pmc1_$TAG.json 2> gpurun_out/pmc1_$TAG.err || { echo PMC1_FAIL; tail -20 gpurun_out/pmc1_$TAG.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_walk_scale|k_walk_bitset|k_topsim" --output-format csv -d gpurun_out/pmc2_$TAG -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-simrank --no-walk10m --no-rmat24 > gpurun_out/pmc2_$TAG.json 2> gpurun_out/pmc2_$TAG.err || { echo PMC2_FAIL; tail -20 gpurun_out/pmc2_$TAG.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_walk_scale|k_walk_bitset|k_topsim" --output-format csv -d gpurun_out/pmc3_$TAG -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-simrank --no-walk10m --no-rmat24 > gpurun_out/pmc3_$TAG.json 2> gpurun_out/pmc3_$TAG.err || { echo PMC3_FAIL; tail -20 gpurun_out/pmc3_$TAG.err; exit 1; }
python tools/kt_summary.py gpurun_out/prof_$TAG/kt_kernel_trace.csv gpurun_out/prof_$TAG/kernel_dispatch_summary.json > /dev/null
echo ALL_OK
find gpurun_out -name "*.csv" | head -20
# TopSim on the 10M-vertex graph (config 5): kernel trace of that workload alone
if [ -n "$P10M" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p10m_$TAG -o kt -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-simrank --no-walk10m --no-rmat24 --topsim-graphs p10m > gpurun_out/prof_p10m_$TAG.json 2> gpurun_out/prof_p10m_$TAG.err || { echo P10M_FAIL; tail -20 gpurun_out/prof_p10m_$TAG.err; exit 1; }
  echo P10M_OK
fi
