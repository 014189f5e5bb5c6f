# Quick perf check of the headline: bench (headline only) x REPS, then one
# rocprofv3 PMC pass (fabric read requests, L2 hit/miss) and a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-perf}
ARGS=${ARGS:-"--secondary none --no-cpu-baseline"}
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_bench$r.json 2> gpurun_out/${TAG}_bench$r.err || { echo BENCH_FAIL; tail -20 gpurun_out/${TAG}_bench$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench$r.json'));r=d['roofline'];print('bench', '%.4g'%d['value'], 'kernel_ms %.3f'%r['kernel_ms'], 'frac %.4f'%r['frac'])"
done
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_walk" --output-format csv -d gpurun_out/${TAG}_pmc -o pmc -- python bench.py $ARGS --steps 2 --warmup 1 > gpurun_out/${TAG}_pmc.json 2> gpurun_out/${TAG}_pmc.err || { echo PMC_FAIL; tail -5 gpurun_out/${TAG}_pmc.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o kt -- python bench.py $ARGS --steps 3 --warmup 1 > gpurun_out/${TAG}_kt.json 2> gpurun_out/${TAG}_kt.err || { echo KT_FAIL; tail -5 gpurun_out/${TAG}_kt.err; exit 1; }
python tools/pmc_lines.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc.json
echo PERF_OK
