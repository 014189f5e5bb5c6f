#!/bin/bash
# A/B timing of diagnostic knobs on the bench workload (no tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--steps 3 --warmup 1 --no-cpu-baseline --no-topsim ${BENCH_ARGS}"
for v in "" "GW_DIAG_NO_BITMAP=1"; do
  env $v timeout -k 10 300 python bench.py $A > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo FAIL; tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', round(d['value']/1e9,3),'G steps/s', round(d['roofline']['kernel_ms'],2),'ms')"
done
