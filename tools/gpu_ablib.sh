#!/bin/bash
# A/B timing of library variants (abl/<name>.so, or "main" for the in-tree
# build) on the bench workload + the north_star 10M graph.
#   LIBS="main orig coop7 main:GW_DIAG_NO_SENT=1" bash tools/gpu_ablib.sh
# (<lib>:<VAR=value> runs that library with one extra environment setting)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--steps 3 --warmup 1 --no-cpu-baseline --no-topsim --no-simrank ${BENCH_ARGS}"
for v in ${LIBS:-main}; do
  lib=${v%%:*}; ev=""; [ "$lib" != "$v" ] && ev=${v#*:}
  if [ "$lib" = main ]; then unset GW_LIB; else export GW_LIB=$PWD/abl/$lib.so; fi
  env $ev timeout -k 10 300 python bench.py $A > gpurun_out/ab_${v//[:=]/_}.json 2>gpurun_out/ab_${v//[:=]/_}.err || { echo "FAIL $v"; tail -5 gpurun_out/ab_${v//[:=]/_}.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_${v//[:=]/_}.json'))
s=d.get('secondary') or {}
print('$v', round(d['value']/1e9,3),'G steps/s', round(d['roofline']['kernel_ms'],2),'ms', *[(k, round(x['value']/1e9,3), round(x.get('kernel_ms',0),2)) for k,x in s.items()])"
done
