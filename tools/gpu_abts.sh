#!/bin/bash
# A/B timing of library variants on the TopSim secondary workloads
#   LIBS="prev main" bash tools/gpu_abts.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--steps 1 --warmup 0 --no-cpu-baseline --no-simrank --no-walk10m --topsim-graphs ${TS_GRAPHS:-p10m,blog,arxiv} ${BENCH_ARGS}"
for v in ${LIBS:-main}; do
  lib=${v%%:*}; ev=""; [ "$lib" != "$v" ] && ev=${v#*:}
  if [ "$lib" = main ]; then unset GW_LIB; else export GW_LIB=$PWD/abl/$lib.so; fi
  tag=ts_${v//[:=]/_}
  env $ev timeout -k 10 400 python bench.py $A > gpurun_out/$tag.json 2>gpurun_out/$tag.err || { echo "FAIL $v"; tail -5 gpurun_out/$tag.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/$tag.json'))
t=d['secondary']['topsim']; r=[t]+t.get('more',[])
print('$v', *[(x['config']['workload'].split(' ')[2], round(x['seconds']*1e3,2),'ms', round(x['value']/1e9,2),'G upd/s') for x in r])"
done
