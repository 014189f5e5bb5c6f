#!/bin/bash
# Walk-steps/s of the headline kernel against the number of walks per launch
# (tail / ramp effects of one launch): NW in walks-per-vertex, same graph and p/q
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for nw in ${NWS:-2 5 10 20 40}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --secondary none --no-cpu-baseline --num-walks $nw > gpurun_out/tail_$nw.json 2> gpurun_out/tail_$nw.err || { echo "FAIL $nw"; tail -5 gpurun_out/tail_$nw.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/tail_$nw.json').readline())
print('num_walks $nw', round(d['value']/1e9,2), 'G steps/s', round(d['roofline']['kernel_ms'],2), 'ms/launch')"
done
