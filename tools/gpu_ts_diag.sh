#!/bin/bash
# Needs the -DGW_DIAG library built beforehand: python graph-embedding_amd/build.py --diag
# TopSim phase timings under diagnostic A/B knobs (GW_DIAG_TS values in DIAGS; timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GRAPHS=${GRAPHS:-p10m}
for dg in ${DIAGS:-0 1 2 3}; do
  GW_LIB=$GRAFT_REPO_ROOT/graph-embedding_amd/gwamd/libgraphwalk_diag.so GW_DIAG_TS=$dg GW_DIAG_TS_PHASES=1 timeout -k 10 600 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-simrank --no-walk10m --topsim-graphs $GRAPHS > gpurun_out/tsd_$dg.json 2> gpurun_out/tsd_$dg.err || { echo FAIL $dg; tail -5 gpurun_out/tsd_$dg.err; exit 1; }
  echo "diag $dg: $(grep phases gpurun_out/tsd_$dg.err | tail -1)"
  python -c "
import json; d=json.load(open('gpurun_out/tsd_$dg.json'))['secondary']['topsim']
for r in [d]+d.get('more',[]): print('   ', r['config']['workload'][:30], round(r['roofline']['kernel_ms'],2), 'ms')"
done
