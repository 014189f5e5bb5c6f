#!/bin/bash
# timing A/B of the bitset walk with diagnostic knobs (wrong walks; timing only).
# Needs the -DGW_DIAG library built beforehand: python graph-embedding_amd/build.py --diag
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for dg in ${DIAGS:-0 1 2 3}; do
  GW_LIB=$GRAFT_REPO_ROOT/graph-embedding_amd/gwamd/libgraphwalk_diag.so GW_DIAG_BS=$dg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --secondary none > gpurun_out/diag_$dg.json 2> gpurun_out/diag_$dg.err || { echo FAIL $dg; tail -5 gpurun_out/diag_$dg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/diag_$dg.json'));print($dg, d['value'], d['roofline']['kernel_ms'])"
done
