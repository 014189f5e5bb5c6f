#!/bin/bash
# round-3 set v: fabric read requests and VALU instructions of the headline
# launch, id-ordered (abl/base_6f5939f5.so) vs degree-ordered tables
# (abl/degree_order.so), one process, dispatches interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum SQ_INSTS_VALU SQ_WAVES --kernel-include-regex k_walk_bitset --output-format csv -d gpurun_out/pmc_deg -o pmc -- python tools/ab_inproc.py abl/base_6f5939f5.so abl/degree_order.so --reps 2 --rebuild 1 > gpurun_out/pmc_deg.json 2> gpurun_out/pmc_deg.err
echo PMC_RC=$?; cat gpurun_out/pmc_deg.json
