#!/bin/bash
# Second-half-of-line reuse test (tools/calib/calib_halfline.hip, built
# in-tree beforehand): timing sweep plus TCC request / hit passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/half
B=./tools/calib/calib_halfline
A="${HALF_ARGS:---sizes 2048,8192}"
timeout -k 10 200 $B $A > gpurun_out/half/sweep.jsonl 2> gpurun_out/half/sweep.err || { echo SWEEP_FAIL; cat gpurun_out/half/sweep.err; exit 1; }
P="--sizes 8192 --reps 1"
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/half/pmc -o pmc -- $B $P > gpurun_out/half/pmc.jsonl 2> gpurun_out/half/pmc.err || { echo PMC_FAIL; tail -5 gpurun_out/half/pmc.err; exit 1; }
cat gpurun_out/half/sweep.jsonl
echo HALF_OK
