#!/bin/bash
# Random-block read-rate calibration (tools/calib/calib_sweep.hip, built in-tree
# beforehand): full sweep (table size x read size x waves/SIMD x dep) plus
# rocprofv3 passes for the fabric request counters of the same kernels.
# Output: gpurun_out/calib/*.  Summarised into profiles/calib_<tag>.json by
# tools/calib/calib_summary.py (run it here or on the box).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
B=./tools/calib/calib_sweep
timeout -k 10 300 $B ${CALIB_ARGS} > gpurun_out/calib/sweep.jsonl 2> gpurun_out/calib/sweep.err || { echo SWEEP_FAIL; cat gpurun_out/calib/sweep.err; exit 1; }
PMC_ARGS="--sizes 256,2048,8192 --waves 5 --dep 1 --reps 1 --rb 32,64,128,256"
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/calib/pmc_rdreq -o pmc -- $B $PMC_ARGS > gpurun_out/calib/pmc_rdreq.jsonl 2> gpurun_out/calib/pmc_rdreq.err || { echo PMC1_FAIL; tail -5 gpurun_out/calib/pmc_rdreq.err; exit 1; }
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/calib/pmc_hit -o pmc -- $B $PMC_ARGS > gpurun_out/calib/pmc_hit.jsonl 2> gpurun_out/calib/pmc_hit.err || { echo PMC2_FAIL; tail -5 gpurun_out/calib/pmc_hit.err; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/pmc_fetch -o pmc -- $B $PMC_ARGS > gpurun_out/calib/pmc_fetch.jsonl 2> gpurun_out/calib/pmc_fetch.err || { echo PMC3_FAIL; tail -5 gpurun_out/calib/pmc_fetch.err; exit 1; }
echo CALIB_OK  # then, here: python3 tools/calib/calib_summary.py gpurun_out/calib <tag>
