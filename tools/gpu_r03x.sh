#!/bin/bash
# round-3 set x: same-box calibration vs the shipped headline kernel — the
# random 64 B block rate at 8 GB (tools/calib/calib_sweep.hip, built in-tree),
# the headline launch in-process, the calibration again
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/calib/calib_sweep --sizes 8192 --rb 64 --waves 5 --dep 1 --reps 3 > gpurun_out/sb_calib1.jsonl 2> gpurun_out/sb_calib1.err || { echo CALIB_FAIL; exit 1; }
cat gpurun_out/sb_calib1.jsonl
timeout -k 10 300 python tools/ab_inproc.py main --reps 6 --rebuild 1 > gpurun_out/sb_kernel.json 2> gpurun_out/sb_kernel.err || { echo AB_FAIL; tail -5 gpurun_out/sb_kernel.err; exit 1; }
cat gpurun_out/sb_kernel.json
timeout -k 10 120 ./tools/calib/calib_sweep --sizes 8192 --rb 64 --waves 5 --dep 1 --reps 3 > gpurun_out/sb_calib2.jsonl 2> gpurun_out/sb_calib2.err || { echo CALIB2_FAIL; exit 1; }
cat gpurun_out/sb_calib2.jsonl
