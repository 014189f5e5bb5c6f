#!/bin/bash
# round-3 check set e: the TopSim / SimRank GPU tests, SQ counters of the two build passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_topsim_law_gpu.py tests/test_topsim_m_gpu.py tests/test_topsim_double_gpu.py tests/test_topsim_gpu.py tests/test_simrank_gpu.py -x -q -s --timeout 400 --timeout-method thread > gpurun_out/t_r03e.log 2>&1
echo TEST_RC=$?; tail -3 gpurun_out/t_r03e.log; grep "\[law\]" gpurun_out/t_r03e.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --kernel-include-regex k_bs_tri --output-format csv -d gpurun_out/pmc_build_sq -o pmc -- python tools/build_time.py --graphs r20 --modes bitset --reps 1 > /dev/null 2> gpurun_out/pmc_build_sq.err
echo PMC_RC=$?
