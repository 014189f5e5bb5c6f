#!/bin/bash
# round-3 check set h: where the bitset build's FILL pass spends its time
# (timing-only knobs of the diag library, LDS and L2-atomic counters)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fill_diag -o fd -- python tools/bs_fill_diag.py --graph r20 > gpurun_out/fill_diag.log 2>&1
echo DIAG_RC=$?
python - <<'PY'
import csv, glob
rows = []
for f in glob.glob('gpurun_out/fill_diag/*kernel_trace.csv'):
    rows += [r for r in csv.DictReader(open(f)) if 'k_bs_tri' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
print([(('FILL' if 'true' in r['Kernel_Name'] else 'COUNT'), round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, 1)) for r in rows])
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM --kernel-include-regex k_bs_tri --output-format csv -d gpurun_out/pmc_build_lds -o pmc -- python tools/build_time.py --graphs r20 --modes bitset --reps 1 > /dev/null 2> gpurun_out/pmc_build_lds.err
echo PMC1_RC=$?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_bs_tri --output-format csv -d gpurun_out/pmc_build_tcc -o pmc -- python tools/build_time.py --graphs r20 --modes bitset --reps 1 > /dev/null 2> gpurun_out/pmc_build_tcc.err
echo PMC2_RC=$?
