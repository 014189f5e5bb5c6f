#!/bin/bash
# round-3 check set k: bitset build (stream rounds in flight, hub chunks skipped per edge)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_n2v_gpu.py -x -q --timeout 300 --timeout-method thread -k "bitset or auto or directory or multichunk" > gpurun_out/t_r03k.log 2>&1
rc=$?; echo TEST_RC=$rc; tail -3 gpurun_out/t_r03k.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_build_k -o bt -- python tools/build_time.py --graphs r20,r24e6 --modes bitset --reps 2 > gpurun_out/build_time_k.json 2> gpurun_out/build_time_k.err
echo BT_RC=$?; grep "\[build\]" gpurun_out/build_time_k.err
python - <<'PY'
import csv, glob
rows = []
for f in glob.glob('gpurun_out/prof_build_k/*kernel_trace.csv'):
    rows += [r for r in csv.DictReader(open(f)) if 'k_bs_tri' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
print([(('FILL' if 'true' in r['Kernel_Name'] else 'COUNT'), round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, 1)) for r in rows])
PY
