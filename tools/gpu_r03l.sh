#!/bin/bash
# round-3 check set l: bitset build passes split into degree > 64 / <= 64 dispatches (diag library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in r20 r24e6; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fill_split_$g -o fd -- python tools/bs_fill_diag.py --graph $g --knobs 8 > gpurun_out/fill_split_$g.log 2>&1 || exit 1
python - $g <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(f'gpurun_out/fill_split_{sys.argv[1]}/*kernel_trace.csv'):
    rows += [r for r in csv.DictReader(open(f)) if 'k_bs_tri' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
print(sys.argv[1], [(('FILL' if 'true' in r['Kernel_Name'] else 'COUNT'), r['Grid_Size'], round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, 1)) for r in rows])
PY
done
