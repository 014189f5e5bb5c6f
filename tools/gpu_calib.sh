#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/calib/calib_gather > gpurun_out/calib.txt 2>&1 && cat gpurun_out/calib.txt && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_p1 -o pmc -- ./tools/calib/calib_gather > /dev/null 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/calib_p2 -o pmc -- ./tools/calib/calib_gather > /dev/null 2>&1 && \
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/calib_p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "gather" in r["Kernel_Name"]:
            print(r["Counter_Name"], r["Counter_Value"])
PY
