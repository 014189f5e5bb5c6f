#!/bin/bash
# Naive SimRank kernels: kernel-trace stats + PMC passes (one group per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-sr}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt -- python tools/sr_time.py blog > gpurun_out/${TAG}_kt.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_sr_gather" --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python tools/sr_time.py blog > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "PASS $i FAIL ($grp)"; tail -5 gpurun_out/${TAG}_p$i.log; }
done
find gpurun_out/${TAG}_kt -name "*stats*.csv" -exec cat {} \; ; ls -R gpurun_out/${TAG}_kt | head
python - <<'PY'
import csv, glob, os
tag = os.environ.get("TAG", "sr")
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/**/pmc_counter_collection.csv", recursive=True)):
    acc = {}
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        key = (kn[kn.find("k_sr"):kn.find("k_sr") + 30] if "k_sr" in kn else kn[:30], r["Counter_Name"])
        acc.setdefault(key, []).append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{k[0]:42s} {k[1]:24s} {sum(v)/len(v):.6g}  (n={len(v)})")
PY
