#!/bin/bash
# PMC passes on the walk kernel (one counter group per pass, kernel-trace only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-cnt}
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-topsim ${BENCH_ARGS}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_walk_scale|k_walk_bitset" --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python bench.py $ARGS > gpurun_out/${TAG}_p$i.json 2> gpurun_out/${TAG}_p$i.err || { echo "PASS $i FAIL ($grp)"; tail -5 gpurun_out/${TAG}_p$i.err; }
done
python - <<'PY'
import csv, glob, os
tag = os.environ.get("TAG", "cnt")
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/pmc_counter_collection.csv")):
    acc = {}
    for r in csv.DictReader(open(f)):
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{k:32s} {sum(v)/len(v):.6g}  (n={len(v)})")
PY
