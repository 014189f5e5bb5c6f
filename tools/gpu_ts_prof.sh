#!/bin/bash
# TopSim kernel on P10M (config 5): kernel trace + SQ/TCC counter passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ts}
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-simrank --no-walk10m --no-rmat24 --no-arxiv --no-p10m --topsim-graphs ${GRAPHS:-p10m}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o kt -- python bench.py $ARGS > gpurun_out/${TAG}_kt.json 2> gpurun_out/${TAG}_kt.err || { echo KT_FAIL; tail -5 gpurun_out/${TAG}_kt.err; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-include-regex "k_topsim" --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python bench.py $ARGS > gpurun_out/${TAG}_p$i.json 2> gpurun_out/${TAG}_p$i.err || { echo "PASS $i FAIL ($grp)"; tail -5 gpurun_out/${TAG}_p$i.err; exit 1; }
done
grep -h "k_topsim" gpurun_out/${TAG}_kt/kt_kernel_stats.csv | cut -c1-200
python - <<'PY'
import csv, glob, os
tag = os.environ.get("TAG", "ts")
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/pmc_counter_collection.csv")):
    acc = {}
    for r in csv.DictReader(open(f)):
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{k:32s} {sum(v)/len(v):.6g}  (n={len(v)})")
PY
