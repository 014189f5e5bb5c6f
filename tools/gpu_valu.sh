#!/bin/bash
# instruction mix per library variant on the bench workload (one PMC pass each)
#   LIBS="prev main" bash tools/gpu_valu.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-topsim --no-simrank --no-walk10m ${BENCH_ARGS}"
for v in ${LIBS:-main}; do
  if [ "$v" = main ]; then unset GW_LIB; else export GW_LIB=$PWD/abl/$v.so; fi
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_walk_bitset|k_walk_scale" --output-format csv -d gpurun_out/valu_$v -o pmc -- python bench.py $ARGS > gpurun_out/valu_$v.json 2> gpurun_out/valu_$v.err || { echo "FAIL $v"; tail -5 gpurun_out/valu_$v.err; exit 1; }
  python - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
acc = {}
for f in glob.glob(f"gpurun_out/valu_{v}/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(v, " ".join(f"{k}={sum(x)/len(x):.4g}" for k, x in sorted(acc.items())))
PY
done
