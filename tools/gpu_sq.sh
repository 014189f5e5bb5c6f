# One PMC pass of SQ counters on the bench headline (wave time split: waiting on
# memory / issue-stalled / issuing; VALU share), printed per walk kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-sq}
ARGS=${ARGS:-"--secondary none --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_walk" --output-format csv -d gpurun_out/${TAG}_pmc -o pmc -- python bench.py $ARGS --steps 2 --warmup 1 > gpurun_out/${TAG}_pmc.json 2> gpurun_out/${TAG}_pmc.err || { echo PMC_FAIL; tail -5 gpurun_out/${TAG}_pmc.err; exit 1; }
python tools/pmc_lines.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc.json
echo SQ_OK
