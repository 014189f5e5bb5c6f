#!/bin/bash
# Counter passes of the headline walk launch for library variants loaded into
# ONE process (tools/ab_inproc.py, interleaved launches; dispatches told apart
# by kernel id / order).  Each pass is its own rocprofv3 run under a time limit.
#   TAG=x tools/pmc_lib_pair.sh LIB_A LIB_B      -> gpurun_out/pmcpair_<TAG>_<i>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-pair}
i=0
for counters in "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex k_walk_bitset --output-format csv \
    -d gpurun_out/pmcpair_${TAG}_$i -o pmc -- python tools/ab_inproc.py "$@" --reps 2 --rebuild 1 \
    > gpurun_out/pmcpair_${TAG}_$i.json 2> gpurun_out/pmcpair_${TAG}_$i.err || { echo "STEP_FAIL pass $i"; tail -5 gpurun_out/pmcpair_${TAG}_$i.err; exit 1; }
  echo "STEP_OK pass $i"
done
