# smoke + GPU tests + the default bench line (one box call)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 ; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  echo BENCH_OK; cut -c1-600 gpurun_out/bench_$TAG.json
fi
