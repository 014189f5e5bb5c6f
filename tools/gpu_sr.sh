set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_simrank_gpu.py -x -q > gpurun_out/sr_tests.log 2>&1 && \
timeout -k 10 300 python tools/sr_time.py g333 moreno blog > gpurun_out/sr_time.log 2>&1
rc=$?; tail -5 gpurun_out/sr_tests.log; cat gpurun_out/sr_time.log; exit $rc
