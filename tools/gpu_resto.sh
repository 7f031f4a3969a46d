set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lmpc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_lmpc_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_lmpc_tests.log; exit 1; }
tail -2 gpurun_out/gpu_lmpc_tests.log
timeout -k 10 300 python -u tools/resto_time.py > gpurun_out/resto_time.log 2>&1 || { echo TIMING_FAILED; tail -20 gpurun_out/resto_time.log; exit 1; }
cat gpurun_out/resto_time.log
