# round 5: GPU tests, then the PMPC restoration stamps (tools/stamps_pmpc_resto.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u tools/stamps_pmpc_resto.py > gpurun_out/stamps_pr31.log 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/stamps_pr31.log; exit 1; }
cat gpurun_out/stamps_pr31.log
DART_STAMPS_N=20 DART_STAMPS_SOC=0 timeout -k 10 200 python -u tools/stamps_pmpc_resto.py > gpurun_out/stamps_pr20.log 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/stamps_pr20.log; exit 1; }
cat gpurun_out/stamps_pr20.log
