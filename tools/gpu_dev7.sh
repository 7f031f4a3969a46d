# round 5: trace of the LMPC restoration instance at N = 32 (two-wave build), then the long-horizon tests and the
# rest of the GPU suite without stopping at the first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/wg2_trace.py 32 > gpurun_out/wg2_trace_32.txt 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/wg2_trace_32.txt; exit 1; }
tail -3 gpurun_out/wg2_trace_32.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc $rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/gpu_tests.log | tail -30
