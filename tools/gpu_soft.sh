# round 5: the soft restoration phase in the N > 31 register kernel: PMPC tests + A/B + restoration lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_pmpc.py tests/test_gpu_serve.py tests/test_gpu_call_form.py tests/test_gpu_batch_server.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pmpc_tests.log 2>&1; echo "tests rc $?"
grep -E "passed|failed|Error|assert" gpurun_out/pmpc_tests.log | head -30
bash tools/ab_soft_only.sh
