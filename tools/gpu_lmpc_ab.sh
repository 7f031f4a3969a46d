# A/B of two library builds on the LMPC workloads (C5 stress batches, bit-for-bit check), then the LMPC GPU tests
set -o pipefail
LIBS=${1:-"libdartmpc_head9.so libdartmpc.so"}
bash tools/ab_variant.sh lmpc "$LIBS" 3 300 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_lmpc.py tests/test_gpu_policy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lmpc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lmpc_tests.log; exit $rc
