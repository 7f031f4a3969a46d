# A/B of two library builds on every LDS-engine workload (bit-for-bit), then the RMPC / PMPC / LMPC tests
set -o pipefail
LIBS=${1:-"libdartmpc_head12.so libdartmpc.so"}
bash tools/ab_variant.sh rmpc "$LIBS" 3 1000 && bash tools/ab_variant.sh rmpc_inf "$LIBS" 2 100 && \
bash tools/ab_variant.sh pmpc_resto "$LIBS" 2 20 && bash tools/ab_variant.sh lmpc "$LIBS" 3 300 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_rmpc.py tests/test_gpu_pmpc.py tests/test_gpu_lmpc.py tests/test_gpu_policy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sync_tests.log 2>&1; rc=$?; tail -2 gpurun_out/sync_tests.log; exit $rc
