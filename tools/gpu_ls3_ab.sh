# A/B of two library builds on C5 stress, C3 and the infeasible start (bit-for-bit), then the LMPC / RMPC tests
set -o pipefail
LIBS=${1:-"libdartmpc_head10.so libdartmpc.so"}
bash tools/ab_variant.sh lmpc "$LIBS" 3 300 && bash tools/ab_variant.sh rmpc_inf "$LIBS" 2 100 && \
bash tools/ab_variant.sh rmpc "$LIBS" 2 1000 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_lmpc.py tests/test_gpu_policy.py tests/test_gpu_rmpc.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ls_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ls_tests.log; exit $rc
