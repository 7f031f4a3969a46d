# A/B of two library builds on C2 (PMPC), C3 (RMPC) and the infeasible start (bit-for-bit check), then their GPU tests
set -o pipefail
LIBS=${1:-"libdartmpc_head12.so libdartmpc.so"}
bash tools/ab_variant.sh pmpc "$LIBS" 4 2000 && bash tools/ab_variant.sh rmpc "$LIBS" 3 1000 && \
bash tools/ab_variant.sh rmpc_inf "$LIBS" 2 100 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_pmpc.py tests/test_gpu_rmpc.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ls_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ls_tests.log; exit $rc
