# A/B of two library builds on the RMPC workloads (C3, infeasible start; bit-for-bit check), then the RMPC GPU tests
set -o pipefail
LIBS=${1:-"libdartmpc_head9.so libdartmpc.so"}
bash tools/ab_variant.sh rmpc_inf "$LIBS" 3 100 && bash tools/ab_variant.sh rmpc "$LIBS" 2 1000 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmpc.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rmpc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/rmpc_tests.log; exit $rc
