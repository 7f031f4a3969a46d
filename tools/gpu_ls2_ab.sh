# A/B of two library builds on C3, the infeasible start and the PMPC restoration launches (bit-for-bit), then the tests
set -o pipefail
LIBS=${1:-"libdartmpc_head10.so libdartmpc.so"}
bash tools/ab_variant.sh rmpc "$LIBS" 3 1000 && bash tools/ab_variant.sh rmpc_inf "$LIBS" 2 100 && \
bash tools/ab_variant.sh pmpc_resto "$LIBS" 2 20 && bash tools/ab_variant.sh pmpc_soc0 "$LIBS" 1 10 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_pmpc.py tests/test_gpu_rmpc.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ls_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ls_tests.log; exit $rc
