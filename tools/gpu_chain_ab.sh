# A/B of two library builds over every LDS-engine workload (bit-for-bit check per workload), then the variant GPU tests
set -o pipefail
LIBS=${1:-"libdartmpc_head7.so libdartmpc.so"}
bash tools/ab_variant.sh rmpc "$LIBS" 2 1000 && bash tools/ab_variant.sh rmpc_inf "$LIBS" 2 100 && \
bash tools/ab_variant.sh lmpc "$LIBS" 2 500 && bash tools/ab_variant.sh pmpc_resto "$LIBS" 2 20 && \
bash tools/ab_variant.sh pmpc_soc0 "$LIBS" 1 10 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_rmpc.py tests/test_gpu_lmpc.py tests/test_gpu_pmpc.py tests/test_gpu_policy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/variant_tests.log 2>&1; rc=$?; tail -3 gpurun_out/variant_tests.log; exit $rc
