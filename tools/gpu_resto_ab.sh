# A/B of two library builds on the PMPC workloads (C4 restoration launches, C2; bit-for-bit check), then the PMPC GPU tests
set -o pipefail
LIBS=${1:-"libdartmpc_head9.so libdartmpc.so"}
bash tools/ab_variant.sh pmpc_resto "$LIBS" 3 20 && bash tools/ab_variant.sh pmpc_soc0 "$LIBS" 2 10 && \
bash tools/ab_variant.sh pmpc "$LIBS" 3 2000 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_pmpc.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/resto_tests.log 2>&1; rc=$?; tail -3 gpurun_out/resto_tests.log; exit $rc
