#!/bin/bash
# Parity tests of every variant on each candidate build (PMPC, RMPC, LMPC), then tools/ab_lib.sh over
# all of them with the C2, C3 and C5 lines.  Usage: bash tools/ab_check_all.sh "<lib file names>" [reps]
set -o pipefail
LIBS=${1:?libs}
REPS=${2:-3}
mkdir -p gpurun_out
for lib in $LIBS; do
  DART_MPC_AB=1 DART_MPC_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_pmpc.py tests/test_gpu_rmpc.py tests/test_gpu_lmpc.py \
    -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/ab_tests_$lib.log 2>&1 || { echo "TESTS_FAILED $lib"; tail -30 gpurun_out/ab_tests_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab_tests_$lib.log)"
done
bash tools/ab_lib.sh "$LIBS" $REPS "${EXTRA:---arm-steps 0 --rmpc-steps 1000 --lmpc-steps 300 --lmpc-policy-steps 300}"
