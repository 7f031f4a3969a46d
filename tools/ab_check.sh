#!/bin/bash
# PMPC parity tests on each candidate build, then tools/ab_lib.sh over all of them (C2 + N=15 lines).
# Usage: bash tools/ab_check.sh "<lib file names>" [reps]
set -o pipefail
LIBS=${1:?libs}
REPS=${2:-3}
mkdir -p gpurun_out
for lib in $LIBS; do
  DART_MPC_AB=1 DART_MPC_LIB=$lib timeout -k 10 240 python -u -m pytest tests/test_gpu_pmpc.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/ab_tests_$lib.log 2>&1 || { echo "TESTS_FAILED $lib"; tail -30 gpurun_out/ab_tests_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab_tests_$lib.log)"
done
bash tools/ab_lib.sh "$LIBS" $REPS "--rmpc-steps 0 --lmpc-steps 0 --arm-steps 0 --n15-steps 2000"
