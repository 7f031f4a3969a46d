#!/bin/bash
# N <= 15 large batches: the one-row build at one wave per SIMD against the short-scan build at two waves
# (DART_PMPC_OCC2_N15).  Usage (on the box): DART_MPC_LIB=<lib> bash tools/occ2_n15.sh [reps]
set -o pipefail
REPS=${1:-2}
mkdir -p gpurun_out
DART_PMPC_OCC2_N15=1 DART_PMPC_OCC2_MIN_B=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_pmpc.py -m gpu -x -q \
    --timeout 180 --timeout-method thread -k "horizons or scan_and_sequential or c2_and_c4 or same_path" > gpurun_out/n15_tests.log 2>&1 \
    || { echo TESTS_FAILED; tail -30 gpurun_out/n15_tests.log; exit 1; }
echo "n15 occ2 parity: $(tail -1 gpurun_out/n15_tests.log)"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --host-calls 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --c4-steps 0 --N 15"
for r in $(seq 1 $REPS); do
  for sb in 2048 18432; do
    for v in off on; do
      if [ $v = on ]; then export DART_PMPC_OCC2_N15=1; else unset DART_PMPC_OCC2_N15; fi
      timeout -k 10 120 python bench.py $ARGS --saturation-batch $sb > gpurun_out/n15.json 2>gpurun_out/n15.err || exit $?
      python -c "import json; d=json.load(open('gpurun_out/n15.json')); print('N 15 B', $sb, 'short-scan two-wave', '$v', round(d['saturation']['solves_per_s']/1e6, 2), 'M')"
    done
  done
done
