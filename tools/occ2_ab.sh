#!/bin/bash
# A/B of the two-waves-per-SIMD PMPC scan instantiation (DART_PMPC_OCC2_MIN_B: batches of at least that many
# N <= 23 instances use it).  Parity first with every N <= 23 batch on it, then saturated / C4 lines alternated.
# Usage (on the box): bash tools/occ2_ab.sh [reps]
set -o pipefail
REPS=${1:-3}
mkdir -p gpurun_out
DART_PMPC_OCC2_MIN_B=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_pmpc.py -m gpu -x -q --timeout 180 \
    --timeout-method thread > gpurun_out/occ2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/occ2_tests.log; exit 1; }
echo "occ2 parity: $(tail -1 gpurun_out/occ2_tests.log)"
ARGS="--steps 200 --warmup 20 --no-cpu-baseline --host-calls 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --c4-steps 50"
for r in $(seq 1 $REPS); do
  for th in off 1024; do
    for sb in 4096 18432; do
      if [ $th = off ]; then export DART_PMPC_OCC2_MIN_B=1000000000; else export DART_PMPC_OCC2_MIN_B=$th; fi
      timeout -k 10 180 python bench.py $ARGS --saturation-batch $sb > gpurun_out/occ2.json 2>gpurun_out/occ2.err || exit $?
      python - "$th" "$sb" <<'PY'
import json, sys
d = json.load(open("gpurun_out/occ2.json"))
print("occ2", sys.argv[1], "sat", sys.argv[2], round(d["saturation"]["solves_per_s"] / 1e6, 2), "M",
      "C4", round(d["pmpc_c4"]["solves_per_s_without_gather"] / 1e6, 2), "M", "C2", round(d["value"]))
PY
    done
  done
done
