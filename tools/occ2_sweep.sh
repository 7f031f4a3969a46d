#!/bin/bash
# Crossover of the two-waves-per-SIMD PMPC scan instantiation over the batch size (saturation line of bench.py).
# Usage (on the box): bash tools/occ2_sweep.sh "<batch sizes>" [reps] [N]
set -o pipefail
BS=${1:-"1536 2048 2560 3072"}
REPS=${2:-2}
HN=${3:-20}
mkdir -p gpurun_out
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --host-calls 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --c4-steps 0 --N $HN"
for r in $(seq 1 $REPS); do
  for sb in $BS; do
    for th in off 1; do
      if [ $th = off ]; then export DART_PMPC_OCC2_MIN_B=1000000000; else export DART_PMPC_OCC2_MIN_B=$th; fi
      timeout -k 10 120 python bench.py $ARGS --saturation-batch $sb > gpurun_out/occ2.json 2>gpurun_out/occ2.err || exit $?
      python -c "import json,sys; d=json.load(open('gpurun_out/occ2.json')); print('N', $HN, 'B', $sb, 'occ2', '$th', round(d['saturation']['solves_per_s']/1e6, 2), 'M')"
    done
  done
done
