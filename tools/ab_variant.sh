#!/bin/bash
# A/B of in-tree library builds on one variant: alternating reps of tools/ab_variant.py, then a bit-for-bit check
# of every build's outputs against the first.  Usage: bash tools/ab_variant.sh <kind> "<libs>" [reps] [launches]
set -o pipefail
KIND=$1; LIBS=$2; REPS=${3:-3}; K=${4:-2000}
mkdir -p gpurun_out/ab
for r in $(seq 1 $REPS); do
  for lib in $LIBS; do
    DART_MPC_AB=1 DART_MPC_LIB=$lib timeout -k 10 200 python -u tools/ab_variant.py $KIND $K gpurun_out/ab/$KIND.$lib.npz 2>/dev/null || exit 1
  done
done
first=$(echo $LIBS | cut -d' ' -f1)
for lib in $LIBS; do
  [ $lib = $first ] || python tools/ab_compare.py gpurun_out/ab/$KIND.$first.npz gpurun_out/ab/$KIND.$lib.npz || exit 1
done
