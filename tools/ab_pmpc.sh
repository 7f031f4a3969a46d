#!/bin/bash
# A/B of the PMPC latency variant on the GPU box: bench main line only, alternating knob settings.
# Usage: bash tools/ab_pmpc.sh "<env A>" "<env B>" [reps]
set -o pipefail
A=${1:-"DART_PMPC_QSCAN_MAX_B=1024"}
B=${2:-"DART_PMPC_QSCAN_MAX_B=0"}
REPS=${3:-3}
mkdir -p gpurun_out
ARGS="--steps 2000 --warmup 50 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --rmpc-steps 0 --lmpc-steps 0 --arm-steps 0"
for r in $(seq 1 $REPS); do
  for cfg in "$A" "$B"; do
    env $cfg timeout -k 10 120 python bench.py $ARGS > gpurun_out/ab.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], round(d['value']), round(d['roofline']['kernel_ms']*1e3,2), 'us')" "$cfg"
  done
done
