#!/bin/bash
# A/B of the host-pointer (PCIe-inclusive) PMPC path of two in-tree builds.
# Usage: bash tools/ab_host.sh "<lib file names>" [reps]
set -o pipefail
LIBS=${1:-"libdartmpc_base.so libdartmpc.so"}
REPS=${2:-2}
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  for lib in $LIBS; do
    DART_MPC_AB=1 DART_MPC_LIB=$lib timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 \
        --host-calls 1000 --c4-steps 0 --rmpc-steps 0 --lmpc-steps 0 --arm-steps 0 > gpurun_out/abh.json 2>gpurun_out/abh.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/abh.json'))['host_path_pcie_inclusive']; print(sys.argv[1], round(d['ms_per_call']*1e3,1), 'us/call B=18,', round(d['single_instance_ms_per_call']*1e3,1), 'us/call B=1')" $lib
  done
done
