#!/bin/bash
# A/B of the round-4 library (queued restoration kernels), the current one (restoration in the solving wave for
# B <= 32) and the current one with DART_RESTO_FUSE=0 (the queued form again).  Usage: bash tools/ab_fuse.sh [reps]
set -o pipefail
REPS=${1:-2}
mkdir -p gpurun_out
ARGS="--steps 1000 --warmup 50 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --resto-steps 0 --lmpc-policy-steps 50 --arm-steps 0 --rmpc-steps 300 --lmpc-steps 200"
for r in $(seq 1 $REPS); do
  for v in r04 cur nofuse; do
    case $v in
      r04) L=libdartmpc_r04.so; F=1 ;;
      cur) L=libdartmpc.so; F=1 ;;
      nofuse) L=libdartmpc.so; F=0 ;;
    esac
    DART_MPC_LIB=$L DART_RESTO_FUSE=$F timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python - "$v" <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab.json"))
l = d["lmpc_c5"]
print(sys.argv[1], "C2", round(d["value"]), round(d["roofline"]["kernel_ms"] * 1e3, 2), "us  C3", round(d["rmpc_c3"]["solves_per_s"]),
      round(d["rmpc_c3"]["kernel_ms"] * 1e3, 1), "us  C5", round(l["solves_per_s"]), "off", round(l["restoration_off"]["solves_per_s"]),
      "fused", round(l["policy_fused"]["solves_per_s"]), flush=True)
PY
  done
done
