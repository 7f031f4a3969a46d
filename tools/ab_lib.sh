#!/bin/bash
# A/B timing of two in-tree builds of libdartmpc on the GPU box (bench main line + supplementary lines).
# Usage: bash tools/ab_lib.sh "<lib file names, space separated>" [reps] [extra bench args]
set -o pipefail
LIBS=${1:-"libdartmpc_base.so libdartmpc.so"}
REPS=${2:-3}
EXTRA=${3:-"--rmpc-steps 0 --lmpc-steps 0 --arm-steps 0"}
mkdir -p gpurun_out
ARGS="--steps 2000 --warmup 50 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --lmpc-policy-steps 0 $EXTRA"
for r in $(seq 1 $REPS); do
  for lib in $LIBS; do
    DART_MPC_AB=1 DART_MPC_LIB=$lib timeout -k 10 180 python bench.py $ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
    python - "$lib" <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab.json"))
out = [sys.argv[1], "C2", round(d["value"]), round(d["roofline"]["kernel_ms"] * 1e3, 2), "us"]
if d.get("saturation"):
    out += ["sat", round(d["saturation"]["solves_per_s"] / 1e6, 2), "M"]
for k in ("rmpc_c3", "lmpc_c5", "arm_qp", "pmpc_n15"):
    if d.get(k):
        out += [k, round(d[k]["solves_per_s"]), round(d[k].get("kernel_ms", d[k]["ms_per_step"]) * 1e3, 1), "us"]
l = d.get("lmpc_c5") or {}
if l.get("restoration_off"):
    out += ["c5_resto_off", round(l["restoration_off"]["solves_per_s"])]
if l.get("policy_fused"):
    out += ["c5_fused", round(l["policy_fused"]["solves_per_s"])]
print(*out)
PY
  done
done
