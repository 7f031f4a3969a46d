# diagnostic: C5 launches with every instance handed to the resume kernel at iteration 0 (libdartmpc_force.so)
# against the normal build: the resume kernel's regular-iteration speed
set -o pipefail
for lib in libdartmpc.so libdartmpc_force.so libdartmpc.so libdartmpc_force.so; do
  DART_MPC_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --arm-steps 0 --lmpc-steps 100 --lmpc-policy-steps 100 > gpurun_out/rs.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/rs.json'))['lmpc_c5']; print(sys.argv[1], 'resto_off', round(d['restoration_off']['solves_per_s']), 'fused', round(d['policy_fused']['solves_per_s']), 'c5', round(d['solves_per_s']))" $lib
done
