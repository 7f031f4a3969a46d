# C3 A/B of the queued RMPC restoration grid (B blocks) against the round's committed library before it, then the
# round-end profile passes again (restoration and long-horizon lines left out of the profiled runs)
set -o pipefail
mkdir -p gpurun_out
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 1000 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --resto-steps 0 --long-steps 0"
for r in 1 2 3; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    DART_MPC_LIB=$lib timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab.json'))['rmpc_c3']
print('$lib', 'C3', round(d['solves_per_s']), round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['kernel_ms']*1e3,2), flush=True)"
  done
done
bash tools/profile_round.sh r05 && bash tools/pmc_sq.sh r05 && echo PROF_OK
