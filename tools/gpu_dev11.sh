# round 5: LMPC tests (incl. the inertia blow-ups now taken through the explicit value function), C5 and C3 A/B
# against the round's first build, then the round-end profile passes again (restoration / long-horizon lines out)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lmpc.py -v --timeout 300 --timeout-method thread > gpurun_out/lmpc_tests.log 2>&1; rc=$?
echo "lmpc tests rc $rc"; grep -E "FAILED|passed|failed" gpurun_out/lmpc_tests.log | tail -20
[ $rc -eq 0 ] || { grep -B2 -A30 "^____" gpurun_out/lmpc_tests.log | grep -E "^E |assert" | head -40; exit 1; }
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 600 --lmpc-steps 300 --lmpc-policy-steps 200 --arm-steps 0 --resto-steps 0 --long-steps 0"
for r in 1 2 3; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    DART_MPC_LIB=$lib timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab.json')); r=d['rmpc_c3']; l=d['lmpc_c5']
print('$lib', 'C3', round(r['solves_per_s']), round(r['kernel_ms']*1e3,2), 'us  C5', round(l['solves_per_s']), 'off', round(l['restoration_off']['solves_per_s']), 'fused', round(l['policy_fused']['solves_per_s']), flush=True)"
  done
done
bash tools/profile_round.sh r05 && bash tools/pmc_sq.sh r05 && echo PROF_OK
