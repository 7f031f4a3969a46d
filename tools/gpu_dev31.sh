# LMPC main sweep (restoration instantiation) stops at the first failed inertia test: LMPC tests, one-/two-wave identity, C5 stress A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lmpc.py tests/test_gpu_policy.py -q --timeout 300 --timeout-method thread > gpurun_out/lm_early_tests2.log 2>&1; rc=$?
tail -2 gpurun_out/lm_early_tests2.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/wg2_ab.py > gpurun_out/wg2_ab8.txt 2>&1; rc=$?
grep -c True gpurun_out/wg2_ab8.txt; grep False gpurun_out/wg2_ab7.txt; [ $rc -eq 0 ] || exit 1
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 300 --lmpc-policy-steps 0 --arm-steps 0 --resto-steps 0 --long-steps 0"
for r in 1 2 3; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    DART_MPC_LIB=$lib timeout -k 10 300 python bench.py $ARGS > gpurun_out/lm_ab.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/lm_ab.json'))['lmpc_c5']
print('$lib', 'C5 stress', round(d['solves_per_s']), 'off', round(d['restoration_off']['solves_per_s']) if isinstance(d.get('restoration_off'),dict) else d.get('restoration_off'), flush=True)"
  done
done
echo DEV31_DONE
