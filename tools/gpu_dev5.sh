# round 5: RMPC tests (incl. the two-wave N = 32..63 build), then C3 A/B of the committed library against the new one
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmpc.py -x -v --timeout 300 --timeout-method thread > gpurun_out/rmpc_tests.log 2>&1; rc=$?
echo "rmpc tests rc $rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/rmpc_tests.log | tail -40
[ $rc -eq 0 ] || exit 1
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 1000 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --resto-steps 0"
for r in 1 2 3; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    DART_MPC_LIB=$lib timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab.json'))['rmpc_c3']
print('$lib', 'C3', round(d['solves_per_s']), round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['kernel_ms']*1e3,2), flush=True)"
  done
done
