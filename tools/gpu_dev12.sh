# RMPC: restoration inlined behind the solve (DART_RMPC_INLINE_RESTO=1) against the queued kernel -- tests and C3 A/B
set -o pipefail
mkdir -p gpurun_out
DART_RMPC_INLINE_RESTO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_rmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/rmpc_inl.log 2>&1; rc=$?
echo "rmpc tests (inline) rc $rc"; tail -3 gpurun_out/rmpc_inl.log
[ $rc -eq 0 ] || exit 1
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 1000 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --resto-steps 0 --long-steps 0"
for r in 1 2 3; do
  for inl in 0 1; do
    DART_RMPC_INLINE_RESTO=$inl timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab.json'))['rmpc_c3']
print('inline=$inl', 'C3', round(d['solves_per_s']), round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['kernel_ms']*1e3,2), flush=True)"
  done
done
