# LMPC-focused GPU check: the LMPC / policy GPU tests, then the C5 bench lines only.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lmpc.py tests/test_gpu_policy.py tests/test_gpu_lmpc_shm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_lmpc_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_lmpc_tests.log; exit 1; }
tail -3 gpurun_out/gpu_lmpc_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --arm-steps 0 > gpurun_out/bench_lmpc.json 2> gpurun_out/bench_lmpc.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_lmpc.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_lmpc.json')); l=d['lmpc_c5']
print('C5', {k: l[k] for k in l if not isinstance(l[k], dict)})
print('fused', {k: v for k, v in l.get('policy_fused', {}).items() if not isinstance(v, dict)})"
