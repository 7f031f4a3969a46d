# round 5: GPU tests, PMPC restoration stamps, restoration bench lines with and without resume, the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u tools/stamps_pmpc_resto.py > gpurun_out/stamps_pr31.log 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/stamps_pr31.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_pr31.log
DART_STAMPS_N=20 DART_STAMPS_SOC=0 timeout -k 10 200 python -u tools/stamps_pmpc_resto.py > gpurun_out/stamps_pr20.log 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/stamps_pr20.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_pr20.log
R="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --arm-steps 0 --resto-steps 10"
for v in 0 1; do
  DART_PMPC_RESUME=$v timeout -k 10 300 python -u bench.py $R > gpurun_out/resto_$v.json 2> gpurun_out/resto_$v.err || { echo RESTO_BENCH_FAILED; tail -20 gpurun_out/resto_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/resto_$v.json'))['pmpc_restoration']
for k in ('c4_n31_default','c4_n20_max_soc0'):
    l=d[k]; print('resume=$v', k, 'restored', l['restored'], 'ms', round(l['ms_per_launch'],3), 'off', round(l['ms_per_launch_restoration_off'],3), 'b18', round(l.get('b18_one_restored_ms',0),3), 'iters', round(l['restored_iters_mean'],2), 'eq', l['restored_status_equal_to_oracle'], 'du', l['restored_max_abs_u0_err_vs_oracle'])"
done
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('C2', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms'], 'C3', round(d['rmpc_c3']['solves_per_s']), 'C5', round(d['lmpc_c5']['solves_per_s']), round(d['lmpc_c5']['policy_fused']['solves_per_s']), 'C4', round(d['pmpc_c4']['solves_per_s']), 'sat', round(d['saturation']['solves_per_s']))"
