# round 5 final set: every GPU test, smoke, bench line, the full parity sweep (C2/C4 115,200, C3 28,800, C5 stress
# 28,800, RMPC restoration, PMPC restoration, horizons 40 / 63)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc $rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('C2', round(d['value']), d['ms_per_step'], 'C3', round(d['rmpc_c3']['solves_per_s']), 'C5', round(d['lmpc_c5']['solves_per_s']), round(d['lmpc_c5']['policy_fused']['solves_per_s']), 'C4', round(d['pmpc_c4']['solves_per_s']), 'sat', round(d['saturation']['solves_per_s']))"
timeout -k 10 900 python -u tools/parity_sweep.py 6400 1600 1600 80 > gpurun_out/parity_sweep_r05.txt 2>&1 || { echo SWEEP_FAILED; tail -20 gpurun_out/parity_sweep_r05.txt; exit 1; }
tail -45 gpurun_out/parity_sweep_r05.txt
