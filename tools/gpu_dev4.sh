# round 5: full GPU tests, the soft-phase A/B and restoration lines, then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "tests rc $?"
grep -E "passed|failed|Error|assert" gpurun_out/gpu_tests.log | head -30
bash tools/ab_soft_only.sh || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('C2', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms'], 'C3', round(d['rmpc_c3']['solves_per_s']), 'C5', round(d['lmpc_c5']['solves_per_s']), round(d['lmpc_c5']['policy_fused']['solves_per_s']), 'C4', round(d['pmpc_c4']['solves_per_s']), 'sat', round(d['saturation']['solves_per_s']))"
