# Development GPU check (round 5): GPU tests, the bench line, bench.py --gpus 2 rehearsal, the RMPC status-2 dump.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('C2', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms'], 'C3', round(d['rmpc_c3']['solves_per_s']), 'C5', round(d['lmpc_c5']['solves_per_s']), round(d['lmpc_c5']['policy_fused']['solves_per_s']), 'C4', round(d['pmpc_c4']['solves_per_s']))"
bash tools/rehearse_ranks.sh || exit 1
timeout -k 10 300 python -u tools/rmpc_dump_status2.py > gpurun_out/rmpc_dump.log 2>&1 || { echo DUMP_FAILED; tail -20 gpurun_out/rmpc_dump.log; exit 1; }
cat gpurun_out/rmpc_dump.log
