set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['host_inclusive_8d']['value'])"
