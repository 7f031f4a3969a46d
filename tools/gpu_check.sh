# GPU check used during development: GPU tests, then a short bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
