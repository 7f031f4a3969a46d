# Round-6 GPU check: every GPU test, then the bench line (stops at the first failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
echo BENCH_OK
