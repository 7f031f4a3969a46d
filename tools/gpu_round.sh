# Round-end measurement set (GPU box): tests, bench line, rocprofv3 trace + HBM passes, SQ counters,
# phase stamps.  Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
bash tools/profile_round.sh $TAG && bash tools/pmc_sq.sh $TAG && bash tools/stamps_all.sh $TAG && echo ROUND_OK
