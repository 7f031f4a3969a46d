# round 5: every GPU test (incl. the two-wave RMPC / LMPC builds for N = 32..63), then the long-horizon bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc $rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/gpu_tests.log | tail -30
[ $rc -eq 0 ] || { grep -B5 -A40 "^____" gpurun_out/gpu_tests.log | head -150; exit 1; }
L="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --resto-steps 0 --long-steps 20"
timeout -k 10 300 python -u bench.py $L > gpurun_out/long.json 2> gpurun_out/long.err || { echo LONG_FAILED; tail -20 gpurun_out/long.err; exit 1; }
python -c "import json;print(json.dumps(json.load(open('gpurun_out/long.json'))['long_horizons'], indent=1))"
