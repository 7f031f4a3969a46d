# PMPC horizons 20..63: per-call time of the two-wave scan build against the one-wave sequential build; GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pmpc_long_speed.py > gpurun_out/pm_long_speed.txt 2>&1; rc=$?
cat gpurun_out/pm_long_speed.txt; [ $rc -eq 0 ] || exit 1
DART_PMPC_SEQ_LONG=1 timeout -k 10 300 python -u tools/pmpc_long_speed.py > gpurun_out/pm_long_speed_seq.txt 2>&1; rc=$?
cat gpurun_out/pm_long_speed_seq.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/pm_long_tests.log 2>&1; rc=$?
tail -4 gpurun_out/pm_long_tests.log
echo DEV15_DONE
