# PMPC two-wave build: one-barrier hand-overs, local filter ballot, merged line-search reductions: same-path check, per-N timing, the PMPC GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pmpc_long_check.py > gpurun_out/pm_long_check3.txt 2>&1; rc=$?
cat gpurun_out/pm_long_check3.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/pmpc_long_speed.py > gpurun_out/pm_long_speed3.txt 2>&1; rc=$?
cat gpurun_out/pm_long_speed3.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/pm_long_tests3.log 2>&1; rc=$?
tail -4 gpurun_out/pm_long_tests3.log
echo DEV18_DONE
