# PMPC N = 32..63 on the two-wave scan build: same-path check against the oracle (both builds), timing, GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pmpc_long_check.py > gpurun_out/pm_long_check.txt 2>&1; rc=$?
cat gpurun_out/pm_long_check.txt; [ $rc -eq 0 ] || exit 1
DART_PMPC_SEQ_LONG=1 timeout -k 10 300 python -u tools/pmpc_long_check.py > gpurun_out/pm_long_check_seq.txt 2>&1; rc=$?
cat gpurun_out/pm_long_check_seq.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/long_diag.py 40 > gpurun_out/long_diag_wg2.txt 2>&1; rc=$?
cat gpurun_out/long_diag_wg2.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/pm_long_tests.log 2>&1; rc=$?
tail -8 gpurun_out/pm_long_tests.log
echo DEV14_DONE
