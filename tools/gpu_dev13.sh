# Two-wave builds with one barrier per cross-wave exchange: A/B identity, speed, the RMPC/LMPC GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/wg2_ab.py > gpurun_out/wg2_ab.txt 2>&1; rc=$?
tail -8 gpurun_out/wg2_ab.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/wg2_speed.py > gpurun_out/wg2_speed.txt 2>&1; rc=$?
cat gpurun_out/wg2_speed.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmpc.py tests/test_gpu_lmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/wg2_tests.log 2>&1; rc=$?
tail -4 gpurun_out/wg2_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/long_diag.py 40 > gpurun_out/long_diag.txt 2>&1; rc=$?
cat gpurun_out/long_diag.txt; [ $rc -eq 0 ] || exit 1
echo DEV13_OK
