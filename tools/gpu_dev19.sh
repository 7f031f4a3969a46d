# Two-wave builds with the wave-local filter test: A/B identity against the one-wave kernels, speed, tests, timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/wg2_ab.py > gpurun_out/wg2_ab4.txt 2>&1; rc=$?
tail -8 gpurun_out/wg2_ab4.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/wg2_speed.py > gpurun_out/wg2_speed4.txt 2>&1; rc=$?
cat gpurun_out/wg2_speed4.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/long_diag.py 40 > gpurun_out/long_diag4.txt 2>&1; rc=$?
cat gpurun_out/long_diag4.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmpc.py tests/test_gpu_lmpc.py tests/test_gpu_pmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/wg2_tests4.log 2>&1; rc=$?
tail -4 gpurun_out/wg2_tests4.log; [ $rc -eq 0 ] || exit 1
echo DEV19_OK
