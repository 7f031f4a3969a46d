# soft-row roles per sweep (aug_soften): RMPC restoration tests + A/B identity, infeasible-start timing A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmpc.py tests/test_gpu_pmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/soften_tests.log 2>&1; rc=$?
tail -3 gpurun_out/soften_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/wg2_ab.py > gpurun_out/wg2_ab5.txt 2>&1; rc=$?
grep -c True gpurun_out/wg2_ab5.txt; grep False gpurun_out/wg2_ab5.txt; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    echo "== $lib"
    DART_MPC_LIB=$lib timeout -k 10 200 python -u tools/rmpc_infeasible_diag.py 20 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
  done
done
echo DEV25_DONE
