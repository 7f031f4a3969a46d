# restoration sweeps stop at the first failed inertia test: exactness, stamps, timing A/B against HEAD's build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pmpc_resto_sweep.py > gpurun_out/pr_sweep3.txt 2>&1; rc=$?
grep -E "restored |N=" gpurun_out/pr_sweep3.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmpc.py tests/test_gpu_pmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/early_tests.log 2>&1; rc=$?
tail -2 gpurun_out/early_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/wg2_ab.py > gpurun_out/wg2_ab6.txt 2>&1; rc=$?
grep -c True gpurun_out/wg2_ab6.txt; grep False gpurun_out/wg2_ab6.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/stamps_pmpc_resto.py > gpurun_out/stamps_pr31d.txt 2>&1; rc=$?
head -6 gpurun_out/stamps_pr31d.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/stamps_rmpc_resto.py > gpurun_out/stamps_rmpc_resto2.txt 2>&1; rc=$?
cat gpurun_out/stamps_rmpc_resto2.txt; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    echo "== $lib"
    DART_MPC_LIB=$lib timeout -k 10 200 python -u tools/rmpc_infeasible_diag.py 20 2>&1 | grep "restoration on" || exit 1
    DART_MPC_LIB=$lib timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --long-steps 0 --resto-steps 20 > gpurun_out/pr_ab2.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/pr_ab2.json'))['pmpc_restoration']; print('pmpc resto ms', round(d['c4_n31_default']['ms_per_launch'],3), round(d['c4_n20_max_soc0']['ms_per_launch'],2))"
  done
done
echo DEV29_DONE
