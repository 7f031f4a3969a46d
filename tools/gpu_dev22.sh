# PMPC restoration restart with exact-arithmetic speedups (node-step roles per sweep, pow terms per iteration, paired
# barrier sums): exactness sweep against the oracle, stamps of the N = 31 instance, bench restoration line A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pmpc_resto_sweep.py > gpurun_out/pr_sweep2.txt 2>&1; rc=$?
cat gpurun_out/pr_sweep2.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/stamps_pmpc_resto.py > gpurun_out/stamps_pr31c.txt 2>&1; rc=$?
head -22 gpurun_out/stamps_pr31c.txt; [ $rc -eq 0 ] || exit 1
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --long-steps 0 --resto-steps 20"
for r in 1 2; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    DART_MPC_LIB=$lib timeout -k 10 240 python bench.py $ARGS > gpurun_out/pr_ab.json 2>gpurun_out/pr_ab.err || { tail -5 gpurun_out/pr_ab.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/pr_ab.json'))['pmpc_restoration']
print('$lib', json.dumps(d)[:400], flush=True)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_pmpc.py -q --timeout 300 --timeout-method thread > gpurun_out/pr_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pr_tests.log
echo DEV22_DONE
