# Scan (one wave per SIMD) against sequential (two per SIMD) PMPC builds over batch sizes: the
# launcher's DART_PMPC_QSCAN_MAX_B knob, saturation line of bench.py.  Usage: bash tools/c4_ab.sh
set -o pipefail
mkdir -p gpurun_out
A="--steps 20 --warmup 5 --no-cpu-baseline --host-calls 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --c4-steps 0"
for b in ${BATCHES:-1152 2048 3072 4096 6144 8192 18432}; do
for q in 1024 1000000; do
  DART_PMPC_QSCAN_MAX_B=$q timeout -k 10 120 python bench.py $A --saturation-batch $b > gpurun_out/sat.json 2>gpurun_out/sat.err || exit 1
  python -c "
import json; l=[x for x in open('gpurun_out/sat.json') if x.startswith('{')][-1]; d=json.loads(l)['saturation']
print('B', $b, 'qscan_max', $q, round(d['solves_per_s']), round(d.get('ms_per_launch', 0) * 1e3, 1), 'us')"
done
done
