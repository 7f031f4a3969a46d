#!/bin/bash
set -o pipefail
ARGS="--steps 2000 --warmup 50 --no-cpu-baseline --saturation-batch 18432 --host-calls 0 --c4-steps 100 --n15-steps 1000 --rmpc-steps 0 --lmpc-steps 0 --lmpc-policy-steps 0 --arm-steps 0 --resto-steps 0"
for r in 1 2 3; do
  for lib in libdartmpc_head.so libdartmpc.so; do
    DART_MPC_LIB=$lib timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab.json'))
print('$lib', 'C2', round(d['value']), round(d['roofline']['kernel_ms']*1e3,2), 'us  N15', round(d['pmpc_n15']['solves_per_s']), ' C4', round(d['pmpc_c4']['solves_per_s']), ' sat', round(d['saturation']['solves_per_s']), flush=True)"
  done
done
R="--steps 20 --warmup 5 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --arm-steps 0 --resto-steps 10"
timeout -k 10 300 python -u bench.py $R > gpurun_out/resto.json 2> gpurun_out/resto.err || { echo RESTO_BENCH_FAILED; tail -20 gpurun_out/resto.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/resto.json'))['pmpc_restoration']
for k in ('c4_n31_default','c4_n20_max_soc0'):
    l=d[k]; print(k, 'restored', l['restored'], 'ms', round(l['ms_per_launch'],3), 'off', round(l['ms_per_launch_restoration_off'],3), 'b18', round(l.get('b18_one_restored_ms',0),3), 'b18 off', round(l.get('b18_restoration_off_ms',0),3), 'iters', round(l['restored_iters_mean'],2), 'eq', l['restored_status_equal_to_oracle'], 'du', l['restored_max_abs_u0_err_vs_oracle'])"
