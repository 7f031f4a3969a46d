# Multi-rank rehearsal of bench.py on a one-GPU box: bench.py --gpus 2 starts its two rank processes itself
# (no torchrun), gloo, both ranks on the card present (RCCL refuses two ranks on one device).  Exercises the
# launcher, rank seeding, max-over-ranks timing and the C4 gather + rank-consistency check; the throughput
# it prints is not a scaling number.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo --no-cpu-baseline \
    --saturation-batch 0 --host-calls 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --arm-steps 0 \
    > gpurun_out/ranks2.json 2> gpurun_out/ranks2.err || { echo REHEARSAL_FAILED; tail -30 gpurun_out/ranks2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ranks2.json')); print('ranks', d['n_gpus'], 'value', round(d['value']), 'c4 consistent', d['pmpc_c4']['rank_blocks_consistent'], d['pmpc_c4']['n_gpus'])"
