# Multi-rank rehearsal of bench.py on a one-GPU box: 2 ranks over gloo, both on the card present
# (RCCL refuses two ranks on one device).  Exercises rank seeding, max-over-ranks timing and the C4
# gather + rank-consistency check; the throughput it prints is not a scaling number.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo --no-cpu-baseline \
    --saturation-batch 0 --host-calls 0 --n15-steps 0 --rmpc-steps 0 --lmpc-steps 0 --arm-steps 0 \
    > gpurun_out/ranks2.json 2> gpurun_out/ranks2.err || { echo REHEARSAL_FAILED; tail -30 gpurun_out/ranks2.err; exit 1; }
cat gpurun_out/ranks2.json
