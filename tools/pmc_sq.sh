#!/bin/bash
# SQ instruction / cycle counters of the bench kernels (one rocprofv3 --pmc pass, <= 8 SQ counters).
# Usage (on the box): bash tools/pmc_sq.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/sq_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM \
    --kernel-trace -d $OUT -o run --output-format csv -- \
    python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 \
    --rmpc-steps 30 --lmpc-steps 30 --lmpc-policy-steps 0 --arm-steps 30 --resto-steps 0 --long-steps 0 > $OUT/bench.json 2> $OUT/err.log || exit $?
# second pass: the matrix-core busy counter (SURVEY 7.8 asks for MFMA-busy even when it is 0: every kernel here
# is FP64 VALU work, no MFMA instruction is issued)
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES \
    --kernel-trace -d $OUT/mfma -o run --output-format csv -- \
    python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 \
    --rmpc-steps 30 --lmpc-steps 30 --lmpc-policy-steps 0 --arm-steps 30 --resto-steps 0 --long-steps 0 > $OUT/bench_mfma.json 2> $OUT/err_mfma.log || exit $?
echo sq_done
