#!/bin/bash
# Instruction-fetch counters of the bench kernels: is the iteration loop of a big kernel (LMPC <false> is
# 110 KB of code) refetching instructions?  Lists the counters the box offers, keeps the instruction-cache
# ones that exist (at most 2 of the SQC block, <= 8 SQ in all), one rocprofv3 --pmc pass.
# Usage (on the box): bash tools/pmc_icache.sh <tag>
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/icache_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
for c in SQ_IFETCH SQ_IFETCH_LEVEL; do
  grep -qw "$c" $OUT/avail.txt && CTRS="$CTRS $c"
done
n=0
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE; do
  if [ $n -lt 2 ] && grep -qw "$c" $OUT/avail.txt; then CTRS="$CTRS $c"; n=$((n+1)); fi
done
echo "counters: $CTRS" | tee $OUT/counters.txt
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace -d $OUT -o run --output-format csv -- \
    python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 --n15-steps 0 \
    --rmpc-steps 30 --lmpc-steps 30 --lmpc-policy-steps 30 --arm-steps 0 > $OUT/bench.json 2> $OUT/err.log || exit $?
echo icache_done
