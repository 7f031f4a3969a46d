#!/bin/bash
# Instruction-fetch counters of the PMPC restoration kernel (257 KB of code) on C4 at N = 31: one rocprofv3 --pmc
# pass over tools/ab_variant.py pmpc_resto.  Usage (on the box): bash tools/pmc_resto_icache.sh <tag>
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/icache_resto_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY"
for c in SQ_IFETCH SQ_INSTS_LDS; do
  grep -qw "$c" $OUT/avail.txt && CTRS="$CTRS $c"
done
n=0
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ; do
  if [ $n -lt 2 ] && grep -qw "$c" $OUT/avail.txt; then CTRS="$CTRS $c"; n=$((n+1)); fi
done
echo "counters: $CTRS" | tee $OUT/counters.txt
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace -d $OUT -o run --output-format csv -- \
    python3 tools/ab_variant.py pmpc_resto 5 $OUT/out.npz > $OUT/log.txt 2>&1 || exit $?
echo icache_done
