#!/bin/bash
# Profiles the bench on the GPU box: kernel trace + stats, then HBM counters in separate passes.
# Usage (on the box, from the repo root): bash tools/profile_round.sh r01
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --saturation-batch 0 --n15-steps 0 --lmpc-policy-steps 0 --resto-steps 0 --long-steps 0 > $OUT/bench_trace.json 2> $OUT/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --saturation-batch 0 --n15-steps 0 --lmpc-policy-steps 0 --host-calls 0 --resto-steps 0 --long-steps 0 > $OUT/bench_fetch.json 2> $OUT/fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --saturation-batch 0 --n15-steps 0 --lmpc-policy-steps 0 --host-calls 0 --resto-steps 0 --long-steps 0 > $OUT/bench_write.json 2> $OUT/write.err || exit $?
echo profile_done
