# Kernel trace of the C2 / C3 / C5 bench lines: per-launch durations and inter-launch gaps.
set -o pipefail
OUT=gpurun_out/gaps
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
    python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --saturation-batch 0 --host-calls 0 --c4-steps 0 \
    --n15-steps 0 --arm-steps 0 --rmpc-steps 100 --lmpc-steps 100 > $OUT/bench.json 2> $OUT/err.log || exit $?
F=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_gaps.py $F pmpc_ipm_kernel && python3 tools/kernel_gaps.py $F rmpc_ipm_kernel && \
python3 tools/kernel_gaps.py $F lmpc_ipm_kernel
