# Round-6 profile set (GPU box): rocprofv3 trace + HBM passes of the bench (tools/profile_round.sh), the saturated
# RMPC / LMPC launches alone, C3 alone (isolates rmpc_ipm_kernel<true> behind C3 launches), the driver's bench form
# (20 steps) twice, and the SQ counters.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile_round.sh r06 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06/sat -o run --output-format csv -- \
    python3 tools/sat_lines.py > gpurun_out/prof_r06/sat_lines.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06/c3 -o run --output-format csv -- \
    python3 tools/ab_variant.py rmpc 500 /tmp/c3.npz > gpurun_out/prof_r06/c3_only.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_k20a.json 2>/dev/null && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_k20b.json 2>/dev/null && \
bash tools/pmc_sq.sh r06 && echo PROF_OK
