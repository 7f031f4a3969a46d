# rocprofv3 kernel trace of the long-horizon lines (two-wave builds of all three variants, batch 18, N = 40 / 63)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_long -o run --output-format csv -- python3 tools/long_diag.py 10 > gpurun_out/prof_long.log 2>&1; rc=$?
tail -14 gpurun_out/prof_long.log; [ $rc -eq 0 ] || exit 1
find gpurun_out/prof_long -name "*kernel_stats.csv" | head -3
echo DEV26_DONE
