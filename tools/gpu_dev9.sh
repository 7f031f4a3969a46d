set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/wg2_trace.py 30 15 3 1 > gpurun_out/wg2_trace_30r.txt 2>&1; tail -1 gpurun_out/wg2_trace_30r.txt
timeout -k 10 120 python -u tools/wg2_trace.py 32 15 3 1 > gpurun_out/wg2_trace_32r.txt 2>&1; tail -1 gpurun_out/wg2_trace_32r.txt
timeout -k 10 120 python -u tools/wg2_trace.py 32 15 3 0 > gpurun_out/wg2_trace_32.txt 2>&1; tail -1 gpurun_out/wg2_trace_32.txt
