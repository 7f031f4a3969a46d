set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/wg2_trace.py 32 > gpurun_out/wg2_trace_32.txt 2>&1; tail -2 gpurun_out/wg2_trace_32.txt
timeout -k 10 400 python -u tools/wg2_ab.py
