# Round 5 end-of-round set: tests, smoke, bench, profile (trace + HBM), SQ counters, stamps, parity sweep.
set -o pipefail
bash tools/gpu_round.sh r05 || exit 1
timeout -k 10 600 python -u tools/parity_sweep.py > gpurun_out/parity_sweep_r05.txt 2>&1 || { echo SWEEP_FAILED; tail -20 gpurun_out/parity_sweep_r05.txt; exit 1; }
tail -30 gpurun_out/parity_sweep_r05.txt
