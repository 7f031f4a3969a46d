#!/bin/bash
# Phase stamps of all kernels (DART_STAMPS build) on the GPU box; writes gpurun_out/stamps_<tag>/.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/stamps_${TAG}
mkdir -p $OUT
timeout -k 10 120 python tools/stamps.py > $OUT/stamps_phase_cycles.txt 2>&1 && \
timeout -k 10 120 python tools/stamps_rmpc.py > $OUT/stamps_rmpc_phase_cycles.txt 2>&1 && \
timeout -k 10 120 python tools/stamps_lmpc.py > $OUT/stamps_lmpc_phase_cycles.txt 2>&1 && \
timeout -k 10 120 python tools/stamps_arm.py > $OUT/stamps_arm_phase_cycles.txt 2>&1
