#!/bin/bash
# Builds and runs tools/host_path_bench.cpp (host-path latency of the PMPC C ABI, no Python).
# Usage (GPU box or here for the build only): bash tools/host_path_bench.sh [B] [reps] [path] [--build-only]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dart-dual-arm-non-prehensile-manipulation_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -Wno-unused-result -Wno-unused-value -I "$ROOT/include" "$ROOT/tools/host_path_bench.cpp" -L "$PKG/dart_mpc" -ldartmpc \
  -Wl,-rpath,"$PKG/dart_mpc" -o "$ROOT/tools/host_path_bench"
[ "$4" = "--build-only" ] && exit 0
timeout -k 10 120 "$ROOT/tools/host_path_bench" "${1:-18}" "${2:-2000}" "${3:-ipopt}"
