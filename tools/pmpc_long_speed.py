"""Diagnostic: PMPC per-call time at horizons 20..63 (batch 18 through the host entry, the same 40 batches at every
N), for the build the launcher picks (two-wave scan build for N > 31 by default, DART_PMPC_SEQ_LONG=1: the one-wave
sequential build).  Usage (on the box): python tools/pmpc_long_speed.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import dart_mpc  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

mode = "sequential" if os.environ.get("DART_PMPC_SEQ_LONG") == "1" else "two-wave"
K = 40
P = [pmpc_batch(1, seed0=700000 + 1000 * i) for i in range(K + 1)]
for N in (20, 31, 32, 36, 40, 44, 48, 56, 63):
    s = dart_mpc.Solver(N=N, Ts=0.002, tol=1e-8, B_max=18)
    s.solve_batch(*P[0])
    ts, bm = [], []
    for i in range(1, K + 1):
        t0 = time.perf_counter()
        r = s.solve_batch(*P[i])
        ts.append(time.perf_counter() - t0)
        bm.append(int(np.max(r["iters"])))
    s.close()
    ts = np.array(ts) * 1e6
    print(f"{mode}: N={N:2d} call median {np.median(ts):7.1f} us  batch-max iterations mean {np.mean(bm):5.2f}  "
          f"median us per batch-max iteration {np.median(ts / np.array(bm)):6.2f}", flush=True)
