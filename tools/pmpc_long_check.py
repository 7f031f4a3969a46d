"""Diagnostic: PMPC at horizons 32..63 against the C oracle -- statuses, iteration equality, max |du0| on C4-sized
batches (1152 instances, default options) -- for the build the launcher picks (two-wave scan build by default,
DART_PMPC_SEQ_LONG=1: the one-wave sequential build).  Usage (on the box): python tools/pmpc_long_check.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"), os.path.join(ROOT, "oracle")]
import dart_mpc  # noqa: E402
import oracle_lib  # noqa: E402  (checker only)
from dart_mpc.workload import pmpc_batch  # noqa: E402

mode = "sequential (one wave)" if os.environ.get("DART_PMPC_SEQ_LONG") == "1" else "two-wave scan"
for N in (32, 40, 50, 63):
    for seed0 in (500000, 400000):
        S, T, P = pmpc_batch(64, seed0=seed0)
        s = dart_mpc.Solver(N=N, Ts=0.002, tol=1e-8, B_max=S.shape[0])
        s.solve_batch(S, T, P)
        t0 = time.perf_counter()
        g = s.solve_batch(S, T, P)
        dt = time.perf_counter() - t0
        s.close()
        o = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=16, want_w=False)
        both = (g["status"] == 0) & (o["status"] == 0)
        print(f"{mode}: N={N} seeds {seed0}+ ({len(S)}): status equal {np.mean(g['status'] == o['status']):.5f}  "
              f"iters equal {np.mean(g['iters'] == o['iters']):.5f}  max|du0| {np.abs(g['u0'] - o['u0']).max(axis=1)[both].max():.2e}"
              f"  statuses {dict(zip(*np.unique(g['status'], return_counts=True)))}  one call {dt * 1e3:.2f} ms", flush=True)
