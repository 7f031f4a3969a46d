"""Diagnostic: per-call time and iteration counts of the long-horizon lines (bench.py `long_horizons`), PMPC at
N = 20 / 31 / 40 / 63 and RMPC / LMPC at 31 / 40 / 63, batch 18 through the host entry.  Prints per-N the median and
max call time, mean / max iterations and the status histogram, so a slow line can be told apart into per-iteration
cost, iteration count and outliers (restoration).  Usage (on the box): python tools/long_diag.py [K]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]


def stats(name, ts, its, sts):
    ts = np.array(ts) * 1e6
    its = np.concatenate(its)
    sts = np.concatenate(sts)
    h = {int(k): int(v) for k, v in zip(*np.unique(sts, return_counts=True))}
    print(f"{name:12s} call median {np.median(ts):8.1f} us  p90 {np.percentile(ts, 90):8.1f}  max {ts.max():8.1f}   "
          f"iters mean {its.mean():5.2f} max {its.max():3d}  batch-max mean {np.mean(np.max(its.reshape(-1, 18), 1)):5.2f}"
          f"   status {h}", flush=True)


def main(K):
    import dart_mpc
    from dart_mpc.workload import lmpc_batch, pmpc_batch, rmpc_batch
    for N in (20, 31, 40, 63):
        P = [pmpc_batch(1, seed0=700000 + 1000 * i) for i in range(K + 1)]
        s = dart_mpc.Solver(N=N, Ts=0.002, tol=1e-8, B_max=18)
        s.solve_batch(*P[0])
        ts, its, sts = [], [], []
        for i in range(1, K + 1):
            t0 = time.perf_counter()
            r = s.solve_batch(*P[i])
            ts.append(time.perf_counter() - t0)
            its.append(np.asarray(r["iters"]))
            sts.append(np.asarray(r["status"]))
        s.close()
        stats(f"PMPC N={N}", ts, its, sts)
    k5 = ("x0", "u_prev", "theta", "Rref", "prm")
    k4 = ("state", "u_prev", "pvec", "target")
    for N in (31, 40, 63):
        R = [rmpc_batch(1, seed0=9500 + i, N=N) for i in range(K + 1)]
        s = dart_mpc.RmpcSolver(N=N, tol=1e-8, B_max=18)
        s.solve_batch(*(R[0][k] for k in k5))
        ts, its, sts = [], [], []
        for i in range(1, K + 1):
            t0 = time.perf_counter()
            r = s.solve_batch(*(R[i][k] for k in k5))
            ts.append(time.perf_counter() - t0)
            its.append(np.asarray(r["iters"]))
            sts.append(np.asarray(r["status"]))
        s.close()
        stats(f"RMPC N={N}", ts, its, sts)
    for N in (30, 40, 63):
        L = [lmpc_batch(1, seed0=7500 + i) for i in range(K + 1)]
        s = dart_mpc.LmpcSolver(N=N, B_max=18)
        s.solve_batch(*(L[0][k] for k in k4))
        ts, its, sts = [], [], []
        for i in range(1, K + 1):
            t0 = time.perf_counter()
            r = s.solve_batch(*(L[i][k] for k in k4))
            ts.append(time.perf_counter() - t0)
            its.append(np.asarray(r["iters"]))
            sts.append(np.asarray(r["status"]))
        s.close()
        stats(f"LMPC N={N}", ts, its, sts)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
