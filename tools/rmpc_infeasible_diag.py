"""Diagnostic: where RMPC's infeasible-start launches spend their time (bench.py rmpc_c3.infeasible_start): C3-shaped
batches with measured velocities x3, timed with IPOPT's restoration phases on and off (off: a failed line search ends
at -2 in the solving kernel, so that launch is the main loop up to the failure), iterations by status.
Usage (on the box): python tools/rmpc_infeasible_diag.py [K]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import dart_mpc  # noqa: E402
from dart_mpc.workload import rmpc_batch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
D = [rmpc_batch(1, seed0=200000 + i) for i in range(K + 1)]
for d in D:
    d["x0"] = d["x0"].copy()
    d["x0"][:, [1, 3]] *= 3.0
k5 = ("x0", "u_prev", "theta", "Rref", "prm")
for resto in (True, False):
    s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=18, restoration=resto)
    s.solve_batch(*(D[0][k] for k in k5))
    ts, st, it = [], [], []
    for i in range(1, K + 1):
        t0 = time.perf_counter()
        r = s.solve_batch(*(D[i][k] for k in k5))
        ts.append(time.perf_counter() - t0)
        st.append(r["status"]); it.append(r["iters"])
    s.close()
    st, it, ts = np.concatenate(st), np.concatenate(it), np.array(ts) * 1e3
    h = {int(a): int(b) for a, b in zip(*np.unique(st, return_counts=True))}
    print(f"restoration {'on ' if resto else 'off'}: call median {np.median(ts):.3f} ms  max {ts.max():.3f}  statuses {h}",
          flush=True)
    for code in sorted(h):
        m = st == code
        print(f"    status {code:2d}: iterations mean {it[m].mean():6.1f}  max {it[m].max():4d}", flush=True)
