"""PMPC restoration phases (pmpc_resto.hip) against the C oracle (GPU box): C4's 1152 instances (64 seeds)
at the reference tol 1e-8 for N / max_soc cases where IPOPT's filter line search fails on some instances.
Per case: status counts, status and iteration agreement, max |du0| over the instances both solve, split into
instances that never enter a restoration phase (the oracle with the phases off solves them) and restored ones.
Usage: python tools/pmpc_resto_sweep.py [n_seeds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import oracle_lib  # noqa: E402  (checker)
import dart_mpc  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

NT = max(1, min(16, len(os.sched_getaffinity(0))))
n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S, T, P = pmpc_batch(n_seeds)
cnt = lambda s: dict(zip(*[a.tolist() for a in np.unique(s, return_counts=True)]))
for N, soc in ((31, 4), (20, 0), (31, 0), (15, 0)):
    t0 = time.time()
    s = dart_mpc.Solver(N=N, Ts=0.002, tol=1e-8, B_max=S.shape[0], max_soc=soc)
    g = s.solve_batch(S, T, P)
    t1 = time.time()
    g2 = s.solve_batch(S, T, P)
    t2 = time.time()
    s.close()
    o = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=NT, want_w=False, soc=soc)
    off = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=NT, want_w=False, soc=soc,
                                 resto=False)
    rest = off["status"] != 0
    both = (g["status"] == 0) & (o["status"] == 0)
    du = np.abs(g["u0"] - o["u0"]).max(axis=1)
    print(f"N={N} max_soc={soc}: kernel {cnt(g['status'])} oracle {cnt(o['status'])}  restored (oracle) {int(rest.sum())}"
          f"  status equal {np.mean(g['status'] == o['status']):.4f}  iterations equal {np.mean(g['iters'] == o['iters']):.4f}"
          f"  repeat identical {np.array_equal(g['u0'], g2['u0'])}", flush=True)
    for name, m in (("plain", both & ~rest), ("restored", both & rest)):
        if m.any():
            print(f"    {name:8s} {int(m.sum()):5d}: iterations equal {np.mean(g['iters'][m] == o['iters'][m]):.4f}  "
                  f"max|du0| {du[m].max():.2e}  median {np.median(du[m]):.2e}  99% {np.quantile(du[m], 0.99):.2e}", flush=True)
    if rest.any():
        i = np.flatnonzero(rest)
        print("    restored: kernel iters", g["iters"][i][:12].tolist(), "oracle", o["iters"][i][:12].tolist(), flush=True)
    print(f"    first call {1e3 * (t1 - t0):.1f} ms, second {1e3 * (t2 - t1):.1f} ms", flush=True)
