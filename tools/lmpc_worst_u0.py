"""Diagnostic (GPU box): the LMPC C5 stress instances of tools/parity_sweep.py (seeds 100000+) that kernel and oracle
both solve (status 0 / 1) but end at different controls -- index, statuses, iterations, u0 of both, and each side's
objective, so that two local solutions of the nonconvex NLP can be told from a wrong one.
Usage: python tools/lmpc_worst_u0.py [seeds] [top]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import oracle_lib  # noqa: E402  (checker)
import dart_mpc  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 6400
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
NT = max(1, min(16, len(os.sched_getaffinity(0))))
D = lmpc_batch(seeds, seed0=100000)
args = (D["state"], D["u_prev"], D["pvec"], D["target"])
s = dart_mpc.LmpcSolver(N=30, B_max=len(D["state"]))
g = s.solve_batch(*args)
s.close()
o = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=NT, want_w=False)
both = np.isin(g["status"], (0, 1)) & np.isin(o["status"], (0, 1))
du = np.abs(g["u0"] - o["u0"]).max(axis=1)
du[~both] = -1.0
idx = np.argsort(-du)[:top]
print(f"{len(du)} instances, solved by both {int(both.sum())}; |du0| > 1e-6 on {int((du > 1e-6).sum())}, > 1e-3 on "
      f"{int((du > 1e-3).sum())}")
for i in idx:
    print(f"  #{i}: |du0| {du[i]:.3e}  status kernel {g['status'][i]} oracle {o['status'][i]}  iters kernel "
          f"{g['iters'][i]} oracle {o['iters'][i]}  f kernel {g['f'][i]:.9e} oracle {o['f'][i]:.9e}  "
          f"u0 kernel {g['u0'][i]} oracle {o['u0'][i]}")
