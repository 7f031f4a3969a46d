"""Diagnostic: the C5 stress instances of the parity sweep (tools/parity_sweep.py, seeds 100000+) where the LMPC
kernel and the oracle end with different statuses, with both iteration counts.  Usage:
python tools/lmpc_mismatch.py [n_seeds, default 1600]; instance i is instance i % 18 of lmpc_batch(1, 100000 + i // 18)
(tools/resto_trace.py <i> 100000 traces the kernel on it)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import oracle_lib  # noqa: E402
import dart_mpc  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1600
D = lmpc_batch(n, seed0=100000)
args = [D[k] for k in ("state", "u_prev", "pvec", "target")]
o = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=16, want_w=False)
s = dart_mpc.LmpcSolver(N=30, B_max=len(D["state"]))
g = s.solve_batch(*args)
s.close()
for i in np.nonzero(g["status"] != o["status"])[0]:
    print(f"instance {i:6d}: oracle {o['status'][i]:3d} / {o['iters'][i]:2d} it   kernel {g['status'][i]:3d} / {g['iters'][i]:2d} it")
