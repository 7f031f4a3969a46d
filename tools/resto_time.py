"""Cost of IPOPT's restoration path on the GPU: the C5 instances whose filter line search fails (found by
the oracle with the phases off) solved as one batch with the phases on, against the same batch with them
off, and a batch of instances that never need them.  Prints launch times and iteration counts."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import oracle_lib  # noqa: E402
import dart_mpc  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

D = lmpc_batch(80, seed0=7000)
args = [D[k] for k in ("state", "u_prev", "pvec", "target")]
o = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=8, want_w=False, resto=False)
fail = np.where(o["status"] == -2)[0][:18]
easy = np.where(o["status"] == 0)[0][:18]
print("resto instances", fail.tolist())


def run(idx, resto, reps=5):
    s = dart_mpc.LmpcSolver(N=30, B_max=64, restoration=resto)
    sub = [a[idx] for a in args]
    out = s.solve_batch(*sub)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = s.solve_batch(*sub)
        t.append(time.perf_counter() - t0)
    s.close()
    return min(t) * 1e3, out


for name, idx in (("needs-resto", fail), ("easy", easy)):
    for resto in (True, False):
        ms, out = run(idx, resto)
        print(f"{name:12s} resto={resto!s:5s} launch {ms:8.3f} ms  iters max {out['iters'].max():3d} "
              f"sum {out['iters'].sum():4d}  ms/iter(max) {ms / max(1, out['iters'].max()):.4f}  "
              f"status {np.unique(out['status'], return_counts=True)}")
# one instance at a time: the cost of each restoration instance alone
for i in fail[:6]:
    ms, out = run(np.array([i]), True, reps=3)
    ms0, out0 = run(np.array([i]), False, reps=3)
    print(f"instance {i}: resto {ms:7.3f} ms / {out['iters'][0]} it ({out['status'][0]}),  "
          f"off {ms0:7.3f} ms / {out0['iters'][0]} it ({out0['status'][0]})")
