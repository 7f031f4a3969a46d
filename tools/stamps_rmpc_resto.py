"""Diagnostic: phase cycles of one RMPC infeasible-start instance (C3 shape, measured velocities x3) in
rmpc_ipm_kernel<true> from the DART_STAMPS build: the main loop (re-run from the start up to the failed line search)
and IPOPT's restoration phase proper.  The instance is put at block 0 of a batch of 18.  Stamps fence the kernel,
so read the shares, not the absolute length.  Usage (on the box): python tools/stamps_rmpc_resto.py [seed]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))
from dart_mpc import _lib  # noqa: E402
from dart_mpc.workload import rmpc_batch  # noqa: E402

_lib.LIB_PATH = os.path.join(_lib.PKG_DIR, os.environ.get("DART_STAMPS_LIB", "libdartmpc_stamps.so"))
L = _lib.lib()
L.dartmpc_read_stamps_rmpc.argtypes = [ctypes.c_void_p]
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 200001
D = rmpc_batch(1, seed0=seed)
D["x0"] = D["x0"].copy()
D["x0"][:, [1, 3]] *= 3.0
k5 = ("x0", "u_prev", "theta", "Rref", "prm")
s = _lib.RmpcSolver(N=20, tol=1e-8, B_max=18)
out = s.solve_batch(*(D[k] for k in k5))
# the slowest status-2 instance first
cand = np.flatnonzero(out["status"] == 2)
j = int(cand[np.argmax(out["iters"][cand])]) if cand.size else 0
order = np.r_[j, np.delete(np.arange(18), j)]
Dj = {k: D[k][order] for k in k5}
for rep in range(2):
    out = s.solve_batch(*(Dj[k] for k in k5))
st = np.zeros(32, dtype=np.uint64)
L.dartmpc_read_stamps_rmpc(ctypes.c_void_p(st.ctypes.data))
names = {0: "setup+rls", 1: "main: eval+errors+mu", 2: "main: qp build", 3: "main: riccati", 4: "main: forward+dz",
         5: "main: slack steps", 6: "main: ls prep", 7: "main: ls trials (+soft phase)", 8: "main: accept",
         16: "resto: start (lsq mults)", 17: "resto: eval + errors", 18: "resto: soft Riccati (inertia)",
         19: "resto: solve + refinement", 20: "resto: line search", 22: "resto: accept + update",
         21: "resto: return to main"}
tot = float(sum(int(st[i]) for i in names))
print(f"instance {j} (seed {seed}): status {out['status'][0]} iters {out['iters'][0]}; total {tot:.0f} cycles")
for i, n in names.items():
    print(f"  {n:32s} {int(st[i]):10d}  {100 * st[i] / tot:5.1f}%")
print(f"  main riccati passes {int(st[9])}, main ls trials {int(st[10])}; restoration iterations {int(st[27])}, "
      f"soft sweeps {int(st[24])}, refinement passes {int(st[25])}, trials {int(st[26])}")
