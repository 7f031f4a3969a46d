"""Diagnostic: per-phase cycle shares of the LMPC kernel (block 0) from the DART_STAMPS build.

Loads dart_mpc/libdartmpc_stamps.so (make -C <pkg>/csrc stamps), solves the C5 batch and prints
s_memtime cycles per phase.  Stamps fence the kernel, so read the shares, not the absolute length.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))
from dart_mpc import _lib  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

_lib.LIB_PATH = os.path.join(_lib.PKG_DIR, os.environ.get("DART_STAMPS_LIB", "libdartmpc_stamps.so"))
L = _lib.lib()
L.dartmpc_read_stamps_lmpc.argtypes = [ctypes.c_void_p]
PHASES = ["setup", "eval+errors+mu", "gradient rows", "riccati", "forward+dz", "bound steps", "ls prep",
          "ls trials", "accept"]
D = lmpc_batch(1)
s = _lib.LmpcSolver(N=30, tol=1e-8, max_iter=500, acceptable_iter=0, B_max=64)
for rep in range(3):
    out = s.solve_batch(D["state"], D["u_prev"], D["pvec"], D["target"])
st = np.zeros(32, dtype=np.uint64)     # the reader copies all 32 slots (16-26: restoration phases)
L.dartmpc_read_stamps_lmpc(ctypes.c_void_p(st.ctypes.data))
tot = float(st[:9].sum() + st[11:15].sum())
it = max(1, out["iters"][0])
print(f"block0 iters={out['iters'][0]} total cycles={tot:.0f}")
for i, n in enumerate(PHASES):
    print(f"  {n:15s} {int(st[i]):10d}  {100 * st[i] / tot:5.1f}%  per-iter {st[i] / it:9.0f}")
for i, n in zip((11, 12, 13, 14), ("closed loop", "forward sweep", "eval: rk4+adjoint", "eval: directions")):
    print(f"  {n:15s} {int(st[i]):10d}  {100 * st[i] / tot:5.1f}%  per-iter {st[i] / it:9.0f}")
print(f"  riccati passes {int(st[9])}, line-search trials {int(st[10])}, second-order corrections {int(st[15])}")
print("batch iters:", out["iters"].tolist())
