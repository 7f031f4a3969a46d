"""Diagnostic: phase cycles of IPOPT's restoration phase in lmpc_ipm_kernel<true> (DART_STAMPS build), for one
C5 instance whose filter line search fails (solved alone: block 0 is that instance).

Slots 0-15 are the iteration phases of the resumed solve (as tools/stamps_lmpc.py), 16-23 the restoration
phases, 24 the soft-row sweeps (inertia attempts), 25 the restoration iterations, 26 its line-search trials.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"), os.path.join(ROOT, "oracle")]
from dart_mpc import _lib  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

_lib.LIB_PATH = os.path.join(_lib.PKG_DIR, os.environ.get("DART_STAMPS_LIB", "libdartmpc_stamps.so"))
L = _lib.lib()
L.dartmpc_read_stamps_lmpc.argtypes = [ctypes.c_void_p]
D = lmpc_batch(80, seed0=7000)
s = _lib.LmpcSolver(N=30, B_max=64)
MAIN = ["setup", "eval+errors+mu", "gradient rows", "riccati", "forward+dz", "bound steps", "ls prep", "ls trials",
        "accept"]
RESTO = ["resto start (p/n, LSQ)", "resto stage (derivatives)", "resto errors+mu+rows", "resto soft sweep(s)",
         "resto step (fwd, p/n)", "resto phi/gTd", "resto line search", "resto accept"]
for i in [int(a) for a in (sys.argv[1:] or ["1", "491", "515"])]:
    sl = slice(i, i + 1)
    for rep in range(2):
        out = s.solve_batch(D["state"][sl], D["u_prev"][sl], D["pvec"][sl], D["target"][sl])
    st = np.zeros(32, dtype=np.uint64)
    L.dartmpc_read_stamps_lmpc(ctypes.c_void_p(st.ctypes.data))
    tot = float(st[:9].sum() + st[11:15].sum() + st[16:24].sum())
    print(f"instance {i}: status {out['status'][0]} iters {out['iters'][0]}, resumed-kernel cycles {tot:.0f}")
    for k, n in enumerate(MAIN):
        print(f"  {n:28s} {int(st[k]):10d}  {100 * st[k] / tot:5.1f}%")
    for k, n in zip((11, 12, 13, 14), ("closed loop", "forward sweep", "eval: rk4+adjoint", "eval: directions")):
        print(f"  {n:28s} {int(st[k]):10d}  {100 * st[k] / tot:5.1f}%")
    for k, n in enumerate(RESTO):
        print(f"  {n:28s} {int(st[16 + k]):10d}  {100 * st[16 + k] / tot:5.1f}%")
    print(f"  line-search trials (regular) {int(st[10])}, riccati passes {int(st[9])}; restoration: iterations "
          f"{int(st[25])}, soft sweeps {int(st[24])}, trials {int(st[26])}")
