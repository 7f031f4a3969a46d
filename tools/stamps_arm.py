"""Diagnostic: per-phase cycle shares of the arm-QP kernel (block 0) from the DART_STAMPS build.

Loads dart_mpc/libdartmpc_stamps.so (make -C <pkg>/csrc stamps), solves one 36-arm batch and prints
s_memtime cycles per phase.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from dart_mpc import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(_lib.PKG_DIR, os.environ.get("DART_STAMPS_LIB", "libdartmpc_stamps.so"))
L = _lib.lib()
L.dartmpc_read_stamps_arm.argtypes = [ctypes.c_void_p]
import arm_qp  # noqa: E402
from dart_mpc.arm import ArmSolver, pack_params, pack_snapshot  # noqa: E402
from dart_mpc.workload import arm_batch  # noqa: E402

PHASES = ["load", "jacobi", "qp build", "iter: residuals+tests", "iter: K + LDL'", "iter: factor rows",
          "iter: pred+corr+update", "outputs"]
S, kinds = arm_batch(1, seed0=int(os.environ.get("ARM_SEED", "0")))
s = ArmSolver(7)
for rep in range(3):
    out = s.solve_batch(pack_snapshot(S), pack_params(arm_qp.default_params()))
st = np.zeros(16, dtype=np.uint64)
L.dartmpc_read_stamps_arm(ctypes.c_void_p(st.ctypes.data))
tot = float(st[:8].sum())
it = max(1, out["iters"][0])
print(f"block0 ({kinds[0]}) iters={out['iters'][0]} jacobi sweeps={int(st[9])} total cycles={tot:.0f}")
for i, n in enumerate(PHASES):
    print(f"  {n:24s} {int(st[i]):10d}  {100 * st[i] / tot:5.1f}%  per-iter {st[i] / it:9.0f}")
print("batch iters:", out["iters"].tolist())
