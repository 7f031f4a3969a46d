"""Diagnostic: per-phase cycle shares of the PMPC kernel (block 0) from the DART_STAMPS build.

Loads dart_mpc/libdartmpc_stamps.so (make -C <pkg>/csrc stamps) in place of the
product library, solves the C2 batch once and prints s_memtime cycles per phase.
Stamps fence the kernel, so read the shares, not the absolute length.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))
from dart_mpc import _lib  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

_lib.LIB_PATH = os.path.join(_lib.PKG_DIR, os.environ.get("DART_STAMPS_LIB", "libdartmpc_stamps.so"))
L = _lib.lib()
N = int(os.environ.get("DART_STAMPS_N", "20"))
B = int(os.environ.get("DART_STAMPS_B", "18"))
# the one-row (N <= 15) and the sequential (B above the scan limit, or N > 31) builds live in the
# PMPC_SEQ object, which has its own stamp array
read = L.dartmpc_read_stamps_seq if (N <= 15 or N > 31 or B > 1664) else L.dartmpc_read_stamps
read.argtypes = [ctypes.c_void_p]
PHASES = ["setup", "eval+errors", "mu update", "riccati", "direction", "ls prep", "ls trials", "update", "outputs"]
S, T, P = pmpc_batch(-(-B // 18))
S, T, P = S[:B], T[:B], P[:B]
s = _lib.Solver(N=N, B_max=B, path=os.environ.get("DART_PMPC_PATH", "ipopt"))
for rep in range(3):
    out = s.solve_batch(S, T, P)
st = np.zeros(16, dtype=np.uint64)
read(ctypes.c_void_p(st.ctypes.data))
tot = float(st[:9].sum())
print(f"block0 iters={out['iters'][0]} total cycles={tot:.0f}")
for i, n in enumerate(PHASES):
    print(f"  {n:12s} {int(st[i]):10d}  {100 * st[i] / tot:5.1f}%  per-iter {st[i] / max(1, out['iters'][0]):9.0f}")
print(f"  scan-path Riccati passes {int(st[11])}")
it0 = int(st[0:9].sum() - st[0] - st[8])
print(f"  first iteration {int(st[12])} cycles, mean iteration {it0 / max(1, out['iters'][0]):.0f} cycles")
print(f"  riccati passes {int(st[9])}, line-search trials {int(st[10])}, iterations with a correction {int(st[15])}")
print("batch iters:", out["iters"].tolist())
