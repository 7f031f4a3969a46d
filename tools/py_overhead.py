"""Where the Python side of a host-pointer PMPC call goes (GPU box): the same C2 batch through
solve_batch, through the in-place Bound path, with and without the GIL released around the call."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dart-dual-arm-non-prehensile-manipulation_amd"))
import dart_mpc  # noqa: E402
from dart_mpc import _lib  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

S, T, P = pmpc_batch(1)
B, n = 18, 3000
s = dart_mpc.Solver(N=20, B_max=B)
s.serve_start(B_serve=B, idle_timeout=10.0)
b = s.bind()
b.x0[:B] = S; b.ref[:B] = T; b.prm[:B] = P


def t(fn, label):
    for _ in range(200):
        fn()
    x = np.empty(n)
    for i in range(n):
        c = time.perf_counter(); fn(); x[i] = time.perf_counter() - c
    print(f"{label:48s} median {np.median(x) * 1e6:7.2f} us", flush=True)


t(lambda: b.solve(B), "bound.solve (CDLL: GIL released)")
py = ctypes.PyDLL(_lib.LIB_PATH)
fn = py.dart_mpc_solve_bound
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
fn.restype = ctypes.c_int
h = s._h
t(lambda: fn(h, B, 0), "dart_mpc_solve_bound via PyDLL (GIL held)")


def copy_and_solve():
    b.x0[:B] = S; b.ref[:B] = T; b.prm[:B] = P
    fn(h, B, 0)


t(copy_and_solve, "3 input copies + PyDLL call")
t(lambda: s.solve_batch(S, T, P), "solve_batch (copies in and out)")
s.close()
