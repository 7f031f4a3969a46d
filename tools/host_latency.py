"""Latency of one PMPC control step through the host-pointer entry (what PMPC.solve / mpc_worker
pay per call) against the kernel alone on the same instance.  Usage (GPU box): python tools/host_latency.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dart-dual-arm-non-prehensile-manipulation_amd"))
import dart_mpc  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

S, T, P = pmpc_batch(1, seed0=42)
s = dart_mpc.Solver(N=15, tol=1e-8, B_max=18)
for i in (0, 5, 9):
    x, t, p = S[i:i + 1], T[i:i + 1], P[i:i + 1]
    for _ in range(50):
        out = s.solve_batch(x, t, p)
    n = 500
    t0 = time.perf_counter()
    for _ in range(n):
        out = s.solve_batch(x, t, p)
    host_us = (time.perf_counter() - t0) / n * 1e6
    dev = torch.device("cuda", 0)
    X, Tt, Pp = (torch.tensor(a, device=dev) for a in (x, t, p))
    U = torch.empty((1, 2), dtype=torch.float64, device=dev); F = torch.empty(1, dtype=torch.float64, device=dev)
    St = torch.empty(1, dtype=torch.int32, device=dev); It = torch.empty(1, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(device=dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    with torch.cuda.stream(stream):
        for a, b in ev:
            a.record(stream)
            s.solve_batch_dev(1, X.data_ptr(), Tt.data_ptr(), Pp.data_ptr(), U.data_ptr(), F.data_ptr(), St.data_ptr(),
                              It.data_ptr(), stream=stream.cuda_stream)
            b.record(stream)
    torch.cuda.synchronize()
    k_us = np.median([a.elapsed_time(b) for a, b in ev]) * 1e3
    print(f"instance {i}: iterations {int(out['iters'][0])}, host call {host_us:.1f} us, kernel (events) {k_us:.1f} us, "
          f"overhead {host_us - k_us:.1f} us", flush=True)

# split of the host overhead: the Python wrapper alone (B = 0 returns right after the argument
# checks), and the raw ctypes call on preallocated arrays
import ctypes  # noqa: E402
from dart_mpc._lib import lib, _ptr  # noqa: E402
x, t, p = S[:1].copy(), T[:1].copy(), P[:1].copy()
n = 2000
t0 = time.perf_counter()
for _ in range(n):
    s.solve_batch(x[:0], t[:0], p[:0])
print(f"python wrapper, B = 0: {(time.perf_counter() - t0) / n * 1e6:.1f} us", flush=True)
u0 = np.empty((1, 2)); f = np.empty(1); st = np.empty(1, np.int32); it = np.empty(1, np.int32)
args = (s._h, 1, _ptr(x), _ptr(t), _ptr(p), None, _ptr(u0), _ptr(f), None, _ptr(st), _ptr(it), None)
L = lib()
for _ in range(50):
    L.dart_mpc_solve_batch(*args)
t0 = time.perf_counter()
for _ in range(500):
    L.dart_mpc_solve_batch(*args)
print(f"raw ctypes call, B = 1 (instance 0): {(time.perf_counter() - t0) / 500 * 1e6:.1f} us", flush=True)
