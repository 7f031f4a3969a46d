"""Launch duration of the C2 PMPC batch against the iteration cap: t(max_iter) = t0 + n t_iter.
The intercept t0 holds the launch's fixed costs (setup, cold instruction fetch, outputs).
Usage (GPU box): [DART_PMPC_PATH=reduced] python tools/iter_cost.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dart-dual-arm-non-prehensile-manipulation_amd"))
import dart_mpc  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

dev = torch.device("cuda", 0)
S, T, P = pmpc_batch(1, seed0=123)
X0, RF, PR = (torch.tensor(a, device=dev) for a in (S, T, P))
U0 = torch.empty((18, 2), dtype=torch.float64, device=dev)
FV = torch.empty(18, dtype=torch.float64, device=dev)
ST = torch.empty(18, dtype=torch.int32, device=dev)
IT = torch.empty(18, dtype=torch.int32, device=dev)
stream = torch.cuda.Stream(device=dev)
rows = []
for mi in (1, 2, 3, 4, 6, 8, 30):
    s = dart_mpc.Solver(N=20, tol=1e-8, max_iter=mi, B_max=18, path=os.environ.get("DART_PMPC_PATH", "ipopt"))
    launch = lambda: s.solve_batch_dev(18, X0.data_ptr(), RF.data_ptr(), PR.data_ptr(), U0.data_ptr(), FV.data_ptr(),
                                       ST.data_ptr(), IT.data_ptr(), stream=stream.cuda_stream)
    for _ in range(20):
        launch()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    with torch.cuda.stream(stream):
        for a, b in ev:
            a.record(stream); launch(); b.record(stream)
    torch.cuda.synchronize()
    ms = np.median([a.elapsed_time(b) for a, b in ev]) * 1e3
    its = IT.cpu().numpy()
    rows.append((mi, int(its.max()), ms))
    print(f"max_iter {mi:3d}: iterations max {its.max():2d} mean {its.mean():5.2f}, launch median {ms:6.1f} us", flush=True)
    s.close()
n = np.array([r[1] for r in rows], float); t = np.array([r[2] for r in rows])
A = np.stack([np.ones_like(n), n], 1)
c = np.linalg.lstsq(A, t, rcond=None)[0]
print(f"fit: t0 = {c[0]:.1f} us, t_iter = {c[1]:.2f} us per iteration (slowest instance)")
