"""The saturated RMPC / LMPC launches of bench.py (batches of 18 x 64 and 18 x 1024, inputs in HBM) on their own, for
a rocprofv3 kernel trace that isolates them (profiles/r06/sat_kernel_stats.csv).  Usage (on the box):
rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sat -o run -- python3 tools/sat_lines.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))
import torch  # noqa: E402
import dart_mpc  # noqa: E402
from dart_mpc._lib import LMPC_PRM_DEFAULT  # noqa: E402
from dart_mpc.workload import lmpc_batch, rmpc_batch  # noqa: E402

dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(device=dev)
sp = stream.cuda_stream
f64 = lambda a: torch.tensor(np.asarray(a), dtype=torch.float64, device=dev).contiguous()
for kind in ("rmpc", "lmpc"):
    for ns in (64, 1024):
        B = 18 * ns
        if kind == "rmpc":
            D = rmpc_batch(ns, seed0=600000)
            X = [f64(D[k]) for k in ("x0", "u_prev", "theta", "Rref", "prm")]
            s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=B, device=0)
        else:
            D = lmpc_batch(ns, seed0=600000)
            X = [f64(D[k]) for k in ("state", "u_prev", "pvec", "target")] + [f64(np.tile(LMPC_PRM_DEFAULT, (B, 1)))]
            s = dart_mpc.LmpcSolver(N=30, B_max=B, device=0)
        U0 = torch.empty((B, 2), dtype=torch.float64, device=dev); FV = torch.empty(B, dtype=torch.float64, device=dev)
        ST = torch.empty(B, dtype=torch.int32, device=dev); IT = torch.empty(B, dtype=torch.int32, device=dev)
        ms = []
        for rep in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            s.solve_batch_dev(B, *[x.data_ptr() for x in X], U0.data_ptr(), FV.data_ptr(), ST.data_ptr(), IT.data_ptr(),
                              stream=sp)
            e1.record(stream)
            torch.cuda.synchronize()
            if rep:
                ms.append(e0.elapsed_time(e1))
        s.close()
        m = float(np.median(ms))
        print(f"{kind} batch {B}: {m:.3f} ms per launch, {B / m * 1e3:.0f} solves/s, iters mean {IT.double().mean():.2f}, "
              f"ok {float(((ST == 0) | (ST == 1)).double().mean()):.4f}", flush=True)
