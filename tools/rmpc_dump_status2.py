"""GPU side of the RMPC status-2 investigation: the kernel's outputs -- u0, the full
iterate w, status, iterations -- on the restoration test batches (rmpc_batch(40, seed0=0) with the C3 velocities
spread 2x / 3x / 6x, tests/test_gpu_rmpc.py) and on the parity sweep's batch (rmpc_batch(80, seed0=200000), 3x,
tools/parity_sweep.py), each solved as one launch (the queued restoration kernel) and in batches of 18 (the
restoration in the solving wave).  Saved to gpurun_out/rmpc_status2_kernel.npz; tools/rmpc_status2_analysis.py
compares them with the oracle on the CPU.
Usage (on the box): [DART_S2_CASES=sweep4_x3] python tools/rmpc_dump_status2.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import dart_mpc  # noqa: E402
from dart_mpc.workload import rmpc_batch  # noqa: E402

CASES = {"test_x2": (40, 0, 2.0), "test_x3": (40, 0, 3.0), "test_x6": (40, 0, 6.0), "sweep_x3": (80, 200000, 3.0),
         "sweep4_x3": (320, 200000, 3.0)}
# DART_S2_CASES=name,name selects cases (default: the round-5 set, without the 4x sweep batch)
_sel = os.environ.get("DART_S2_CASES", "test_x2,test_x3,test_x6,sweep_x3").split(",")
CASES = {k: v for k, v in CASES.items() if k in _sel}


def batch(n, seed0, spread):
    D = rmpc_batch(n, seed0=seed0)
    D["x0"] = D["x0"].copy()
    D["x0"][:, [1, 3]] *= spread
    return D


def main():
    out = {}
    keys = ("x0", "u_prev", "theta", "Rref", "prm")
    for name, (n, seed0, spread) in CASES.items():
        D = batch(n, seed0, spread)
        B = len(D["x0"])
        s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=B)
        g = s.solve_batch(*(D[k] for k in keys), want_w=True)
        s.close()
        s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=18)
        parts = [s.solve_batch(*(D[k][i:i + 18] for k in keys), want_w=True) for i in range(0, B, 18)]
        s.close()
        for k in ("u0", "w", "status", "iters"):
            out[f"{name}/{k}"] = g[k]
            out[f"{name}/b18_{k}"] = np.concatenate([p[k] for p in parts])
        same = all(np.array_equal(out[f"{name}/{k}"], out[f"{name}/b18_{k}"]) for k in ("status", "iters", "u0", "w"))
        print(f"{name}: {B} instances, status 2 on {int(np.sum(g['status'] == 2))}; batches of 18 bit-identical "
              f"to one launch: {same}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "rmpc_status2_kernel.npz"), **out)


if __name__ == "__main__":
    main()
