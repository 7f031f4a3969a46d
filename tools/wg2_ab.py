"""Diagnostic: the two-wave builds of the RMPC and LMPC kernels (DART_WG=2, used for N = 32..63) against the one-wave
kernels on the same instances at N <= 31 (DART_FORCE_WG2=1 routes every N to the two-wave build).  With N <= 31
the second wave owns only idle nodes, whose terms are exact zeros in every reduction, so the two builds must agree
bit for bit: any difference is a defect of the two-wave machinery, not rounding.
Usage (on the box): python tools/wg2_ab.py            (runs both modes as child processes and compares)"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def run(mode):
    sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
    import dart_mpc
    from dart_mpc.workload import lmpc_batch, rmpc_batch
    res = {}
    D = lmpc_batch(1, seed0=3)
    k4 = ("state", "u_prev", "pvec", "target")
    s = dart_mpc.LmpcSolver(N=30, tol=1e-10, max_iter=500, acceptable_iter=0, B_max=64, max_cpu_time=0.0)
    g = s.solve_batch(*(D[k] for k in k4), want_w=True)
    s.close()
    for k in ("status", "iters", "u0", "w"):
        res[f"lmpc_tight/{k}"] = g[k]
    D = lmpc_batch(10, seed0=7000)
    s = dart_mpc.LmpcSolver(N=30, B_max=256, max_cpu_time=0.0)
    g = s.solve_batch(*(D[k] for k in k4), want_w=True)
    s.close()
    for k in ("status", "iters", "u0", "w"):
        res[f"lmpc_ref/{k}"] = g[k]
    D = lmpc_batch(40, seed0=0)         # 720 instances, 5 of them through IPOPT's restoration phases
    s = dart_mpc.LmpcSolver(N=30, B_max=1024, max_cpu_time=0.0)
    g = s.solve_batch(*(D[k] for k in k4), want_w=True)
    s.close()
    for k in ("status", "iters", "u0", "w"):
        res[f"lmpc_resto/{k}"] = g[k]
    k5 = ("x0", "u_prev", "theta", "Rref", "prm")
    D = rmpc_batch(4, seed0=60)
    s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=128)
    g = s.solve_batch(*(D[k] for k in k5), want_w=True)
    s.close()
    for k in ("status", "iters", "u0", "w"):
        res[f"rmpc/{k}"] = g[k]
    D = rmpc_batch(2, seed0=70)
    D["x0"] = D["x0"].copy(); D["x0"][:, [1, 3]] *= 3.0
    s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=64)
    g = s.solve_batch(*(D[k] for k in k5), want_w=True)
    s.close()
    for k in ("status", "iters", "u0", "w"):
        res[f"rmpc_resto/{k}"] = g[k]
    np.savez(os.path.join(OUT, f"wg2_ab_{mode}.npz"), **res)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        sys.exit(0)
    os.makedirs(OUT, exist_ok=True)
    for mode, force in (("wg1", "0"), ("wg2", "1")):
        env = dict(os.environ, DART_FORCE_WG2=force)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), mode], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
    A = np.load(os.path.join(OUT, "wg2_ab_wg1.npz"))
    B = np.load(os.path.join(OUT, "wg2_ab_wg2.npz"))
    for key in A.files:
        a, b = A[key], B[key]
        same = np.array_equal(a, b)
        line = f"{key:22s} equal {same}"
        if not same:
            d = a != b if a.dtype.kind in "iu" else np.abs(a - b) > 0
            rows = np.unique(np.nonzero(d)[0])
            line += f"  rows {rows[:12].tolist()}"
            if a.dtype.kind not in "iu":
                line += f"  max |diff| {np.max(np.abs(a - b)):.3e}"
            else:
                line += f"  wg1 {a[rows][:8].tolist()} wg2 {b[rows][:8].tolist()}"
        print(line, flush=True)
