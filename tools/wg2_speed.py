"""Diagnostic: the cost of the two-wave machinery -- RMPC (C3, N = 31) and LMPC (C5 stress inputs, reference options,
N = 30) batches of 18 through the host entry on the one-wave kernels and, with DART_FORCE_WG2=1, on the two-wave
builds (same instances, same results: tools/wg2_ab.py).  Usage (on the box): python tools/wg2_speed.py
(runs both modes as child processes)."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(mode):
    sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
    import dart_mpc
    from dart_mpc.workload import lmpc_batch, rmpc_batch
    K = 200
    R = [rmpc_batch(1, seed0=9000 + i, N=31) for i in range(K + 5)]
    k5 = ("x0", "u_prev", "theta", "Rref", "prm")
    s = dart_mpc.RmpcSolver(N=31, tol=1e-8, B_max=18)
    for i in range(5):
        s.solve_batch(*(R[i][k] for k in k5))
    t0 = time.perf_counter()
    for i in range(5, K + 5):
        s.solve_batch(*(R[i][k] for k in k5))
    dr = time.perf_counter() - t0
    s.close()
    L = [lmpc_batch(1, seed0=7000 + i) for i in range(K + 5)]
    k4 = ("state", "u_prev", "pvec", "target")
    s = dart_mpc.LmpcSolver(N=30, B_max=18, max_cpu_time=0.0)
    for i in range(5):
        s.solve_batch(*(L[i][k] for k in k4))
    t0 = time.perf_counter()
    for i in range(5, K + 5):
        s.solve_batch(*(L[i][k] for k in k4))
    dl = time.perf_counter() - t0
    s.close()
    print(f"{mode}: RMPC N=31 {18 * K / dr:9.0f} solves/s ({dr / K * 1e3:.3f} ms per batch)   "
          f"LMPC N=30 {18 * K / dl:9.0f} solves/s ({dl / K * 1e3:.3f} ms per batch)", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        sys.exit(0)
    for rep in range(2):
        for mode, force in (("one-wave", "0"), ("two-wave", "1")):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), mode], env=dict(os.environ, DART_FORCE_WG2=force),
                               timeout=300)
            if r.returncode:
                sys.exit(r.returncode)
