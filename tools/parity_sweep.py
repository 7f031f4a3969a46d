"""Parity sweep (GPU box): every kernel against the C oracle on many seeded batches beyond the test suite's,
at the reference's options -- PMPC tol 1e-8 (C2/C4 workload), RMPC tol 1e-8 (C3), LMPC tol 1e-4 / max_iter 50
/ acceptable 1e-3 x 5 with IPOPT's restoration phases (C5 stress workload).  Per variant: instances, status
agreement, iteration agreement, max |du0| over the instances the oracle solves (status 0 / 1) and the
status counts of both.  Round 4 adds the restoration phases: RMPC with the C3 velocities spread 3x (infeasible starts) and PMPC at
N = 31 and with max_soc = 0 (instances whose filter line search fails).
Round 5 adds horizons 40 and 63 on all three variants (DART_SWEEP_LONG=0 skips them).
Usage: python tools/parity_sweep.py [pmpc_seeds rmpc_seeds lmpc_seeds [rmpc_spread_seeds]]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import oracle_lib  # noqa: E402  (checker)
import dart_mpc  # noqa: E402
from dart_mpc.workload import lmpc_batch, pmpc_batch, rmpc_batch  # noqa: E402

NT = max(1, min(16, len(os.sched_getaffinity(0))))
ns = [int(a) for a in sys.argv[1:5]] if len(sys.argv) > 3 else [640, 160, 160, 80]


def report(name, g, o, solved):
    st_eq = np.mean(g["status"] == o["status"])
    it_eq = np.mean(g["iters"] == o["iters"])
    both = solved(g["status"]) & solved(o["status"])
    du = np.max(np.abs(g["u0"][both] - o["u0"][both])) if both.any() else float("nan")
    it_both = np.mean(g["iters"][both] == o["iters"][both]) if both.any() else float("nan")
    only_o = int(np.sum(solved(o["status"]) & ~solved(g["status"])))
    only_g = int(np.sum(solved(g["status"]) & ~solved(o["status"])))
    cnt = lambda s: dict(zip(*[a.tolist() for a in np.unique(s, return_counts=True)]))
    print(f"{name}: {len(g['status'])} instances  status equal {st_eq:.5f}  iterations equal {it_eq:.5f}\n"
          f"    solved by both {int(both.sum())}: iterations equal {it_both:.5f}, max|du0| {du:.2e};  solved by the "
          f"oracle only {only_o}, by the kernel only {only_g}\n    kernel {cnt(g['status'])}\n    oracle {cnt(o['status'])}",
          flush=True)


t0 = time.time()
S, T, P = pmpc_batch(ns[0], seed0=100000)
s = dart_mpc.Solver(N=20, Ts=0.002, tol=1e-8, B_max=S.shape[0])
g = s.solve_batch(S, T, P)
s.close()
o = oracle_lib.solve_batch(S, T, P, N=20, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=NT, want_w=False)
report("PMPC C2/C4 (seeds 100000+)", g, o, lambda st: st == 0)

D = rmpc_batch(ns[1], seed0=100000)
args = (D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=len(D["x0"]))
g = s.solve_batch(*args)
s.close()
o = oracle_lib.rmpc_solve_batch(*args, N=20, tol=1e-8, nthreads=NT)
report("RMPC C3 (seeds 100000+)", g, o, lambda st: st == 0)

D = lmpc_batch(ns[2], seed0=100000)
args = (D["state"], D["u_prev"], D["pvec"], D["target"])
s = dart_mpc.LmpcSolver(N=30, B_max=len(D["state"]))
g = s.solve_batch(*args)
s.close()
o = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=NT, want_w=False)
report("LMPC C5 stress (seeds 100000+, restoration on)", g, o, lambda st: np.isin(st, (0, 1)))

# the restoration phases of RMPC and PMPC (round 4): infeasible RMPC starts (measured velocities 3x the C3
# spread: |v| > vmax at the pinned node 0) and PMPC instances whose filter line search fails (N = 31 at the
# defaults; max_soc = 0 at N = 20)
if len(ns) > 3 or len(sys.argv) <= 4:
    n_r = ns[3] if len(ns) > 3 else 80
    D = rmpc_batch(n_r, seed0=200000)
    D["x0"] = D["x0"].copy(); D["x0"][:, [1, 3]] *= 3.0
    args = (D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=len(D["x0"]))
    g = s.solve_batch(*args)
    s.close()
    o = oracle_lib.rmpc_solve_batch(*args, N=20, tol=1e-8, nthreads=NT)
    report("RMPC C3 velocities x3 (seeds 200000+, restoration)", g, o, lambda st: st == 0)
    inf = (o["status"] == 2) & (g["status"] == 2)
    if inf.any():
        du = np.abs(g["u0"] - o["u0"]).max(axis=1)[inf]
        print(f"    status 2 by both {int(inf.sum())}: |du0| median {np.median(du):.2e}, 99 % {np.quantile(du, 0.99):.2e}, "
              f"max {du.max():.2e}", flush=True)
    for N, soc, seeds in ((31, 4, 128), (20, 0, 32)):
        S, T, P = pmpc_batch(seeds, seed0=300000)
        s = dart_mpc.Solver(N=N, Ts=0.002, tol=1e-8, B_max=S.shape[0], max_soc=soc)
        g = s.solve_batch(S, T, P)
        s.close()
        o = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=NT, want_w=False, soc=soc)
        off = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=NT, want_w=False, soc=soc,
                                     resto=False)
        report(f"PMPC N={N} max_soc={soc} (seeds 300000+; {int(np.sum(off['status'] != 0))} need restoration)", g, o,
               lambda st: st == 0)
# horizons beyond 31 (round 5): PMPC two registers per lane, RMPC / LMPC the two-wave builds
if os.environ.get("DART_SWEEP_LONG", "1") == "1":
    for N in (40, 63):
        S, T, P = pmpc_batch(80, seed0=400000)
        s = dart_mpc.Solver(N=N, Ts=0.002, tol=1e-8, B_max=S.shape[0])
        g = s.solve_batch(S, T, P)
        s.close()
        o = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=NT, want_w=False)
        report(f"PMPC N={N} (seeds 400000+)", g, o, lambda st: st == 0)
        D = rmpc_batch(80, seed0=400000, N=N)
        args = (D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
        s = dart_mpc.RmpcSolver(N=N, tol=1e-8, B_max=len(D["x0"]))
        g = s.solve_batch(*args)
        s.close()
        o = oracle_lib.rmpc_solve_batch(*args, N=N, tol=1e-8, nthreads=NT)
        report(f"RMPC N={N} (seeds 400000+)", g, o, lambda st: st == 0)
        D = lmpc_batch(80, seed0=400000)
        args = (D["state"], D["u_prev"], D["pvec"], D["target"])
        s = dart_mpc.LmpcSolver(N=N, B_max=len(D["state"]), max_cpu_time=0.0)
        g = s.solve_batch(*args)
        s.close()
        o = oracle_lib.lmpc_solve_batch(*args, N=N, nthreads=NT, want_w=False)
        report(f"LMPC stress N={N} (seeds 400000+, restoration on)", g, o, lambda st: np.isin(st, (0, 1)))
print(f"({time.time() - t0:.0f} s, oracle on {NT} threads)")
