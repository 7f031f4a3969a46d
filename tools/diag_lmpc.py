import sys, numpy as np
sys.path.insert(0, 'dart-dual-arm-non-prehensile-manipulation_amd'); sys.path.insert(0, 'oracle')
import dart_mpc, oracle_lib
from dart_mpc.workload import lmpc_batch
D = lmpc_batch(1, seed0=3)
for N in (25, 28, 29, 30, 31):
    for tol in (1e-4, 1e-8, 1e-10):
        s = dart_mpc.LmpcSolver(N=N, tol=tol, max_iter=500, acceptable_iter=0, B_max=32)
        out = s.solve_batch(D["state"], D["u_prev"], D["pvec"], D["target"], want_w=True)
        s.close()
        bad = np.nonzero(out["status"] != 0)[0]
        print(N, tol, "bad", bad.tolist(), "st", out["status"][bad].tolist(), "it", out["iters"][bad].tolist(), "maxit", out["iters"].max())
i = 15
print("pvec", np.round(D["pvec"][i], 3).tolist())
print("state", D["state"][i], "target", D["target"][i], "u_prev", D["u_prev"][i])
r = oracle_lib.lmpc_solve_batch(D["state"][i:i+1], D["u_prev"][i:i+1], D["pvec"][i:i+1], D["target"][i:i+1], N=31, tol=1e-10, acc_iter=0, max_iter=500)
print("oracle", r["status"], r["iters"], r["u0"])
