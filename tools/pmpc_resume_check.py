"""Diagnostic: PMPC restoration resumed from the register kernel's failed iteration (DART_PMPC_RESUME=1) against the
restoration solve started over (the default; DART_PMPC_RESUME=1 resumes), per restored instance, against the oracle's
iterations.  Usage (on the box): python tools/pmpc_resume_check.py [N] [max_soc]  (resume = DART_PMPC_RESUME=1)"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 15
SOC = int(sys.argv[2]) if len(sys.argv) > 2 else 0

if os.environ.get("_CHILD"):
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(64)
    g = dart_mpc.Solver(N=N, tol=1e-8, B_max=S.shape[0], max_soc=SOC).solve_batch(S, T, P)
    off = dart_mpc.Solver(N=N, tol=1e-8, B_max=S.shape[0], max_soc=SOC, restoration=False).solve_batch(S, T, P)
    np.savez(os.environ["_CHILD"], status=g["status"], iters=g["iters"], u0=g["u0"], off_status=off["status"],
             off_iters=off["iters"])
    sys.exit(0)

out = {}
for tag, res in (("resume", "1"), ("restart", "0")):
    fn = os.path.join(ROOT, "gpurun_out", f"resume_{tag}.npz")
    subprocess.run([sys.executable, __file__, str(N), str(SOC)], env=dict(os.environ, _CHILD=fn, DART_PMPC_RESUME=res),
                   check=True, timeout=300)
    out[tag] = np.load(fn)
import oracle_lib  # noqa: E402  (checker)
from dart_mpc.workload import pmpc_batch  # noqa: E402
S, T, P = pmpc_batch(64)
o = oracle_lib.solve_batch(S, T, P, N=N, tol=1e-8, max_iter=3000, nthreads=8, want_w=False, soc=SOC)
rest = out["resume"]["off_status"] != 0
idx = np.flatnonzero(rest)
print(f"N={N} max_soc={SOC}: {idx.size} restored")
for tag in ("resume", "restart"):
    g = out[tag]
    eq = g["iters"][idx] == o["iters"][idx]
    print(f"  {tag}: statuses equal {np.array_equal(g['status'], o['status'])}, restored iterations equal "
          f"{eq.mean():.3f}, max|du0| restored {np.abs(g['u0'][idx] - o['u0'][idx]).max():.2e}")
r, s_ = out["resume"], out["restart"]
for i in idx:
    if r["iters"][i] != o["iters"][i] or s_["iters"][i] != o["iters"][i]:
        print(f"    #{i}: fails at {r['off_iters'][i]}, oracle {o['iters'][i]}, resume {r['iters'][i]}, "
              f"restart {s_['iters'][i]}")
