"""Diagnostic: per-iteration trace (DART_RESTO_TRACE build, libdartmpc_trace.so) of one LMPC instance at a given
horizon -- instance 15 of lmpc_batch(1, seed0=3) at tol 1e-10, the one test_horizons sends through IPOPT's
restoration phase -- to set beside the oracle's ORACLE_DEBUG trace of the same solve (built on the CPU).
Usage (on the box): python tools/wg2_trace.py N [instance seed0 ref]   (ref = 1: the reference's IPOPT options)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
os.environ.setdefault("DART_MPC_LIB", "libdartmpc_trace.so")
import dart_mpc  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

N = int(sys.argv[1])
i = int(sys.argv[2]) if len(sys.argv) > 2 else 15
seed0 = int(sys.argv[3]) if len(sys.argv) > 3 else 3
D = lmpc_batch(1, seed0=seed0)
ref = len(sys.argv) > 4 and sys.argv[4] == "1"
kw = dict(max_cpu_time=0.0) if ref else dict(tol=1e-10, max_iter=500, acceptable_iter=0, max_cpu_time=0.0)
s = dart_mpc.LmpcSolver(N=N, B_max=4, **kw)
g = s.solve_batch(*[D[k][i:i + 1] for k in ("state", "u_prev", "pvec", "target")])
s.close()
print("kernel status", g["status"], g["iters"], flush=True)
