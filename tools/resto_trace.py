"""Diagnostic: per-iteration trace of IPOPT's restoration phase in the LMPC kernel for one C5 instance (seed
7000 batch of tools/resto_time.py), from the DART_RESTO_TRACE build (libdartmpc_trace.so): the same line as the
oracle's ORACLE_DEBUG build prints, plus the step's residual on the linearised restoration rows and on the
closed-loop rows of the forward sweep.  Build it first (`make -C dart-dual-arm-non-prehensile-manipulation_amd/csrc
trace`; the library stays out of the shipped tree).  Usage: python tools/resto_trace.py <instance> [seed0, default 7000]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
os.environ.setdefault("DART_MPC_LIB", "libdartmpc_trace.so")
import dart_mpc  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

i = int(sys.argv[1])
seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 7000      # instance i of lmpc_batch(., seed0): seed seed0 + i // 18
D = lmpc_batch(1, seed0=seed0 + i // 18)
s = dart_mpc.LmpcSolver(N=30, B_max=4)
g = s.solve_batch(*[D[k][i % 18:i % 18 + 1] for k in ("state", "u_prev", "pvec", "target")])
s.close()
print("kernel status", g["status"], g["iters"], flush=True)
