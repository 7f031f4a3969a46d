"""Diagnostic (GPU box): the kernel's full iterate w of chosen LMPC C5 stress instances of the parity sweep (seeds
100000+, solved as one launch like tools/parity_sweep.py), saved to gpurun_out/lmpc_instances.npz for a
solver-independent KKT check on the CPU (oracle/lmpc_nlp.py kkt_certificate).
Usage: python tools/lmpc_dump_instance.py <seeds> <index> [<index> ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import dart_mpc  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

seeds, idx = int(sys.argv[1]), [int(a) for a in sys.argv[2:]]
D = lmpc_batch(seeds, seed0=100000)
s = dart_mpc.LmpcSolver(N=30, B_max=len(D["state"]))
g = s.solve_batch(D["state"], D["u_prev"], D["pvec"], D["target"], want_w=True)
s.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "lmpc_instances.npz"), idx=np.array(idx), w=g["w"][idx], u0=g["u0"][idx],
         status=g["status"][idx], iters=g["iters"][idx], f=g["f"][idx])
print("saved", idx, g["status"][idx], g["iters"][idx])
