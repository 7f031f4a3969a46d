"""Diagnostic: the PMPC instances that need IPOPT's soft restoration phase at N = 40 / 50 (C4-sized batches, default
options) -- the kernel's and the oracle's end points side by side: iterations, |du0|, and the solver-independent KKT
certificate of the reference NLP (oracle/pmpc_nlp.kkt_certificate) for both.  Usage (on the box):
python tools/pmpc_long_resto_cert.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"), os.path.join(ROOT, "oracle")]
import dart_mpc  # noqa: E402
import oracle_lib  # noqa: E402  (checker only)
from pmpc_nlp import PMPCProblem, kkt_certificate  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

for N in (40, 50):
    for seed0 in (0, 500000, 400000):
        S, T, P = pmpc_batch(64, seed0=seed0)
        s = dart_mpc.Solver(N=N, Ts=0.002, tol=1e-8, B_max=S.shape[0])
        g = s.solve_batch(S, T, P, want_w=True)
        s.close()
        kw = dict(N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=16)
        o = oracle_lib.solve_batch(S, T, P, want_w=True, **kw)
        off = oracle_lib.solve_batch(S, T, P, resto=False, want_w=False, **kw)
        idx = np.flatnonzero(off["status"] != 0)
        eq = np.mean(g["iters"][idx] == o["iters"][idx]) if idx.size else 1.0
        print(f"N={N} seeds {seed0}+: restored {idx.size}, iterations equal on {eq:.3f}, statuses equal "
              f"{np.array_equal(g['status'], o['status'])}", flush=True)
        for i in idx:
            mu, qp, qv, r, lo, hi = P[i]
            prob = PMPCProblem(N=N, Ts=0.002, Qp=qp, Qv=qv, R=r, mu=mu, u_bounds=(lo, hi))
            p = np.concatenate([S[i], T[i]])
            cg = kkt_certificate(prob, g["w"][i], p, act_tol=1e-6)
            co = kkt_certificate(prob, o["w"][i], p, act_tol=1e-6)
            print(f"  #{i:4d} iters {g['iters'][i]:3d} / {o['iters'][i]:3d}  |du0| {np.abs(g['u0'][i] - o['u0'][i]).max():.1e}"
                  f"  kernel primal {cg['primal']:.1e} stat {max(cg['stat_free'], cg['stat_sign']):.1e}"
                  f"  oracle primal {co['primal']:.1e} stat {max(co['stat_free'], co['stat_sign']):.1e}"
                  f"  grad scale {cg['grad_scale']:.1e}", flush=True)
