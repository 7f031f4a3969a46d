"""Generate the LMPC golden fixtures (tests/golden/lmpc_goldens.npz).

CasADi+IPOPT cannot run here and the reference holds no LMPC fixtures.
Each golden optimum of the LMPC NLP (LMPC/src/controller/rlmpc2.py:239-491, restated in
oracle/lmpc_nlp.py) comes from two independent solvers:
  1. scipy SLSQP on the numpy restatement (complex-step Jacobians);
  2. the C oracle oracle/lmpc_ipm.c (IPOPT's algorithm restated, second-order jets) on the
     exact NLP (bound_relax_factor 0) to tol 1e-11.
An instance is kept only if both agree to <= 5e-8 in every control and the KKT certificate
(oracle/lmpc_nlp.py) holds for the stored point, which is whichever optimum has the smaller
stationarity residual.  pvec is an input fixture (the policy checkpoints are not loaded,
SURVEY.md §0.4).

Run:  python tests/golden/make_lmpc_goldens.py
"""
from __future__ import annotations

import os
import sys
from multiprocessing import Pool

import numpy as np
from scipy.optimize import minimize

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))

import oracle_lib  # noqa: E402
from lmpc_nlp import LMPCProblem, kkt_certificate  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

AGREE_TOL = 5e-8


def _prob(N, prm):
    return LMPCProblem(N=N, Q=prm[:8], Qt=prm[8:16], R=prm[16:20], u_bounds=(prm[20], prm[21]))


def slsqp(args):
    N, st, up, pv, tg, prm = args
    prob = _prob(N, prm)
    p = np.concatenate([st, up, pv, tg])
    lbx, ubx = prob.bounds()
    cons = [dict(type="eq", fun=lambda w: prob.constraints(w, p), jac=lambda w: prob.constraint_jac(w, p))]
    res = minimize(lambda w: prob.objective(w, p), np.zeros(prob.nw), jac=lambda w: prob.objective_grad(w, p),
                   method="SLSQP", bounds=list(zip(lbx, ubx)), constraints=cons,
                   options=dict(ftol=1e-16, maxiter=1000))
    return res.x, kkt_certificate(prob, res.x, p)


def cases():
    prm0 = oracle_lib.LMPC_PRM_DEFAULT
    out = []
    D = lmpc_batch(1)
    for i in range(18):
        out.append(("c5", 30, D["state"][i], D["u_prev"][i], D["pvec"][i], D["target"][i], prm0))
    D = lmpc_batch(1, seed0=31)
    for i in range(0, 18, 3):
        out.append(("n20", 20, D["state"][i], D["u_prev"][i], D["pvec"][i], D["target"][i], prm0))
    D = lmpc_batch(1, seed0=57)
    # edge: origin at rest with zero target (u* = 0 by symmetry), u_prev at the bound, far target (U saturated),
    # short horizons
    out.append(("edge", 30, np.zeros(8), np.zeros(2), D["pvec"][0], np.zeros(8), prm0))
    out.append(("edge", 30, D["state"][1], np.array([0.4, -0.4]), D["pvec"][1], D["target"][1], prm0))
    far = D["target"][2].copy(); far[0] = 0.35; far[2] = -0.3
    out.append(("edge", 30, D["state"][2], D["u_prev"][2], D["pvec"][2], far, prm0))
    out.append(("edge", 1, D["state"][3], D["u_prev"][3], D["pvec"][3], D["target"][3], prm0))
    out.append(("edge", 2, D["state"][4], D["u_prev"][4], D["pvec"][4], D["target"][4], prm0))
    return out


def main():
    cs = cases()
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(slsqp, [c[1:] for c in cs])
    keep = []
    for i, (c, r) in enumerate(zip(cs, res)):
        N = c[1]
        orc = oracle_lib.lmpc_solve_batch(c[2][None], c[3][None], c[4][None], c[5][None], c[6][None], N=N,
                                          tol=1e-11, acc_iter=0, max_iter=500, relax=0.0)
        nX = 8 * (N + 1)
        agree = float(np.max(np.abs(orc["w"][0][nX:] - r[0][nX:])))
        prob = _prob(N, c[6])
        p = np.concatenate([c[2], c[3], c[4], c[5]])
        cert_o = kkt_certificate(prob, orc["w"][0], p)
        w_best, cert = (r[0], r[1]) if r[1]["stat"] <= cert_o["stat"] else (orc["w"][0], cert_o)
        print(f"{i:3d} {c[0]:5s} N={N:2d} agree={agree:.1e} oracle_status={orc['status'][0]} it={orc['iters'][0]} "
              f"stat={cert['stat']:.1e} prim={cert['primal']:.1e} u0={w_best[nX:nX + 2]}")
        if agree > AGREE_TOL or cert["stat"] > 1e-8 or cert["primal"] > 1e-10 or orc["status"][0] != 0:
            raise SystemExit(f"instance {i} failed the two-solver agreement / certificate gate")
        keep.append(w_best)
    nwmax = max(w.size for w in keep)
    W = np.full((len(cs), nwmax), np.nan)
    for i, w in enumerate(keep):
        W[i, : w.size] = w
    np.savez_compressed(os.path.join(HERE, "lmpc_goldens.npz"),
                        group=np.array([c[0] for c in cs]), N=np.array([c[1] for c in cs]),
                        state=np.stack([c[2] for c in cs]), u_prev=np.stack([c[3] for c in cs]),
                        pvec=np.stack([c[4] for c in cs]), target=np.stack([c[5] for c in cs]),
                        prm=np.stack([c[6] for c in cs]), w=W)
    print("wrote", len(cs), "goldens")


if __name__ == "__main__":
    main()
