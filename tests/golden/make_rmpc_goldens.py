"""Generate the RMPC golden fixtures (tests/golden/rmpc_goldens.npz).

CasADi+IPOPT cannot run here.  Each golden optimum of the RMPC NLP
(RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py:35-168, restated in
oracle/rmpc_nlp.py) comes from two independent solvers:
  1. scipy SLSQP on the full NLP (defects, Delta-u rows, velocity caps, U box);
  2. the C oracle oracle/rmpc_ipm.c (IPOPT's algorithm restated, exact jet Hessians)
     run on the exact NLP (bound_relax_factor 0) to tol 1e-12.
An instance is kept only if both agree to <= 5e-8 in every control and the
solver-independent KKT certificate (oracle/rmpc_nlp.py) holds for the stored point;
the fixture stores whichever of the two optima has the smaller stationarity residual.

Run:  python tests/golden/make_rmpc_goldens.py
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
from rmpc_nlp import RMPC_DEFAULTS, RMPCProblem, kkt_certificate  # noqa: E402
from dart_mpc.workload import rmpc_batch  # noqa: E402

AGREE_TOL = 5e-8


def slsqp(args):
    N, x0, up, th, R, prm = args
    kw = dict(N=N, Qp=prm[0], Qv=prm[1], Ru=prm[2], Rdu=prm[3], u_bounds=(prm[4], prm[5]),
              du_bounds=(prm[6], prm[7]), vmax=prm[8], v_eps=prm[9])
    prob = RMPCProblem(**kw)
    p = np.concatenate([x0, up, th, R])
    lbg, ubg = prob.gbounds()
    lbx, ubx = prob.bounds()
    eq = lbg == ubg
    lo_m = (~eq) & np.isfinite(lbg)
    up_m = (~eq) & np.isfinite(ubg)
    cons = [dict(type="eq", fun=lambda w: prob.constraints(w, p)[eq], jac=lambda w: prob.constraint_jac(w, p)[eq]),
            dict(type="ineq",
                 fun=lambda w: np.concatenate([(prob.constraints(w, p) - lbg)[lo_m], (ubg - prob.constraints(w, p))[up_m]]),
                 jac=lambda w: np.concatenate([prob.constraint_jac(w, p)[lo_m], -prob.constraint_jac(w, p)[up_m]]))]
    res = minimize(lambda w: prob.objective(w, p), np.zeros(prob.nw), jac=lambda w: prob.objective_grad(w, p),
                   method="SLSQP", bounds=list(zip(lbx, ubx)), constraints=cons, options=dict(ftol=1e-15, maxiter=600))
    cert = kkt_certificate(prob, res.x, p)
    return res.x, prob.objective(res.x, p), cert


def cases():
    out = []
    D = rmpc_batch(1)
    for i in range(18):
        out.append(("c3", 20, D["x0"][i], D["u_prev"][i], D["theta"][i], D["Rref"][i], D["prm"][i]))
    D = rmpc_batch(1, seed0=11, N=15)
    for i in range(0, 18, 3):
        out.append(("n15", 15, D["x0"][i], D["u_prev"][i], D["theta"][i], D["Rref"][i], D["prm"][i]))
    # edge: velocity cap active along the horizon, and a du-saturated start
    D = rmpc_batch(1, seed0=23)
    x0 = D["x0"][0].copy(); x0[1] = 0.195; x0[3] = -0.19
    out.append(("edge", 20, x0, D["u_prev"][0], D["theta"][0], D["Rref"][0], D["prm"][0]))
    up = np.array([0.55, -0.55])
    out.append(("edge", 20, D["x0"][1], up, D["theta"][1], D["Rref"][1], D["prm"][1]))
    # velocity caps (np_mpc...:123-127) active: fast start toward a far reference, tightened vmax
    R = np.zeros((21, 4)); R[:, 0] = 0.15; R[:, 2] = -0.1
    for vm, vx in ((0.2, 0.199), (0.05, 0.049), (0.05, 0.0), (0.03, 0.0)):
        x0 = D["x0"][2].copy(); x0[0] = -0.15; x0[1] = vx; x0[2] = 0.1; x0[3] = -vx
        prm = D["prm"][2].copy(); prm[8] = vm
        out.append(("vcap", 20, x0, np.zeros(2), D["theta"][2], R.reshape(-1), prm))
    return out


def main():
    cs = cases()
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(slsqp, [c[1:] for c in cs])
    keep_w = []
    for i, (c, r) in enumerate(zip(cs, res)):
        N = c[1]
        orc = oracle_lib.rmpc_solve_batch(c[2][None], c[3][None], c[4][None], c[5][None], c[6][None], N=N,
                                          tol=1e-12, relax=0.0, max_iter=500)
        nX = 4 * (N + 1)
        agree = float(np.max(np.abs(orc["w"][0][nX:] - r[0][nX:])))
        kw = dict(N=N, Qp=c[6][0], Qv=c[6][1], Ru=c[6][2], Rdu=c[6][3], u_bounds=(c[6][4], c[6][5]),
                  du_bounds=(c[6][6], c[6][7]), vmax=c[6][8], v_eps=c[6][9])
        prob = RMPCProblem(**kw)
        p = np.concatenate([c[2], c[3], c[4], c[5]])
        cert_o = kkt_certificate(prob, orc["w"][0], p)
        w_best, cert = (r[0], r[2]) if r[2]["stat"] <= cert_o["stat"] else (orc["w"][0], cert_o)
        print(f"{i:3d} {c[0]:5s} N={N:2d} agree={agree:.1e} oracle_status={orc['status'][0]} "
              f"stat={cert['stat']:.1e} prim={cert['primal']:.1e}")
        if agree > AGREE_TOL or cert["stat"] > 1e-8 or cert["primal"] > 1e-10 or orc["status"][0] != 0:
            raise SystemExit(f"instance {i} failed the two-solver agreement / certificate gate")
        keep_w.append(w_best)
    nwmax = max(w.size for w in keep_w)
    W = np.full((len(cs), nwmax), np.nan)
    for i, w in enumerate(keep_w):
        W[i, : w.size] = w
    np.savez_compressed(os.path.join(HERE, "rmpc_goldens.npz"),
                        group=np.array([c[0] for c in cs]), N=np.array([c[1] for c in cs]),
                        x0=np.stack([c[2] for c in cs]), u_prev=np.stack([c[3] for c in cs]),
                        theta=np.stack([c[4] for c in cs]),
                        Rref=np.stack([np.pad(c[5], (0, 4 * 21 - c[5].size)) for c in cs]),
                        prm=np.stack([c[6] for c in cs]), w=W)
    print("wrote", len(cs), "goldens")


if __name__ == "__main__":
    main()
