"""CPU tests of the LMPC oracle (rows L1-L4): the C IPOPT restatement against the two-solver
goldens, the KKT certificate, the model/RK4 against the numpy restatement, and the reference's
IPOPT options (max_iter 50, tol 1e-4, acceptable_tol 1e-3, acceptable_iter 5).

Tolerances: exact NLP (bound_relax 0, tol 1e-12) reproduces the goldens to 5e-8 (the golden
gate); with IPOPT's bound_relax_factor 1e-8 and tol 1e-10, 1e-6.  The reference options stop
at tol 1e-4: u0 within 5e-3 of the exact optimum (observed <= 1.1e-3).
"""
import numpy as np
import pytest

import lmpc_nlp
import oracle_lib
from lmpc_nlp import LMPCProblem, kkt_certificate


def _prob(N, prm):
    return LMPCProblem(N=N, Q=prm[:8], Qt=prm[8:16], R=prm[16:20], u_bounds=(prm[20], prm[21]))


def _solve(G, idx, N, **kw):
    return oracle_lib.lmpc_solve_batch(G["state"][idx], G["u_prev"][idx], G["pvec"][idx], G["target"][idx],
                                       G["prm"][idx], N=N, nthreads=4, **kw)


@pytest.mark.parametrize("relax,tol,bound", [(0.0, 1e-12, 5e-8), (1e-8, 1e-10, 1e-6)])
def test_c_oracle_vs_goldens(lmpc_goldens, relax, tol, bound):
    G = lmpc_goldens
    for N in np.unique(G["N"]):
        N = int(N)
        idx = np.nonzero(G["N"] == N)[0]
        out = _solve(G, idx, N, tol=tol, relax=relax, acc_iter=0, max_iter=500)
        assert np.all(out["status"] == 0), out["status"]
        nX, nw = 8 * (N + 1), 8 * (N + 1) + 2 * N
        err = np.max(np.abs(out["w"][:, nX:] - G["w"][idx][:, nX:nw]))
        assert err <= bound, (N, err)


def test_goldens_certificate_and_coverage(lmpc_goldens):
    G = lmpc_goldens
    n_sat = 0
    for i in range(len(G["N"])):
        N = int(G["N"][i]); nX = 8 * (N + 1)
        w = G["w"][i][: nX + 2 * N]
        p = np.concatenate([G["state"][i], G["u_prev"][i], G["pvec"][i], G["target"][i]])
        c = kkt_certificate(_prob(N, G["prm"][i]), w, p)
        assert c["stat"] <= 1e-8 and c["primal"] <= 1e-10 and c["bound"] <= 1e-12, (i, c)
        n_sat += int(np.sum(np.abs(np.abs(w[nX:]) - 0.4) < 1e-7))
    assert n_sat > 0                                   # U box active somewhere
    e = np.nonzero(G["group"] == "edge")[0][0]         # origin at rest, zero target: u* = 0
    assert np.max(np.abs(G["w"][e][8 * 31:8 * 31 + 60])) == 0.0


def test_rk4_c_matches_numpy():
    from dart_mpc.workload import lmpc_batch
    D = lmpc_batch(2)
    rng = np.random.default_rng(3)
    U = rng.uniform(-0.4, 0.4, (36, 2))
    X = D["state"].copy(); X[::4, 1] = 0.0; X[1::4, 5] = 0.0       # exercise |v| at v = 0
    xc = oracle_lib.lmpc_rk4(X, U, D["pvec"])
    xn = np.stack([lmpc_nlp.rk4(X[i], U[i], D["pvec"][i], 0.002) for i in range(36)])
    assert np.max(np.abs(xc - xn)) <= 1e-15


def test_dynamics_kat_free_sliding():
    """With every force but the tilt switched off the translational rows integrate a constant
    acceleration g sin(a) exactly (RK4 is exact for quadratics in t)."""
    pv = np.zeros(34)                     # squashed params -> 1e-6; raw Stribeck / damping -> 0
    pv[0] = pv[1] = 1.0 - 1e-6            # m = 1
    x = np.array([0.01, 0.02, -0.03, 0.04, 0.0, 0.0, 0.0, 0.0]); u = np.array([0.1, -0.2]); Ts = 0.002
    xn = lmpc_nlp.rk4(x, u, pv, Ts)
    ax, ay = 9.81 * np.sin(0.1), 9.81 * np.sin(-0.2)
    k = 1e-6                              # residual spring / damper / radius from the squash floor
    assert abs(xn[0] - (x[0] + x[1] * Ts + 0.5 * ax * Ts ** 2)) < 1e-9 + k
    assert abs(xn[3] - (x[3] + ay * Ts)) < 1e-7 + k


def test_reference_options_and_warm_start(lmpc_goldens):
    G = lmpc_goldens
    idx = np.nonzero(G["group"] == "c5")[0]
    ref = _solve(G, idx, 30)                                     # tol 1e-4, acceptable 1e-3 x 5, max_iter 50
    assert np.all(ref["status"] >= 0) and np.all(ref["iters"] <= 50)
    assert np.max(np.abs(ref["u0"] - G["w"][idx][:, 8 * 31:8 * 31 + 2])) <= 5e-3
    warm = _solve(G, idx, 30, w_init=ref["w"])                   # worker loop w0 <- w_opt (:519-520)
    assert np.all(warm["status"] >= 0) and warm["iters"].mean() <= ref["iters"].mean()


def test_lmpc_workload_shapes_and_determinism():
    from dart_mpc.workload import lmpc_batch
    a, b = lmpc_batch(1), lmpc_batch(1)
    assert a["state"].shape == (18, 8) and a["pvec"].shape == (18, 34) and a["target"].shape == (18, 8)
    assert np.all((a["pvec"] >= 0.01) & (a["pvec"] <= 1.9))
    for k in a:
        assert np.array_equal(a[k], b[k])


def test_soc_switch_changes_path_not_solution(lmpc_goldens):
    """The oracle's second-order correction (IPOPT default) can be switched off to mirror the GPU
    kernel's line search; both end at the same optimum on the goldens."""
    G = lmpc_goldens
    idx = np.nonzero(G["group"] == "c5")[0][:6]
    a = _solve(G, idx, 30, tol=1e-11, acc_iter=0, max_iter=500, soc=True)
    b = _solve(G, idx, 30, tol=1e-11, acc_iter=0, max_iter=500, soc=False)
    assert np.all(a["status"] == 0) and np.all(b["status"] == 0)
    assert np.max(np.abs(a["u0"] - b["u0"])) <= 1e-7


def test_restoration_phase_recovers_failed_line_searches():
    """IPOPT's soft restoration and restoration phases (MinC_1NrmRestorationPhase, restated in
    oracle/lmpc_ipm.c): on the cold-started C5 batch of 720 instances (reference options) the filter line
    search fails on five instances; IPOPT leaves through the restoration phase there, and every one of
    them then converges (no status -2 left), while the other 715 instances never touch it."""
    from dart_mpc.workload import lmpc_batch
    D = lmpc_batch(40, seed0=0)
    args = (D["state"], D["u_prev"], D["pvec"], D["target"])
    off = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=8, want_w=False, resto=False)
    on = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=8, want_w=False)
    failed = off["status"] == -2
    assert failed.sum() == 5
    assert not np.any(np.isin(on["status"], (2, -2)))
    assert np.all(on["status"][failed] >= -1)
    assert np.mean(on["status"][failed] == 0) >= 0.6
    same = ~failed
    assert np.array_equal(on["status"][same], off["status"][same])
    assert np.array_equal(on["iters"][same], off["iters"][same])
    assert np.array_equal(on["u0"][same], off["u0"][same])


def test_restoration_reports_local_infeasibility():
    """IPOPT's two restoration outcomes (ApplicationReturnStatus): the restoration problem converging means
    a point of local infeasibility, Infeasible_Problem_Detected = 2; with the phases off those instances end
    at the failed filter line search, -2.  Six stress instances of the seed-7000 batch (tools/resto_time.py)
    take the first branch, after more iterations than the failed line search took."""
    from dart_mpc.workload import lmpc_batch
    D = lmpc_batch(80, seed0=7000)
    idx = np.array([477, 509, 925, 1145, 1188, 1372])
    args = tuple(D[k][idx] for k in ("state", "u_prev", "pvec", "target"))
    on = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=6, want_w=False)
    off = oracle_lib.lmpc_solve_batch(*args, N=30, nthreads=6, want_w=False, resto=False)
    assert np.all(on["status"] == 2), on["status"]
    assert np.all(off["status"] == -2), off["status"]
    assert np.all(on["iters"] > off["iters"]) and np.all(on["iters"] <= 50)


def test_least_square_multipliers_match_dense_solve():
    """IPOPT's least-square starting multipliers (constr_mult_init_max 1000) on an unstable C5 stress draw
    (instance 13542 of the parity sweep): the dense solution of [I J^T; J 0] [d; y] = [-r; 0] at the start point
    (numpy lstsq, IPOPT's gradient-based row scaling) has max |y| = 547, below the cap, so IPOPT keeps the
    estimate.  The oracle's Riccati recursion once overflowed there (an unsymmetrised P lost its positive
    definiteness) and started from zero multipliers.  Pinned through the cap itself: just above the dense
    max |y| the oracle's path differs from the zero-multiplier path, just below it is identical."""
    from dart_mpc.workload import lmpc_batch
    i = 13542
    D = lmpc_batch(1, seed0=100000 + i // 18)
    j = i % 18
    args = [D[k][j:j + 1] for k in ("state", "u_prev", "pvec", "target")]
    prm = oracle_lib.LMPC_PRM_DEFAULT
    N = 30
    prob = _prob(N, prm)
    p = np.concatenate([a[0] for a in args])
    w = np.zeros(prob.nw)                                    # the cold start (u = 0 is inside the box)
    g = prob.objective_grad(w, p)
    sc = 100.0 / np.abs(g).max() if np.abs(g).max() > 100.0 else 1.0
    J = prob.constraint_jac(w, p)
    d = np.ones(prob.ng)
    for r in range(8, prob.ng):
        m = max(1.0, np.abs(J[r]).max())
        d[r] = 100.0 / m if m > 100.0 else 1.0
    ys = np.linalg.lstsq((d[:, None] * J).T, -sc * g, rcond=None)[0]     # z_L = z_U = 1 cancel on u
    ymax = np.abs(ys).max()
    assert 100.0 < ymax < 1000.0, ymax
    run = lambda cap: oracle_lib.lmpc_solve_batch(*args, N=N, nthreads=1, max_iter=3, mult_init_max=cap)
    zero = run(0.0)
    above, below = run(ymax * (1 + 1e-6)), run(ymax * (1 - 1e-6))
    assert not np.array_equal(above["w"], zero["w"])
    assert np.array_equal(below["w"], zero["w"])
