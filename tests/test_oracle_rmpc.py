"""CPU tests of the RMPC oracle (rows R1-R6): the C IPOPT restatement against the
two-solver goldens, the KKT certificate, the RLS filter, and the driver-side host logic.

Tolerances: the exact-NLP oracle (bound_relax 0, tol 1e-12) must reproduce the
goldens to 5e-8 (the golden gate); with IPOPT's default bound_relax_factor 1e-8 the
solution moves by O(relax) on active rows, so 1e-6 there.
"""
import numpy as np
import pytest

import oracle_lib
import rmpc_nlp
from rmpc_nlp import RMPCProblem, kkt_certificate


def _prob(N, prm):
    return RMPCProblem(N=N, Qp=prm[0], Qv=prm[1], Ru=prm[2], Rdu=prm[3], u_bounds=(prm[4], prm[5]),
                       du_bounds=(prm[6], prm[7]), vmax=prm[8], v_eps=prm[9])


def _group(G, N):
    return np.nonzero(G["N"] == N)[0]


def _rref(G, idx, N):
    return G["Rref"][idx][:, : 4 * (N + 1)]


@pytest.mark.parametrize("N", [20, 15])
@pytest.mark.parametrize("relax,tol,bound", [(0.0, 1e-12, 5e-8), (1e-8, 1e-11, 1e-6)])
def test_c_oracle_vs_goldens(rmpc_goldens, N, relax, tol, bound):
    G = rmpc_goldens
    idx = _group(G, N)
    out = oracle_lib.rmpc_solve_batch(G["x0"][idx], G["u_prev"][idx], G["theta"][idx], _rref(G, idx, N),
                                      G["prm"][idx], N=N, tol=tol, relax=relax, max_iter=500, nthreads=4)
    assert np.all(out["status"] == 0), out["status"]
    nX, nw = 4 * (N + 1), 4 * (N + 1) + 2 * N
    err = np.max(np.abs(out["w"][:, nX:] - G["w"][idx][:, nX:nw]))
    assert err <= bound, err


def test_goldens_certificate_and_activity(rmpc_goldens):
    """Every stored optimum satisfies the KKT certificate; the set exercises Delta-u rows,
    the U box and the velocity caps."""
    G = rmpc_goldens
    act = dict(u=0, du=0, v=0)
    for i in range(len(G["N"])):
        N = int(G["N"][i]); prm = G["prm"][i]; nX = 4 * (N + 1)
        w = G["w"][i][: nX + 2 * N]
        p = np.concatenate([G["x0"][i], G["u_prev"][i], G["theta"][i], G["Rref"][i][:nX]])
        c = kkt_certificate(_prob(N, prm), w, p)
        assert c["stat"] <= 1e-8 and c["primal"] <= 1e-10 and c["bound"] <= 1e-12, (i, c)
        X = w[:nX].reshape(N + 1, 4); U = w[nX:].reshape(N, 2)
        du = np.diff(np.vstack([G["u_prev"][i], U]), axis=0)
        act["u"] += int(np.sum(np.minimum(np.abs(U - prm[4]), np.abs(U - prm[5])) < 1e-7))
        act["du"] += int(np.sum(np.minimum(np.abs(du - prm[6]), np.abs(du - prm[7])) < 1e-7))
        act["v"] += int(np.sum(np.abs(np.abs(X[:, [1, 3]]) - prm[8]) < 1e-7))
    assert min(act.values()) > 0, act


def test_oracle_warm_start_and_status(rmpc_goldens):
    """Warm start from the solution converges in few iterations (np_mpc...:220-221)."""
    G = rmpc_goldens
    idx = _group(G, 20)[:4]
    a = oracle_lib.rmpc_solve_batch(G["x0"][idx], G["u_prev"][idx], G["theta"][idx], _rref(G, idx, 20),
                                    G["prm"][idx], N=20, tol=1e-8)
    b = oracle_lib.rmpc_solve_batch(G["x0"][idx], G["u_prev"][idx], G["theta"][idx], _rref(G, idx, 20),
                                    G["prm"][idx], N=20, tol=1e-8, w_init=a["w"])
    assert np.all(b["status"] == 0)
    assert np.max(np.abs(a["u0"] - b["u0"])) <= 1e-6


def test_rls_c_oracle_matches_numpy():
    rng = np.random.default_rng(5)
    r = rmpc_nlp.RLS(7, P0=1e3, lam=0.995)
    th, P = np.zeros(7), np.eye(7) * 1e3
    for _ in range(200):
        phi = rng.normal(size=7); phi[6] = 1.0
        y = float(rng.normal())
        r.update(phi, y)
        th, P = oracle_lib.rls_update(th, P, phi, y, 0.995)
    assert np.allclose(th, r.theta, rtol=1e-10, atol=1e-10)
    assert np.allclose(P, r.P, rtol=1e-9, atol=1e-9 * np.max(np.abs(r.P)))


def test_rls_identifies_linear_model():
    """RLS on noise-free data of a linear-in-features model predicts it (vx and tanh(vx/v_eps)
    are nearly collinear on this range, so the check is on predictions, not parameters)."""
    rng = np.random.default_rng(9)
    truth = np.array([0.0, -1.2, 0.0, 0.0, -0.4, 0.0, 0.05])
    r = rmpc_nlp.RLS(7)
    for _ in range(300):
        x = rng.uniform(-0.15, 0.15, 4)
        f = rmpc_nlp.rls_features(x, 0.1)
        r.update(f, f @ truth)
    X = rng.uniform(-0.15, 0.15, (100, 4))
    F = np.stack([rmpc_nlp.rls_features(x, 0.1) for x in X])
    assert np.max(np.abs(F @ r.get() - F @ truth)) < 2e-3     # P0 = 1e3 prior bias


def test_driver_host_logic_matches_shim():
    """The shim's staged reference equals the oracle restatement (np_mpc...:201-210)."""
    from dart_mpc.rmpc import AdaptiveNPMPCSmooth, rls_features
    r_v = np.array([0.01, 0.0, -0.02, 0.0]); tgt = np.array([0.1, 0.0, 0.05, 0.0])
    for N in (1, 15, 20, 31):
        a = AdaptiveNPMPCSmooth.build_ref_traj(None, r_v, tgt, N, 4)
        b = rmpc_nlp.build_ref_traj(None, r_v, tgt, N)
        assert np.array_equal(a, b)
    s = np.array([0.02, -0.03, 0.01, 0.05])
    assert np.array_equal(rls_features(s, 0.1), rmpc_nlp.rls_features(s, 0.1))
    g = rmpc_nlp.governor_step(r_v, tgt)
    assert np.allclose(g, [0.015, 0.0, -0.015, 0.0])


def test_rmpc_workload_shapes_and_determinism():
    from dart_mpc.workload import rmpc_batch
    a = rmpc_batch(1); b = rmpc_batch(1)
    assert a["x0"].shape == (18, 4) and a["Rref"].shape == (18, 84) and a["prm"].shape == (18, 10)
    assert a["rls_P"].shape == (18, 2, 7, 7)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_second_order_correction_never_engages_on_c3():
    """IPOPT's second-order correction (max_soc 4) leaves every C3 solve bit-identical to the solve
    without it (720 instances, tol 1e-8 and 1e-11): on this workload the full step is never rejected
    with theta(trial) >= theta, so the kernel's line search (no correction) follows IPOPT's path."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(40, seed0=0)
    args = (D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    for tol in (1e-8, 1e-11):
        a = oracle_lib.rmpc_solve_batch(*args, N=20, tol=tol, nthreads=8, want_w=False, soc=True)
        b = oracle_lib.rmpc_solve_batch(*args, N=20, tol=tol, nthreads=8, want_w=False, soc=False)
        np.testing.assert_array_equal(a["u0"], b["u0"])
        np.testing.assert_array_equal(a["iters"], b["iters"])
        np.testing.assert_array_equal(a["status"], b["status"])


def _spread_batch(n_seeds, factor):
    """C3-type instances with the measured velocities scaled: a |v| above vmax at node 0 (x_0 pinned,
    np_mpc...:88-91, caps at every node :123-127) makes the NLP locally infeasible."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(n_seeds, seed0=0)
    D["x0"] = D["x0"].copy()
    D["x0"][:, [1, 3]] *= factor
    return D


def test_restoration_phase_leaves_feasible_solves_unchanged():
    """IPOPT's soft restoration and restoration phases (default on) never engage on the C3 batch: every
    solve is bit-identical with the phases off (720 instances)."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(40, seed0=0)
    args = (D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    on = oracle_lib.rmpc_solve_batch(*args, nthreads=8, want_w=False)
    off = oracle_lib.rmpc_solve_batch(*args, nthreads=8, want_w=False, resto=False)
    for k in ("u0", "iters", "status"):
        np.testing.assert_array_equal(on[k], off[k])
    assert np.all(on["status"] == 0)


def test_restoration_phase_on_infeasible_starts():
    """Measured velocities 2x the C3 spread (72 instances, about half of them above vmax at node 0).  With
    the phases off the filter line search fails there (-2); IPOPT's restoration phase (oracle/rmpc_ipm.c,
    MinC_1NrmRestorationPhase) instead converges to a point of local infeasibility, status 2
    (Infeasible_Problem_Detected), and never fails.  Solver-independent check (rmpc_nlp.l1_stationarity): at
    the returned point the linearised l1 violation cannot decrease within |d| <= 1e-4 (LP decrease <= 1e-7;
    observed <= 2e-8), at the failed line search's point it can (>= 1e-4; observed >= 4.6e-4), and the
    violation is lower there.  Instances the line search solves are unchanged."""
    D = _spread_batch(4, 2.0)
    args = (D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    on = oracle_lib.rmpc_solve_batch(*args, nthreads=8)
    off = oracle_lib.rmpc_solve_batch(*args, nthreads=8, resto=False)
    failed = off["status"] == -2
    assert failed.sum() >= 20 and set(np.unique(off["status"])) <= {0, -2}
    assert np.all(on["status"][failed] == 2), on["status"][failed]
    for k in ("u0", "iters", "status"):
        np.testing.assert_array_equal(on[k][~failed], off[k][~failed])
    assert np.all(on["iters"][failed] > off["iters"][failed]) and on["iters"].max() <= 200
    for i in np.nonzero(failed)[0][:12]:
        p = (D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i])
        dec_on, th_on = rmpc_nlp.l1_stationarity(on["w"][i], *p)
        dec_off, th_off = rmpc_nlp.l1_stationarity(off["w"][i], *p)
        assert dec_on <= 1e-7 and dec_off >= 1e-4 and th_on < th_off, (i, dec_on, dec_off, th_on, th_off)
