"""CPU tests of the oracle (numpy restatement + C IPM) against the goldens and
the analytic known-answer tests of SURVEY §8c.  No GPU."""
import numpy as np
import pytest

from pmpc_nlp import PMPCProblem, dynamics, kkt_certificate, rk4_step


def test_rk4_closed_form_mu0():
    """RK4 is exact for theta const, mu = 0: px(Ts) = px + vx Ts + 1/2 g sin(theta) Ts^2 (SURVEY §8c ii)."""
    x = np.array([0.1, 0.2, -0.05, 0.03, 0.43, 0.0]); u = np.array([0.3, -0.2])
    Ts, g = 0.002, -9.81
    xn = rk4_step(x, u, 0.0, Ts)
    assert abs(xn[0] - (x[0] + x[1] * Ts + 0.5 * g * np.sin(u[0]) * Ts ** 2)) < 1e-16
    assert abs(xn[1] - (x[1] + g * np.sin(u[0]) * Ts)) < 1e-15
    assert abs(xn[2] - (x[2] + x[3] * Ts + 0.5 * g * np.sin(u[1]) * Ts ** 2)) < 1e-16


def test_dynamics_matches_reference_formula():
    x = np.array([0.0, 0.1, 0.0, -0.2, 0.43, 0.01]); u = np.array([0.2, 0.1]); mu, Ts = 0.1, 0.002
    xd = dynamics(x, u, mu, Ts)
    vz_new = 9.81 * (0.2 ** 2 + 0.1 ** 2)                      # -g (tx^2 + ty^2), g = -9.81
    np.testing.assert_allclose(xd, [0.1, -9.81 * np.sin(0.2) - 0.01, -0.2, -9.81 * np.sin(0.1) + 0.02,
                                    vz_new, (vz_new - 0.01) / Ts], rtol=1e-15)


def test_c_oracle_rk4_matches_numpy():
    import oracle_lib
    rng = np.random.default_rng(3)
    for _ in range(20):
        x = rng.normal(size=6) * 0.1; u = rng.uniform(-0.6, 0.6, 2); mu = rng.uniform(0.0, 0.5)
        np.testing.assert_allclose(oracle_lib.rk4(0.002, mu, x, u), rk4_step(x, u, mu, 0.002), rtol=0, atol=1e-15)


def test_goldens_pass_kkt_certificate(goldens):
    G = goldens
    for i in range(len(G["N"])):
        N = int(G["N"][i]); mu, qp, qv, r, lo, hi = G["prm"][i]
        prob = PMPCProblem(N=N, Ts=float(G["Ts"][i]), Qp=qp, Qv=qv, R=r, mu=mu, u_bounds=(lo, hi))
        w = G["w"][i][: prob.nw]
        c = kkt_certificate(prob, w, np.concatenate([G["state"][i], G["target"][i]]), relax=0.0)
        assert c["primal"] <= 1e-12 and c["bound"] == 0.0 and c["stat_sign"] == 0.0
        assert c["stat_free"] <= 1e-9
        assert G["agree"][i] <= 2e-8
        assert abs(prob.objective(w, np.concatenate([G["state"][i], G["target"][i]])) - G["f"][i]) <= 1e-12 * max(1, G["f"][i])


def test_golden_edge_cases_known_answers(goldens):
    G = goldens
    edge = [i for i in range(len(G["N"])) if G["group"][i] == "edge"]
    rest = edge[0]                       # at rest on the target: u* = 0 (SURVEY §8c i)
    N = int(G["N"][rest])
    assert np.max(np.abs(G["w"][rest][6 * (N + 1): 6 * (N + 1) + 2 * N])) == 0.0
    a, b = edge[1], edge[2]              # mirror pair: u*(-e) = -u*(e) (SURVEY §8c iii)
    N = int(G["N"][a])
    ua = G["w"][a][6 * (N + 1): 6 * (N + 1) + 2 * N]; ub = G["w"][b][6 * (N + 1): 6 * (N + 1) + 2 * N]
    assert np.max(np.abs(ua + ub)) <= 1e-10


def test_c_oracle_matches_goldens(goldens):
    import oracle_lib
    G = goldens
    for i in range(len(G["N"])):
        N = int(G["N"][i])
        r = oracle_lib.solve_batch(G["state"][i:i + 1], G["target"][i:i + 1], G["prm"][i:i + 1], N=N,
                                   Ts=float(G["Ts"][i]), tol=1e-8)
        nX = 6 * (N + 1)
        assert r["status"][0] == 0, i
        assert np.max(np.abs(r["u0"][0] - G["w"][i][nX:nX + 2])) <= 1e-6, i
        assert np.max(np.abs(r["w"][0][nX:] - G["w"][i][nX:nX + 2 * N])) <= 1e-5, i
        # states: x/y sub-states to 1e-6; the z sub-state amplifies control differences by
        # d vz / d theta = 0.625 * 2 |g| theta (mpc_3d.py:93-95), so it gets 1e-4
        dX = np.abs(r["w"][0][:nX] - G["w"][i][:nX]).reshape(N + 1, 6)
        assert dX[:, :4].max() <= 1e-6 and dX[:, 4:].max() <= 1e-4, i
        assert abs(r["f"][0] - G["f"][i]) <= 1e-7 * max(1.0, G["f"][i]), i


def test_c_oracle_tight_tol_is_exact(goldens):
    import oracle_lib
    G = goldens
    for i in range(0, len(G["N"]), 5):
        N = int(G["N"][i])
        r = oracle_lib.solve_batch(G["state"][i:i + 1], G["target"][i:i + 1], G["prm"][i:i + 1], N=N,
                                   Ts=float(G["Ts"][i]), tol=1e-11)
        nX = 6 * (N + 1)
        assert np.max(np.abs(r["w"][0][nX:] - G["w"][i][nX:nX + 2 * N])) <= 1e-7, i


def test_workload_is_seeded_and_matches_survey():
    from dart_mpc.workload import pmpc_batch, config_params, config_name
    a = pmpc_batch(2); b = pmpc_batch(2)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    S, T, P = a
    assert S.shape == (36, 6)
    assert np.all(np.abs(S[:, 0]) <= 0.18) and np.all(np.abs(S[:, 2]) <= 0.13)
    assert np.all(S[:, 4] == 0.43) and np.all(T[:, 4] == 0.4)
    np.testing.assert_array_equal(config_params(0), [0.05, 600, 5, 0.1, -0.6, 0.6])     # cube, mu 0.05
    np.testing.assert_array_equal(config_params(17), [0.2, 200, 2, 0.2, -0.6, 0.6])     # sphere, mu 0.2
    assert config_name(4) == "cube_m2_mu0.1"


@pytest.mark.parametrize("N,soc", [(31, 4), (20, 0)])
def test_c_oracle_restoration_phases(N, soc):
    """IPOPT's soft restoration and restoration phases in the PMPC oracle (TrySoftRestoStep,
    MinC_1NrmRestorationPhase; oracle/pmpc_ipm.c restoration()).  C4's 1152 instances at the reference
    tol 1e-8: at N = 31 three, and with the second-order correction off about a tenth, fail the filter
    line search; IPOPT (and the oracle with the phases on) solves every one.  Instances that never enter a
    restoration phase take the identical path with the phases on or off; the restored ones end at a KKT
    point (the certificate of pmpc_nlp.py, tolerances of an interior-point answer at tol 1e-8)."""
    import oracle_lib
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(64)
    kw = dict(N=N, Ts=0.002, tol=1e-8, max_iter=3000, nthreads=8, soc=soc)
    on = oracle_lib.solve_batch(S, T, P, resto=True, **kw)
    off = oracle_lib.solve_batch(S, T, P, resto=False, **kw)
    assert np.all(on["status"] == 0)
    failed = off["status"] != 0
    assert failed.any() and np.all(off["status"][failed] == -2)
    same = ~failed
    np.testing.assert_array_equal(on["iters"][same], off["iters"][same])
    np.testing.assert_array_equal(on["u0"][same], off["u0"][same])
    for i in np.flatnonzero(failed)[:12]:
        mu, qp, qv, r, lo, hi = P[i]
        prob = PMPCProblem(N=N, Ts=0.002, Qp=qp, Qv=qv, R=r, mu=mu, u_bounds=(lo, hi))
        c = kkt_certificate(prob, on["w"][i], np.concatenate([S[i], T[i]]), act_tol=1e-5)
        assert c["primal"] <= 1e-8 and c["bound"] == 0.0, i
        assert c["stat_free"] <= 1e-6 * max(1.0, c["grad_scale"]) and c["stat_sign"] <= 1e-6 * max(1.0, c["grad_scale"]), i
