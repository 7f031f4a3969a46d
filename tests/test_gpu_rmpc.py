"""GPU parity tests of the batched RMPC kernel + RLS (through the C ABI).

Tolerances (fp64 path, IPOPT-equivalent algorithm with bound_relax 1e-8):
  * against the two-solver goldens (exact NLP): every control within 1e-6 at
    tol 1e-11 (the relaxation moves active rows by O(1e-8 / multiplier));
  * against the C oracle with the same options: every control within 1e-6 at
    tol 1e-11, u0 within 1e-5 at the reference's tol 1e-8;
  * RLS (theta, P): relative 1e-12 against oracle/rmpc_ipm.c's oracle_rls_update.
"""
import numpy as np
import pytest

import oracle_lib
import rmpc_nlp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dm():
    import dart_mpc
    return dart_mpc


def _nw(N):
    return 4 * (N + 1) + 2 * N


def test_goldens_tight_tol(dm, rmpc_goldens):
    G = rmpc_goldens
    for N in np.unique(G["N"]):
        N = int(N)
        idx = np.nonzero(G["N"] == N)[0]
        s = dm.RmpcSolver(N=N, tol=1e-11, max_iter=500, B_max=64)
        out = s.solve_batch(G["x0"][idx], G["u_prev"][idx], G["theta"][idx], G["Rref"][idx][:, : 4 * (N + 1)],
                            G["prm"][idx], want_w=True)
        s.close()
        assert np.all(out["status"] == 0), (N, out["status"], out["iters"])
        nX = 4 * (N + 1)
        err = np.abs(out["w"][:, nX:] - G["w"][idx][:, nX:_nw(N)]).max(axis=1)
        assert np.all(err <= 1e-6), (N, err)


@pytest.mark.parametrize("tol,u0_bound,U_bound", [(1e-8, 1e-5, 1e-4), (1e-11, 1e-6, 1e-6)])
def test_c3_batch_vs_oracle(dm, tol, u0_bound, U_bound):
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(2)
    s = dm.RmpcSolver(N=20, tol=tol, max_iter=500, B_max=64)
    out = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], want_w=True)
    s.close()
    ref = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], N=20, tol=tol,
                                      max_iter=500, nthreads=4)
    assert np.all(out["status"] == 0) and np.all(ref["status"] == 0), (out["status"], out["iters"])
    assert np.max(np.abs(out["u0"] - ref["u0"])) <= u0_bound
    assert np.max(np.abs(out["w"][:, 84:] - ref["w"][:, 84:])) <= U_bound
    assert np.allclose(out["f"], ref["f"], rtol=1e-6, atol=1e-10)
    # the same path as the oracle (test_same_path_as_oracle's bound): equal iteration counts, bar at most one
    # instance where rounding near the end shifts convergence by one iteration
    d = np.abs(out["iters"] - ref["iters"])
    assert np.sum(d != 0) <= 1 and d.max() <= 1, (out["iters"], ref["iters"])


def test_wide_tilt_box_library_trig_path(dm):
    """u box [-1.2, 1.2] (library sin/cos instead of the Taylor path) against the C oracle."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(1)
    prm = D["prm"].copy(); prm[:, 4] = -1.2; prm[:, 5] = 1.2
    s = dm.RmpcSolver(N=20, tol=1e-11, max_iter=500, B_max=64)
    out = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], prm, want_w=True)
    s.close()
    ref = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], prm, N=20, tol=1e-11,
                                      max_iter=500, nthreads=4)
    assert np.all(out["status"] == 0) and np.all(ref["status"] == 0), (out["status"], ref["status"])
    assert np.max(np.abs(out["u0"] - ref["u0"])) <= 1e-6
    assert np.allclose(out["f"], ref["f"], rtol=1e-6, atol=1e-10)


@pytest.mark.parametrize("N", [1, 2, 15, 21, 22, 31, 32, 40, 63])
def test_horizons(dm, N):
    """N <= 31: one wave per instance; N = 32..63: the two-wave build (rmpc_ipm.hip with DART_WG=2)."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(1, seed0=3, N=N)
    s = dm.RmpcSolver(N=N, tol=1e-11, max_iter=500, B_max=32)
    out = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], want_w=True)
    s.close()
    ref = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], N=N, tol=1e-11,
                                      max_iter=500, nthreads=4)
    assert np.all(out["status"] == 0), out["status"]
    nX = 4 * (N + 1)
    assert np.max(np.abs(out["w"][:, nX:] - ref["w"][:, nX:])) <= 1e-6


@pytest.mark.parametrize("N", [20, 40])
def test_fused_rls_matches_oracle_and_unfused(dm, N):
    """The RLS update fused into the solve launch (one wave; at N = 40 the two-wave build, whose first wave writes
    theta and P back) against the oracle's RLS and against the unfused solve with the updated estimate."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(1, seed0=5, N=N)
    B = D["x0"].shape[0]
    s = dm.RmpcSolver(N=N, tol=1e-10, max_iter=500, B_max=32)
    fused = s.solve_batch(D["x0"], D["u_prev"], D["rls_theta"], D["Rref"], D["prm"], want_w=True,
                          rls_P=D["rls_P"], rls_phi=D["phi_prev"], rls_y=D["y"], rls_lambda=0.995)
    th_ref = np.zeros((B, 14)); P_ref = np.zeros((B, 2, 7, 7))
    for b in range(B):
        for a in range(2):
            th_ref[b, 7 * a:7 * a + 7], P_ref[b, a] = oracle_lib.rls_update(
                D["rls_theta"][b, 7 * a:7 * a + 7], D["rls_P"][b, a], D["phi_prev"][b], D["y"][b, a], 0.995)
    assert np.allclose(fused["theta"], th_ref, rtol=1e-12, atol=1e-12)
    assert np.allclose(fused["rls_P"], P_ref, rtol=1e-11, atol=1e-11 * np.abs(P_ref).max())
    plain = s.solve_batch(D["x0"], D["u_prev"], th_ref, D["Rref"], D["prm"], want_w=True)
    s.close()
    assert np.max(np.abs(fused["w"] - plain["w"])) <= 1e-9


def test_standalone_rls_batch(dm):
    rng = np.random.default_rng(17)
    B = 300
    th = rng.normal(size=(B, 7)); A = rng.normal(size=(B, 7, 7)); P = A @ A.transpose(0, 2, 1) + np.eye(7)
    phi = rng.normal(size=(B, 7)); y = rng.normal(size=B)
    gt, gP = dm.rls_update_batch(th, P, phi, y, 0.99)
    for b in range(0, B, 37):
        t2, P2 = oracle_lib.rls_update(th[b], P[b], phi[b], y[b], 0.99)
        assert np.allclose(gt[b], t2, rtol=1e-12, atol=1e-12) and np.allclose(gP[b], P2, rtol=1e-11, atol=1e-11)
    r = dm.RLS(7)
    ro = rmpc_nlp.RLS(7)
    for _ in range(20):
        f = rng.normal(size=7); yy = float(rng.normal())
        r.update(f, yy); ro.update(f, yy)
    assert np.allclose(r.get(), ro.get(), rtol=1e-10, atol=1e-10)


def test_warm_start_and_edge_batches(dm):
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(1)
    s = dm.RmpcSolver(N=20, tol=1e-8, B_max=32)
    cold = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], want_w=True)
    warm = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], w_warm=cold["w"], want_w=True)
    assert np.all(warm["status"] == 0) and np.max(np.abs(warm["u0"] - cold["u0"])) <= 1e-5
    e = s.solve_batch(np.zeros((0, 4)), np.zeros((0, 2)), np.zeros((0, 14)), np.zeros((0, 84)), np.zeros((0, 10)))
    assert e["u0"].shape == (0, 2)
    with pytest.raises(dm.DartMPCError):
        s.solve_batch(np.zeros((40, 4)), np.zeros((40, 2)), np.zeros((40, 14)), np.zeros((40, 84)),
                      np.tile(D["prm"][0], (40, 1)))
    s.close()


def test_closed_loop_driver_matches_oracle_loop(dm):
    """RMPCStep (rob_ctrl.py:331-352, RLS fused on the GPU) driving a plant integrated with the
    true model; at every step the oracle (numpy RLS + C IPOPT restatement, own warm start) is
    fed the same measurements and must give the same estimate and control."""
    from dart_mpc.rmpc import AdaptiveNPMPCSmooth, RMPCStep
    kw = dict(Ts=0.002, N=20, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0, u_bounds=(-0.6, 0.6), du_bounds=(-0.06, 0.06),
              vmax=0.2, v_eps=0.1)
    ctrl = AdaptiveNPMPCSmooth(None, None, tol=1e-10, max_iter=500, **kw)
    target = np.array([0.08, 0.0, -0.05, 0.0])
    x = np.zeros(4); xprev = x.copy(); up = np.zeros(2)
    step = RMPCStep(ctrl, target, r_v0=x.copy())
    truth = np.concatenate([[0, -1.0, 0, 0, -0.2, 0, 0], [0, 0, 0, -1.0, 0, -0.2, 0]])
    rls = [rmpc_nlp.RLS(7), rmpc_nlp.RLS(7)]
    r_v = x.copy(); w0 = np.zeros(_nw(20))
    for k in range(25):
        u, _ = step(x, xprev, up)
        y = rmpc_nlp.rls_targets(x, xprev, 0.002)
        f = rmpc_nlp.rls_features(xprev, 0.1)
        rls[0].update(f, y[0]); rls[1].update(f, y[1])
        th = np.concatenate([rls[0].get(), rls[1].get()])
        assert np.allclose(step.theta, th, rtol=1e-9, atol=1e-9 * max(1.0, np.abs(th).max())), k
        r_v = rmpc_nlp.governor_step(r_v, target)
        assert np.allclose(step.r_v, r_v, rtol=0, atol=1e-15)
        R = rmpc_nlp.build_ref_traj(x, r_v, target, 20)
        o = oracle_lib.rmpc_solve_batch(x[None], up[None], step.theta[None], R[None], ctrl.params()[None], N=20,
                                        tol=1e-10, w_init=w0[None], max_iter=500)
        w0 = o["w"][0]
        assert o["status"][0] == 0 and ctrl.w0 is not None
        assert np.max(np.abs(u - o["u0"][0])) <= 1e-6, (k, u, o["u0"][0])
        xprev, x = x, rmpc_nlp.rk4(x, u, truth, 0.1, 0.002)
        up = u


@pytest.mark.parametrize("mult_init", [1000.0, 0.0])
def test_least_square_starting_multipliers_same_path(dm, mult_init):
    """IPOPT starts y_c and y_d (the slack rows) from its least-square estimate (constr_mult_init_max 1000;
    np_mpc...:158-162 leaves it): on C3 it changes a third of the iteration counts.  With the estimate and
    with zero multipliers the kernel follows the oracle: same statuses, >= 99 % same iterations,
    |du0| <= 1e-6 at the reference's tol 1e-8."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(8, seed0=60)
    s = dm.RmpcSolver(N=20, tol=1e-8, B_max=256, constr_mult_init_max=mult_init)
    g = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    s.close()
    args = (D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    o = oracle_lib.rmpc_solve_batch(*args, N=20, tol=1e-8, nthreads=8, mult_init_max=mult_init)
    other = oracle_lib.rmpc_solve_batch(*args, N=20, tol=1e-8, nthreads=8, mult_init_max=1000.0 - mult_init)
    assert np.mean(o["iters"] != other["iters"]) > 0.05
    assert np.array_equal(g["status"], o["status"])
    assert np.mean(g["iters"] == o["iters"]) >= 0.99, (g["iters"], o["iters"])
    assert np.max(np.abs(g["u0"] - o["u0"])) <= 1e-6


@pytest.mark.parametrize("soc", [False, True])
def test_same_path_as_oracle(dm, soc):
    """Exact derivatives in the kernel: against the C oracle with its second-order correction off
    (the kernel's line search has none) and on (IPOPT's default; it never engages on the C3 workload,
    test_oracle_rmpc.py) every instance takes the same iterations, ends with the same status and
    returns the same control at the reference's tol 1e-8."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(8, seed0=40)
    s = dm.RmpcSolver(N=20, tol=1e-8, B_max=256)
    g = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    s.close()
    o = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], N=20, tol=1e-8,
                                    nthreads=8, soc=soc)
    assert np.array_equal(g["status"], o["status"])
    assert np.mean(g["iters"] == o["iters"]) >= 0.99, (g["iters"], o["iters"])
    assert np.max(np.abs(g["u0"] - o["u0"])) <= 1e-6


@pytest.mark.parametrize("N", [40, 63])
def test_long_horizons_same_path_as_oracle(dm, N):
    """The two-wave build (N = 32..63) on the C3 workload at the reference's tol 1e-8: IPOPT's path as the oracle's --
    statuses equal, iteration counts equal on >= 95 % and never more than one apart (at N = 63 the longer sums
    shift convergence by one iteration on 2 of 72 instances), u0 within 1e-6."""
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(4, seed0=60, N=N)
    s = dm.RmpcSolver(N=N, tol=1e-8, B_max=128)
    g = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    s.close()
    o = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], N=N, tol=1e-8, nthreads=8)
    assert np.array_equal(g["status"], o["status"]), (g["status"], o["status"])
    d = np.abs(g["iters"] - o["iters"])
    assert np.mean(d == 0) >= 0.95 and d.max() <= 1, (g["iters"], o["iters"])
    ok = np.isin(o["status"], (0, 1))
    assert ok.all()
    assert np.max(np.abs(g["u0"] - o["u0"])) <= 1e-6


@pytest.mark.parametrize("N", [40, 63])
def test_long_horizons_restoration(dm, N):
    """Measured velocities 3x the C3 spread at N = 40 / 63: IPOPT's soft restoration and restoration phases in the
    two-wave build (their state in a per-stream device area instead of LDS) take the oracle's path -- statuses
    equal (2 where the restoration converges to local infeasibility, 0 where it returns), iterations equal on
    >= 95 %, u0 within 1e-6 where solved; every status-2 point passes the l1 local-infeasibility certificate."""
    from dart_mpc.workload import rmpc_batch
    D = _spread(rmpc_batch(2, seed0=70, N=N), 3.0)
    s = dm.RmpcSolver(N=N, tol=1e-8, B_max=64)
    g = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], want_w=True)
    s.close()
    o = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], N=N, tol=1e-8,
                                    nthreads=8)
    inf = o["status"] == 2
    assert inf.sum() >= 5
    assert np.array_equal(g["status"], o["status"]), (g["status"], o["status"])
    assert np.mean(g["iters"] == o["iters"]) >= 0.95, (g["iters"], o["iters"])
    du = np.abs(g["u0"] - o["u0"]).max(axis=1)
    if (~inf).any():
        assert np.max(du[~inf]) <= 1e-6
    for i in np.nonzero(inf)[0]:
        a = (D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i])
        dec, _ = rmpc_nlp.l1_stationarity(g["w"][i], *a, N=N)
        assert dec <= 2e-7, (i, dec)


def _spread(D, factor):
    D["x0"] = D["x0"].copy()
    D["x0"][:, [1, 3]] *= factor
    return D


@pytest.mark.parametrize("spread", [2.0, 3.0, 6.0])
def test_restoration_phase_same_path_as_oracle(dm, spread):
    """Measured velocities 2x / 3x / 6x the C3 spread (720 instances each; a |v| above vmax at the pinned node 0,
    np_mpc...:123-127, makes the NLP locally infeasible).  The filter line search fails there, and IPOPT's soft
    restoration and restoration phases (rmpc_ipm_kernel<true>, the resume launch) take the oracle's path:
    statuses equal everywhere (2 = Infeasible_Problem_Detected where the restoration converges, 0 where it
    returns to a solvable problem), iteration counts equal on >= 99 %.  Controls: |du0| <= 1e-6 where the problem
    is solved (status 0).
    At a point of local infeasibility (status 2) the NLP does not determine the iterate (tools/rmpc_status2_analysis.py,
    profiles/r05/rmpc_status2.txt): the restoration phase minimises the l1 violation V of the reference NLP's rows,
    whose minimisers form a face -- V is flat to ~1e-10 on the segment between the kernel's and the oracle's
    points -- and only its proximity term (weight sqrt(mu)) picks the point; the oracle's own tol-1e-8 point moves
    1e-3..4e-2 in u0 when re-solved at tol 1e-10.  So on EVERY status-2 instance the kernel's point must pass the
    solver-independent local-infeasibility certificate (rmpc_nlp.l1_stationarity: no decrease of the linearised l1
    violation within |d| <= 1e-4, <= 2e-7) and reach the oracle's violation (V within 1e-5 relative; measured max
    3.9e-6); where the two u0 differ by more than 1e-6 they must lie on one face (V between them flat to 1e-7
    relative); and |du0| <= 5e-5 on 99 %, max <= 2e-4 (measured on these batches: 99 % <= 2e-5, max 1.54e-4).
    The returned iterate is the next control step's warm start (np_mpc...:214-217)."""
    from dart_mpc.workload import rmpc_batch
    D = _spread(rmpc_batch(40, seed0=0), spread)
    s = dm.RmpcSolver(N=20, tol=1e-8, B_max=720)
    g = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], want_w=True)
    s.close()
    o = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], N=20, tol=1e-8,
                                    nthreads=8)
    inf = o["status"] == 2
    assert inf.sum() >= 300
    assert np.array_equal(g["status"], o["status"]), np.nonzero(g["status"] != o["status"])
    assert np.mean(g["iters"] == o["iters"]) >= 0.99, np.nonzero(g["iters"] != o["iters"])
    du = np.abs(g["u0"] - o["u0"]).max(axis=1)
    assert np.max(du[~inf]) <= 1e-6
    assert np.percentile(du[inf], 99) <= 5e-5 and np.max(du[inf]) <= 2e-4, np.percentile(du[inf], [50, 99, 100])
    for i in np.nonzero(inf)[0]:
        a = (D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i])
        dec, Vk = rmpc_nlp.l1_stationarity(g["w"][i], *a)
        assert dec <= 2e-7, (i, dec)
        Vo = rmpc_nlp.l1_violation(o["w"][i], *a)
        Vk = rmpc_nlp.l1_violation(g["w"][i], *a)
        assert abs(Vk - Vo) <= 1e-5 * Vo, (i, Vk, Vo)
        if du[i] > 1e-6:
            seg = [rmpc_nlp.l1_violation(o["w"][i] + t * (g["w"][i] - o["w"][i]), *a) for t in (0.25, 0.5, 0.75)]
            assert max(abs(v - Vo) for v in seg) <= 1e-7 * Vo, (i, seg, Vo)
    if spread == 3.0:
        # batches of 18 (C3's size, one launch and its queued restoration kernel) -- the same statuses and
        # iterations as the oracle
        s = dm.RmpcSolver(N=20, tol=1e-8, B_max=18)
        parts = [s.solve_batch(*(D[k][i:i + 18] for k in ("x0", "u_prev", "theta", "Rref", "prm")))
                 for i in range(0, 720, 18)]
        s.close()
        gs = {k: np.concatenate([p_[k] for p_ in parts]) for k in ("status", "iters", "u0")}
        assert np.array_equal(gs["status"], o["status"]), np.nonzero(gs["status"] != o["status"])
        assert np.mean(gs["iters"] == o["iters"]) >= 0.99
        dus = np.abs(gs["u0"] - o["u0"]).max(axis=1)
        assert np.max(dus[~inf]) <= 1e-6


def test_restoration_off_matches_oracle_without_restoration(dm):
    """restoration=False (IPOPT's phases off): a failed filter line search ends the solve at status -2, as the
    oracle with resto=False -- same statuses, iterations and controls."""
    from dart_mpc.workload import rmpc_batch
    D = _spread(rmpc_batch(4, seed0=0), 2.0)
    s = dm.RmpcSolver(N=20, tol=1e-8, B_max=256, restoration=False)
    g = s.solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"])
    s.close()
    off = oracle_lib.rmpc_solve_batch(D["x0"], D["u_prev"], D["theta"], D["Rref"], D["prm"], N=20, tol=1e-8,
                                      nthreads=8, resto=False)
    assert (off["status"] == -2).sum() >= 20
    assert np.array_equal(g["status"], off["status"])
    assert np.mean(g["iters"] == off["iters"]) >= 0.99, (g["iters"], off["iters"])
    ok = off["status"] == 0          # (where the line search fails, the iterate is ill-conditioned: ~1e-6 apart)
    assert np.max(np.abs(g["u0"][ok] - off["u0"][ok])) <= 1e-6


def test_restoration_with_fused_rls(dm):
    """The resume launch re-solves a handed-over instance from its start: with the RLS update fused, the
    estimate is updated once (by the first launch) and the re-solve reads it.  Fused = unfused with the
    updated estimate, on an infeasible batch."""
    from dart_mpc.workload import rmpc_batch
    D = _spread(rmpc_batch(1, seed0=5), 3.0)
    s = dm.RmpcSolver(N=20, tol=1e-8, B_max=32)
    fused = s.solve_batch(D["x0"], D["u_prev"], D["rls_theta"], D["Rref"], D["prm"], want_w=True,
                          rls_P=D["rls_P"], rls_phi=D["phi_prev"], rls_y=D["y"], rls_lambda=0.995)
    plain = s.solve_batch(D["x0"], D["u_prev"], fused["theta"], D["Rref"], D["prm"], want_w=True)
    s.close()
    assert (fused["status"] == 2).sum() >= 5
    B = D["x0"].shape[0]
    th_ref = np.zeros((B, 14))
    for b in range(B):
        for a in range(2):
            th_ref[b, 7 * a:7 * a + 7], _ = oracle_lib.rls_update(
                D["rls_theta"][b, 7 * a:7 * a + 7], D["rls_P"][b, a], D["phi_prev"][b], D["y"][b, a], 0.995)
    assert np.allclose(fused["theta"], th_ref, rtol=1e-12, atol=1e-12)
    assert np.array_equal(fused["status"], plain["status"]) and np.array_equal(fused["iters"], plain["iters"])
    assert np.max(np.abs(fused["w"] - plain["w"])) <= 1e-9


def test_closed_loop_leaving_the_velocity_cap(dm):
    """RMPCStep (rob_ctrl.py:331-352) on a plant that starts above the velocity cap (vx = 0.225, vy = -0.21,
    vmax = 0.2): the first nine solves are locally infeasible (status 2, IPOPT's restoration phase) and their
    iterate is the next step's warm start (np_mpc...:214-217); then the plant is back under the cap and the
    solves succeed (status 0) from those warm starts.  At every one of 25 steps the oracle chain (numpy RLS +
    C restatement with its own warm start) gets the same measurements and gives the same status and
    control."""
    from dart_mpc.rmpc import AdaptiveNPMPCSmooth, RMPCStep
    kw = dict(Ts=0.002, N=20, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0, u_bounds=(-0.6, 0.6), du_bounds=(-0.06, 0.06),
              vmax=0.2, v_eps=0.1)
    ctrl = AdaptiveNPMPCSmooth(None, None, tol=1e-8, max_iter=200, **kw)
    target = np.array([0.08, 0.0, -0.05, 0.0])
    x = np.array([0.0, 0.225, 0.0, -0.21]); xprev = x.copy(); up = np.zeros(2)
    step = RMPCStep(ctrl, target, r_v0=x.copy())
    truth = np.concatenate([[0, -1.0, 0, 0, -0.2, 0, 0], [0, 0, 0, -1.0, 0, -0.2, 0]])
    rls = [rmpc_nlp.RLS(7), rmpc_nlp.RLS(7)]
    r_v = x.copy(); w0 = np.zeros(_nw(20))
    seen = set()
    for k in range(25):
        u, _ = step(x, xprev, up)
        y = rmpc_nlp.rls_targets(x, xprev, 0.002)
        f = rmpc_nlp.rls_features(xprev, 0.1)
        rls[0].update(f, y[0]); rls[1].update(f, y[1])
        th = np.concatenate([rls[0].get(), rls[1].get()])
        assert np.allclose(step.theta, th, rtol=1e-9, atol=1e-9 * max(1.0, np.abs(th).max())), k
        r_v = rmpc_nlp.governor_step(r_v, target)
        R = rmpc_nlp.build_ref_traj(x, r_v, target, 20)
        o = oracle_lib.rmpc_solve_batch(x[None], up[None], step.theta[None], R[None], ctrl.params()[None], N=20,
                                        tol=1e-8, w_init=w0[None], max_iter=200)
        w0 = o["w"][0]
        seen.add(int(o["status"][0]))
        assert ctrl.last_status == int(o["status"][0]), (k, ctrl.last_status, o["status"][0])
        assert np.max(np.abs(u - o["u0"][0])) <= 1e-6, (k, u, o["u0"][0], o["status"][0])
        xprev, x = x, rmpc_nlp.rk4(x, u, truth, 0.1, 0.002)
        up = u
    assert seen == {0, 2}, seen
