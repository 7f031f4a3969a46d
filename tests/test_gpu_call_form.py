"""The reference's own call form: ``ctrl.solve(target)`` with the state read from ``data`` (PMPC
mpc_3d.py:115-123 via get_state :106-113; AdaptiveNPMPCSmooth via get_state np_mpc...:195-198 and
solve :212-222; RLMPC.solve rlmpc2.py:986-988 via get_state :1034-1042), here with the MjData
stand-in dart_mpc.BodyData.  Each must equal the explicit-state form and the oracle, and
reassigning ``target_body`` (main_parallel_enhanced.py:41) must switch the body that is read."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_pmpc_solve_reads_state_from_data():
    import dart_mpc
    import oracle_lib
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(1)
    data = dart_mpc.BodyData()
    data.set_pmpc_state("cube", S[0])
    data.set_pmpc_state("sphere", S[1])
    mu, qp, qv, r, lo, hi = P[0]
    c = dart_mpc.PMPC(None, data, Ts=0.002, N=20, Qp=qp, Qv=qv, R=r, mu=mu, u_bounds=(lo, hi))
    u, loss = c.solve(T[0])
    u_s, loss_s = c.solve(T[0], state=S[0])
    np.testing.assert_array_equal(u, u_s)
    np.testing.assert_array_equal(loss, loss_s)
    ref = oracle_lib.solve_batch(S[:2], np.stack([T[0], T[0]]), np.tile(P[0], (2, 1)), N=20, tol=1e-8)
    assert np.max(np.abs(u - ref["u0"][0])) <= 1e-6
    c.target_body = "sphere"
    u2, _ = c.solve(T[0])
    np.testing.assert_array_equal(u2, c.solve(T[0], state=S[1])[0])
    assert np.max(np.abs(u2 - ref["u0"][1])) <= 1e-6


def test_worker_injects_state_into_data():
    """mpc_worker writes each received state into data.body(target_body) and calls solve(target)
    (main_parallel_enhanced.py:47-52); run in-process with plain queues."""
    import queue
    import dart_mpc
    import oracle_lib
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(1)
    sq, cq = queue.Queue(), queue.Queue()
    params = dict(Ts=0.002, nx=6, nu=2, N=15, Qp=600, Qv=5, R=0.1, u_bounds=(-0.6, 0.6), mu=0.1)
    for i in range(4):
        sq.put((S[i], T[i]))
    sq.put("STOP")
    dart_mpc.mpc_worker("unused.xml", "sphere", params, sq, cq)
    ref = oracle_lib.solve_batch(S[:4], T[:4], np.tile([0.1, 600, 5, 0.1, -0.6, 0.6], (4, 1)), N=15, tol=1e-8)
    for i in range(4):
        u, loss, t = cq.get_nowait()
        assert np.max(np.abs(u - ref["u0"][i])) <= 1e-6 and loss.shape == (1,) and t >= 0.0


def test_rmpc_get_state_call_form():
    import dart_mpc
    from dart_mpc.workload import rmpc_batch
    D = rmpc_batch(1)
    data = dart_mpc.BodyData()
    x0 = D["x0"][0]
    data.set_pmpc_state("cube", [x0[0], x0[1], x0[2], x0[3], 0.43, 0.0])
    kw = dict(Ts=0.002, N=20, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0, u_bounds=(-0.6, 0.6), du_bounds=(-0.06, 0.06),
              vmax=0.2, v_eps=0.1)
    a = dart_mpc.AdaptiveNPMPCSmooth(None, data, **kw)
    b = dart_mpc.AdaptiveNPMPCSmooth(None, None, **kw)
    for step in range(3):                        # warm-started from w0 after the first call
        ua, la = a.solve(a.get_state(), D["u_prev"][0], D["theta"][0], D["Rref"][0])
        ub, lb = b.solve(x0, D["u_prev"][0], D["theta"][0], D["Rref"][0])
        np.testing.assert_array_equal(ua, ub)
        np.testing.assert_array_equal(la, lb)


def test_rlmpc_solve_reads_state_from_data():
    import dart_mpc
    rng = np.random.default_rng(11)
    data = dart_mpc.BodyData()
    a = dart_mpc.RLMPC(None, data, dict(N=20), seed=5)
    b = dart_mpc.RLMPC(None, None, dict(N=20), seed=5)
    target = np.array([0.1, 0, -0.05, 0, 0, 0, 0, 0])
    for step in range(4):
        s = np.array([*rng.uniform(-0.1, 0.1, 4), *rng.uniform(-0.05, 0.05, 4)])
        data.set_lmpc_state(a.params["body_name"], s)
        ua, la = a.solve(target)
        ub, lb = b.solve(target, state=a.get_state())
        np.testing.assert_array_equal(ua, ub)
        np.testing.assert_array_equal(la, lb)
        np.testing.assert_allclose(a.get_state(), s, atol=1e-14)
