"""The resident PMPC solver (dart_mpc_serve_start): one long-lived grid takes requests from a mailbox
in mapped host memory.  Its answers must be bit-identical to ordinary launches (the same solve code),
for every scan instantiation (N = 15 one-row, 20 SHORT2, 24 full scan), for batches smaller than the
grid, with a warm start and with w_out; it must leave on stop, drain by itself after the idle timeout
(and be restarted transparently by the next call), and serve two threads sharing the handle."""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N", [15, 20, 24])
def test_served_equals_launched(N):
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(4)
    ref = dart_mpc.Solver(N=N, tol=1e-8, B_max=18)
    expect = [ref.solve_batch(S[i:i + 18], T[i:i + 18], P[i:i + 18], want_w=True) for i in range(0, 72, 18)]
    one = ref.solve_batch(S[5:6], T[5:6], P[5:6])
    ref.close()
    with dart_mpc.Solver(N=N, tol=1e-8, B_max=18) as s:
        s.serve_start(B_serve=18, idle_timeout=5.0)
        assert s.serving()
        for rep in range(3):
            for j, i in enumerate(range(0, 72, 18)):
                got = s.solve_batch(S[i:i + 18], T[i:i + 18], P[i:i + 18], want_w=(rep == 0))
                for k in ("u0", "f", "status", "iters"):
                    np.testing.assert_array_equal(got[k], expect[j][k], err_msg=f"{N} {rep} {i} {k}")
                if rep == 0:
                    np.testing.assert_array_equal(got["w"], expect[j]["w"])
        got1 = s.solve_batch(S[5:6], T[5:6], P[5:6])
        for k in ("u0", "f", "status", "iters"):
            np.testing.assert_array_equal(got1[k], one[k])
        # warm start through the mailbox flags: from the optimum, one or two iterations
        w = expect[0]["w"]
        warm = s.solve_batch(S[:18], T[:18], P[:18], w_warm=w)
        assert np.all(warm["status"] == 0) and warm["iters"].mean() < expect[0]["iters"].mean()
        assert s.serving()
        s.serve_stop()
        assert not s.serving()
        again = s.solve_batch(S[:18], T[:18], P[:18])            # an ordinary launch again
        np.testing.assert_array_equal(again["u0"], expect[0]["u0"])


def test_short_idle_timeout_serves_from_the_grid():
    """An idle timeout of a few ms (the host's pre-drain margin is at most half of it): back-to-back requests
    are answered by the resident grid -- the same results as launches -- and it is still resident after them."""
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(1)
    with dart_mpc.Solver(N=20, tol=1e-8, B_max=18) as s:
        base = s.solve_batch(S, T, P)
        s.serve_start(B_serve=18, idle_timeout=0.004)
        for _ in range(20):
            got = s.solve_batch(S, T, P)
            for k in ("u0", "f", "status", "iters"):
                np.testing.assert_array_equal(got[k], base[k])
        assert s.serving()
        s.serve_stop()


def test_requests_spaced_near_half_a_short_idle_timeout():
    """Requests spaced ~0.45 of a short idle timeout apart: the host's pre-drain margin is at
    least 2 ms, so whether a request is served from the grid or after a host-side drain and relaunch, its
    results equal a launch's and it never waits out a further idle period."""
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(1)
    with dart_mpc.Solver(N=20, tol=1e-8, B_max=18) as s:
        base = s.solve_batch(S, T, P)
        for idle in (0.004, 0.01):
            s.serve_start(B_serve=18, idle_timeout=idle)
            worst = 0.0
            for _ in range(12):
                time.sleep(0.45 * idle)
                t0 = time.perf_counter()
                got = s.solve_batch(S, T, P)
                worst = max(worst, time.perf_counter() - t0)
                for k in ("u0", "f", "status", "iters"):
                    np.testing.assert_array_equal(got[k], base[k])
            assert worst < 0.05, (idle, worst)
            s.serve_stop()


def test_idle_timeout_drains_and_restarts():
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(1)
    with dart_mpc.Solver(N=20, tol=1e-8, B_max=18) as s:
        base = s.solve_batch(S, T, P)
        s.serve_start(B_serve=18, idle_timeout=0.2)
        np.testing.assert_array_equal(s.solve_batch(S, T, P)["u0"], base["u0"])
        time.sleep(0.6)
        assert not s.serving()                                     # the grid has drained by itself
        np.testing.assert_array_equal(s.solve_batch(S, T, P)["u0"], base["u0"])   # served after a relaunch
        assert s.serving()
        s.serve_stop()


def test_requests_near_the_idle_timeout():
    """Requests posted around the idle timeout (0.2 s) -- where part of the grid may have left on its own
    clock while the rest still waits -- are answered promptly and correctly: the host drains and relaunches
    the grid itself from 90 % of the timeout on, so no request meets a partly drained grid and waits out a
    further idle period."""
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(1)
    with dart_mpc.Solver(N=20, tol=1e-8, B_max=18) as s:
        base = s.solve_batch(S, T, P)
        s.serve_start(B_serve=18, idle_timeout=0.2)
        worst = 0.0
        for gap in (0.15, 0.17, 0.178, 0.182, 0.19, 0.195, 0.2, 0.205, 0.21, 0.22, 0.3):
            time.sleep(gap)
            t0 = time.perf_counter()
            got = s.solve_batch(S, T, P)
            worst = max(worst, time.perf_counter() - t0)
            np.testing.assert_array_equal(got["u0"], base["u0"])
            np.testing.assert_array_equal(got["iters"], base["iters"])
        assert worst < 0.1, worst          # a request that waited for a partly drained grid takes >= 0.2 s
        s.serve_stop()


def test_two_threads_share_a_served_handle():
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(2)
    with dart_mpc.Solver(N=20, tol=1e-8, B_max=18) as s:
        base = [s.solve_one(S[i], T[i], P[i])[0] for i in range(36)]
        s.serve_start(B_serve=4, idle_timeout=5.0)
        bad = []

        def run(t):
            for rep in range(20):
                for i in range(t, 36, 2):
                    u = s.solve_one(S[i], T[i], P[i])[0]
                    if not np.array_equal(u, base[i]):
                        bad.append((t, rep, i))

        th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not bad, bad[:5]
        s.serve_stop()


@pytest.mark.parametrize("serve", [False, True])
def test_bound_in_place_io(serve):
    """dart_mpc_bind / dart_mpc_solve_bound: inputs written in place into the mapped I/O area, results read
    from it; the same answers as solve_batch, with a launch per call and served, incl. w_warm / w_out."""
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(2)
    with dart_mpc.Solver(N=20, tol=1e-8, B_max=36) as s:
        ref = s.solve_batch(S, T, P, want_w=True)
        if serve:
            s.serve_start(B_serve=36, idle_timeout=5.0)
        b = s.bind()
        for B in (36, 7, 1):
            b.x0[:B] = S[:B]; b.ref[:B] = T[:B]; b.prm[:B] = P[:B]
            b.solve(B, want_w=True)
            np.testing.assert_array_equal(b.u0[:B], ref["u0"][:B])
            np.testing.assert_array_equal(b.f[:B], ref["f"][:B])
            np.testing.assert_array_equal(b.iters[:B], ref["iters"][:B])
            np.testing.assert_array_equal(b.w_out[:B], ref["w"][:B])
        b.w_warm[:36] = ref["w"]
        b.x0[:36] = S; b.ref[:36] = T; b.prm[:36] = P
        b.solve(36, w_warm=True)
        assert np.all(b.status[:36] == 0) and b.iters[:36].mean() < ref["iters"].mean()
        assert s.serving() == serve
