"""RLMPCAsync with the real GPU workers (dart_mpc.lmpc_shm): the solver process answers the
front-end through shared memory with plans that solve the NLP of the inputs it read, and the
policy process moves model_params through the reference's EMA + soft clip."""
import time

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu


def test_async_front_end_with_gpu_workers():
    from dart_mpc.lmpc_shm import RLMPCAsync
    state = np.array([0.03, 0.0, -0.02, 0.0, 0.01, 0.0, -0.01, 0.0])
    target = np.array([0.1, 0, -0.05, 0, 0, 0, 0, 0])
    with RLMPCAsync(params=dict(N=20), seed=3) as c:
        p0 = c.views["model_params"].copy()
        fresh = 0
        for _ in range(40):
            c.solve(target, state=state)
            if c.wait_solution(60.0):
                u, loss = c.solve(target, state=state)
                fresh += 1
                assert np.all(np.abs(u) <= 0.4 + 1e-6) and np.isfinite(loss).all()
            time.sleep(0.01)
        assert fresh >= 10
        time.sleep(0.1)
        # the inputs of the solver's most recent solves: state, target, control (u_prev), params
        c.events["terminate"].set()
        for pr in c.procs:
            pr.join(timeout=30)
        st, tg = c.views["state"].copy(), c.views["target"].copy()
        up, pv = c.views["control"].copy(), c.views["model_params"].copy()
        w = c.views["w_opt"].copy()
        assert not np.allclose(pv, p0)                  # the policy process wrote new parameters
        assert np.all((pv > 1e-2) & (pv < 2.0 - 0.1))    # inside the soft-clip band (:606-616)
    # the published plan solves the NLP of those inputs to the reference's loose tolerance
    # (tol 1e-4, acceptable 1e-3): u0 within 5e-3 of the exact optimum, as tests/test_gpu_lmpc.py
    ref = oracle_lib.lmpc_solve_batch(st[None], up[None], pv[None], tg[None], N=20, tol=1e-11, acc_iter=0,
                                      max_iter=500, nthreads=1)
    if ref["status"][0] == 0:
        nX = 8 * 21
        assert np.max(np.abs(w[nX:nX + 2] - ref["u0"][0])) <= 5e-3
