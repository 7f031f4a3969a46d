"""Shared-memory / Event protocol of the LMPC front-end (dart_mpc.lmpc_shm, rlmpc2.py:110-164,
494-524, 986-1021) on CPU: a stand-in solver worker (tests/lmpc_fake_worker.py) publishes plans
that encode the state it read, so every reply of the non-blocking front-end can be attributed to a
fresh plan, a shift of the previous plan, or the held control."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def test_front_end_takes_fresh_plans_and_shifts_stale_ones():
    from dart_mpc.lmpc_shm import RLMPCAsync, shm_shapes
    import lmpc_fake_worker
    N = 6
    c = RLMPCAsync(params=dict(N=N), policy=False, solver_worker=lmpc_fake_worker.fake_solver)
    try:
        assert set(c.views) == set(shm_shapes(8, 2, N))
        assert c.views["w_opt"].shape == (8 * (N + 1) + 2 * N,)
        tgt = np.array([0.1, 0, -0.05, 0, 0, 0, 0, 0])
        s = np.zeros(8); s[0] = 1.0
        u, _ = c.solve(tgt, state=s)
        # the worker cannot have answered yet, or it answered this very state
        assert np.allclose(u, 0.0) or np.allclose(u, [1.0, 0.0])
        np.testing.assert_array_equal(c.views["state"], s)
        np.testing.assert_array_equal(c.views["target"], tgt)
        assert c.wait_solution(20.0)
        u, loss = c.solve(tgt, state=s)                 # fresh plan: U[0]
        np.testing.assert_allclose(u, [1.0, 0.0])
        np.testing.assert_allclose(loss, [1.0])
        np.testing.assert_array_equal(c.views["control"], u)
        for k in (1, 2, 3):                             # same state: no new plan, shift (:1013-1018)
            time.sleep(0.05)
            u, _ = c.solve(tgt, state=s)
            np.testing.assert_allclose(u, [1.0 + k, -k])
        s2 = s.copy(); s2[0] = 5.0
        c.solve(tgt, state=s2)
        assert c.wait_solution(20.0)
        u, _ = c.solve(tgt, state=s2)
        np.testing.assert_allclose(u, [5.0, 0.0])
        for _ in range(N + 2):                          # a plan shifted to its last node is held
            time.sleep(0.02)
            u, _ = c.solve(tgt, state=s2)
        np.testing.assert_allclose(u, [5.0 + N - 1, -(N - 1)])
        assert c.views["RLstatus"][0] == 2
    finally:
        names = list(c.shm_names.values())
        c.close()
    assert all(not p.is_alive() for p in c.procs)
    from multiprocessing import shared_memory
    for n in names:                                     # segments unlinked
        try:
            shared_memory.SharedMemory(name=n).close()
            raise AssertionError(f"{n} still exists")
        except FileNotFoundError:
            pass


def test_write_params_is_the_reference_ema_and_soft_clip():
    from dart_mpc.lmpc_shm import write_params
    prev = np.linspace(0.0, 2.0, 34)
    k = np.linspace(2.0, 0.0, 34)
    out = write_params(prev, k, 1e-2, 2.0, 0.1)
    sm = 0.5 * k + 0.5 * prev                           # rlmpc2.py:606-616
    c, s = (1.9 + 1e-2) / 2, (1.9 - 1e-2) / 2 - 1e-3
    np.testing.assert_allclose(out, c + s * np.tanh((sm - c) / s), rtol=0, atol=1e-15)
    assert np.all(out > 1e-2) and np.all(out < 1.9)
