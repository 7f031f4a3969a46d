"""Stand-in LMPC solver worker for the CPU protocol test of dart_mpc.lmpc_shm (no GPU).

It speaks the worker side of rlmpc2.py:494-524 (wait on state_ready with a 10 ms timeout, clear
it, publish w_opt / loss, set ctrl_ready) but "solves" by writing a plan that encodes the state it
read: U[k] = [state[0] + k, -k].  It publishes only when the state changed since its last plan, so
a test can tell a fresh plan from the front-end's shifting of the previous one."""
import numpy as np

from dart_mpc.lmpc_shm import _attach, _detach


def fake_solver(shm_names, events, packet, shapes):
    shms, views = _attach(shm_names, shapes)
    N, nx, nu = int(packet["N"]), int(packet["nx"]), int(packet["nu"])
    last = None
    try:
        while True:
            events["state_ready"].wait(timeout=0.01)
            if events["terminate"].is_set():
                break
            events["state_ready"].clear()
            s = views["state"].copy()
            if last is not None and np.array_equal(s, last):
                continue
            last = s
            w = np.zeros(shapes["w_opt"])
            U = np.stack([s[0] + np.arange(N), -np.arange(N, dtype=float)], axis=1)
            w[nx * (N + 1):] = U.reshape(-1)
            views["w_opt"][:] = w
            views["loss"][:] = s[0]
            views["RLstatus"][0] += 1          # number of plans published (test bookkeeping)
            events["ctrl_ready"].set()
    finally:
        _detach(shms)
