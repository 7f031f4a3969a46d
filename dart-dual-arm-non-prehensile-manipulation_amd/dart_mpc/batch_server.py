"""One GPU process serving many simulations' MPC queues in batches.

The reference runs one ``mpc_worker`` process per simulation (PMPC/main_parallel_enhanced.py:200-207,
the worker at :22-55), so a sweep over object configurations and seeds runs as many CasADi/IPOPT
processes as simulations.  ``mpc_batch_server`` keeps every simulation's side of that protocol
unchanged -- the same ``(state, target)`` / ``"STOP"`` messages on its own ``state_queue`` and the same
``(u_cmd, loss, solve_time)`` replies on its own ``control_queue`` -- but one process drains all
pending requests into ONE batched solve (the resident GPU solver with in-place I/O,
``dart_mpc_serve_start`` / ``dart_mpc_bind``) and replies to each client.

Per client: one request is taken per round, so each client's replies stay in its request order
(FIFO), and a client that sends its next state only after the reply (the reference driver) is never
starved.  Clients may have different objects and weights (their ``params`` dicts, as passed to
``mpc_worker``); clients are grouped by (N, Ts), one GPU handle per group.  A client leaves with
``"STOP"``; the server returns when every client has left.

Waiting on many queues uses only their public API: one forwarding thread per client blocks in
``state_queue.get()`` and hands each message, stamped with its arrival time, to one in-process inbox.
The ``solve_time`` of a reply is that request's own time in the server, from its arrival to its reply
(the batch it waited for and the solve), the server-side counterpart of the worker's timed
``mpc.solve`` (:44-46).
"""
from __future__ import annotations

import queue
import threading
import time
from collections import deque

import numpy as np


def _prm_row(params):
    lo, hi = params.get("u_bounds", (-0.5, 0.5))
    return np.array([float(params.get("mu", 0.4)), float(params.get("Qp", 100.0)), float(params.get("Qv", 0.0)),
                     float(params.get("R", 0.1)), float(lo), float(hi)])


def mpc_batch_server(model_path, clients, idle_timeout=1.0, device=0, tol=1e-8, max_iter=3000,
                     solver_factory=None):
    """Serve ``clients`` = [(target_body, params, state_queue, control_queue), ...] until all stop.

    ``model_path`` and the target bodies are accepted for symmetry with ``mpc_worker``; the states
    arrive in the messages (the worker's inject-then-``get_state`` round trip, :47-52, returns the
    same vector).  Gravity is -9.81 (``model.opt.gravity[2]`` of the reference worlds).
    ``solver_factory(N, Ts, B_max)`` replaces the GPU handle (host-logic tests only).
    Returns the list of batch sizes it solved, in order."""
    if solver_factory is None:
        from ._lib import Solver

        def solver_factory(N, Ts, B_max):
            s = Solver(N=N, Ts=Ts, tol=tol, max_iter=max_iter, B_max=B_max, device=device)
            if N <= 31:                  # the resident grid serves N <= 31 (dart_mpc_serve_start)
                s.serve_start(B_serve=B_max, idle_timeout=idle_timeout)
            return s

    groups = {}         # (N, Ts) -> dict(solver, bound, clients)
    for i, (_body, params, _sq, _cq) in enumerate(clients):
        if int(params.get("nx", 6)) != 6 or int(params.get("nu", 2)) != 2:
            raise ValueError("PMPC dynamics are defined for nx=6, nu=2 only (mpc_3d.py:87-97)")
        key = (int(params.get("N", 20)), float(params.get("Ts", 0.002)))
        groups.setdefault(key, {"clients": []})["clients"].append(i)
    prm = [_prm_row(c[1]) for c in clients]
    for (N, Ts), g in groups.items():
        s = solver_factory(N, Ts, len(g["clients"]))
        g["solver"], g["bound"] = s, s.bind()

    inbox = queue.Queue()

    def forward(i, q):
        while True:
            item = q.get()
            inbox.put((i, item, time.perf_counter()))
            if isinstance(item, str) and item == "STOP":
                return

    for i, c in enumerate(clients):
        threading.Thread(target=forward, args=(i, c[2]), daemon=True, name=f"mpc-client-{i}").start()
    active = set(range(len(clients)))
    backlog = {i: deque() for i in active}       # arrived, not yet taken (one per client per round)
    sizes = []
    try:
        while active:
            if not any(backlog[i] for i in active):
                i, item, t = inbox.get()
                backlog[i].append((item, t))
            while True:
                try:
                    i, item, t = inbox.get_nowait()
                except queue.Empty:
                    break
                backlog[i].append((item, t))
            pending = {}
            for i in sorted(active):
                if not backlog[i]:
                    continue
                item, t = backlog[i].popleft()
                if isinstance(item, str) and item == "STOP":
                    active.discard(i)
                    continue
                pending[i] = (item, t)
            for g in groups.values():
                idx = [i for i in g["clients"] if i in pending]
                if not idx:
                    continue
                bd, B = g["bound"], len(idx)
                for r, i in enumerate(idx):
                    state, target = pending[i][0]
                    bd.x0[r] = state
                    bd.ref[r] = target
                    bd.prm[r] = prm[i]
                bd.solve(B)
                sizes.append(B)
                for r, i in enumerate(idx):
                    clients[i][3].put((bd.u0[r].copy(), np.array([bd.f[r]]), time.perf_counter() - pending[i][1]))
    finally:
        for g in groups.values():
            g["solver"].close()
    return sizes
