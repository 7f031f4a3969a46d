"""MPC worker process speaking the reference's queue protocol.

Drop-in for ``mpc_worker`` of PMPC/main_parallel_enhanced.py:22-55 (same
signature, same messages): it reads ``(state[6], target[6])`` or ``"STOP"``
from ``state_queue`` (FIFO, blocking, one reply per request) and writes
``(u_cmd[2], loss[1], solve_time)`` to ``control_queue``.  Start it with the
``spawn`` method (main_parallel_enhanced.py:106): the GPU context is created
inside the worker.

``model_path`` is accepted for signature compatibility; when MuJoCo is
importable the model's gravity is used (mpc_3d.py:23), otherwise it is ignored.
"""
from __future__ import annotations

import time

import numpy as np


def _gravity_from_model(model_path):
    if not model_path:
        return None
    try:
        import mujoco  # noqa: F401  (absent in this image)
    except Exception:
        return None
    try:
        return float(mujoco.MjModel.from_xml_path(model_path).opt.gravity[2])
    except Exception:
        return None


def mpc_worker(model_path, target_body, params, state_queue, control_queue):
    from .pmpc import PMPC

    params = dict(params)
    g = _gravity_from_model(model_path)

    class _Opt:                     # minimal stand-in exposing opt.gravity for the shim
        def __init__(self, gz):
            self.opt = type("opt", (), {"gravity": np.array([0.0, 0.0, gz])})()

    ctrl = PMPC(_Opt(g) if g is not None else None, None, **params)
    ctrl.target_body = target_body
    while True:
        item = state_queue.get()
        if isinstance(item, str) and item == "STOP":
            break
        state, target = item
        t0 = time.time()
        u_cmd, loss = ctrl.solve(target, state=np.asarray(state, float))
        solve_time = time.time() - t0
        control_queue.put((u_cmd, loss, solve_time))
