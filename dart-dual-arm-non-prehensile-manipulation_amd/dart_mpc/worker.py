"""MPC worker process speaking the reference's queue protocol.

Drop-in for ``mpc_worker`` of PMPC/main_parallel_enhanced.py:22-55 (same
signature, same messages): it reads ``(state[6], target[6])`` or ``"STOP"``
from ``state_queue`` (FIFO, blocking, one reply per request) and writes
``(u_cmd[2], loss[1], solve_time)`` to ``control_queue``.  Start it with the
``spawn`` method (main_parallel_enhanced.py:106): the GPU context is created
inside the worker.

The loop is the reference's: the received state is written into
``data.body(ctrl.target_body).xpos / .cvel`` and ``ctrl.solve(target)`` reads
it back through ``get_state`` (main_parallel_enhanced.py:47-52).  When MuJoCo
is importable the model (its gravity, mpc_3d.py:23) and ``MjData`` come from
``model_path``; otherwise ``data`` is a ``dart_mpc.mjdata.BodyData`` and
``model_path`` is ignored.
"""
from __future__ import annotations

import time

import numpy as np


def _mujoco_model(model_path):
    """(model, MjData) from the xml when MuJoCo is importable, else (None, None)."""
    if not model_path:
        return None, None
    try:
        import mujoco  # absent in this image
        model = mujoco.MjModel.from_xml_path(model_path)
        return model, mujoco.MjData(model)
    except Exception:
        return None, None


def mpc_worker(model_path, target_body, params, state_queue, control_queue):
    from .mjdata import BodyData
    from .pmpc import PMPC

    model, data = _mujoco_model(model_path)
    if data is None:
        data = BodyData(target_body)
    ctrl = PMPC(model, data, **dict(params))
    ctrl.target_body = target_body                                      # main_parallel_enhanced.py:41
    while True:
        item = state_queue.get()
        if isinstance(item, str) and item == "STOP":
            break
        state, target = item
        data.body(ctrl.target_body).xpos[:] = [state[0], state[2], state[4]]      # :48
        data.body(ctrl.target_body).cvel[3:6] = [state[1], state[3], state[5]]    # :49
        t0 = time.time()
        u_cmd, loss = ctrl.solve(np.asarray(target, float))
        solve_time = time.time() - t0
        control_queue.put((u_cmd, loss, solve_time))
