"""A minimal stand-in for ``mujoco.MjData`` body access, for running the reference's call form
``ctrl.solve(target)`` without MuJoCo.

The reference controllers read their state from ``data.body(name)`` (``PMPC.get_state``,
PMPC/src/controller/mpc_3d.py:106-113; ``AdaptiveNPMPCSmooth.get_state``,
RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py:195-198; ``RLMPC.get_state``,
LMPC/src/controller/rlmpc2.py:1034-1042), and ``mpc_worker`` writes the received state into
``data.body(ctrl.target_body).xpos`` / ``.cvel`` before calling ``ctrl.solve(target)``
(PMPC/main_parallel_enhanced.py:47-52).  ``BodyData`` keeps, per body name, the same fields as
MuJoCo's body view (``xpos[3]``, ``xmat[9]`` row-major, ``cvel[6]`` and ``cacc[6]`` as
[angular; linear]) as writable float64 arrays, so that code runs unchanged.  MuJoCo's own
``MjData`` can be passed wherever this is accepted.
"""
from __future__ import annotations

import numpy as np


class BodyView:
    """Writable per-body fields with MuJoCo's names and layouts."""

    __slots__ = ("name", "xpos", "xmat", "cvel", "cacc")

    def __init__(self, name):
        self.name = name
        self.xpos = np.zeros(3)
        self.xmat = np.eye(3).reshape(9)
        self.cvel = np.zeros(6)
        self.cacc = np.zeros(6)


class BodyData:
    """``data.body(name)`` returns the (created on first use) ``BodyView`` of that body."""

    def __init__(self, *names):
        self._bodies = {}
        for n in names:
            self.body(n)

    def body(self, name):
        v = self._bodies.get(name)
        if v is None:
            v = self._bodies[name] = BodyView(name)
        return v

    # -- helpers writing a controller's state vector into the body fields ------------------
    def set_pmpc_state(self, name, state):
        """[px, vx, py, vy, pz, vz] (the write of main_parallel_enhanced.py:48-49)."""
        b = self.body(name)
        b.xpos[:] = [state[0], state[2], state[4]]
        b.cvel[3:6] = [state[1], state[3], state[5]]

    def set_lmpc_state(self, name, state):
        """[px, vx, py, vy, theta_x, omega_x, theta_y, omega_y] (read back by rlmpc2.py:1034-1042):
        the body frame is the xyz Euler rotation (theta_x, theta_y, 0)."""
        b = self.body(name)
        b.xpos[:2] = [state[0], state[2]]
        b.cvel[3:5] = [state[1], state[3]]
        b.cvel[0:2] = [state[5], state[7]]
        cx, sx = np.cos(state[4]), np.sin(state[4])
        cy, sy = np.cos(state[6]), np.sin(state[6])
        # R = Rz(0) Ry(theta_y) Rx(theta_x) (scipy's extrinsic "xyz" = intrinsic z-y-x product)
        R = np.array([[cy, sy * sx, sy * cx],
                      [0.0, cx, -sx],
                      [-sy, cy * sx, cy * cx]])
        b.xmat[:] = R.reshape(9)
