"""Drop-in PMPC controller backed by the MI355X batched interior-point kernel.

Mirrors ``PMPC`` of PMPC/src/controller/mpc_3d.py:11-138 (same constructor
keywords, ``target_body`` attribute, ``get_state()``, ``solve(target) ->
(u_cmd[2], loss[1])``, ``w0``), and adds the batch/step API the north star
asks for: ``step(state, target) -> tilt_cmd`` and ``solve_batch``.

``model``/``data`` are optional: MuJoCo is only used, as in the reference, to
read ``model.opt.gravity[2]`` (mpc_3d.py:23) and the object state
(mpc_3d.py:106-113).  All numerics run in libdartmpc.so on the GPU.
"""
from __future__ import annotations

import threading

import numpy as np

from ._lib import Solver

# Controllers with the same configuration share one handle.  The library serialises calls on a
# handle (its mutex, include/dart_mpc.h), so controllers on different threads stay correct; the
# cache itself is guarded here.
_SOLVERS = {}
_SOLVERS_LOCK = threading.Lock()


def _solver(N, Ts, tol, max_iter, device, gravity, B_max, path="ipopt"):
    key = (int(N), float(Ts), float(tol), int(max_iter), int(device), float(gravity), path)
    with _SOLVERS_LOCK:
        s = _SOLVERS.get(key)
        if s is None or s.cfg.B_max < B_max:
            s = Solver(N=N, Ts=Ts, tol=tol, max_iter=max_iter, B_max=max(B_max, 1024), device=device, gravity=gravity,
                       path=path)
            _SOLVERS[key] = s
        return s


class PMPC:
    """Tray-tilt NMPC, reference constructor signature (mpc_3d.py:12)."""

    def __init__(self, model=None, data=None, Ts=0.002, nx=6, nu=2, N=20, Qp=100, Qv=0, R=0.1, mu=0.4,
                 u_bounds=(-0.5, 0.5), *, device=0, tol=1e-8, max_iter=3000, path="ipopt"):
        if nx != 6 or nu != 2:
            # the reference dynamics (mpc_3d.py:87-97) are hard-wired to 6 states / 2 tilts
            raise ValueError("PMPC dynamics are defined for nx=6, nu=2 only (mpc_3d.py:87-97)")
        if not (1 <= int(N) <= 63):
            raise ValueError("horizon N must be in [1, 63]")
        if not (u_bounds[1] > u_bounds[0]):
            raise ValueError("u_bounds must satisfy lower < upper")
        self.model = model
        self.data = data
        self.Ts = float(Ts)
        self.nx, self.nu, self.N = nx, nu, int(N)
        self.Qp, self.Qv, self.R, self.mu = float(Qp), float(Qv), float(R), float(mu)
        self.g = float(model.opt.gravity[2]) if model is not None else -9.81     # mpc_3d.py:23
        self.h_cube = 0.1
        self.u_bounds = (float(u_bounds[0]), float(u_bounds[1]))
        self.target_body = "cube"                                                # mpc_3d.py:26
        self.tol, self.max_iter, self.device = float(tol), int(max_iter), int(device)
        if path not in Solver.PATHS:
            raise ValueError(f"path must be one of {sorted(Solver.PATHS)}")
        self.path = path          # "ipopt": IPOPT's iterates (default); "reduced": the faster opt-in
        self.nw = self.nx * (self.N + 1) + self.nu * self.N
        self.w0 = np.zeros(self.nw)                                              # mpc_3d.py:85
        self.lbx = [-np.inf] * (self.nx * (self.N + 1)) + [self.u_bounds[0]] * (self.nu * self.N)
        self.ubx = [np.inf] * (self.nx * (self.N + 1)) + [self.u_bounds[1]] * (self.nu * self.N)
        self.last_status = None
        self.last_iters = None

    # -- parameter row of the C ABI -----------------------------------------
    @property
    def _prm(self):
        return np.array([self.mu, self.Qp, self.Qv, self.R, self.u_bounds[0], self.u_bounds[1]])

    def params(self):
        return np.array([self.mu, self.Qp, self.Qv, self.R, self.u_bounds[0], self.u_bounds[1]])

    def _engine(self, B):
        return _solver(self.N, self.Ts, self.tol, self.max_iter, self.device, self.g, B, self.path)

    # -- reference API --------------------------------------------------------
    def get_state(self):
        """[px, vx, py, vy, pz, vz] of ``target_body`` (mpc_3d.py:106-113)."""
        if self.data is None:
            raise RuntimeError("get_state() needs MuJoCo data; use step(state, target) instead")
        pos = self.data.body(self.target_body).xpos
        vel = self.data.body(self.target_body).cvel[3:6]
        return np.array([pos[0], vel[0], pos[1], vel[1], pos[2], vel[2]])

    def solve(self, target, state=None):
        """Reference semantics (mpc_3d.py:115-138): cold start, returns (U_opt[0], loss)."""
        x = self.get_state() if state is None else state
        u, f, st, it, w = self._engine(1).solve_one(x, target, self._prm, want_w=True)
        self.w0 = w                                                              # mpc_3d.py:135
        self.last_status, self.last_iters = st, it
        return u, np.array([f])

    # -- new API ----------------------------------------------------------------
    def step(self, state, target):
        """mpc.step(state, target) -> tilt_cmd[2] (north-star interface)."""
        u, _ = self.solve(target, state=state)
        return u

    def solve_batch(self, states, targets, params=None, w_warm=None, want_w=False):
        """Solve B independent instances in one launch.  ``params`` rows are
        [mu, Qp, Qv, R, u_lo, u_hi]; default: this controller's own row."""
        states = np.asarray(states, float).reshape(-1, 6)
        B = states.shape[0]
        prm = np.tile(self.params(), (B, 1)) if params is None else np.asarray(params, float).reshape(B, 6)
        return self._engine(B).solve_batch(states, np.asarray(targets, float).reshape(B, 6), prm,
                                           w_warm=w_warm, want_w=want_w)


def tilt_to_quat(u_cmd):
    """Tilt command -> MuJoCo (w,x,y,z) quaternion of the tray, Euler xyz
    [u1, -u0, 0] (PMPC/main_parallel_enhanced.py:333-348)."""
    angles = np.array([u_cmd[1], -u_cmd[0], 0.0])
    cx, cy, cz = np.cos(angles / 2.0)
    sx, sy, sz = np.sin(angles / 2.0)
    return np.array([cx * cy * cz + sx * sy * sz,
                     sx * cy * cz - cx * sy * sz,
                     cx * sy * cz + sx * cy * sz,
                     cx * cy * sz - sx * sy * cz])
