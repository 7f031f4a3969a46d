"""Drop-in RMPC (regressor NMPC + online RLS) backed by the MI355X kernels.

Mirrors RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py:
  - ``RLS(p, theta0, P0, lam)`` with ``update(phi, y)`` / ``get()``         (:10-30)
  - ``AdaptiveNPMPCSmooth(model, data, Ts, nx, nu, N, Qp, Qv, Ru, Rdu, u_bounds,
    du_bounds, vmax, v_eps, target_body)`` with ``get_state()``,
    ``build_ref_traj`` (static) and ``solve(x0, u_prev, theta_hat, Rref_flat)``
    returning ``(U_opt[0], loss)`` and warm-starting from ``self.w0``          (:33-222)
plus the per-step driver logic of RMPC/dev_dual/rob_ctrl.py:331-352 as
``RMPCStep`` (RLS update fused into the solve launch) and ``solve_batch``.

All numerics of the solve and of the RLS update run in libdartmpc.so on the
GPU; the reference governor / staged reference are the driver's O(N) host
arithmetic, kept on the host as in the reference.
"""
from __future__ import annotations

import threading

import numpy as np

from ._lib import RmpcSolver, rls_update_batch

# Controllers with the same configuration share one handle.  The library serialises calls on a
# handle (its mutex, include/dart_mpc.h), so controllers on different threads stay correct; the
# cache itself is guarded here.
_SOLVERS = {}
_SOLVERS_LOCK = threading.Lock()


def _solver(N, Ts, tol, max_iter, device, gravity, B):
    key = (int(N), float(Ts), float(tol), int(max_iter), int(device), float(gravity))
    with _SOLVERS_LOCK:
        s = _SOLVERS.get(key)
        if s is None or s.cfg.B_max < B:
            s = RmpcSolver(N=N, Ts=Ts, tol=tol, max_iter=max_iter, B_max=max(B, 256), device=device, gravity=gravity)
            _SOLVERS[key] = s
        return s


class RLS:
    """Exponentially weighted recursive least squares, update on the GPU (np_mpc...:10-30)."""

    def __init__(self, p, theta0=None, P0=1e3, lam=0.995):
        if p != 7:
            raise ValueError("the GPU RLS filter is specialised to the reference's p = 7 features")
        self.p = p
        self.theta = np.zeros(p) if theta0 is None else np.asarray(theta0, float).copy()
        self.P = np.eye(p) * float(P0)
        self.lam = float(lam)

    def update(self, phi, y):
        th, P = rls_update_batch(self.theta[None], self.P[None], np.asarray(phi, float).reshape(1, 7),
                                 np.asarray([float(np.asarray(y).reshape(()))]), self.lam)
        self.theta, self.P = th[0], P[0]

    def get(self):
        return self.theta.copy()


class AdaptiveNPMPCSmooth:
    """Reference constructor (np_mpc...:35-38); rob_ctrl.py:281-284 uses N=20, Qp=80, Qv=2,
    Ru=0.02, Rdu=1.0, u_bounds=(-0.6,0.6), du_bounds=(-0.06,0.06), vmax=0.2, v_eps=0.1."""

    def __init__(self, model=None, data=None, Ts=0.002, nx=4, nu=2, N=20, Qp=100.0, Qv=1.0, Ru=0.05, Rdu=1.0,
                 u_bounds=(-0.4, 0.4), du_bounds=(-0.05, 0.05), vmax=0.25, v_eps=0.1, target_body="cube",
                 *, device=0, tol=1e-8, max_iter=200):
        if nx != 4 or nu != 2:
            raise ValueError("the regressor model is defined for nx=4, nu=2 (np_mpc...:178-186)")
        if not (1 <= int(N) <= 63):
            raise ValueError("horizon N must be in [1, 63]")
        self.model, self.data = model, data
        self.Ts = float(Ts)
        self.nx, self.nu, self.N = nx, nu, int(N)
        self.Qp, self.Qv, self.Ru, self.Rdu = float(Qp), float(Qv), float(Ru), float(Rdu)
        self.u_bounds, self.du_bounds = tuple(map(float, u_bounds)), tuple(map(float, du_bounds))
        self.vmax, self.v_eps = float(vmax), float(v_eps)
        self.target_body = target_body
        self.gz = float(model.opt.gravity[2]) if model is not None else -9.81        # :56
        self.px = self.py = 7
        self.p_total = 14
        self.tol, self.max_iter, self.device = float(tol), int(max_iter), int(device)
        self.nw = self.nx * (self.N + 1) + self.nu * self.N
        self.w0 = np.zeros(self.nw)                                                   # :168
        self.last_status = None
        self.last_iters = None

    def params(self):
        return np.array([self.Qp, self.Qv, self.Ru, self.Rdu, *self.u_bounds, *self.du_bounds, self.vmax, self.v_eps])

    def _engine(self, B):
        return _solver(self.N, self.Ts, self.tol, self.max_iter, self.device, self.gz, B)

    def get_state(self):
        """[px, vx, py, vy] of ``target_body`` (np_mpc...:195-198)."""
        if self.data is None:
            raise RuntimeError("get_state() needs MuJoCo data")
        pos = self.data.body(self.target_body).xpos[:2]
        vxy = self.data.body(self.target_body).cvel[3:5]
        return np.array([pos[0], vxy[0], pos[1], vxy[1]], dtype=float)

    @staticmethod
    def build_ref_traj(x_now, r_v, target, N, nx, step_fraction=0.2):
        """Staged reference from r_v toward target (np_mpc...:201-210)."""
        R = np.zeros(((N + 1), nx), dtype=float)
        for i in range(N + 1):
            w = 1.0 - (1.0 - step_fraction) ** (i + 1)
            r_i = np.asarray(r_v) + w * (np.asarray(target) - np.asarray(r_v))
            R[i, :] = np.array([r_i[0], 0.0, r_i[2], 0.0])
        return R.reshape(-1)

    def solve(self, x0, u_prev, theta_hat, Rref_flat):
        """np_mpc...:212-222: warm start from w0, returns (U_opt[0], loss)."""
        out = self._engine(1).solve_batch(np.asarray(x0, float)[None], np.asarray(u_prev, float)[None],
                                          np.asarray(theta_hat, float)[None], np.asarray(Rref_flat, float)[None],
                                          self.params()[None], w_warm=self.w0[None], want_w=True)
        self.w0 = out["w"][0]
        self.last_status = int(out["status"][0])
        self.last_iters = int(out["iters"][0])
        return out["u0"][0].copy(), np.array([out["f"][0]])

    def solve_batch(self, x0, u_prev, theta, Rref, params=None, w_warm=None, want_w=False, rls=None):
        """B instances in one launch; ``rls`` = dict(P=[B,2,7,7], phi=[B,7], y=[B,2], lam) fuses the
        RLS update (theta is then the RLS estimate and is updated)."""
        x0 = np.asarray(x0, float).reshape(-1, 4)
        B = x0.shape[0]
        prm = np.tile(self.params(), (B, 1)) if params is None else np.asarray(params, float).reshape(B, 10)
        kw = {}
        if rls is not None:
            kw = dict(rls_P=rls["P"], rls_phi=rls["phi"], rls_y=rls["y"], rls_lambda=rls.get("lam", 0.995))
        return self._engine(B).solve_batch(x0, u_prev, theta, Rref, prm, w_warm=w_warm, want_w=want_w, **kw)


def rls_features(prev_state, v_eps):
    """phi_prev (rob_ctrl.py:338-339)."""
    return np.array([prev_state[0], prev_state[1], prev_state[2], prev_state[3],
                     np.tanh(prev_state[1] / v_eps), np.tanh(prev_state[3] / v_eps), 1.0])


class RMPCStep:
    """One control step of RMPC/dev_dual/rob_ctrl.py:331-352 with the two RLS updates fused
    into the solve launch: features/targets (:335-339), RLS (:340-343), reference governor
    (:346-348), staged reference (:351), warm-started solve (:352)."""

    def __init__(self, ctrl: AdaptiveNPMPCSmooth, target, r_v0, dr_max=0.01, alpha_rg=0.5, P0=1e3, lam=0.995):
        self.ctrl = ctrl
        self.target = np.asarray(target, float)
        self.r_v = np.asarray(r_v0, float).copy()
        self.dr_max, self.alpha_rg, self.lam = dr_max, alpha_rg, lam
        self.theta = np.zeros(14)
        self.P = np.stack([np.eye(7) * P0, np.eye(7) * P0])

    def __call__(self, xk, prev_state, u_prev):
        Ts, c = self.ctrl.Ts, self.ctrl
        y = np.array([(xk[1] - prev_state[1]) / Ts, (xk[3] - prev_state[3]) / Ts])
        phi = rls_features(prev_state, c.v_eps)
        err = np.array([self.target[0] - self.r_v[0], 0.0, self.target[2] - self.r_v[2], 0.0])
        step = np.array([np.clip(err[0], -self.dr_max, self.dr_max), 0.0, np.clip(err[2], -self.dr_max, self.dr_max), 0.0])
        self.r_v = self.r_v + self.alpha_rg * step
        Rref = c.build_ref_traj(xk, self.r_v, self.target, c.N, c.nx, step_fraction=0.2)
        out = c._engine(1).solve_batch(np.asarray(xk, float)[None], np.asarray(u_prev, float)[None], self.theta[None],
                                       Rref[None], c.params()[None], w_warm=c.w0[None], want_w=True,
                                       rls_P=self.P[None], rls_phi=phi[None], rls_y=y[None], rls_lambda=self.lam)
        self.theta, self.P = out["theta"][0], out["rls_P"][0]
        c.w0 = out["w"][0]          # whatever the status (np_mpc...:214-217: an infeasible start's iterate too)
        c.last_status = int(out["status"][0])
        c.last_iters = int(out["iters"][0])
        return out["u0"][0].copy(), np.array([out["f"][0]])
