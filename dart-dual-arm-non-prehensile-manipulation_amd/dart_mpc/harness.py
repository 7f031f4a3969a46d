"""Headless closed-loop harness and the reference's result formats.

The reference evaluates its controllers end to end in MuJoCo (PMPC/main_parallel_enhanced.py:290-419,
RMPC/dev_dual/rob_ctrl.py:331-420) and writes
  * PMPC / LMPC: one ``.npz`` per experiment with the per-step logs of AsyncLogger
    (PMPC/src/logger.py:90-111) plus three metrics (:158-183): steady-state error, convergence
    time (first step with error < 1 cm) and control effort (sum |U_cmd| dt);
  * RMPC: a JSON file ``{"data": {"ep1": {"pos_err", "pos_err_norm", "u_cmd", "torque",
    "timestep"}}}`` (rob_ctrl.py:51-86), one episode per run until the 1 cm tolerance is reached.

MuJoCo is not part of this package.  ``TrayPlant`` is a batched stand-in for the scene: the tray tilt
follows the commanded tilt through a first-order lag (the arms' impedance tracking), and the object
obeys the reference model (mpc_3d.py:87-97) driven by the *actual* tilt plus a Coulomb friction term
the MPC model does not have -- so the loop sees model mismatch, as the reference's does.  Many
experiments (object configs, targets) run in lock step: one batched GPU solve per simulation step.
Times in the logs are simulation time (the reference logs wall time); ``solve_time`` is the wall
time of the step's batched solve, shared by every experiment of that step.
"""
from __future__ import annotations

import json
import os
import time
from datetime import datetime
from pathlib import Path

import numpy as np

from ._lib import RmpcSolver, Solver
from .pmpc import tilt_to_quat
from .rmpc import AdaptiveNPMPCSmooth, rls_features

G_Z = -9.81
ERROR_THRESHOLD = 0.01          # logger.py:162 and rob_ctrl.py:323 (1 cm)
NPZ_KEYS = ("t", "X", "X_target", "U_cmd", "quat_tray", "loss", "solve_time", "L_torques", "R_torques", "L_qpos",
            "R_qpos", "L_qvel", "R_qvel", "L_ee_pos", "R_ee_pos", "L_ee_vel", "R_ee_vel")


class TrayPlant:
    """B objects on B tilting trays, integrated with RK4 at ``dt`` (tilt held within a step).

    state x = [px, vx, py, vy, pz, vz] (mpc_3d.py:106-113); tilt = [theta_x, theta_y] follows the
    command: tilt += (1 - exp(-dt / tau)) (u_cmd - tilt)."""

    def __init__(self, x0, mu, tau=0.03, mu_c=0.02, v_c=0.01, dt=0.002, g=G_Z):
        self.x = np.array(x0, dtype=float).reshape(-1, 6).copy()
        B = self.x.shape[0]
        self.mu = np.broadcast_to(np.asarray(mu, float), (B,)).copy()
        self.tilt = np.zeros((B, 2))
        self.a_lag = 1.0 - np.exp(-dt / tau) if tau > 0 else 1.0
        self.mu_c, self.v_c, self.dt, self.g = float(mu_c), float(v_c), float(dt), float(g)

    def _f(self, x, s):
        vx, vy = x[:, 1], x[:, 3]
        fric = self.mu_c * abs(self.g)
        ax = self.g * s[:, 0] - self.mu * vx - fric * np.tanh(vx / self.v_c)
        ay = self.g * s[:, 1] - self.mu * vy - fric * np.tanh(vy / self.v_c)
        return np.stack([vx, ax, vy, ay, np.zeros_like(vx), np.zeros_like(vx)], axis=1)

    def step(self, u_cmd):
        self.tilt += self.a_lag * (np.asarray(u_cmd, float).reshape(-1, 2) - self.tilt)
        s = np.sin(self.tilt)
        h, x = self.dt, self.x
        k1 = self._f(x, s)
        k2 = self._f(x + h / 2 * k1, s)
        k3 = self._f(x + h / 2 * k2, s)
        k4 = self._f(x + h * k3, s)
        self.x = x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
        return self.x


# ---------------------------------------------------------------------------------------------
# formats
def logger_metrics(logs: dict, dt: float) -> dict:
    """AsyncLogger's metrics (PMPC/src/logger.py:158-183)."""
    X, Xt, t = np.asarray(logs["X"]), np.asarray(logs["X_target"]), np.asarray(logs["t"])
    if len(t) == 0:
        return {}
    sse = float(np.linalg.norm(X[-1, [0, 2]] - Xt[-1, [0, 2]]))
    errors = np.linalg.norm(X[:, [0, 2]] - Xt[:, [0, 2]], axis=1)
    idx = np.where(errors < ERROR_THRESHOLD)[0]
    conv = float(t[idx[0]]) if len(idx) > 0 else float(t[-1])
    effort = float(np.sum(np.linalg.norm(np.asarray(logs["U_cmd"]), axis=1)) * dt)
    return {"steady_state_error": sse, "convergence_time": conv, "control_effort": effort}


def save_npz(logs: dict, metrics: dict, log_dir, experiment_name: str, object_name: str, mass, friction) -> str:
    """np.savez(logs + metrics) at ``{log_dir}/{object}/mass={m}_friction={f}/{name}_{timestamp}.npz``
    (logger.py:186-196)."""
    save_dir = os.path.join(str(log_dir), object_name, f"mass={mass}_friction={friction}")
    os.makedirs(save_dir, exist_ok=True)
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    path = os.path.join(save_dir, f"{experiment_name}_{stamp}.npz")
    np.savez(path, **{**logs, **metrics})
    return path


def to_jsonable(obj):
    """rob_ctrl.py:51-62."""
    if isinstance(obj, dict):
        return {k: to_jsonable(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [to_jsonable(v) for v in obj]
    if isinstance(obj, np.ndarray):
        return to_jsonable(obj.tolist())
    if isinstance(obj, np.generic):
        return to_jsonable(obj.item())
    if isinstance(obj, float):
        return obj if np.isfinite(obj) else None
    return obj


def add_episode(store: dict, ep_name: str, pos_err, error_norm, u_cmd, torque, timestep) -> None:
    """rob_ctrl.py:64-76."""
    store[ep_name] = {"pos_err": pos_err, "pos_err_norm": error_norm, "u_cmd": u_cmd, "torque": torque,
                      "timestep": timestep}


def save_episodes_json(path, episodes: dict, pretty: bool = True) -> None:
    """rob_ctrl.py:78-83: ``{"data": episodes}``, NaN-free."""
    with Path(path).open("w", encoding="utf-8") as f:
        json.dump({"data": to_jsonable(episodes)}, f, indent=2 if pretty else None, ensure_ascii=False,
                  allow_nan=False)


# ---------------------------------------------------------------------------------------------
# closed loops
def run_pmpc(states0, targets, prm, steps: int, N: int = 20, Ts: float = 0.002, tol: float = 1e-8, device: int = 0,
             plant_kw: dict | None = None):
    """B PMPC experiments in lock step (main_parallel_enhanced.py:290-419 without MuJoCo): per step the
    state of every object, one batched cold-started solve, tilt -> quaternion (:333-348), plant step.

    states0, targets [B, 6]; prm [B, 6] = [mu, Qp, Qv, R, u_lo, u_hi] (the solver's parameter rows).
    Returns a list of per-experiment log dicts in the AsyncLogger schema, metrics included, and the
    per-step solver statuses [steps, B]."""
    states0 = np.asarray(states0, float).reshape(-1, 6)
    B = states0.shape[0]
    targets = np.asarray(targets, float).reshape(B, 6)
    prm = np.asarray(prm, float).reshape(B, 6)
    solver = Solver(N=N, Ts=Ts, tol=tol, B_max=max(B, 1), device=device)
    plant = TrayPlant(states0, prm[:, 0], dt=Ts, **(plant_kw or {}))
    X = np.zeros((steps, B, 6)); U = np.zeros((steps, B, 2)); Q = np.zeros((steps, B, 4))
    L = np.zeros((steps, B)); ST = np.zeros((steps, B), np.int32); TS = np.zeros(steps)
    try:
        for k in range(steps):
            X[k] = plant.x
            t0 = time.perf_counter()
            out = solver.solve_batch(plant.x, targets, prm)
            TS[k] = time.perf_counter() - t0
            U[k], L[k], ST[k] = out["u0"], out["f"], out["status"]
            Q[k] = np.stack([tilt_to_quat(u) for u in out["u0"]])
            plant.step(out["u0"])
    finally:
        solver.close()
    t = np.arange(steps) * Ts
    logs = []
    for b in range(B):
        lg = {"t": t, "X": X[:, b], "X_target": np.tile(targets[b], (steps, 1)), "U_cmd": U[:, b],
              "quat_tray": Q[:, b], "loss": L[:, b], "solve_time": TS.copy()}
        for key, w in (("torques", 7), ("qpos", 7), ("qvel", 7), ("ee_pos", 3), ("ee_vel", 6)):
            lg["L_" + key] = np.zeros((steps, w))       # arms are not simulated here
            lg["R_" + key] = np.zeros((steps, w))
        lg.update(logger_metrics(lg, Ts))
        logs.append(lg)
    return logs, ST


def run_rmpc(x0, targets, steps: int, N: int = 20, Ts: float = 0.002, prm=None, device: int = 0,
             pos_tol: float = ERROR_THRESHOLD, plant_kw: dict | None = None, mu=0.1, dr_max: float = 0.01,
             alpha_rg: float = 0.5, lam: float = 0.995, P0: float = 1e3):
    """B RMPC experiments in lock step (rob_ctrl.py:320-420 without MuJoCo): RLS on the measured
    accelerations fused into the solve launch, reference governor, staged reference, warm-started
    solve; an experiment's episode closes when its error first drops below ``pos_tol`` (the
    reference then stops).  Returns (episodes per experiment in the rob_ctrl.py JSON layout,
    statuses [steps, B])."""
    x0 = np.asarray(x0, float).reshape(-1, 4)
    B = x0.shape[0]
    targets = np.asarray(targets, float).reshape(B, 4)
    ctl = AdaptiveNPMPCSmooth(None, None, Ts=Ts, N=N, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0, u_bounds=(-0.6, 0.6),
                              du_bounds=(-0.06, 0.06), vmax=0.2, v_eps=0.1)          # rob_ctrl.py:280-283
    prm = np.tile(ctl.params(), (B, 1)) if prm is None else np.asarray(prm, float).reshape(B, 10)
    solver = RmpcSolver(N=N, Ts=Ts, B_max=max(B, 1), device=device)
    full = np.zeros((B, 6)); full[:, :4] = x0
    plant = TrayPlant(full, mu, dt=Ts, **(plant_kw or {}))
    theta = np.zeros((B, 14)); P = np.tile(np.eye(7) * P0, (B, 2, 1, 1))
    r_v = np.zeros((B, 4)); u_prev = np.zeros((B, 2)); w = np.zeros((B, ctl.w0.shape[0]))
    prev = x0.copy()
    done = np.zeros(B, bool)
    logs = [{"pos_err": [], "pos_err_norm": [], "u_cmd": [], "torque": [], "timestep": []} for _ in range(B)]
    ST = np.zeros((steps, B), np.int32)
    try:
        for k in range(steps):
            xk = plant.x[:, :4].copy()
            y = (xk[:, [1, 3]] - prev[:, [1, 3]]) / Ts
            phi = np.stack([rls_features(p, ctl.v_eps) for p in prev])
            err = np.stack([targets[:, 0] - r_v[:, 0], np.zeros(B), targets[:, 2] - r_v[:, 2], np.zeros(B)], axis=1)
            r_v = r_v + alpha_rg * np.clip(err, -dr_max, dr_max) * np.array([1.0, 0.0, 1.0, 0.0])
            Rref = np.stack([ctl.build_ref_traj(xk[b], r_v[b], targets[b], N, 4, step_fraction=0.2) for b in range(B)])
            out = solver.solve_batch(xk, u_prev, theta, Rref, prm, w_warm=w, want_w=True, rls_P=P, rls_phi=phi,
                                     rls_y=y, rls_lambda=lam)
            theta, P, w = out["theta"], out["rls_P"], out["w"]
            u = out["u0"]
            ST[k] = out["status"]
            en = np.linalg.norm(xk[:, [0, 2]] - targets[:, [0, 2]], axis=1)
            for b in np.where(~done)[0]:
                lg = logs[b]
                lg["pos_err"].append([targets[b, 0] - xk[b, 0], targets[b, 2] - xk[b, 2]])
                lg["pos_err_norm"].append(float(en[b]))
                lg["u_cmd"].append(u[b].copy())
                lg["torque"].append(np.zeros(14))                # arms are not simulated here
                lg["timestep"].append(k * Ts)
                if en[b] < pos_tol:
                    done[b] = True
            prev = xk
            u_prev = u.copy()
            plant.step(u)
            if done.all():
                break
    finally:
        solver.close()
    episodes = []
    for b in range(B):
        eps = {}
        add_episode(eps, "ep1", logs[b]["pos_err"], logs[b]["pos_err_norm"], logs[b]["u_cmd"], logs[b]["torque"],
                    logs[b]["timestep"])
        episodes.append(eps)
    return episodes, ST[:k + 1], done
