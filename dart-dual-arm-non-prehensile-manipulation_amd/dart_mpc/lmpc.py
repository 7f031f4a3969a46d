"""Drop-in LMPC front-end backed by the MI355X kernels.

Mirrors LMPC/src/controller/rlmpc2.py:
  - ``LmpcPolicy``: the inference / parameter-write half of ``RLMPC._rl_worker`` (:537-769) for B
    controllers on the GPU (Welford-normalised 10-step history, mean_net MLP 520->64->64->34,
    Normal.rsample, logit-space update every 8th step, EMA + soft clip of write_params_to_shm).
    Weights follow ``Policy._init_weights`` (orthogonal, gain sqrt(2), zero bias; log_std =
    log(policy_std_init)) because the reference checkpoints are not loaded.
  - ``RLMPC``: ``RLMPC.solve(target)`` (:986-1021) run synchronously: state from MjData, one
    policy step producing pvec, one warm-started LMPC solve (the worker loop :494-524), returns
    ``(U_opt[0], loss)``.  The reference runs the three parts in separate processes; here they
    are one launch (``dart_lmpc_policy_solve_batch``: the policy step is the prologue of the
    solve kernel), or two launches on one stream with ``fused=False``.
  - ``policy_solve_batch``: the fused policy step + solve for B controllers.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import DartMPCError, LMPC_PRM_DEFAULT, LmpcSolver, _ptr, lib

HIST, PB, PH, PA = 10, 52, 64, 34
NWEIGHTS = 520 * 64 + 64 + 64 * 64 + 64 + 64 * 34 + 34 + 34


class PolicyConfig(ctypes.Structure):
    """Mirror of ``struct dart_lmpc_policy_config``."""
    _fields_ = [("update_every", ctypes.c_int32), ("reserved", ctypes.c_int32), ("max_delta", ctypes.c_double),
                ("k_max", ctypes.c_double), ("min_k", ctypes.c_double), ("k_ceiling_margin", ctypes.c_double),
                ("action_scale", ctypes.c_double), ("smooth_alpha", ctypes.c_double),
                ("log_std_min", ctypes.c_double), ("log_std_max", ctypes.c_double)]


def policy_config(**over) -> PolicyConfig:
    c = PolicyConfig()
    L = lib()
    L.dart_lmpc_policy_config_default(ctypes.byref(c))
    for k, v in over.items():
        setattr(c, k, v)
    return c


def _orthogonal(rng, rows, cols, gain):
    """torch.nn.init.orthogonal_ on a [rows, cols] weight (Policy._init_weights, :63-68)."""
    flat = rng.standard_normal((rows, cols))
    if rows < cols:
        flat = flat.T
    q, r = np.linalg.qr(flat)
    q = q * np.sign(np.diag(r))
    if rows < cols:
        q = q.T
    return gain * q


def init_policy_weights(seed=0, std_init=0.1):
    """Packed fp32 weights (input-major) of a freshly initialised Policy.mean_net + log_std."""
    rng = np.random.default_rng(seed)
    g = np.sqrt(2.0)
    W1 = _orthogonal(rng, 64, 520, g).T          # nn.Linear stores [out, in]; packed as [in][out]
    W2 = _orthogonal(rng, 64, 64, g).T
    W3 = _orthogonal(rng, 34, 64, g).T
    parts = [W1, np.zeros(64), W2, np.zeros(64), W3, np.zeros(34), np.full(34, np.log(std_init))]
    return np.concatenate([np.asarray(p, np.float32).reshape(-1) for p in parts]).astype(np.float32)


class LmpcPolicy:
    """B independent parameter policies; state arrays live on the host and are staged per call."""

    def __init__(self, B, weights=None, current_k=None, seed=0, **cfg):
        self.B = int(B)
        self.cfg = policy_config(**cfg)
        self.weights = np.ascontiguousarray(init_policy_weights(seed) if weights is None else weights, np.float32)
        if self.weights.size != NWEIGHTS:
            raise ValueError(f"policy weights must have {NWEIGHTS} floats")
        if current_k is None:     # :566-568: mid-range with +-5 % jitter
            rng = np.random.default_rng(seed + 1)
            k_max = self.cfg.k_max
            current_k = np.clip(0.5 * k_max + rng.uniform(-0.05, 0.05, (self.B, PA)) * k_max, self.cfg.min_k,
                                k_max - self.cfg.k_ceiling_margin)
        self.current_k = np.ascontiguousarray(np.broadcast_to(current_k, (self.B, PA)), np.float64).copy()
        self.model_params = self.current_k.copy()
        self.obs_mean = np.zeros((self.B, PB)); self.obs_M2 = np.zeros((self.B, PB))
        self.obs_count = np.zeros(self.B, np.int32); self.timestep = np.zeros(self.B, np.int32)
        self.history = np.zeros((self.B, HIST, PB), np.float32)

    def step(self, state, target, control, noise=None, rng=None):
        """One policy step for all B controllers; returns the raw actions [B, 34] and leaves the
        new parameter vectors in ``model_params``."""
        c = lambda a, n: np.ascontiguousarray(a, np.float64).reshape(self.B, n)
        state, target, control = c(state, 8), c(target, 8), c(control, 2)
        if noise is None:
            noise = (rng or np.random.default_rng()).standard_normal((self.B, PA))
        noise = np.ascontiguousarray(noise, np.float32).reshape(self.B, PA)
        act = np.empty((self.B, PA), np.float32)
        rc = lib().dart_lmpc_policy_step(ctypes.byref(self.cfg), self.B, _ptr(self.weights), _ptr(state), _ptr(target),
                                         _ptr(control), _ptr(self.current_k), _ptr(self.obs_mean), _ptr(self.obs_M2),
                                         _ptr(self.obs_count), _ptr(self.history), _ptr(self.timestep), _ptr(noise),
                                         _ptr(self.model_params), _ptr(act))
        if rc != 0:
            raise DartMPCError(f"dart_lmpc_policy_step failed ({rc})")
        return act


def policy_solve_batch(solver: LmpcSolver, policy: LmpcPolicy, state, u_prev, target, prm=None, w_warm=None,
                       want_w=False, noise=None, rng=None):
    """One LMPC control step for ``policy.B`` controllers in ONE launch: the policy step (control =
    u_prev, :650 / :505) updates the policy state and ``policy.model_params``, then the solve uses
    those parameters as pvec (:506).  Same results as ``policy.step`` followed by
    ``solver.solve_batch``.  Returns the solve dict plus ``action`` (raw actions [B, 34])."""
    B = policy.B
    c = lambda a, n: np.ascontiguousarray(a, np.float64).reshape(B, n)
    state, u_prev, target = c(state, 8), c(u_prev, 2), c(target, 8)
    prm = c(np.tile(LMPC_PRM_DEFAULT, (B, 1)) if prm is None else prm, 22)
    ww = None if w_warm is None else c(w_warm, solver.nw)
    if noise is None:
        noise = (rng or np.random.default_rng()).standard_normal((B, PA))
    noise = np.ascontiguousarray(noise, np.float32).reshape(B, PA)
    act = np.empty((B, PA), np.float32)
    u0 = np.empty((B, 2)); f = np.empty(B)
    w = np.empty((B, solver.nw)) if want_w else None
    st = np.empty(B, np.int32); it = np.empty(B, np.int32)
    rc = lib().dart_lmpc_policy_solve_batch(
        solver._h, ctypes.byref(policy.cfg), B, _ptr(policy.weights), _ptr(state), _ptr(u_prev), _ptr(target),
        _ptr(policy.current_k), _ptr(policy.obs_mean), _ptr(policy.obs_M2), _ptr(policy.obs_count),
        _ptr(policy.history), _ptr(policy.timestep), _ptr(noise), _ptr(policy.model_params), _ptr(act), _ptr(prm),
        _ptr(ww), _ptr(u0), _ptr(f), _ptr(w), _ptr(st), _ptr(it), None)
    if rc != 0:
        solver._err(rc, "dart_lmpc_policy_solve_batch")
    return dict(u0=u0, f=f, w=w, status=st, iters=it, action=act)


class RLMPC:
    """Front-end of RLMPC (:110-226, :986-1021) with the solver and policy on the GPU."""

    def __init__(self, model=None, data=None, params=None, *, policy_weights=None, seed=0, device=0, fused=True):
        p = dict(Ts=0.002, nx=8, nu=2, N=20, Q=LMPC_PRM_DEFAULT[:8], Qt=LMPC_PRM_DEFAULT[8:16], R=LMPC_PRM_DEFAULT[16:20],
                 u_bounds=tuple(LMPC_PRM_DEFAULT[20:22]), body_name="cube2", max_param_abs=2.0, max_delta_abs=0.02)
        p.update(params or {})
        if p["nx"] != 8 or p["nu"] != 2:
            raise ValueError("the LMPC model is defined for nx=8, nu=2 (rlmpc2.py:260-429)")
        self.model, self.data, self.params = model, data, p
        self.N = int(p["N"])
        self.solver = LmpcSolver(N=self.N, Ts=float(p["Ts"]), B_max=1, device=device)
        self.prm = np.concatenate([p["Q"], p["Qt"], p["R"], p["u_bounds"]]).astype(np.float64)[None]
        k_max = float(p["max_param_abs"])
        self.policy = LmpcPolicy(1, weights=policy_weights, seed=seed, k_max=k_max,
                                 max_delta=float(p["max_delta_abs"]), k_ceiling_margin=max(1e-3, 0.05 * k_max))
        self.w0 = np.zeros(lib().dart_lmpc_nw(self.N))
        self.last_control = np.zeros(2)
        self.loss = np.zeros(1)
        self._rng = np.random.default_rng(seed + 2)
        self.fused = bool(fused)

    def get_state(self):
        """[px, vx, py, vy, theta_x, omega_x, theta_y, omega_y] (:1034-1042)."""
        if self.data is None:
            raise RuntimeError("get_state() needs MuJoCo data")
        from scipy.spatial.transform import Rotation as Rot
        b = self.data.body(self.params["body_name"])
        th = Rot.from_matrix(np.asarray(b.xmat).reshape(3, 3)).as_euler("xyz", degrees=False)[:2]
        return np.array([b.xpos[0], b.cvel[3], b.xpos[1], b.cvel[4], th[0], b.cvel[0], th[1], b.cvel[1]])

    def solve(self, target, state=None):
        state = self.get_state() if state is None else np.asarray(state, float)
        tg = np.asarray(target, float)[None]
        if self.fused:
            out = policy_solve_batch(self.solver, self.policy, state[None], self.last_control[None], tg, self.prm,
                                     w_warm=self.w0[None], want_w=True, rng=self._rng)
        else:
            self.policy.step(state, target, self.last_control, rng=self._rng)
            out = self.solver.solve_batch(state[None], self.last_control[None], self.policy.model_params, tg,
                                          self.prm, w_warm=self.w0[None], want_w=True)
        self.w0 = out["w"][0]
        self.loss = out["f"].copy()
        self.last_control = out["u0"][0].copy()
        return self.last_control.copy(), self.loss
