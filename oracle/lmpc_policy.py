"""LMPC parameter policy step restated in numpy -- TEST INFRASTRUCTURE ONLY.

Oracle for SURVEY.md §8a row L5: the inference / parameter-write half of RLMPC._rl_worker
(LMPC/src/controller/rlmpc2.py:537-769), for one controller:
  base vector [state, target, control, current_k] as fp32 -> fp64          :648-653
  Welford mean / M2 (fp64), std = sqrt(max(var, 1e-12)) (fp32)              :656-665
  normalised (fp32), 10-step history deque (oldest first)                    :667-670
  Policy.mean_net: Linear(520,64)-Tanh-Linear(64,64)-Tanh-Linear(64,34), fp32 :33-56
  raw = mean + exp(clamp(log_std, log 1e-2, log 2)) * eps (Normal.rsample)    :57-80, :674-680
  every 8th step: logit-space update in fp32                                  :742-756
  write_params_to_shm: EMA (alpha 0.5) + tanh soft clip in fp64               :606-616
The policy weights are an input (checkpoints are not loaded).  Weights are kept
in the packed input-major layout of include/dart_mpc.h (W1[520][64] ... log_std[34]).

Parity status: unpinned against the reference's torch worker (torch runs here, but the
reference's process / shared-memory wrapper is not executed); this restatement follows the
quoted lines operation by operation, in the same precisions.
"""
from __future__ import annotations

from collections import deque

import numpy as np

HIST, PB, PH, PA = 10, 52, 64, 34
NWEIGHTS = 520 * 64 + 64 + 64 * 64 + 64 + 64 * 34 + 34 + 34
DEFAULTS = dict(update_every=8, max_delta=0.02, k_max=2.0, min_k=1e-2, k_ceiling_margin=max(1e-3, 0.05 * 2.0),
                action_scale=1.0, smooth_alpha=0.5, log_std_min=float(np.log(1e-2)), log_std_max=float(np.log(2.0)))


def unpack(w):
    w = np.asarray(w, np.float32)
    o = 0
    out = []
    for shape in ((520, 64), (64,), (64, 64), (64,), (64, 34), (34,), (34,)):
        n = int(np.prod(shape))
        out.append(w[o:o + n].reshape(shape)); o += n
    return out


class PolicyState:
    """Per-controller state of the worker loop (:550-569)."""

    def __init__(self, current_k, model_params=None):
        self.obs_mean = np.zeros(PB)
        self.obs_M2 = np.zeros(PB)
        self.obs_count = 0
        self.history = deque([np.zeros(PB, np.float32) for _ in range(HIST)], maxlen=HIST)
        self.timestep = 0
        self.current_k = np.asarray(current_k, np.float64).copy()
        self.model_params = self.current_k.copy() if model_params is None else np.asarray(model_params, float).copy()


def smooth_clip(x, lo, hi, margin=1e-3):
    c = (hi + lo) / 2
    s = (hi - lo) / 2 - margin
    return c + s * np.tanh((x - c) / s)


def policy_step(st: PolicyState, weights, state, target, control, eps, cfg=DEFAULTS):
    """One loop body (:641-756).  Returns the raw action (fp32); updates st in place."""
    W1, b1, W2, b2, W3, b3, log_std = unpack(weights)
    base = np.concatenate([np.asarray(state).astype(np.float32), np.asarray(target).astype(np.float32),
                           np.asarray(control).astype(np.float32),
                           st.current_k.astype(np.float32)]).astype(np.float64)
    st.obs_count += 1
    delta = base - st.obs_mean
    st.obs_mean = st.obs_mean + delta / st.obs_count
    delta2 = base - st.obs_mean
    st.obs_M2 = st.obs_M2 + delta * delta2
    var = st.obs_M2 / (st.obs_count - 1) if st.obs_count > 1 else np.ones_like(st.obs_M2) * 1e-6
    std = np.sqrt(np.maximum(var, 1e-12)).astype(np.float32)
    nv = ((base.astype(np.float32) - st.obs_mean.astype(np.float32)) / (std + np.float32(1e-8))).astype(np.float32)
    st.history.append(nv)
    obs = np.concatenate(list(st.history)).astype(np.float32)
    h1 = np.tanh(obs @ W1 + b1).astype(np.float32)
    h2 = np.tanh(h1 @ W2 + b2).astype(np.float32)
    mean = (h2 @ W3 + b3).astype(np.float32)
    sd = np.exp(np.clip(log_std, np.float32(cfg["log_std_min"]), np.float32(cfg["log_std_max"]))).astype(np.float32)
    raw = (mean + sd * np.asarray(eps, np.float32)).astype(np.float32)
    if st.timestep % cfg["update_every"] == 0:
        kmax = np.float32(cfg["k_max"])
        cur = st.model_params.astype(np.float32)
        frac = np.clip(cur / kmax, np.float32(cfg["min_k"] / cfg["k_max"]), np.float32(1.0 - 1e-6))
        z = np.log(frac / (np.float32(1) - frac)).astype(np.float32)
        zn = (z + raw * np.float32(cfg["max_delta"]) * np.float32(cfg["action_scale"])).astype(np.float32)
        kn = (kmax * (np.float32(1) / (np.float32(1) + np.exp(-zn)))).astype(np.float32)
        sm = cfg["smooth_alpha"] * kn.astype(np.float64) + (1 - cfg["smooth_alpha"]) * st.model_params
        st.model_params = smooth_clip(sm, cfg["min_k"], cfg["k_max"] - cfg["k_ceiling_margin"])
    st.timestep += 1
    return raw
