"""Seeded synthetic PMPC workloads.

Instances are laid out seed-major, config-minor: instance ``i = 18*seed + b``
with object config ``b = 6*shape_idx + 3*mass_idx + fric_idx``.  Shapes pick
the per-object weights of ``PMPC/main_parallel_enhanced.py:171-179``; mass does
not enter the PMPC NLP (``mpc_3d.py:87-97`` is mass-free), friction is the
``--friction`` value that becomes ``mu``.
"""
from __future__ import annotations

import numpy as np

# PMPC/main_parallel_enhanced.py:171-179
SHAPE_WEIGHTS = (
    ("cube", 600.0, 5.0, 0.1),
    ("cylinder", 400.0, 2.5, 0.2),
    ("sphere", 200.0, 2.0, 0.2),
)
MASSES = (1.0, 2.0)
FRICTIONS = (0.05, 0.10, 0.20)
U_BOUNDS = (-0.6, 0.6)
N_CONFIGS = 18
SEED_BASE = 20251024
TRAY_CENTER = np.array([0.0, 0.0, 0.4])   # world_cube_m=1.0_mu=0.1.xml:141

# parameter row layout shared with the C ABI (include/dart_mpc.h)
PRM_MU, PRM_QP, PRM_QV, PRM_R, PRM_ULO, PRM_UHI = range(6)
N_PRM = 6


def config_params(b: int) -> np.ndarray:
    """Parameter row [mu, Qp, Qv, R, u_lo, u_hi] of object config ``b``."""
    shape_idx, rest = divmod(int(b), 6)
    _mass_idx, fric_idx = divmod(rest, 3)
    _name, qp, qv, r = SHAPE_WEIGHTS[shape_idx]
    return np.array([FRICTIONS[fric_idx], qp, qv, r, U_BOUNDS[0], U_BOUNDS[1]])


def config_name(b: int) -> str:
    shape_idx, rest = divmod(int(b), 6)
    mass_idx, fric_idx = divmod(rest, 3)
    return f"{SHAPE_WEIGHTS[shape_idx][0]}_m{MASSES[mass_idx]:g}_mu{FRICTIONS[fric_idx]:g}"


def pmpc_batch(n_seeds: int = 1, seed0: int = 0):
    """Return (states[B,6], targets[B,6], params[B,6]) for B = 18*n_seeds.

    Per seed s: ``rng = default_rng(20251024 + s)``; the 18 configs draw in
    order b = 0..17.  25 % of instances get a target within 5 mm of the object
    (interior, unsaturated optimum).
    """
    B = N_CONFIGS * n_seeds
    states = np.zeros((B, 6))
    targets = np.zeros((B, 6))
    params = np.zeros((B, N_PRM))
    for s in range(n_seeds):
        rng = np.random.default_rng(SEED_BASE + seed0 + s)
        for b in range(N_CONFIGS):
            i = N_CONFIGS * s + b
            px = TRAY_CENTER[0] + rng.uniform(-0.18, 0.18)
            py = TRAY_CENTER[1] + rng.uniform(-0.13, 0.13)
            vx = rng.uniform(-0.15, 0.15)
            vy = rng.uniform(-0.15, 0.15)
            vz = rng.uniform(-0.01, 0.01)
            states[i] = [px, vx, py, vy, 0.43, vz]
            if rng.uniform() < 0.25:
                tx = px + rng.uniform(-5e-3, 5e-3)
                ty = py + rng.uniform(-5e-3, 5e-3)
            else:
                tx = TRAY_CENTER[0] + rng.uniform(-0.15, 0.15)
                ty = TRAY_CENTER[1] + rng.uniform(-0.12, 0.12)
            targets[i] = [tx, 0.0, ty, 0.0, TRAY_CENTER[2], 0.0]
            params[i] = config_params(b)
    return states, targets, params


def pmpc_c1():
    """C1: cube, mu=0.10, object at rest at the tray centre, target 10 cm in +x
    (PMPC/README.md:226-227 experiment 1)."""
    state = np.array([[0.0, 0.0, 0.0, 0.0, 0.43, 0.0]])
    target = np.array([[0.1, 0.0, 0.0, 0.0, 0.4, 0.0]])
    prm = np.array([[0.10, 600.0, 5.0, 0.1, -0.6, 0.6]])
    return state, target, prm


# ---------------------------------------------------------------------------
# C3: RMPC batch.  Controller weights are the rob_ctrl.py defaults
# (RMPC/dev_dual/rob_ctrl.py:281-284); the object config enters through the
# regressor estimate theta_hat, which is produced by 50 seeded RLS updates
# (np_mpc...:10-30, lambda 0.995, P0 1e3) on synthetic features / accelerations.
# ---------------------------------------------------------------------------
RMPC_PRM = np.array([80.0, 2.0, 0.02, 1.0, -0.6, 0.6, -0.06, 0.06, 0.2, 0.1])
N_RMPC_PRM = 10
RMPC_PRM_NAMES = ("Qp", "Qv", "Ru", "Rdu", "u_lo", "u_hi", "du_lo", "du_hi", "vmax", "v_eps")


def _rls_update(theta, P, phi, y, lam=0.995):
    denom = lam + phi @ P @ phi
    K = (P @ phi) / denom
    err = y - phi @ theta
    theta = theta + K * err
    P = (P - np.outer(K, phi) @ P) / lam
    return theta, P


def _features(x, v_eps=0.1):
    return np.array([x[0], x[1], x[2], x[3], np.tanh(x[1] / v_eps), np.tanh(x[3] / v_eps), 1.0])


def rmpc_batch(n_seeds: int = 1, seed0: int = 0, N: int = 20, n_rls: int = 50):
    """Return dict of C3 inputs for B = 18*n_seeds instances:
    x0[B,4], u_prev[B,2], theta[B,14], Rref[B,4(N+1)], prm[B,10], and the RLS state
    (rls_theta[B,14], rls_P[B,2,7,7], phi_prev[B,7], y[B,2]) for one more fused update."""
    B = N_CONFIGS * n_seeds
    out = dict(x0=np.zeros((B, 4)), u_prev=np.zeros((B, 2)), theta=np.zeros((B, 14)),
               Rref=np.zeros((B, 4 * (N + 1))), prm=np.tile(RMPC_PRM, (B, 1)),
               rls_theta=np.zeros((B, 14)), rls_P=np.zeros((B, 2, 7, 7)), phi_prev=np.zeros((B, 7)), y=np.zeros((B, 2)))
    for s in range(n_seeds):
        rng = np.random.default_rng(SEED_BASE + 7919 + seed0 + s)
        for b in range(N_CONFIGS):
            i = N_CONFIGS * s + b
            shape_idx, rest = divmod(b, 6)
            mass_idx, fric_idx = divmod(rest, 3)
            mu, m = FRICTIONS[fric_idx], MASSES[mass_idx]
            # synthetic ground truth of the linear-in-features acceleration model
            tx = np.array([0.0, -mu / m, 0.0, 0.0, -0.3 * mu * (1 + 0.5 * shape_idx), 0.0, 0.0])
            ty = np.array([0.0, 0.0, 0.0, -mu / m, 0.0, -0.3 * mu * (1 + 0.5 * shape_idx), 0.0])
            th = [np.zeros(7), np.zeros(7)]
            Pm = [np.eye(7) * 1e3, np.eye(7) * 1e3]
            for _ in range(n_rls):
                xs = np.array([rng.uniform(-0.15, 0.15), rng.uniform(-0.15, 0.15),
                               rng.uniform(-0.12, 0.12), rng.uniform(-0.15, 0.15)])
                ph = _features(xs)
                for a, tt in enumerate((tx, ty)):
                    th[a], Pm[a] = _rls_update(th[a], Pm[a], ph, ph @ tt + rng.normal(0, 0.01))
            x0 = np.array([rng.uniform(-0.18, 0.18), rng.uniform(-0.15, 0.15),
                           rng.uniform(-0.13, 0.13), rng.uniform(-0.15, 0.15)])
            target = np.array([rng.uniform(-0.15, 0.15), 0.0, rng.uniform(-0.12, 0.12), 0.0])
            r_v = np.array([x0[0], 0.0, x0[2], 0.0])
            # reference governor step (rob_ctrl.py:346-348) then staged reference (np_mpc...:201-210)
            err = target - r_v
            r_v = r_v + 0.5 * np.array([np.clip(err[0], -0.01, 0.01), 0.0, np.clip(err[2], -0.01, 0.01), 0.0])
            R = np.zeros((N + 1, 4))
            for k in range(N + 1):
                w = 1.0 - 0.8 ** (k + 1)
                rk = r_v + w * (target - r_v)
                R[k] = [rk[0], 0.0, rk[2], 0.0]
            out["x0"][i] = x0
            out["u_prev"][i] = rng.uniform(-0.3, 0.3, 2)
            out["theta"][i] = np.concatenate(th)
            out["Rref"][i] = R.reshape(-1)
            out["rls_theta"][i] = np.concatenate(th)
            out["rls_P"][i] = np.stack(Pm)
            xp = x0 + rng.normal(0, 1e-3, 4)
            out["phi_prev"][i] = _features(xp)
            out["y"][i] = (x0[[1, 3]] - xp[[1, 3]]) / 0.002
    return out


# ---------------------------------------------------------------------------------------------
# C5: LMPC batch = 18, N = 30.  The 34-vector model parameters are an input
# fixture (the policy checkpoints cannot be loaded): pvec ~ U(0.01, 1.9)^34, the
# output range of the policy's soft clip (LMPC/src/controller/rlmpc2.py:759-769).
LMPC_SEED_BASE = 20251024 + 15485863


def lmpc_batch(n_seeds: int = 1, seed0: int = 0):
    """Return dict of C5 inputs for B = 18*n_seeds instances: state[B,8], u_prev[B,2],
    pvec[B,34], target[B,8] (x0 as the PMPC workload plus theta, omega ~ U(-0.05, 0.05))."""
    B = N_CONFIGS * n_seeds
    out = dict(state=np.zeros((B, 8)), u_prev=np.zeros((B, 2)), pvec=np.zeros((B, 34)), target=np.zeros((B, 8)))
    for s in range(n_seeds):
        rng = np.random.default_rng(LMPC_SEED_BASE + seed0 + s)
        for b in range(N_CONFIGS):
            i = N_CONFIGS * s + b
            out["state"][i] = [rng.uniform(-0.18, 0.18), rng.uniform(-0.15, 0.15),
                               rng.uniform(-0.13, 0.13), rng.uniform(-0.15, 0.15),
                               rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05),
                               rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05)]
            out["u_prev"][i] = rng.uniform(-0.2, 0.2, 2)
            out["pvec"][i] = rng.uniform(0.01, 1.9, 34)
            out["target"][i] = [rng.uniform(-0.15, 0.15), 0.0, rng.uniform(-0.12, 0.12), 0.0, 0.0, 0.0, 0.0, 0.0]
    return out


# ---------------------------------------------------------------------------------------------
# Per-arm impedance QP (PMPC/src/controller/arm.py:266-457).  MuJoCo is not in
# this image, so the shared-memory snapshot that compute_dynamics (arm.py:111-199) publishes is
# synthesised with the same structure: a revolute 7-DOF chain (joint axes z_i, origins p_i) gives
# J = [z_i x (p_ee - p_i); z_i], a link-inertia sum gives an SPD M, Mx_inv = J M^-1 J^T as
# arm.py:133-138 forms it for a fixed-base arm.  Scenario mix per instance: 60 % nominal tracking,
# 20 % large task error (torque bounds active), 10 % joint at its limit drifting outward
# (position-row bound active), 10 % near-singular task Jacobian (|det Mx_inv| <= 1e-8 -> the
# pinv(rcond=1e-3) branch of arm.py:346-350).
ARM_SEED_BASE = 20251024 + 32452843
ARM_N = 7


def _arm_instance(rng, kind: str, n: int = ARM_N):
    from_lim = 0.3
    qmin = np.array([-6.28319, -2.059, -6.28319, -0.19198, -6.28319, -1.69297, -6.28319])[:n]
    qmax = np.array([6.28319, 2.0944, 6.28319, 3.927, 6.28319, 3.14159, 6.28319])[:n]
    lo_q = np.maximum(qmin + from_lim, -2.5)
    hi_q = np.minimum(qmax - from_lim, 2.5)
    q = rng.uniform(lo_q, hi_q)
    qd = rng.normal(0.0, 0.05, n)
    # kinematic chain
    z = np.zeros((n, 3))
    p = np.zeros((n, 3))
    axis = np.array([0.0, 0.0, 1.0])
    pos = np.array([0.0, 0.0, 0.27])
    for i in range(n):
        a = axis + rng.normal(0.0, 0.6, 3)
        z[i] = a / np.linalg.norm(a)
        p[i] = pos
        pos = pos + rng.normal(0.0, 0.12, 3) + np.array([0.0, 0.0, 0.05])
    p_ee = pos + np.array([0.0, 0.0, 0.125])
    J = np.zeros((6, n))
    for i in range(n):
        J[:3, i] = np.cross(z[i], p_ee - p[i])
        J[3:, i] = z[i]
    if kind == "singular":
        J[5] *= 1e-4                                   # task direction nearly unreachable
    # mass matrix: sum of link contributions + armature
    Jb = rng.normal(0.0, 0.35, (12, n)) * np.linspace(1.0, 0.3, n)
    M = Jb.T @ np.diag(rng.uniform(0.5, 3.0, 12)) @ Jb + np.diag(rng.uniform(0.01, 0.05, n))
    M = 0.5 * (M + M.T)
    Mx_inv = J @ np.linalg.inv(M) @ J.T
    Mx_inv = 0.5 * (Mx_inv + Mx_inv.T)
    Jd = rng.normal(0.0, 0.4, (6, n)) * (0.2 + np.mean(np.abs(qd)))
    h = np.clip(rng.normal(0.0, 8.0, n), -25.0, 25.0)
    ee_pos = p_ee.copy()
    if kind == "large":
        d = rng.normal(0.0, 1.0, 3)
        mocap = ee_pos + d / np.linalg.norm(d) * rng.uniform(0.08, 0.2)
        rotvec = rng.normal(0.0, 0.3, 3)
    else:
        mocap = ee_pos + rng.normal(0.0, 0.003, 3)
        rotvec = rng.normal(0.0, 0.02, 3)
    if kind == "limit":
        j = int(rng.integers(0, n))
        if rng.uniform() < 0.5:
            q[j] = qmax[j] - rng.uniform(0.0, 2e-5)
            qd[j] = rng.uniform(0.002, 0.02)
        else:
            q[j] = qmin[j] + rng.uniform(0.0, 2e-5)
            qd[j] = -rng.uniform(0.002, 0.02)
    return {"q": q, "qd": qd, "qdd_prev": rng.normal(0.0, 1.0, n), "mocap_pos": mocap, "ee_pos": ee_pos,
            "rotvec": rotvec, "jac": J, "jacDot": Jd, "M": M, "h": h, "Mx_inv": Mx_inv}


def arm_batch(n_seeds: int = 1, seed0: int = 0, n: int = ARM_N):
    """Return (snaps, kinds) for B = 36*n_seeds arm instances (18 configs x 2 arms per seed):
    snaps[key] = [B, ...] arrays with the fields of arm.py:185-199."""
    kinds_cycle = ["nominal"] * 6 + ["large"] * 2 + ["limit", "singular"]
    out, kinds = None, []
    B = 2 * N_CONFIGS * n_seeds
    for s in range(n_seeds):
        rng = np.random.default_rng(ARM_SEED_BASE + seed0 + s)
        for b in range(2 * N_CONFIGS):
            kind = kinds_cycle[int(rng.integers(0, len(kinds_cycle)))]
            inst = _arm_instance(rng, kind, n)
            if out is None:
                out = {k: np.zeros((B,) + np.shape(v)) for k, v in inst.items()}
            for k, v in inst.items():
                out[k][2 * N_CONFIGS * s + b] = v
            kinds.append(kind)
    return out, kinds
