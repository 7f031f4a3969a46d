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
