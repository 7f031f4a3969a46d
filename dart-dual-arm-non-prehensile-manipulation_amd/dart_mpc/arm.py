"""Drop-in per-arm impedance controller backed by the MI355X arm-QP kernel.

Mirrors ARMCONTROL (PMPC/src/controller/arm.py; the same class lives in
RMPC/dev_dual/controller/parallel.py and LMPC/src/controller/parallel.py):

  - ``ArmSolver``: the batched C ABI ``dart_arm_solve_batch(_dev)`` -- the body of
    ``ARMCONTROL.solver_worker`` (:266-457) for B arm snapshots per launch.
  - ``ArmControl``: ``ARMCONTROL.compute_torque`` (:201-231) with the solver run in-process:
    feed it the dict ``compute_dynamics`` (:111-199) returns, get ``(torque_cmd, loss)``; the
    solution is kept as the next ``qdd_prev`` exactly as the worker writes ``views["qdd_prev"]``
    (:431).  MuJoCo is not part of this package, so the dynamics dict is an input.

Snapshot / parameter row layouts are those of include/dart_mpc.h (``pack_snapshot``,
``pack_params``).  The kernel cold-starts the bound multipliers and warm-starts qdd from
qdd_prev; the QP is strictly convex, so the answer does not depend on the reference's IPOPT
warm-start duals (:401-417).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import DartMPCError, _ptr, lib

SOLVED, ACCEPTABLE, MAXITER, BREAKDOWN, INFEASIBLE = 0, 1, -1, -2, -3
SNAP_FIELDS = (("q", "n"), ("qd", "n"), ("qdd_prev", "n"), ("mocap_pos", 3), ("ee_pos", 3), ("rotvec", 3),
               ("jac", "6n"), ("jacDot", "6n"), ("M", "nn"), ("h", "n"), ("Mx_inv", 36))
PARAM_FIELDS = (("Wimp", 36), ("Wpos", "nn"), ("Wsmooth", "nn"), ("Qmin", "n"), ("Qmax", "n"), ("Qdotmin", "n"),
                ("Qdotmax", "n"), ("taumin", "n"), ("taumax", "n"), ("K", 36), ("K_null", "nn"), ("dt", 1))


class ArmConfig(ctypes.Structure):
    """Mirror of ``struct dart_arm_config``."""
    _fields_ = [("tol", ctypes.c_double), ("acceptable_tol", ctypes.c_double), ("max_iter", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


def _width(w, n):
    return {"n": n, "6n": 6 * n, "nn": n * n}.get(w, w)


def pack_snapshot(snaps: dict) -> np.ndarray:
    """[B, snapshot_len] rows from a dict of [B, ...] arrays (or one snapshot of unbatched arrays)."""
    one = np.ndim(snaps["q"]) == 1
    n = np.shape(snaps["q"])[-1]
    cols = [np.reshape(np.asarray(snaps[k], dtype=np.float64), (1 if one else -1, _width(w, n)))
            for k, w in SNAP_FIELDS]
    return np.ascontiguousarray(np.concatenate(cols, axis=1))


def pack_params(prm: dict) -> np.ndarray:
    """One parameter row (dict of arrays, the reference's params) or [B, param_len] when batched."""
    n = np.shape(prm["Qmin"])[-1]
    batched = np.ndim(prm["Qmin"]) == 2
    cols = []
    for k, w in PARAM_FIELDS:
        v = np.asarray(prm[k], dtype=np.float64)
        cols.append(np.reshape(v, (-1 if batched else 1, _width(w, n))))
    out = np.concatenate(cols, axis=1)
    return np.ascontiguousarray(out if batched else out[0])


def arm_config(**over) -> ArmConfig:
    c = ArmConfig()
    lib().dart_arm_config_default(ctypes.byref(c))
    for k, v in over.items():
        setattr(c, k, v)
    return c


class ArmSolver:
    """Batched ``dart_arm_solve_batch``: B arm QPs per call (n joints, one shared or per-instance
    parameter row)."""

    def __init__(self, n: int = 7, **cfg):
        self.n = int(n)
        self.cfg = arm_config(**cfg)
        L = lib()
        self.snap_len = L.dart_arm_snapshot_len(self.n)
        self.param_len = L.dart_arm_param_len(self.n)
        if self.snap_len < 0:
            raise DartMPCError(f"unsupported joint count n={n}")

    def solve_batch(self, snap_rows: np.ndarray, prm_rows: np.ndarray):
        """Host arrays: snap_rows [B, snapshot_len], prm_rows [param_len] (shared) or [B, param_len]."""
        snap_rows = np.ascontiguousarray(snap_rows, dtype=np.float64)
        prm_rows = np.ascontiguousarray(prm_rows, dtype=np.float64)
        B = snap_rows.shape[0]
        if snap_rows.shape[1] != self.snap_len:
            raise DartMPCError(f"snapshot rows must have {self.snap_len} entries")
        stride = 0 if prm_rows.ndim == 1 else self.param_len
        if prm_rows.shape[-1] != self.param_len or (stride and prm_rows.shape[0] != B):
            raise DartMPCError(f"parameter rows must have {self.param_len} entries")
        out = {"qdd": np.zeros((B, self.n)), "tau": np.zeros((B, self.n)), "loss": np.zeros(B),
               "status": np.zeros(B, dtype=np.int32), "iters": np.zeros(B, dtype=np.int32)}
        rc = lib().dart_arm_solve_batch(ctypes.byref(self.cfg), B, self.n, _ptr(snap_rows), _ptr(prm_rows), stride,
                                        _ptr(out["qdd"]), _ptr(out["tau"]), _ptr(out["loss"]), _ptr(out["status"]),
                                        _ptr(out["iters"]))
        if rc != 0:
            raise DartMPCError(f"dart_arm_solve_batch failed ({rc})")
        return out

    def solve_batch_dev(self, B, snap_ptr, prm_ptr, prm_shared, qdd_ptr, tau_ptr, loss_ptr, status_ptr, iters_ptr,
                        stream=None):
        """Device pointers (ints), asynchronous on ``stream`` (a hipStream_t as int, None = default)."""
        rc = lib().dart_arm_solve_batch_dev(ctypes.byref(self.cfg), B, self.n, ctypes.c_void_p(snap_ptr),
                                            ctypes.c_void_p(prm_ptr), 0 if prm_shared else self.param_len,
                                            ctypes.c_void_p(qdd_ptr), ctypes.c_void_p(tau_ptr),
                                            ctypes.c_void_p(loss_ptr), ctypes.c_void_p(status_ptr),
                                            ctypes.c_void_p(iters_ptr), ctypes.c_void_p(stream or 0))
        if rc != 0:
            raise DartMPCError(f"dart_arm_solve_batch_dev failed ({rc})")


class ArmControl:
    """ARMCONTROL.compute_torque with the solve in-process on the GPU.

    ``params`` is the reference's parameter dict (Wimp, Wpos, Wsmooth, Qmin, Qmax, Qdotmin, Qdotmax,
    taumin, taumax, K, K_null, dt; joint/actuator/body names are MuJoCo bindings and not needed).
    """

    def __init__(self, params: dict, n: int = 7):
        self.params = params
        self.solver = ArmSolver(n)
        self.prm_row = pack_params(params)
        self.qdd_prev = np.zeros(n)          # views["qdd_prev"], zero-initialised (arm.py:95)
        self.last_status = None

    def compute_torque(self, dynamics: dict):
        """dynamics: the dict of compute_dynamics (arm.py:185-199); qdd_prev is taken from this
        controller (the worker's own last solution) unless the dict carries one."""
        snap = dict(dynamics)
        snap.setdefault("qdd_prev", self.qdd_prev)
        out = self.solver.solve_batch(pack_snapshot(snap), self.prm_row)
        self.last_status = int(out["status"][0])
        self.qdd_prev = out["qdd"][0].copy()
        return out["tau"][0].copy(), float(out["loss"][0])
