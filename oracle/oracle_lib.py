"""ctypes loader for the C oracle (liboracle_pmpc.so) -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  See pmpc_ipm.c for what is restated and where from.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_pmpc.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def _max_soc(soc):
    """IPOPT max_soc from the ``soc`` argument: True = IPOPT's default 4, False = off, or a count."""
    if soc is True:
        return 4
    if soc is False or soc is None:
        return 0
    return max(0, int(soc))


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_pmpc_solve_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp, _dp, _dp,
                                              ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                              _dp, _dp, _dp, _ip, _ip]
        L.oracle_pmpc_solve_batch.restype = ctypes.c_int
        L.oracle_pmpc_rk4.argtypes = [ctypes.c_double, ctypes.c_double, _dp, _dp, _dp]
        L.oracle_pmpc_rk4.restype = None
        _lib = L
    return _lib


def _p(a, t=_dp):
    return a.ctypes.data_as(t)


def solve_batch(states, targets, params, N=20, Ts=0.002, max_iter=200, tol=1e-9, nthreads=1, want_w=True, soc=True,
                mult_init_max=1000.0, resto=True):
    """PMPC oracle.  resto: IPOPT's soft restoration and restoration phases (default on, as IPOPT); off, a
    failed filter line search ends the solve at status -2."""
    states = np.ascontiguousarray(states, np.float64)
    targets = np.ascontiguousarray(targets, np.float64)
    params = np.ascontiguousarray(params, np.float64)
    B = states.shape[0]
    nw = 6 * (N + 1) + 2 * N
    u0 = np.zeros((B, 2))
    f = np.zeros(B)
    w = np.zeros((B, nw)) if want_w else None
    st = np.zeros(B, np.int32)
    it = np.zeros(B, np.int32)
    lib().oracle_pmpc_set_soc(_max_soc(soc))
    lib().oracle_pmpc_set_mult_init_max(ctypes.c_double(float(mult_init_max)))
    lib().oracle_pmpc_set_resto(int(bool(resto)))
    lib().oracle_pmpc_solve_batch(B, N, Ts, _p(states), _p(targets), _p(params), max_iter, tol, nthreads,
                                  _p(u0), _p(f), _p(w) if want_w else None, _p(st, _ip), _p(it, _ip))
    return dict(u0=u0, f=f, w=w, status=st, iters=it)


def rk4(Ts, mu, x, u):
    x = np.ascontiguousarray(x, np.float64)
    u = np.ascontiguousarray(u, np.float64)
    out = np.zeros(6)
    lib().oracle_pmpc_rk4(Ts, mu, _p(x), _p(u), _p(out))
    return out


# --------------------------------------------------------------------------- RMPC
_rlib = None
_RLIB_PATH = os.path.join(_HERE, "liboracle_rmpc.so")


def rlib():
    global _rlib
    if _rlib is None:
        if not os.path.exists(_RLIB_PATH):
            build()
        L = ctypes.CDLL(_RLIB_PATH)
        L.oracle_rmpc_solve_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp, _dp, _dp, _dp, _dp,
                                              _dp, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                              _dp, _dp, _dp, _ip, _ip]
        L.oracle_rmpc_solve_batch.restype = ctypes.c_int
        L.oracle_rls_update.argtypes = [_dp, _dp, _dp, ctypes.c_double, ctypes.c_double]
        L.oracle_rls_update.restype = None
        L.oracle_rmpc_set_relax.argtypes = [ctypes.c_double]
        L.oracle_rmpc_set_relax.restype = None
        L.oracle_rmpc_set_soc.argtypes = [ctypes.c_int]
        L.oracle_rmpc_set_soc.restype = None
        L.oracle_rmpc_set_resto.argtypes = [ctypes.c_int]
        L.oracle_rmpc_set_resto.restype = None
        L.oracle_rmpc_set_slack_shift.argtypes = [ctypes.c_int]
        L.oracle_rmpc_set_slack_shift.restype = None
        _rlib = L
    return _rlib


def rmpc_solve_batch(x0, u_prev, theta, Rref, prm, N=20, Ts=0.002, w_init=None, max_iter=200, tol=1e-8,
                     nthreads=1, want_w=True, relax=1e-8, soc=True, mult_init_max=1000.0, resto=True, slack_shift=False):
    """resto: IPOPT's soft restoration and restoration phases (default on, as IPOPT); off, a failed filter
    line search ends the solve at status -2.  soc: max_soc of the original and the restoration line
    searches.  slack_shift: IPOPT's inertia shift of the slack block (delta_s = delta_x; off by default,
    never engaged on the RMPC workloads)."""
    c = lambda a: np.ascontiguousarray(a, np.float64)
    x0, u_prev, theta, Rref, prm = c(x0), c(u_prev), c(theta), c(Rref), c(prm)
    B = x0.shape[0]
    nw = 4 * (N + 1) + 2 * N
    wi = None if w_init is None else c(w_init)
    u0 = np.zeros((B, 2)); f = np.zeros(B); w = np.zeros((B, nw)) if want_w else None
    st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
    rlib().oracle_rmpc_set_relax(float(relax))
    rlib().oracle_rmpc_set_soc(_max_soc(soc))
    rlib().oracle_rmpc_set_mult_init_max(ctypes.c_double(float(mult_init_max)))
    rlib().oracle_rmpc_set_resto(int(bool(resto)))
    rlib().oracle_rmpc_set_slack_shift(int(bool(slack_shift)))
    rlib().oracle_rmpc_solve_batch(B, N, Ts, _p(x0), _p(u_prev), _p(theta), _p(Rref), _p(prm),
                                   _p(wi) if wi is not None else None, max_iter, tol, nthreads,
                                   _p(u0), _p(f), _p(w) if want_w else None, _p(st, _ip), _p(it, _ip))
    return dict(u0=u0, f=f, w=w, status=st, iters=it)


def rls_update(theta, P, phi, y, lam=0.995):
    th = np.ascontiguousarray(theta, np.float64).copy()
    Pm = np.ascontiguousarray(P, np.float64).copy()
    rlib().oracle_rls_update(_p(th), _p(Pm), _p(np.ascontiguousarray(phi, np.float64)), float(y), lam)
    return th, Pm


_llib = None


def llib():
    global _llib
    if _llib is None:
        L = ctypes.CDLL(os.path.join(_HERE, "liboracle_lmpc.so"))
        L.oracle_lmpc_solve_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp, _dp, _dp, _dp, _dp,
                                              _dp, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                              ctypes.c_int, _dp, _dp, _dp, _ip, _ip]
        L.oracle_lmpc_solve_batch.restype = ctypes.c_int
        L.oracle_lmpc_set_relax.argtypes = [ctypes.c_double]
        L.oracle_lmpc_set_relax.restype = None
        L.oracle_lmpc_set_soc.argtypes = [ctypes.c_int]
        L.oracle_lmpc_set_soc.restype = None
        L.oracle_lmpc_set_soft_resto.argtypes = [ctypes.c_int]
        L.oracle_lmpc_set_soft_resto.restype = None
        L.oracle_lmpc_set_resto.argtypes = [ctypes.c_int]
        L.oracle_lmpc_set_resto.restype = None
        L.oracle_lmpc_set_resto_refine.argtypes = [ctypes.c_int]
        L.oracle_lmpc_set_resto_refine.restype = None
        L.oracle_lmpc_rk4.argtypes = [ctypes.c_int, ctypes.c_double, _dp, _dp, _dp, _dp]
        L.oracle_lmpc_rk4.restype = None
        _llib = L
    return _llib


LMPC_PRM_DEFAULT = np.array([200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0,      # Q   (LMPC/src/run.py:118)
                             200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0,      # Qt  (:119)
                             0.1, 0.1, 1.0, 1.0,                              # R   (:120)
                             -0.4, 0.4])                                      # u_bounds (:121)


def lmpc_solve_batch(state, u_prev, pvec, target, prm=None, N=20, Ts=0.002, w_init=None, max_iter=50, tol=1e-4,
                     acc_tol=1e-3, acc_iter=5, nthreads=1, want_w=True, relax=1e-8, soc=True, mult_init_max=1000.0,
                     resto=True, resto_refine=3):
    """LMPC oracle; defaults are the reference's IPOPT options (rlmpc2.py:480-489).  resto=False turns
    IPOPT's soft restoration and restoration phases off (a failed line search then ends with status -2);
    resto_refine caps the iterative-refinement solves per restoration step (0: none)."""
    c = lambda a: np.ascontiguousarray(a, np.float64)
    state, u_prev, pvec, target = c(state), c(u_prev), c(pvec), c(target)
    B = state.shape[0]
    prm = c(np.tile(LMPC_PRM_DEFAULT, (B, 1)) if prm is None else prm)
    nw = 8 * (N + 1) + 2 * N
    wi = None if w_init is None else c(w_init)
    u0 = np.zeros((B, 2)); f = np.zeros(B); w = np.zeros((B, nw)) if want_w else None
    st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
    llib().oracle_lmpc_set_relax(float(relax))
    llib().oracle_lmpc_set_soc(_max_soc(soc))
    llib().oracle_lmpc_set_mult_init_max(ctypes.c_double(float(mult_init_max)))
    llib().oracle_lmpc_set_soft_resto(int(bool(resto)))
    llib().oracle_lmpc_set_resto(int(bool(resto)))
    llib().oracle_lmpc_set_resto_refine(int(resto_refine))
    llib().oracle_lmpc_solve_batch(B, N, Ts, _p(state), _p(u_prev), _p(pvec), _p(target), _p(prm),
                                   _p(wi) if wi is not None else None, max_iter, tol, acc_tol, acc_iter, nthreads,
                                   _p(u0), _p(f), _p(w) if want_w else None, _p(st, _ip), _p(it, _ip))
    return dict(u0=u0, f=f, w=w, status=st, iters=it)


def lmpc_rk4(x, u, pvec, Ts=0.002):
    x, u, pvec = (np.ascontiguousarray(a, np.float64) for a in (x, u, pvec))
    xn = np.zeros_like(x)
    llib().oracle_lmpc_rk4(x.shape[0], Ts, _p(x), _p(u), _p(pvec), _p(xn))
    return xn
