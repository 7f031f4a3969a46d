"""PMPC NLP restatement in numpy -- TEST INFRASTRUCTURE ONLY.

This module is part of the *oracle*: a CPU fp64 restatement of the tray-tilt
MPC nonlinear program that the reference hands to CasADi+IPOPT.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it, and only as the checker.  The shipped solver never calls it.

Parity status: CasADi/IPOPT are not importable in this image,
so parity against the reference *solver* is unpinned.  The formulation below is
pinned instead by (i) the analytic known-answer tests of SURVEY §8c (RK4 closed
form, u*=0 at rest on target, mirror symmetry), (ii) two independent
solvers that must agree (scipy SLSQP on the full multiple-shooting NLP, and
``projected_newton`` on the condensed single-shooting problem), and (iii) the solver-independent KKT
certificate ``kkt_certificate``.

Every function cites the reference line it restates
(paths relative to the reference root).
"""
from __future__ import annotations

import numpy as np

GRAVITY_Z = -9.81          # model.opt.gravity[2]  (PMPC/src/controller/mpc_3d.py:23; world xml line 5)
TS_DEFAULT = 0.002         # MuJoCo default timestep
NX, NU = 6, 2              # mpc_3d.py:12


# --------------------------------------------------------------------------
# P1  continuous dynamics            PMPC/src/controller/mpc_3d.py:87-97
# --------------------------------------------------------------------------
def dynamics(x, u, mu, Ts, g=GRAVITY_Z):
    """x[...,6]=[px,vx,py,vy,pz,vz], u[...,2]=[theta_x,theta_y] -> xdot[...,6].

    Works on real or complex arrays (complex-step differentiation)."""
    vx, vy, vz = x[..., 1], x[..., 3], x[..., 5]
    tx, ty = u[..., 0], u[..., 1]
    ax = g * np.sin(tx) - mu * vx                     # :91
    ay = g * np.sin(ty) - mu * vy                     # :92
    vz_new = -g * (tx ** 2 + ty ** 2)                 # :93  (pz-rate is vz_new, not vz)
    az = (vz_new - vz) / Ts                           # :95
    return np.stack([vx, ax, vy, ay, vz_new, az], axis=-1)   # :97


# --------------------------------------------------------------------------
# P2  RK4 with u held constant        mpc_3d.py:99-104 (self.f at :28-30)
# --------------------------------------------------------------------------
def rk4_step(x, u, mu, Ts, g=GRAVITY_Z):
    k1 = dynamics(x, u, mu, Ts, g)
    k2 = dynamics(x + Ts / 2 * k1, u, mu, Ts, g)
    k3 = dynamics(x + Ts / 2 * k2, u, mu, Ts, g)
    k4 = dynamics(x + Ts * k3, u, mu, Ts, g)
    return x + Ts / 6 * (k1 + 2 * k2 + 2 * k3 + k4)


# --------------------------------------------------------------------------
# P3  NLP transcription               mpc_3d.py:32-85
# --------------------------------------------------------------------------
class PMPCProblem:
    """Direct multiple shooting NLP of ``PMPC.__init__``.

    w = [x_0 .. x_N (6 each, = vec(X) column-major), u_0 .. u_{N-1} (2 each)]   (:69)
    p = [state(6); target(6)]                                                     (:34)
    g = [x_0 - state; x_{k+1} - f(x_k,u_k) for k<N]  with lbg = ubg = 0             (:37,:48,:129)
    f = sum_{k<N} Qp|pos-r|^2 + Qv|vel-r|^2 + R|u_k|^2  + terminal Qp,Qv terms     (:44-46,:63-66)
    bounds: X free, U in [u_lo, u_hi]                                              (:71-79)
    """

    def __init__(self, N=20, Ts=TS_DEFAULT, Qp=100.0, Qv=0.0, R=0.1, mu=0.4,
                 u_bounds=(-0.5, 0.5), g=GRAVITY_Z):
        self.N, self.Ts = int(N), float(Ts)
        self.Qp, self.Qv, self.R, self.mu = float(Qp), float(Qv), float(R), float(mu)
        self.u_lo, self.u_hi = float(u_bounds[0]), float(u_bounds[1])
        self.g = float(g)
        self.nX = NX * (self.N + 1)
        self.nU = NU * self.N
        self.nw = self.nX + self.nU
        self.ng = NX * (self.N + 1)

    # -- layout helpers ----------------------------------------------------
    def unpack(self, w):
        w = np.asarray(w)
        X = w[: self.nX].reshape(self.N + 1, NX)
        U = w[self.nX:].reshape(self.N, NU)
        return X, U

    def pack(self, X, U):
        return np.concatenate([np.asarray(X).reshape(-1), np.asarray(U).reshape(-1)])

    def bounds(self):
        lbx = np.concatenate([np.full(self.nX, -np.inf), np.full(self.nU, self.u_lo)])
        ubx = np.concatenate([np.full(self.nX, np.inf), np.full(self.nU, self.u_hi)])
        return lbx, ubx

    def init_guess(self, state):
        """Cold start of ``PMPC.solve``: state tiled N+1 times, zero controls (:123)."""
        return np.concatenate([np.tile(np.asarray(state, float), self.N + 1), np.zeros(self.nU)])

    # -- objective -----------------------------------------------------------
    def objective(self, w, p):
        X, U = self.unpack(w)
        ref = np.asarray(p)[NX:]
        ep = (X[:, 0] - ref[0]) ** 2 + (X[:, 2] - ref[2]) ** 2
        ev = (X[:, 1] - ref[1]) ** 2 + (X[:, 3] - ref[3]) ** 2
        return (self.Qp * ep.sum() + self.Qv * ev.sum() + self.R * (U ** 2).sum())

    def objective_grad(self, w, p):
        X, U = self.unpack(w)
        ref = np.asarray(p)[NX:]
        gX = np.zeros_like(X)
        gX[:, 0] = 2 * self.Qp * (X[:, 0] - ref[0])
        gX[:, 2] = 2 * self.Qp * (X[:, 2] - ref[2])
        gX[:, 1] = 2 * self.Qv * (X[:, 1] - ref[1])
        gX[:, 3] = 2 * self.Qv * (X[:, 3] - ref[3])
        gU = 2 * self.R * U
        return self.pack(gX, gU)

    # -- constraints ---------------------------------------------------------
    def step(self, X, U):
        return rk4_step(X, U, self.mu, self.Ts, self.g)

    def constraints(self, w, p):
        X, U = self.unpack(w)
        state = np.asarray(p)[:NX]
        g0 = X[0] - state
        gk = X[1:] - self.step(X[:-1], U)
        return np.concatenate([g0, gk.reshape(-1)])

    def step_jacobians(self, X, U, h=1e-30):
        """Complex-step Jacobians of the RK4 map: A[k]=d x+/d x_k, B[k]=d x+/d u_k."""
        N = X.shape[0]
        A = np.zeros((N, NX, NX))
        B = np.zeros((N, NX, NU))
        Xc = X.astype(complex)
        Uc = U.astype(complex)
        for j in range(NX):
            Xp = Xc.copy()
            Xp[:, j] += 1j * h
            A[:, :, j] = self.step(Xp, Uc).imag / h
        for j in range(NU):
            Up = Uc.copy()
            Up[:, j] += 1j * h
            B[:, :, j] = self.step(Xc, Up).imag / h
        return A, B

    def constraint_jac(self, w, p):
        X, U = self.unpack(w)
        A, B = self.step_jacobians(X[:-1], U)
        J = np.zeros((self.ng, self.nw))
        J[:NX, :NX] = np.eye(NX)
        for k in range(self.N):
            r = NX * (k + 1)
            J[r:r + NX, NX * (k + 1):NX * (k + 2)] = np.eye(NX)
            J[r:r + NX, NX * k:NX * (k + 1)] = -A[k]
            J[r:r + NX, self.nX + NU * k:self.nX + NU * (k + 1)] = -B[k]
        return J


# --------------------------------------------------------------------------
# Solver-independent KKT certificate
# --------------------------------------------------------------------------
def multipliers_from_state_rows(prob: PMPCProblem, w, p):
    """Equality multipliers that zero the state rows of grad L (unique: triangular).

    L = f + lam^T g.  State rows: grad_x f + J_x^T lam = 0, J_x is block lower
    bidiagonal with identity diagonal, so lam is recovered by back substitution.
    """
    X, U = prob.unpack(w)
    gf = prob.objective_grad(w, p)
    gX = gf[: prob.nX].reshape(prob.N + 1, NX)
    A, _ = prob.step_jacobians(X[:-1], U)
    lam = np.zeros((prob.N + 1, NX))
    lam[prob.N] = -gX[prob.N]
    for k in range(prob.N - 1, -1, -1):
        lam[k] = -gX[k] + A[k].T @ lam[k + 1]
    return lam.reshape(-1)


def kkt_certificate(prob: PMPCProblem, w, p, relax=1e-8, act_tol=1e-6):
    """Return a dict of KKT residuals for a candidate optimum ``w``.

    - primal: ||g(w)||_inf
    - bound: max violation of the (IPOPT bound_relax_factor-relaxed) box
    - stat_free: ||grad_u L||_inf over controls strictly inside the box
    - stat_sign: worst sign violation of grad_u L at active bounds
      (at the upper bound grad_u L <= 0, at the lower bound >= 0)
    - lam: the recovered equality multipliers
    A control within ``act_tol`` of a bound counts as active (an interior-point
    answer at tolerance tol sits mu/z inside a weakly active bound).
    """
    w = np.asarray(w, float)
    X, U = prob.unpack(w)
    gval = prob.constraints(w, p)
    lam = multipliers_from_state_rows(prob, w, p)
    J = prob.constraint_jac(w, p)
    gradL = prob.objective_grad(w, p) + J.T @ lam
    gu = gradL[prob.nX:]
    u = w[prob.nX:]
    lo = prob.u_lo - relax * max(1.0, abs(prob.u_lo))
    hi = prob.u_hi + relax * max(1.0, abs(prob.u_hi))
    at_hi = u >= prob.u_hi - act_tol
    at_lo = u <= prob.u_lo + act_tol
    free = ~(at_hi | at_lo)
    stat_free = float(np.max(np.abs(gu[free]), initial=0.0))
    stat_sign = float(max(np.max(gu[at_hi], initial=-np.inf), np.max(-gu[at_lo], initial=-np.inf), 0.0))
    bound = float(max(np.max(lo - u, initial=0.0), np.max(u - hi, initial=0.0), 0.0))
    return dict(primal=float(np.max(np.abs(gval))), bound=bound, stat_free=stat_free,
                stat_sign=stat_sign, lam=lam, grad_scale=float(np.max(np.abs(prob.objective_grad(w, p)))))


# --------------------------------------------------------------------------
# Condensed single-shooting view (used only by the independent golden solver)
# --------------------------------------------------------------------------
def rollout(prob: PMPCProblem, state, U):
    X = np.zeros((prob.N + 1, NX), dtype=np.result_type(U, float))
    X[0] = state
    for k in range(prob.N):
        X[k + 1] = prob.step(X[k], U[k])
    return X


def condensed_cost_grad(prob: PMPCProblem, p, uflat):
    """Single-shooting cost and its adjoint gradient w.r.t. the controls."""
    U = uflat.reshape(prob.N, NU)
    state = np.asarray(p)[:NX]
    X = rollout(prob, state, U)
    w = prob.pack(X, U)
    cost = prob.objective(w, p)
    gf = prob.objective_grad(w, p)
    gX = gf[: prob.nX].reshape(prob.N + 1, NX)
    gU = gf[prob.nX:].reshape(prob.N, NU).copy()
    A, B = prob.step_jacobians(X[:-1], U)
    adj = gX[prob.N].copy()
    for k in range(prob.N - 1, -1, -1):
        gU[k] += B[k].T @ adj
        adj = gX[k] + A[k].T @ adj
    return cost, gU.reshape(-1)


# --------------------------------------------------------------------------
# Reference parameter tables
# --------------------------------------------------------------------------
# PMPC/main_parallel_enhanced.py:171-179 (per-shape weights, N=15 in the driver;
# the BASELINE configs use N=20), u in [-0.6, 0.6]
SHAPE_PARAMS = {
    "cube": dict(Qp=600.0, Qv=5.0, R=0.1),
    "cylinder": dict(Qp=400.0, Qv=2.5, R=0.2),
    "sphere": dict(Qp=200.0, Qv=2.0, R=0.2),
    "general": dict(Qp=300.0, Qv=2.0, R=0.2),
}
SHAPES = ("cube", "cylinder", "sphere")
MASSES = (1.0, 2.0)           # no effect on the PMPC NLP
FRICTIONS = (0.05, 0.10, 0.20)
U_BOUNDS = (-0.6, 0.6)


def projected_newton(prob: PMPCProblem, p, u0=None, iters=60, fd_h=1e-6):
    """Independent golden solver: projected Newton on the condensed problem.

    Gradient: exact adjoint (``condensed_cost_grad``).  Hessian: central
    differences of that gradient (affects only the rate, not the fixed point).
    Active set: a control at a bound whose gradient points outward is fixed.
    Returns (u[N*2], n_iter).
    """
    lo, hi = prob.u_lo, prob.u_hi
    u = np.zeros(prob.nU) if u0 is None else np.clip(np.asarray(u0, float), lo, hi)
    n = prob.nU
    for it in range(iters):
        f, g = condensed_cost_grad(prob, p, u)
        act = ((u <= lo + 1e-14) & (g > 0)) | ((u >= hi - 1e-14) & (g < 0))
        free = ~act
        pg = np.where(free, g, 0.0)
        if np.max(np.abs(pg)) < 1e-13 * max(1.0, abs(f)):
            return u, it
        H = np.zeros((n, n))
        for j in range(n):
            e = np.zeros(n); e[j] = fd_h
            H[:, j] = (condensed_cost_grad(prob, p, u + e)[1] - condensed_cost_grad(prob, p, u - e)[1]) / (2 * fd_h)
        H = 0.5 * (H + H.T)
        d = np.zeros(n)
        Hf = H[np.ix_(free, free)]
        # guard against indefiniteness far from the optimum
        ev = np.linalg.eigvalsh(Hf) if Hf.size else np.array([1.0])
        shift = max(0.0, 1e-8 - ev.min())
        d[free] = -np.linalg.solve(Hf + shift * np.eye(Hf.shape[0]), g[free])
        t = 1.0
        while t > 1e-12:
            un = np.clip(u + t * d, lo, hi)
            fn, _ = condensed_cost_grad(prob, p, un)
            if fn <= f + 1e-4 * g @ (un - u) or np.max(np.abs(un - u)) < 1e-15:
                break
            t *= 0.5
        u = un
    return u, iters
