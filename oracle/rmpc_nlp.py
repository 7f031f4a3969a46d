"""RMPC (regressor NMPC + online RLS) restated in numpy -- TEST INFRASTRUCTURE ONLY.

Oracle for SURVEY.md §8a rows R1-R6.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it, as the checker.  Restates (paths
relative to the reference root, file RMPC/dev_dual/controller/
np_mpc_adaptive_with_linear_regressor.py unless noted):

  R1  RLS                        :10-30
  R2  feature/target build       RMPC/dev_dual/rob_ctrl.py:335-343
  R3  reference governor         rob_ctrl.py:346-348, build_ref_traj :201-210
  R4  _phi/_dyn_regressor/_rk4   :171-193
  R5  NLP                        :35-168
  R6  solve (warm start w0)      :212-222

Parity status: unpinned against CasADi+IPOPT (not installed) and the
reference has no RMPC fixtures; the goldens (tests/golden/make_rmpc_goldens.py) are
pinned by two independent solvers (scipy SLSQP on this restatement and the C
oracle oracle/rmpc_ipm.c on the exact NLP) agreeing to <= 5e-8, plus the
solver-independent KKT certificate ``kkt_certificate``.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import lsq_linear

GRAVITY_Z = -9.81
NX, NU, NTH = 4, 2, 14


# R1 -------------------------------------------------------------------------
class RLS:
    """Exponentially weighted recursive least squares (np_mpc...:10-30)."""

    def __init__(self, p, theta0=None, P0=1e3, lam=0.995):
        self.p = p
        self.theta = np.zeros(p) if theta0 is None else np.asarray(theta0, float).copy()
        self.P = np.eye(p) * float(P0)
        self.lam = float(lam)

    def update(self, phi, y):
        phi = np.asarray(phi, dtype=float).reshape(-1)
        y = float(np.asarray(y).reshape(()))
        denom = self.lam + phi @ self.P @ phi                 # :22
        K = (self.P @ phi) / denom                            # :23
        err = y - (phi @ self.theta)                          # :24
        self.theta = self.theta + K * err                     # :26
        self.P = (self.P - np.outer(K, phi) @ self.P) / self.lam   # :27

    def get(self):
        return self.theta.copy()


# R2 -------------------------------------------------------------------------
def rls_features(prev_state, v_eps):
    """phi_prev = [px, vx, py, vy, tanh(vx/v_eps), tanh(vy/v_eps), 1] (rob_ctrl.py:338-339)."""
    px, vx, py, vy = prev_state
    return np.array([px, vx, py, vy, np.tanh(vx / v_eps), np.tanh(vy / v_eps), 1.0])


def rls_targets(state, prev_state, Ts):
    """Measured accelerations by finite difference, gravity not removed (rob_ctrl.py:336-337)."""
    return (state[1] - prev_state[1]) / Ts, (state[3] - prev_state[3]) / Ts


# R3 -------------------------------------------------------------------------
def governor_step(r_v, target, dr_max=0.01, alpha_rg=0.5):
    """r_v += alpha * clip(target - r_v, +-dr_max) on x, y (rob_ctrl.py:345-348)."""
    err = np.array([target[0] - r_v[0], 0.0, target[2] - r_v[2], 0.0])
    step = np.array([np.clip(err[0], -dr_max, dr_max), 0.0, np.clip(err[2], -dr_max, dr_max), 0.0])
    return r_v + alpha_rg * step


def build_ref_traj(x_now, r_v, target, N, nx=4, step_fraction=0.2):
    """Staged reference (np_mpc...:201-210)."""
    R = np.zeros((N + 1, nx))
    for i in range(N + 1):
        w = 1.0 - (1.0 - step_fraction) ** (i + 1)
        r_i = r_v + w * (target - r_v)
        R[i, :] = np.array([r_i[0], 0.0, r_i[2], 0.0])
    return R.reshape(-1)


# R4 -------------------------------------------------------------------------
def phi(x, v_eps):
    return np.stack([x[..., 0], x[..., 1], x[..., 2], x[..., 3],
                     np.tanh(x[..., 1] / v_eps), np.tanh(x[..., 3] / v_eps), np.ones_like(x[..., 0])], axis=-1)


def dyn(x, u, th, v_eps, gz=GRAVITY_Z):
    f = phi(x, v_eps)
    ax = gz * np.sin(u[..., 0]) + (f * th[:7]).sum(-1)      # :184
    ay = gz * np.sin(u[..., 1]) + (f * th[7:]).sum(-1)      # :185
    return np.stack([x[..., 1], ax, x[..., 3], ay], axis=-1)


def rk4(x, u, th, v_eps, Ts, gz=GRAVITY_Z):
    k1 = dyn(x, u, th, v_eps, gz)
    k2 = dyn(x + Ts / 2 * k1, u, th, v_eps, gz)
    k3 = dyn(x + Ts / 2 * k2, u, th, v_eps, gz)
    k4 = dyn(x + Ts * k3, u, th, v_eps, gz)
    return x + Ts / 6 * (k1 + 2 * k2 + 2 * k3 + k4)


# R5 -------------------------------------------------------------------------
class RMPCProblem:
    """NLP of AdaptiveNPMPCSmooth.__init__ (np_mpc...:35-168).

    w = [x_0..x_N (4 each); u_0..u_{N-1} (2 each)]
    p = [x0(4); u_prev(2); theta_hat(14); Rref((N+1)*4)]
    g = [x_0 - x0 (4)] + per k: [defect(4); du_k(2); vx-vmax, -vx-vmax, vy-vmax, -vy-vmax (4)]
    """

    def __init__(self, Ts=0.002, N=20, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0, u_bounds=(-0.6, 0.6),
                 du_bounds=(-0.06, 0.06), vmax=0.2, v_eps=0.1, gz=GRAVITY_Z):
        self.Ts, self.N = float(Ts), int(N)
        self.Qp, self.Qv, self.Ru, self.Rdu = float(Qp), float(Qv), float(Ru), float(Rdu)
        self.u_lo, self.u_hi = map(float, u_bounds)
        self.du_lo, self.du_hi = map(float, du_bounds)
        self.vmax, self.v_eps, self.gz = float(vmax), float(v_eps), float(gz)
        self.nX = NX * (self.N + 1)
        self.nU = NU * self.N
        self.nw = self.nX + self.nU
        self.ng = NX + 10 * self.N
        self.np = NX + NU + NTH + (self.N + 1) * NX

    def unpack(self, w):
        w = np.asarray(w)
        return w[: self.nX].reshape(self.N + 1, NX), w[self.nX:].reshape(self.N, NU)

    def pack(self, X, U):
        return np.concatenate([np.asarray(X).reshape(-1), np.asarray(U).reshape(-1)])

    def split_p(self, p):
        p = np.asarray(p, float)
        x0, up, th = p[:4], p[4:6], p[6:20]
        R = p[20:].reshape(self.N + 1, NX)
        return x0, up, th, R

    def bounds(self):
        lbx = np.concatenate([np.full(self.nX, -np.inf), np.full(self.nU, self.u_lo)])
        ubx = np.concatenate([np.full(self.nX, np.inf), np.full(self.nU, self.u_hi)])
        return lbx, ubx

    def gbounds(self):
        lbg = [0.0] * NX
        ubg = [0.0] * NX
        for _ in range(self.N):
            lbg += [0.0] * NX + [self.du_lo] * NU + [-np.inf] * 4      # :111, :120, :126
            ubg += [0.0] * NX + [self.du_hi] * NU + [0.0] * 4
        return np.array(lbg), np.array(ubg)

    def du(self, U, up):
        return U - np.vstack([up[None, :], U[:-1]])               # :115-118

    def objective(self, w, p):
        X, U = self.unpack(w)
        _, up, _, R = self.split_p(p)
        D = self.du(U, up)
        ep = (X[:, 0] - R[:, 0]) ** 2 + (X[:, 2] - R[:, 2]) ** 2
        ev = (X[:, 1] - R[:, 1]) ** 2 + (X[:, 3] - R[:, 3]) ** 2
        return float(self.Qp * ep.sum() + self.Qv * ev.sum() + self.Ru * (U ** 2).sum() + self.Rdu * (D ** 2).sum())

    def objective_grad(self, w, p):
        X, U = self.unpack(w)
        _, up, _, R = self.split_p(p)
        gX = np.zeros_like(X)
        gX[:, 0] = 2 * self.Qp * (X[:, 0] - R[:, 0]); gX[:, 2] = 2 * self.Qp * (X[:, 2] - R[:, 2])
        gX[:, 1] = 2 * self.Qv * (X[:, 1] - R[:, 1]); gX[:, 3] = 2 * self.Qv * (X[:, 3] - R[:, 3])
        D = self.du(U, up)
        gU = 2 * self.Ru * U + 2 * self.Rdu * D
        gU[:-1] -= 2 * self.Rdu * D[1:]
        return self.pack(gX, gU)

    def step(self, X, U, th):
        return rk4(X, U, th, self.v_eps, self.Ts, self.gz)

    def constraints(self, w, p):
        X, U = self.unpack(w)
        x0, up, th, _ = self.split_p(p)
        D = self.du(U, up)
        F = self.step(X[:-1], U, th)
        out = [X[0] - x0]
        for k in range(self.N):
            vx, vy = X[k, 1], X[k, 3]
            out += [X[k + 1] - F[k], D[k], np.array([vx - self.vmax, -vx - self.vmax, vy - self.vmax, -vy - self.vmax])]
        return np.concatenate(out)

    def step_jacobians(self, X, U, th, h=1e-30):
        n = X.shape[0]
        A = np.zeros((n, NX, NX)); B = np.zeros((n, NX, NU))
        Xc, Uc = X.astype(complex), U.astype(complex)
        for j in range(NX):
            Xp = Xc.copy(); Xp[:, j] += 1j * h
            A[:, :, j] = self.step(Xp, Uc, th).imag / h
        for j in range(NU):
            Up = Uc.copy(); Up[:, j] += 1j * h
            B[:, :, j] = self.step(Xc, Up, th).imag / h
        return A, B

    def constraint_jac(self, w, p):
        X, U = self.unpack(w)
        _, _, th, _ = self.split_p(p)
        A, B = self.step_jacobians(X[:-1], U, th)
        J = np.zeros((self.ng, self.nw))
        J[:NX, :NX] = np.eye(NX)
        for k in range(self.N):
            r = NX + 10 * k
            J[r:r + NX, NX * (k + 1):NX * (k + 2)] = np.eye(NX)
            J[r:r + NX, NX * k:NX * (k + 1)] = -A[k]
            J[r:r + NX, self.nX + NU * k:self.nX + NU * (k + 1)] = -B[k]
            J[r + 4:r + 6, self.nX + NU * k:self.nX + NU * (k + 1)] = np.eye(NU)
            if k > 0:
                J[r + 4:r + 6, self.nX + NU * (k - 1):self.nX + NU * k] = -np.eye(NU)
            J[r + 6, NX * k + 1] = 1.0; J[r + 7, NX * k + 1] = -1.0
            J[r + 8, NX * k + 3] = 1.0; J[r + 9, NX * k + 3] = -1.0
        return J


def kkt_certificate(prob: RMPCProblem, w, p, act_tol=1e-6):
    """Solver-independent KKT check: primal feasibility of every row/bound, and the
    smallest stationarity residual ||grad f + J^T y - z|| over multipliers with
    the sign pattern of the active set (inactive inequalities/bounds forced to 0)."""
    w = np.asarray(w, float)
    g = prob.constraints(w, p)
    lbg, ubg = prob.gbounds()
    lbx, ubx = prob.bounds()
    prim = max(float(np.max(np.maximum(lbg - g, 0.0))), float(np.max(np.maximum(g - ubg, 0.0))))
    eq = lbg == ubg
    prim = max(prim, float(np.max(np.abs(g[eq]))))
    bnd = max(float(np.max(np.maximum(lbx - w, 0.0))), float(np.max(np.maximum(w - ubx, 0.0))))
    J = prob.constraint_jac(w, p)
    gf = prob.objective_grad(w, p)
    cols, lo, hi = [], [], []
    for i in range(prob.ng):          # L = f + y^T g: y free on equalities, >= 0 at upper, <= 0 at lower
        if eq[i]:
            cols.append(J[i]); lo.append(-np.inf); hi.append(np.inf)
        elif g[i] >= ubg[i] - act_tol:
            cols.append(J[i]); lo.append(0.0); hi.append(np.inf)
        elif g[i] <= lbg[i] + act_tol:
            cols.append(J[i]); lo.append(-np.inf); hi.append(0.0)
    for j in range(prob.nw):          # bound multipliers: + at upper, - at lower
        if np.isfinite(ubx[j]) and w[j] >= ubx[j] - act_tol:
            e = np.zeros(prob.nw); e[j] = 1.0; cols.append(e); lo.append(0.0); hi.append(np.inf)
        elif np.isfinite(lbx[j]) and w[j] <= lbx[j] + act_tol:
            e = np.zeros(prob.nw); e[j] = 1.0; cols.append(e); lo.append(-np.inf); hi.append(0.0)
    M = np.array(cols).T
    res = lsq_linear(M, -gf, bounds=(np.array(lo), np.array(hi)), method="bvls", tol=1e-14, max_iter=5000)
    stat = float(np.max(np.abs(M @ res.x + gf)))
    return dict(primal=prim, bound=bnd, stat=stat, grad_scale=float(np.max(np.abs(gf))))


# R6 / driver loop pieces ---------------------------------------------------
RMPC_DEFAULTS = dict(N=20, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0, u_bounds=(-0.6, 0.6), du_bounds=(-0.06, 0.06),
                     vmax=0.2, v_eps=0.1)       # rob_ctrl.py:281-284


# Restoration certificate ---------------------------------------------------
# IPOPT ends at Infeasible_Problem_Detected (status 2) when its restoration problem converges: the point is
# then a stationary point of the l1 constraint violation.  Solver-independent check: the l1 violation of the
# linearised rows cannot decrease within a small box around the point (an LP), while at a point where the
# filter line search merely failed it can.
def l1_model(w, x0, up, th, prm, N=20, Ts=0.002):
    """rows of the reference NLP at w: equality values c (x0 pin + RK4 defects) with Jacobian Jc, inequality values g with
    bounds (lb, ub) and Jacobian Jg (du rows, velocity caps), over w = [X (4(N+1)), U (2N)]"""
    nX, n = 4 * (N + 1), 4 * (N + 1) + 2 * N
    X = w[:nX].reshape(N + 1, 4); U = w[nX:].reshape(N, 2)
    c = [X[0] - x0]; Jc = [np.hstack([np.eye(4), np.zeros((4, n - 4))])]
    for k in range(N):
        f = lambda xu: rk4(xu[:4], xu[4:], th, prm[9], Ts)
        xu = np.concatenate([X[k], U[k]]); h = 1e-7
        Jf = np.stack([(f(xu + h * e) - f(xu - h * e)) / (2 * h) for e in np.eye(6)], 1)
        c.append(X[k + 1] - f(xu))
        J = np.zeros((4, n)); J[:, 4 * (k + 1):4 * (k + 2)] = np.eye(4)
        J[:, 4 * k:4 * k + 4] -= Jf[:, :4]; J[:, nX + 2 * k:nX + 2 * k + 2] -= Jf[:, 4:]
        Jc.append(J)
    g, lb, ub, Jg = [], [], [], []
    for k in range(N):
        for a in range(2):
            row = np.zeros(n); row[nX + 2 * k + a] = 1
            if k > 0: row[nX + 2 * (k - 1) + a] = -1
            g.append(U[k, a] - (up[a] if k == 0 else U[k - 1, a])); lb.append(prm[6]); ub.append(prm[7]); Jg.append(row)
        for j in (1, 3):
            row = np.zeros(n); row[4 * k + j] = 1
            g.append(X[k, j]); lb.append(-prm[8]); ub.append(prm[8]); Jg.append(row)
    return np.concatenate(c), np.vstack(Jc), np.array(g), np.array(lb), np.array(ub), np.array(Jg)

def l1_violation(w, x0, up, th, prm, N=20, Ts=0.002, relax=1e-8):
    """l1 violation V(w) of the reference NLP's rows (np_mpc...:103-127): |x0 pin| + |RK4 defects| (equalities) and
    the du rows / velocity caps outside their bounds (relaxed by IPOPT's bound_relax_factor); the U box is kept by
    both solvers.  IPOPT's restoration phase (MinC_1NrmRestorationPhase) minimises this quantity."""
    nX = 4 * (N + 1)
    X = w[:nX].reshape(N + 1, 4)
    U = w[nX:].reshape(N, 2)
    v = np.abs(X[0] - x0).sum()
    for k in range(N):
        v += np.abs(X[k + 1] - rk4(X[k], U[k], th, prm[9], Ts)).sum()
    lo, hi = prm[6] - relax * max(1, abs(prm[6])), prm[7] + relax * max(1, abs(prm[7]))
    du = np.diff(np.vstack([np.asarray(up)[None], U]), axis=0)
    v += np.maximum(0, du - hi).sum() + np.maximum(0, lo - du).sum()
    vm = prm[8] + relax * max(1, prm[8])
    v += np.maximum(0, np.abs(X[:N][:, [1, 3]]) - vm).sum()
    return float(v)


def l1_stationarity(w, x0, up, th, prm, N=20, delta=1e-4, relax=1e-8):
    """decrease of the linearised l1 infeasibility within |d|_inf <= delta, U box kept; and the value at d = 0"""
    c, Jc, g, lb, ub, Jg = l1_model(w, x0, up, th, prm, N)
    lb = lb - relax * np.maximum(1, np.abs(lb)); ub = ub + relax * np.maximum(1, np.abs(ub))
    n, me, mi = w.size, c.size, g.size
    # variables [d (n), ep (me), en (me), t (mi)]
    cost = np.concatenate([np.zeros(n), np.ones(2 * me + mi)])
    Aeq = np.hstack([Jc, -np.eye(me), np.eye(me), np.zeros((me, mi))]); beq = -c
    Aub = np.vstack([np.hstack([Jg, np.zeros((mi, 2 * me)), -np.eye(mi)]),
                     np.hstack([-Jg, np.zeros((mi, 2 * me)), -np.eye(mi)])])
    bub = np.concatenate([ub - g, g - lb])
    ulo, uhi = prm[4] - relax, prm[5] + relax
    nX = 4 * (N + 1)
    bounds = [(-delta, delta)] * nX + [(max(-delta, ulo - w[i]), min(delta, uhi - w[i])) for i in range(nX, n)] + [(0, None)] * (2 * me + mi)
    from scipy.optimize import linprog
    res = linprog(cost, A_ub=Aub, b_ub=bub, A_eq=Aeq, b_eq=beq, bounds=bounds, method='highs')
    base = np.abs(c).sum() + np.maximum(0, g - ub).sum() + np.maximum(0, lb - g).sum()
    return base - res.fun, base
