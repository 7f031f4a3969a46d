"""LMPC (learned-parameter NMPC) restated in numpy -- TEST INFRASTRUCTURE ONLY.

Oracle for SURVEY.md §8a rows L1-L4.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it, as the checker.  Restates (paths
relative to the reference root, file LMPC/src/controller/rlmpc2.py unless noted):

  L1  safe_dynamics (8-state translational + rotational Stribeck / rolling model)  :260-429
      (the code's index map :301-334 is authoritative; the docstring :273-285 is stale)
  L2  _rk4                                                                         :431-436
  L3  NLP: w = [X (8 x N+1) ; U (2 x N)], p = [state(8); u_prev(2); pvec(34); target(8)]
      (:241-258), g = [x_0 - state; defects] (:251, :456), cost :444-464 with
      Q = Qt = [200,2,200,2,0,0,0,0], R = [0.1,0.1,1,1], U box +-0.4 (LMPC/src/run.py:118-126)
  L4  IPOPT options max_iter 50, tol 1e-4, acceptable_tol 1e-3, acceptable_iter 5 (:480-489)
      and the warm start w0 <- w_opt of the worker loop (:494-524)

Non-smooth points follow CasADi: d|v|/dv = sign(v) with sign(0) = 0.  Derivatives
here use the complex step with |v| written as sign(Re v) * v, which reproduces that
convention exactly.

Parity status: unpinned against CasADi+IPOPT (not installed) and the
reference holds no LMPC fixtures; goldens (tests/golden/make_lmpc_goldens.py) are
pinned by scipy SLSQP on this restatement and the C oracle oracle/lmpc_ipm.c agreeing
on the exact NLP, plus ``kkt_certificate``.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import lsq_linear

NX, NU, NPV = 8, 2, 34
G_ACC = 9.81                                              # :354 (g = 9.81, tilt forcing)
LMPC_DEFAULTS = dict(N=20, Ts=0.002, Q=(200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0),
                     Qt=(200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0), R=(0.1, 0.1, 1.0, 1.0),
                     u_bounds=(-0.4, 0.4))               # LMPC/src/run.py:114-126
IPOPT_OPTIONS = dict(max_iter=50, tol=1e-4, acceptable_tol=1e-3, acceptable_iter=5)   # :480-489


def _abs(v):
    """|v| with CasADi's derivative convention (sign(0) = 0), complex-step safe."""
    return np.sign(np.real(v)) * v


def squash(p):
    """squash_param (:296-298): |p| + 1e-6 (the bounds arguments are unused)."""
    return _abs(p) + 1e-6


def stribeck(v, F_s, F_c, B, v_s, eps):
    """:372-376: tanh(v/eps) (F_c + (F_s - F_c) exp(-|v|/(v_s + 1e-12))) + B v."""
    e = np.exp(-_abs(v) / (v_s + 1e-12))
    return np.tanh(v / eps) * (F_c + (F_s - F_c) * e) + B * v


def model_params(pv):
    """Unpacked, squashed model parameters (:300-344), as a dict of scalars."""
    pv = np.asarray(pv, float)
    s = squash
    return dict(m_x=s(pv[0]), m_y=s(pv[1]), c_x=s(pv[2]), c_y=s(pv[3]), k_x=s(pv[4]), k_y=s(pv[5]),
                F_s_x=pv[6], F_c_x=pv[7], B_x=pv[8], v_s_x=s(pv[9]), eps_x=s(pv[10]),
                F_s_y=pv[11], F_c_y=pv[12], B_y=pv[13], v_s_y=s(pv[14]), eps_y=s(pv[15]),
                I_x=s(pv[16]), I_y=s(pv[17]), r_x=s(pv[18]), r_y=s(pv[19]),
                c_rot_x=s(pv[20]), c_rot_y=s(pv[21]),
                F_s_rot_x=pv[22], F_c_rot_x=pv[23], B_rot_x=pv[24], v_s_rot_x=s(pv[25]), eps_rot_x=s(pv[26]),
                F_s_rot_y=pv[27], F_c_rot_y=pv[28], B_rot_y=pv[29], v_s_rot_y=s(pv[30]), eps_rot_y=s(pv[31]),
                h_com_x=s(pv[32]), h_com_y=s(pv[33]))


def dyn(x, u, pv):
    """safe_dynamics (:260-429): x[..., 8], u[..., 2] -> xdot[..., 8]."""
    P = model_params(pv)
    px, vx, py, vy = x[..., 0], x[..., 1], x[..., 2], x[..., 3]
    th_x, om_x, th_y, om_y = x[..., 4], x[..., 5], x[..., 6], x[..., 7]
    a, b = u[..., 0], u[..., 1]
    g = G_ACC
    Gx = P["m_x"] * (g * np.sin(a))                                   # :353-357
    Gy = P["m_y"] * (g * np.sin(b))
    Ff_x = stribeck(vx, P["F_s_x"], P["F_c_x"], P["B_x"], P["v_s_x"], P["eps_x"])        # :379-380
    Ff_y = stribeck(vy, P["F_s_y"], P["F_c_y"], P["B_y"], P["v_s_y"], P["eps_y"])
    v_slip_x = vx - P["r_x"] * om_y                                   # :387-391
    v_slip_y = vy - (-P["r_y"] * om_x)
    F_roll_x = stribeck(v_slip_x, P["F_s_x"], P["F_c_x"], P["B_x"], P["v_s_x"], P["eps_x"])   # :395-396
    F_roll_y = stribeck(v_slip_y, P["F_s_y"], P["F_c_y"], P["B_y"], P["v_s_y"], P["eps_y"])
    tau_slip_x = -P["r_y"] * F_roll_y                                 # :402-403
    tau_slip_y = -P["r_x"] * F_roll_x
    T_noslip_x = stribeck(om_x, P["F_s_rot_x"], P["F_c_rot_x"], P["B_rot_x"], P["v_s_rot_x"], P["eps_rot_x"])
    T_noslip_y = stribeck(om_y, P["F_s_rot_y"], P["F_c_rot_y"], P["B_rot_y"], P["v_s_rot_y"], P["eps_rot_y"])
    T_damp_x = P["c_rot_x"] * om_x                                    # :410-411
    T_damp_y = P["c_rot_y"] * om_y
    tau_topple_x = -P["m_y"] * g * P["h_com_x"] * np.sin(th_x)        # :414-415
    tau_topple_y = -P["m_x"] * g * P["h_com_y"] * np.sin(th_y)
    tau_x = tau_slip_x - T_noslip_x - T_damp_x + tau_topple_x         # :418-419
    tau_y = tau_slip_y - T_noslip_y - T_damp_y + tau_topple_y
    al_x = tau_x / (P["I_x"] + 1e-12)                                 # :422-423
    al_y = tau_y / (P["I_y"] + 1e-12)
    rhs_x = Gx - P["c_x"] * vx - P["k_x"] * px - Ff_x - F_roll_x      # :427
    rhs_y = Gy - P["c_y"] * vy - P["k_y"] * py - Ff_y - F_roll_y
    qdd_x = rhs_x / P["m_x"]                                          # :429 (inv of the diagonal M)
    qdd_y = rhs_y / P["m_y"]
    return np.stack([vx, qdd_x, vy, qdd_y, om_x, al_x, om_y, al_y], axis=-1)


def rk4(x, u, pv, Ts):
    """_rk4 (:431-436)."""
    k1 = dyn(x, u, pv)
    k2 = dyn(x + 0.5 * Ts * k1, u, pv)
    k3 = dyn(x + 0.5 * Ts * k2, u, pv)
    k4 = dyn(x + Ts * k3, u, pv)
    return x + Ts * (k1 + 2 * k2 + 2 * k3 + k4) / 6


class LMPCProblem:
    """NLP built by _solver_worker (:236-491).

    w = [x_0..x_N (8 each); u_0..u_{N-1} (2 each)]   (ca.reshape(X,(-1,1)) is column-major: node-major)
    p = [state(8); u_prev(2); pvec(34); target(8)]
    g = [x_0 - state (8)] + per k: [x_{k+1} - F(x_k, u_k, pvec) (8)], all equalities
    """

    def __init__(self, N=20, Ts=0.002, Q=LMPC_DEFAULTS["Q"], Qt=LMPC_DEFAULTS["Qt"], R=LMPC_DEFAULTS["R"],
                 u_bounds=LMPC_DEFAULTS["u_bounds"]):
        self.N, self.Ts = int(N), float(Ts)
        self.Q, self.Qt, self.R = np.asarray(Q, float), np.asarray(Qt, float), np.asarray(R, float)
        self.u_lo, self.u_hi = map(float, u_bounds)
        self.nX = NX * (self.N + 1)
        self.nU = NU * self.N
        self.nw = self.nX + self.nU
        self.ng = NX * (self.N + 1)
        self.np = NX + NU + NPV + NX

    def unpack(self, w):
        w = np.asarray(w)
        return w[: self.nX].reshape(self.N + 1, NX), w[self.nX:].reshape(self.N, NU)

    def pack(self, X, U):
        return np.concatenate([np.asarray(X).reshape(-1), np.asarray(U).reshape(-1)])

    @staticmethod
    def split_p(p):
        p = np.asarray(p, float)
        return p[:8], p[8:10], p[10:44], p[44:52]

    def bounds(self):
        lbx = np.concatenate([np.full(self.nX, -np.inf), np.full(self.nU, self.u_lo)])
        ubx = np.concatenate([np.full(self.nX, np.inf), np.full(self.nU, self.u_hi)])
        return lbx, ubx

    def gbounds(self):
        return np.zeros(self.ng), np.zeros(self.ng)

    def du(self, U, up):
        return U - np.vstack([up[None, :], U[:-1]])                   # :450

    def objective(self, w, p):
        X, U = self.unpack(w)
        _, up, _, tgt = self.split_p(p)
        E = X[:-1] - tgt
        D = self.du(U, up)
        C = np.concatenate([U, D], axis=1)
        eN = X[-1] - tgt
        return float((E * E * self.Q).sum() + (C * C * self.R).sum() + (eN * eN * self.Qt).sum())

    def objective_grad(self, w, p):
        X, U = self.unpack(w)
        _, up, _, tgt = self.split_p(p)
        gX = np.zeros_like(X)
        gX[:-1] = 2 * self.Q * (X[:-1] - tgt)
        gX[-1] = 2 * self.Qt * (X[-1] - tgt)
        D = self.du(U, up)
        gU = 2 * self.R[:2] * U + 2 * self.R[2:] * D
        gU[:-1] -= 2 * self.R[2:] * D[1:]
        return self.pack(gX, gU)

    def constraints(self, w, p):
        X, U = self.unpack(w)
        st, _, pv, _ = self.split_p(p)
        F = rk4(X[:-1], U, pv, self.Ts)
        return np.concatenate([X[0] - st, (X[1:] - F).reshape(-1)])

    def step_jacobians(self, X, U, pv, h=1e-30):
        n = X.shape[0]
        A = np.zeros((n, NX, NX)); B = np.zeros((n, NX, NU))
        Xc, Uc = X.astype(complex), U.astype(complex)
        for j in range(NX):
            Xp = Xc.copy(); Xp[:, j] += 1j * h
            A[:, :, j] = rk4(Xp, Uc, pv, self.Ts).imag / h
        for j in range(NU):
            Up = Uc.copy(); Up[:, j] += 1j * h
            B[:, :, j] = rk4(Xc, Up, pv, self.Ts).imag / h
        return A, B

    def constraint_jac(self, w, p):
        X, U = self.unpack(w)
        _, _, pv, _ = self.split_p(p)
        A, B = self.step_jacobians(X[:-1], U, pv)
        J = np.zeros((self.ng, self.nw))
        J[:NX, :NX] = np.eye(NX)
        for k in range(self.N):
            r = NX * (k + 1)
            J[r:r + NX, NX * (k + 1):NX * (k + 2)] = np.eye(NX)
            J[r:r + NX, NX * k:NX * (k + 1)] = -A[k]
            J[r:r + NX, self.nX + NU * k:self.nX + NU * (k + 1)] = -B[k]
        return J


def kkt_certificate(prob: LMPCProblem, w, p, act_tol=1e-6):
    """Solver-independent KKT check: primal feasibility, and the smallest stationarity
    residual ||grad f + J^T y - z|| over free equality multipliers y and sign-constrained
    multipliers of the active U-box bounds."""
    w = np.asarray(w, float)
    g = prob.constraints(w, p)
    lbx, ubx = prob.bounds()
    prim = float(np.max(np.abs(g)))
    bnd = max(float(np.max(np.maximum(lbx - w, 0.0))), float(np.max(np.maximum(w - ubx, 0.0))))
    J = prob.constraint_jac(w, p)
    gf = prob.objective_grad(w, p)
    cols, lo, hi = list(J), [-np.inf] * prob.ng, [np.inf] * prob.ng
    for j in range(prob.nw):
        if np.isfinite(ubx[j]) and w[j] >= ubx[j] - act_tol:
            e = np.zeros(prob.nw); e[j] = 1.0; cols.append(e); lo.append(0.0); hi.append(np.inf)
        elif np.isfinite(lbx[j]) and w[j] <= lbx[j] + act_tol:
            e = np.zeros(prob.nw); e[j] = 1.0; cols.append(e); lo.append(-np.inf); hi.append(0.0)
    M = np.array(cols).T
    res = lsq_linear(M, -gf, bounds=(np.array(lo), np.array(hi)), method="bvls", tol=1e-14, max_iter=5000)
    stat = float(np.max(np.abs(M @ res.x + gf)))
    return dict(primal=prim, bound=bnd, stat=stat, grad_scale=float(np.max(np.abs(gf))))
