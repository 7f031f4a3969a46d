"""CPU oracle for the per-arm impedance QP (ARMCONTROL.solver_worker) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the
product path (dart_mpc.ArmControl -> libdartmpc.so) never does.

What it restates (PMPC/src/controller/arm.py; RMPC/dev_dual/controller/parallel.py and
LMPC/src/controller/parallel.py carry the same solver_worker):

* QP construction from one shared-memory snapshot, arm.py:335-392, with the same numpy calls:
  ``pinv(M, rcond=1e-6)`` (:339-342), ``inv(Mx_inv)`` when ``|det| > 1e-8`` else
  ``pinv(Mx_inv, rcond=1e-3)`` (:344-350), ``mu = Mx (J Minv h + Jdot qd)`` (:353),
  ``D = sqrtm_safe(Mx) sqrt(K) + sqrt(K) sqrtm_safe(Mx)`` with the eigenvalue-|.| square root
  (:355-362, elementwise ``np.sqrt(K)``), ``F = -D J qd + K twist + mu`` (:376),
  ``Eimp = J qdd + Jdot qd - Mx_inv F`` (:377), ``beta = 2 sqrt(diag(K_null)) (-qd) + K_null (-q)``
  (:379), ``Epos = qdd - beta`` (:380), ``qddd = (qdd - qdd_prev)/dt`` (:382) and the cost
  ``Eimp^T Wimp Eimp + Epos^T Wpos Epos + qddd^T Wsmooth qddd`` (:384-388);
  constraints ``[0.5 dt^2 qdd + qd dt + q ; qdd dt + qd ; M qdd + h]`` in
  ``[Qmin, Qdotmin, taumin] .. [Qmax, Qdotmax, taumax]`` (:391-398).
* The solve: the reference hands this strictly convex QP (Wpos > 0) to IPOPT (``ca.nlpsol``,
  tol 1e-8, bound_relax_factor 1e-8 on the constraint bounds, warm start).  IPOPT converges to the
  unique KKT point of the relaxed problem, so the oracle computes that point with a
  Mehrotra predictor-corrector interior-point method (converged to 1e-10 scaled KKT error) on
      min 1/2 x^T H x + c^T x   s.t.  l~ <= A x + b <= u~
  (the same algorithm the GPU kernel runs) and certifies it with an independent KKT check
  (``kkt_certificate``).  Outputs as the reference publishes them (:428-437):
  ``tau = M x + h``, ``loss = f(x)`` and ``x`` (the next ``qdd_prev``).

Parity status: casadi / IPOPT and MuJoCo are absent from this image and the reference holds no
stored ARMCONTROL outputs, so this row is **parity unpinned** against reference-produced numbers;
it is anchored by the KKT certificate of the reference's own NLP (unique optimum) and by a
cross-check against scipy's SLSQP in tests/test_oracle_arm.py.
"""
from __future__ import annotations

import numpy as np

N_TASK = 6
BOUND_RELAX = 1e-8          # IPOPT bound_relax_factor default
INF_BOUND = 1e19            # IPOPT nlp_lower/upper_bound_inf

# parameter set of PMPC/src/main_parallel_enhanced / RMPC/dev_dual/rob_ctrl.py:232-275 (both arms)
QMIN = np.array([-6.28319, -2.059, -6.28319, -0.19198, -6.28319, -1.69297, -6.28319])
QMAX = np.array([6.28319, 2.0944, 6.28319, 3.927, 6.28319, 3.14159, 6.28319])


def default_params(n: int = 7, dt: float = 0.002) -> dict:
    """The reference's arm parameters (rob_ctrl.py:238-251; identical for L and R)."""
    assert n == 7, "the reference parameter set is for the 7-DOF xArm"
    return {
        "Wimp": np.diag([10.0, 10.0, 10.0, 1.0, 1.0, 1.0]),
        "Wpos": np.eye(7) * 0.1,
        "Wsmooth": np.eye(7) * 0.0,
        "Qmin": QMIN.copy(), "Qmax": QMAX.copy(),
        "Qdotmin": np.ones(7) * -20.0, "Qdotmax": np.ones(7) * 20.0,
        "taumin": np.array([-50.0, -50, -30, -30, -30, -20, -20]),
        "taumax": np.array([50.0, 50, 30, 30, 30, 20, 20]),
        "K": np.diag([5000.0, 5000.0, 5000.0, 50.0, 50.0, 50.0]) * 0.1 * 10,
        "K_null": np.diag([1.0] * 7),
        "dt": float(dt),
    }


def _safe_sqrtm(Mx):
    """arm.py:355-358 (eigh, sqrt of |eigenvalues|)."""
    w, V = np.linalg.eigh(Mx)
    return V @ np.diag(np.sqrt(np.abs(w))) @ V.T


def build_qp(snap: dict, prm: dict):
    """QP data (H, c, const, A, b, lo, hi) of one arm snapshot, as arm.py:335-398 defines it.

    f(x) = 1/2 x^T H x + c^T x + const equals the reference cost; A x + b are the reference
    constraint rows g; lo/hi are the bounds relaxed as IPOPT does (bound_relax_factor).
    """
    q, qd, qdd_prev = snap["q"], snap["qd"], snap["qdd_prev"]
    J, Jd, M, h, Mx_inv = snap["jac"], snap["jacDot"], snap["M"], snap["h"], snap["Mx_inv"]
    n = q.shape[0]
    dt = prm["dt"]
    twist = np.zeros(N_TASK)
    twist[:3] = snap["mocap_pos"] - snap["ee_pos"]
    twist[3:] = snap["rotvec"]
    try:
        Minv = np.linalg.pinv(M, rcond=1e-6)
    except Exception:       # pragma: no cover - mirrors arm.py:339-342
        Minv = np.linalg.pinv(M)
    try:
        if abs(np.linalg.det(Mx_inv)) > 1e-8:
            Mx = np.linalg.inv(Mx_inv)
        else:
            Mx = np.linalg.pinv(Mx_inv, rcond=1e-3)
    except Exception:       # pragma: no cover
        Mx = np.linalg.pinv(Mx_inv, rcond=1e-3)
    mu = Mx @ (J @ (Minv @ h) + Jd @ qd)
    K = prm["K"]
    D = _safe_sqrtm(Mx) @ np.sqrt(K) + np.sqrt(K) @ _safe_sqrtm(Mx)
    F = -D @ (J @ qd) + K @ twist + mu
    e0 = Jd @ qd - Mx_inv @ F                       # Eimp = J x + e0
    Kn = prm["K_null"]
    beta = 2.0 * np.sqrt(np.diag(Kn)) * (-qd) + Kn @ (-q)
    sym = lambda W: 0.5 * (W + W.T)                  # noqa: E731  (x^T W x only sees sym(W))
    Wi, Wp, Ws = sym(prm["Wimp"]), sym(prm["Wpos"]), sym(prm["Wsmooth"]) / dt ** 2
    H = 2.0 * (J.T @ Wi @ J + Wp + Ws)
    c = 2.0 * (J.T @ Wi @ e0 - Wp @ beta - Ws @ qdd_prev)
    const = e0 @ Wi @ e0 + beta @ Wp @ beta + qdd_prev @ Ws @ qdd_prev
    A = np.vstack([0.5 * dt ** 2 * np.eye(n), dt * np.eye(n), M])
    b = np.concatenate([qd * dt + q, qd, h])
    lo = np.concatenate([prm["Qmin"], prm["Qdotmin"], prm["taumin"]]).astype(float)
    hi = np.concatenate([prm["Qmax"], prm["Qdotmax"], prm["taumax"]]).astype(float)
    lo = np.where(lo <= -INF_BOUND, -np.inf, lo - BOUND_RELAX * np.maximum(1.0, np.abs(lo)))
    hi = np.where(hi >= INF_BOUND, np.inf, hi + BOUND_RELAX * np.maximum(1.0, np.abs(hi)))
    aux = {"e0": e0, "beta": beta, "Mx": Mx, "D": D, "mu": mu, "F": F}
    return H, c, const, A, b, lo, hi, aux


def reference_cost(x, snap, prm, aux):
    """The reference's objective expression (arm.py:377-388) at x."""
    J = snap["jac"]
    Eimp = J @ x + aux["e0"]
    Epos = x - aux["beta"]
    qddd = (x - snap["qdd_prev"]) / prm["dt"]
    return float(Eimp @ prm["Wimp"] @ Eimp + Epos @ prm["Wpos"] @ Epos + (-qddd) @ prm["Wsmooth"] @ (-qddd))


def qp_ipm(H, c, A, b, lo, hi, x0=None, tol=1e-10, acc_tol=1e-7, max_iter=60):
    """Mehrotra predictor-corrector IPM for min 1/2 x'Hx + c'x s.t. lo <= Ax + b <= hi.

    Inequalities G x <= g with G = [A; -A], g = [hi - b; b - lo] (infinite rows dropped),
    slacks s = g - G x > 0, multipliers z > 0, start s = max(g - G x0, 1), z = (1 + |c|max) / #rows.  Per iteration
    the normal matrix K = H + G' S^-1 Z G is factored once (Cholesky) and solved for the affine
    direction (rc = s z) and the corrector (rc = s z + ds_a dz_a - sigma mu, sigma = (mu_a/mu)^3);
    one common step 0.99 x the fraction to the boundary for (x, s, z).
    Converged when max(|rd|/sd, |rp|/sp, mu/sd) <= tol (sd = 1 + |c|max, sp = 1 + |g|max).
    Status: 0 converged, 1 acceptable (factorisation lost definiteness with the test met at
    acc_tol), -1 max_iter, -2 breakdown, -3 diverging multipliers (infeasible bounds).
    Returns (x, status, iterations, z_hi, z_lo).
    """
    n = H.shape[0]
    m = A.shape[0]
    onu, onl = np.isfinite(hi), np.isfinite(lo)
    G = np.vstack([A, -A])
    g = np.concatenate([np.where(onu, hi - b, 0.0), np.where(onl, b - lo, 0.0)])
    on = np.concatenate([onu, onl])
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=float)
    r = g - G @ x
    s = np.where(on, np.maximum(r, 1.0), 1.0)
    nact = max(1, int(on.sum()))
    sd = 1.0 + np.max(np.abs(c))
    z = np.where(on, sd / nact, 0.0)              # multipliers on the scale of the cost gradient
    sp = 1.0 + np.max(np.abs(np.where(on, g, 0.0)))
    status, it = -1, 0
    for it in range(max_iter):
        rd = H @ x + c + G.T @ z
        rp = np.where(on, G @ x + s - g, 0.0)
        mu = float(s[on] @ z[on]) / nact
        err = max(np.max(np.abs(rd)) / sd, np.max(np.abs(rp)) / sp, mu / sd)
        if err <= tol:
            status = 0
            break
        if np.max(z) > 1e14 * sd:
            status = -3
            break
        w = np.where(on, z / s, 0.0)
        Kmat = H + G.T @ (w[:, None] * G)
        try:
            L = np.linalg.cholesky(Kmat)
        except np.linalg.LinAlgError:
            status = 1 if err <= acc_tol else -2
            break

        def solve(rc):
            rhs = -rd - G.T @ np.where(on, (z * rp - rc) / s, 0.0)
            dx = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
            ds = np.where(on, -rp - G @ dx, 0.0)
            dz = np.where(on, (-rc - z * ds) / s, 0.0)
            return dx, ds, dz

        def max_step(v, dv):
            neg = on & (dv < 0)
            return min(1.0, float(np.min(-v[neg] / dv[neg]))) if neg.any() else 1.0

        dxa, dsa, dza = solve(np.where(on, s * z, 0.0))
        aa = min(max_step(s, dsa), max_step(z, dza))
        mu_aff = float((s + aa * dsa)[on] @ (z + aa * dza)[on]) / nact
        sigma = (mu_aff / mu) ** 3 if mu > 0.0 else 0.0
        rc = np.where(on, s * z + dsa * dza - sigma * mu, 0.0)
        dx, ds, dz = solve(rc)
        a = min(1.0, 0.99 * min(max_step(s, ds), max_step(z, dz)))
        x = x + a * dx
        s = np.where(on, s + a * ds, 1.0)
        z = np.where(on, z + a * dz, 0.0)
    else:
        it = max_iter
    return x, status, it, z[:m], z[m:]


def kkt_certificate(H, c, A, b, lo, hi, x, zu, zl):
    """Scaled KKT residuals of (x, zu, zl): stationarity, primal feasibility, complementarity."""
    r = A @ x + b
    stat = H @ x + c + A.T @ (zu - zl)
    feas = max(0.0, float(np.max(np.maximum(r - hi, lo - r))))
    gap_u = np.abs(np.where(np.isfinite(hi), hi, r) - r)
    gap_l = np.abs(r - np.where(np.isfinite(lo), lo, r))
    comp = float(np.max(np.concatenate([zu * gap_u, zl * gap_l])))
    return {"stat": float(np.max(np.abs(stat))) / (1.0 + float(np.max(np.abs(c)))),
            "feas": feas, "comp": comp, "dual_min": float(min(zu.min(), zl.min()))}


def solve_arm(snap: dict, prm: dict, tol: float = 1e-10):
    """One ARMCONTROL solve: returns dict(qdd, tau, loss, status, iters, kkt)."""
    H, c, const, A, b, lo, hi, aux = build_qp(snap, prm)
    x, st, it, zu, zl = qp_ipm(H, c, A, b, lo, hi, x0=snap.get("qdd_prev"), tol=tol)
    return {"qdd": x, "tau": snap["M"] @ x + snap["h"], "loss": reference_cost(x, snap, prm, aux),
            "status": st, "iters": it, "kkt": kkt_certificate(H, c, A, b, lo, hi, x, zu, zl),
            "qp": (H, c, const, A, b, lo, hi)}


def solve_batch(snaps: dict, prms: dict, tol: float = 1e-10):
    """Batched wrapper: snaps/prms hold [B, ...] arrays (see dart_mpc.workload.arm_batch)."""
    B = snaps["q"].shape[0]
    n = snaps["q"].shape[1]
    shared = np.ndim(prms["Qmin"]) == 1
    out = {"qdd": np.zeros((B, n)), "tau": np.zeros((B, n)), "loss": np.zeros(B),
           "status": np.zeros(B, dtype=np.int32), "iters": np.zeros(B, dtype=np.int32)}
    for i in range(B):
        r = solve_arm({k: v[i] for k, v in snaps.items()}, prms if shared else {k: v[i] for k, v in prms.items()},
                      tol=tol)
        out["qdd"][i], out["tau"][i], out["loss"][i] = r["qdd"], r["tau"], r["loss"]
        out["status"][i], out["iters"][i] = r["status"], r["iters"]
    return out
