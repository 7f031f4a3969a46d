/*
 * lmpc_ipm.c -- CPU oracle for the LMPC solve (8-state Stribeck / rolling model, pvec input).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker / timed CPU baseline.  Never
 * linked into the shipped solver.
 *
 * Restates (LMPC/src/controller/rlmpc2.py): safe_dynamics :260-429 (the code's
 * index map :301-334), _rk4 :431-436, the NLP :239-491 (w = [X; U] node-major,
 * g = [x_0 - state; x_{k+1} - F(x_k, u_k)], cost :444-464 with the Delta-u rows
 * u_0 - u_prev, u_k - u_{k-1}), solve with warm start w0 <- w_opt :494-524, and
 * IPOPT with print_level 0 and max_iter / tol / acceptable_tol / acceptable_iter
 * as passed (the reference: 50 / 1e-4 / 1e-3 / 5, :480-489; max_cpu_time 0.05 s
 * is a wall-clock cap and is not restated).
 * IPOPT's algorithm as in pmpc_ipm.c / rmpc_ipm.c: monotone mu, filter line
 * search with second-order correction, inertia correction, bound_relax 1e-8,
 * gradient-based scaling of the objective AND of the constraint rows
 * (nlp_scaling_max_gradient 100), exact Hessian (second-order jets), and IPOPT's
 * termination tests: optimal (scaled error <= tol, unscaled dual infeasibility
 * <= 1, constraint violation <= 1e-4, complementarity <= 1e-4) and "acceptable"
 * (acceptable_iter consecutive iterates with error <= acceptable_tol, violation
 * and complementarity <= 1e-2).  The Delta-u coupling is carried by the
 * augmented state [x_k; u_{k-1}] in the Riccati recursion.
 * |v| is differentiated as CasADi does: sign(v), sign(0) = 0.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef ORACLE_DEBUG
#include <stdio.h>
#endif

/* IPOPT Compare_le: lhs <= rhs up to 10 machine epsilons of |base| */
#define LE(l, r, b) ((l) - (r) <= 10.0 * 2.220446049250313e-16 * fabs(b))

#define NXS 8           /* physical states px vx py vy th_x om_x th_y om_y */
#define NA 10           /* augmented state [x; u_prev] */
#define NU 2
#define NZ 12           /* jet variables [x(8) up(2) u(2)] (up unused by the dynamics) */
#define NH 78
#define NMAX 64
#define NPV 34
#define GACC 9.81

typedef struct { double v, d[NZ], h[NH]; } jet;
static inline int hx(int i, int j) { if (i < j) { int t = i; i = j; j = t; } return i * (i + 1) / 2 + j; }
static inline jet jconst(double c) { jet r; memset(&r, 0, sizeof r); r.v = c; return r; }
static inline jet jvar(double v, int i) { jet r = jconst(v); r.d[i] = 1.0; return r; }
static inline jet jaxpy(jet a, double s, jet b) {
    jet r; r.v = a.v + s * b.v;
    for (int i = 0; i < NZ; ++i) r.d[i] = a.d[i] + s * b.d[i];
    for (int i = 0; i < NH; ++i) r.h[i] = a.h[i] + s * b.h[i];
    return r;
}
static inline jet jadd(jet a, jet b) { return jaxpy(a, 1.0, b); }
static inline jet jsub(jet a, jet b) { return jaxpy(a, -1.0, b); }
static inline jet jscale(jet a, double s) {
    jet r; r.v = s * a.v;
    for (int i = 0; i < NZ; ++i) r.d[i] = s * a.d[i];
    for (int i = 0; i < NH; ++i) r.h[i] = s * a.h[i];
    return r;
}
static inline jet jaddc(jet a, double c) { a.v += c; return a; }
static inline jet jmul(jet a, jet b) {
    jet r; r.v = a.v * b.v;
    for (int i = 0; i < NZ; ++i) r.d[i] = a.v * b.d[i] + b.v * a.d[i];
    for (int i = 0; i < NZ; ++i) for (int j = 0; j <= i; ++j)
        r.h[hx(i, j)] = a.v * b.h[hx(i, j)] + b.v * a.h[hx(i, j)] + a.d[i] * b.d[j] + a.d[j] * b.d[i];
    return r;
}
/* f(a) with f' = f1, f'' = f2 at a.v */
static inline jet junary(jet a, double f, double f1, double f2) {
    jet r; r.v = f;
    for (int i = 0; i < NZ; ++i) r.d[i] = f1 * a.d[i];
    for (int i = 0; i < NZ; ++i) for (int j = 0; j <= i; ++j) r.h[hx(i, j)] = f1 * a.h[hx(i, j)] + f2 * a.d[i] * a.d[j];
    return r;
}
static inline jet jsin(jet a) { return junary(a, sin(a.v), cos(a.v), -sin(a.v)); }
static inline jet jtanh(jet a) { double t = tanh(a.v), d1 = 1.0 - t * t; return junary(a, t, d1, -2.0 * t * d1); }
static inline jet jexp(jet a) { double e = exp(a.v); return junary(a, e, e, e); }
static inline double sgn(double v) { return (v > 0) - (v < 0); }
static inline jet jfabs(jet a) { return junary(a, fabs(a.v), sgn(a.v), 0.0); }

typedef struct {
    double m_x, m_y, c_x, c_y, k_x, k_y;
    double F_s_x, F_c_x, B_x, v_s_x, eps_x, F_s_y, F_c_y, B_y, v_s_y, eps_y;
    double I_x, I_y, r_x, r_y, c_rot_x, c_rot_y;
    double F_s_rx, F_c_rx, B_rx, v_s_rx, eps_rx, F_s_ry, F_c_ry, B_ry, v_s_ry, eps_ry;
    double h_x, h_y;
} mparams;

/* squash_param (:296-298) and the index map (:301-344) */
static void unpack_params(const double *p, mparams *M) {
#define SQ(v) (fabs(v) + 1e-6)
    M->m_x = SQ(p[0]); M->m_y = SQ(p[1]); M->c_x = SQ(p[2]); M->c_y = SQ(p[3]); M->k_x = SQ(p[4]); M->k_y = SQ(p[5]);
    M->F_s_x = p[6]; M->F_c_x = p[7]; M->B_x = p[8]; M->v_s_x = SQ(p[9]); M->eps_x = SQ(p[10]);
    M->F_s_y = p[11]; M->F_c_y = p[12]; M->B_y = p[13]; M->v_s_y = SQ(p[14]); M->eps_y = SQ(p[15]);
    M->I_x = SQ(p[16]); M->I_y = SQ(p[17]); M->r_x = SQ(p[18]); M->r_y = SQ(p[19]);
    M->c_rot_x = SQ(p[20]); M->c_rot_y = SQ(p[21]);
    M->F_s_rx = p[22]; M->F_c_rx = p[23]; M->B_rx = p[24]; M->v_s_rx = SQ(p[25]); M->eps_rx = SQ(p[26]);
    M->F_s_ry = p[27]; M->F_c_ry = p[28]; M->B_ry = p[29]; M->v_s_ry = SQ(p[30]); M->eps_ry = SQ(p[31]);
    M->h_x = SQ(p[32]); M->h_y = SQ(p[33]);
#undef SQ
}

/* stribeck_fric (:372-376) */
static jet jstribeck(jet v, double Fs, double Fc, double B, double vs, double eps) {
    jet e = jexp(jscale(jfabs(v), -1.0 / (vs + 1e-12)));
    jet s = jtanh(jscale(v, 1.0 / eps));
    jet c = jaddc(jscale(e, Fs - Fc), Fc);
    return jaxpy(jmul(s, c), B, v);
}
static double stribeck(double v, double Fs, double Fc, double B, double vs, double eps) {
    double e = exp(-fabs(v) / (vs + 1e-12));
    return tanh(v / eps) * (Fc + (Fs - Fc) * e) + B * v;
}

/* safe_dynamics (:260-429) on jets */
static void dyn_jet(const mparams *M, const jet *x, const jet *u, jet *xd) {
    jet Gx = jscale(jsin(u[0]), M->m_x * GACC), Gy = jscale(jsin(u[1]), M->m_y * GACC);
    jet Ffx = jstribeck(x[1], M->F_s_x, M->F_c_x, M->B_x, M->v_s_x, M->eps_x);
    jet Ffy = jstribeck(x[3], M->F_s_y, M->F_c_y, M->B_y, M->v_s_y, M->eps_y);
    jet vsx = jaxpy(x[1], -M->r_x, x[7]);             /* vx - r_x om_y */
    jet vsy = jaxpy(x[3], M->r_y, x[5]);              /* vy - (-r_y om_x) */
    jet Frx = jstribeck(vsx, M->F_s_x, M->F_c_x, M->B_x, M->v_s_x, M->eps_x);
    jet Fry = jstribeck(vsy, M->F_s_y, M->F_c_y, M->B_y, M->v_s_y, M->eps_y);
    jet Tnx = jstribeck(x[5], M->F_s_rx, M->F_c_rx, M->B_rx, M->v_s_rx, M->eps_rx);
    jet Tny = jstribeck(x[7], M->F_s_ry, M->F_c_ry, M->B_ry, M->v_s_ry, M->eps_ry);
    jet tx = jscale(Fry, -M->r_y);
    tx = jsub(tx, Tnx);
    tx = jaxpy(tx, -M->c_rot_x, x[5]);
    tx = jaxpy(tx, -M->m_y * GACC * M->h_x, jsin(x[4]));
    jet ty = jscale(Frx, -M->r_x);
    ty = jsub(ty, Tny);
    ty = jaxpy(ty, -M->c_rot_y, x[7]);
    ty = jaxpy(ty, -M->m_x * GACC * M->h_y, jsin(x[6]));
    jet rx = jsub(jsub(jaxpy(jaxpy(Gx, -M->c_x, x[1]), -M->k_x, x[0]), Ffx), Frx);
    jet ry = jsub(jsub(jaxpy(jaxpy(Gy, -M->c_y, x[3]), -M->k_y, x[2]), Ffy), Fry);
    xd[0] = x[1]; xd[1] = jscale(rx, 1.0 / M->m_x);
    xd[2] = x[3]; xd[3] = jscale(ry, 1.0 / M->m_y);
    xd[4] = x[5]; xd[5] = jscale(tx, 1.0 / (M->I_x + 1e-12));
    xd[6] = x[7]; xd[7] = jscale(ty, 1.0 / (M->I_y + 1e-12));
}
static void dyn_val(const mparams *M, const double *x, const double *u, double *xd) {
    const double Gx = M->m_x * (GACC * sin(u[0])), Gy = M->m_y * (GACC * sin(u[1]));
    const double Ffx = stribeck(x[1], M->F_s_x, M->F_c_x, M->B_x, M->v_s_x, M->eps_x);
    const double Ffy = stribeck(x[3], M->F_s_y, M->F_c_y, M->B_y, M->v_s_y, M->eps_y);
    const double Frx = stribeck(x[1] - M->r_x * x[7], M->F_s_x, M->F_c_x, M->B_x, M->v_s_x, M->eps_x);
    const double Fry = stribeck(x[3] - (-M->r_y * x[5]), M->F_s_y, M->F_c_y, M->B_y, M->v_s_y, M->eps_y);
    const double Tnx = stribeck(x[5], M->F_s_rx, M->F_c_rx, M->B_rx, M->v_s_rx, M->eps_rx);
    const double Tny = stribeck(x[7], M->F_s_ry, M->F_c_ry, M->B_ry, M->v_s_ry, M->eps_ry);
    const double tx = -M->r_y * Fry - Tnx - M->c_rot_x * x[5] + (-M->m_y * GACC * M->h_x * sin(x[4]));
    const double ty = -M->r_x * Frx - Tny - M->c_rot_y * x[7] + (-M->m_x * GACC * M->h_y * sin(x[6]));
    const double rx = Gx - M->c_x * x[1] - M->k_x * x[0] - Ffx - Frx;
    const double ry = Gy - M->c_y * x[3] - M->k_y * x[2] - Ffy - Fry;
    xd[0] = x[1]; xd[1] = rx / M->m_x; xd[2] = x[3]; xd[3] = ry / M->m_y;
    xd[4] = x[5]; xd[5] = tx / (M->I_x + 1e-12); xd[6] = x[7]; xd[7] = ty / (M->I_y + 1e-12);
}

typedef struct {
    int N; double Ts, Q[8], Qt[8], R[4], ulo, uhi;
    mparams M;
} prob_t;

/* _rk4 (:431-436) */
static void rk4_val(const prob_t *P, const double *x, const double *u, double *xn) {
    double k1[8], k2[8], k3[8], k4[8], y[8], h = P->Ts;
    dyn_val(&P->M, x, u, k1);
    for (int i = 0; i < 8; ++i) y[i] = x[i] + 0.5 * h * k1[i];
    dyn_val(&P->M, y, u, k2);
    for (int i = 0; i < 8; ++i) y[i] = x[i] + 0.5 * h * k2[i];
    dyn_val(&P->M, y, u, k3);
    for (int i = 0; i < 8; ++i) y[i] = x[i] + h * k3[i];
    dyn_val(&P->M, y, u, k4);
    for (int i = 0; i < 8; ++i) xn[i] = x[i] + h * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]) / 6;
}
/* RK4 on jets over z = [x(8), up(2), u(2)]: value, Jacobian rows and nlam-contracted Hessian */
static void rk4_derivs(const prob_t *P, const double *x, const double *u, const double *nlam,
                       double *xn, double J[8][NZ], double H[NZ][NZ]) {
    jet xj[8], uj[2], k1[8], k2[8], k3[8], k4[8], y[8];
    const double h = P->Ts;
    for (int i = 0; i < 8; ++i) xj[i] = jvar(x[i], i);
    for (int i = 0; i < 2; ++i) uj[i] = jvar(u[i], NA + i);
    dyn_jet(&P->M, xj, uj, k1);
    for (int i = 0; i < 8; ++i) y[i] = jaxpy(xj[i], 0.5 * h, k1[i]);
    dyn_jet(&P->M, y, uj, k2);
    for (int i = 0; i < 8; ++i) y[i] = jaxpy(xj[i], 0.5 * h, k2[i]);
    dyn_jet(&P->M, y, uj, k3);
    for (int i = 0; i < 8; ++i) y[i] = jaxpy(xj[i], h, k3[i]);
    dyn_jet(&P->M, y, uj, k4);
    for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) H[a][b] = 0.0;
    for (int i = 0; i < 8; ++i) {
        jet s = jaxpy(jaxpy(jaxpy(k1[i], 2.0, k2[i]), 2.0, k3[i]), 1.0, k4[i]);
        jet r = jaxpy(xj[i], h / 6, s);
        xn[i] = r.v;
        for (int j = 0; j < NZ; ++j) J[i][j] = r.d[j];
        for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) H[a][b] += nlam[i] * r.h[hx(a, b)];
    }
}

typedef struct {
    double X[NA * (NMAX + 1)], U[NU * NMAX];
    double lam[NA * (NMAX + 1)];                /* multipliers of the (unscaled) defect rows */
    double zL[NU * NMAX], zU[NU * NMAX];
    double A[NMAX][NA][NA], Bm[NMAX][NA][NU], Hs[NMAX][NZ][NZ];
    double Lq[NMAX][3], Qux[NMAX][NU][NA], K[NMAX][NU][NA], Pm[NMAX + 1][NA][NA];
    double kff[NMAX][NU], pv[NMAX + 1][NA];
    double dX[NA * (NMAX + 1)], dU[NU * NMAX], lamp[NA * (NMAX + 1)], dzL[NU * NMAX], dzU[NU * NMAX];
    double Xt[NA * (NMAX + 1)], Ut[NU * NMAX];
    double dsc[NA * (NMAX + 1)];                /* constraint-row scaling factors */
    double filt_th[256], filt_ph[256];
} work_t;

struct resto_s;
typedef struct {
    const prob_t *P; const double *x0, *up0, *tgt; double sc, mu, lo, hi;
    struct resto_s *R;      /* restoration phase data (NULL: the original problem) */
    int mode;               /* 0 original problem, 1 restoration Newton step, 2 restoration least-square multipliers */
} ctx_t;

/* IPOPT's restoration phase (MinC_1NrmRestorationPhase, RestoIpoptNLP): the feasibility problem
 *   min rho sum(p + n) + eta/2 ||D_R (x - x_R)||^2   s.t.  d c(x) + n - p = 0,  p, n >= 0,  lo <= u <= hi
 * over the reference NLP's variables x = [X; U] and a pair (p, n) per physical defect row (scaled by
 * the row scaling d; the Delta-u copy rows of the augmented formulation are not rows of the reference
 * NLP and stay hard).  Eliminating p, n from the Newton system leaves each physical row soft:
 * J dx - D dlam = rhs with D = (1/(Sigma_p + delta) + 1/(Sigma_n + delta)) / d^2, which the Riccati
 * recursion absorbs per node as P~ = P (I + D P)^-1, p~ = (I + P D)^-1 p (value function seen through
 * the soft rows) and dx+ = (I + D P)^-1 (A dx + B du - rg - D p). */
typedef struct resto_s {
    double pc[NA * (NMAX + 1)], nc[NA * (NMAX + 1)], zp[NA * (NMAX + 1)], zn[NA * (NMAX + 1)];
    double dpc[NA * (NMAX + 1)], dnc[NA * (NMAX + 1)], dzp[NA * (NMAX + 1)], dzn[NA * (NMAX + 1)];
    double rp[NA * (NMAX + 1)], rn[NA * (NMAX + 1)];   /* p / n rows of the barrier Lagrangian gradient */
    double D[NA * (NMAX + 1)], Spd[NA * (NMAX + 1)], Snd[NA * (NMAX + 1)];   /* of the current factorisation */
    double XR[NA * (NMAX + 1)], UR[NU * NMAX], DRx[NA * (NMAX + 1)], DRu[NU * NMAX];
    double M[NMAX + 1][NA][NA], Pt[NMAX + 1][NA][NA];
    double filt_th[256], filt_ph[256];
    double pt_[NA * (NMAX + 1)], nt_[NA * (NMAX + 1)];    /* trial p, n */
    double rho, eta, delta;
    const double *dsc;
    /* iterative refinement (resto_refine): residuals of the full Newton system, gradient override */
    int ovr;
    double gov[NMAX + 1][NZ], ex[NMAX + 1][NZ], ec[NMAX + 1][NA], ep[NA * (NMAX + 1)], en[NA * (NMAX + 1)];
} resto_t;

/* solve A X = B (n x n, nrhs columns of B stored row-major with stride NA + 1 ... ) by Gaussian
   elimination with partial pivoting; A and B are overwritten */
static void gauss_solve(int n, double A[NA][NA], double B[NA][NA], int nrhs) {
    for (int c = 0; c < n; ++c) {
        int piv = c;
        for (int r = c + 1; r < n; ++r) if (fabs(A[r][c]) > fabs(A[piv][c])) piv = r;
        if (piv != c) {
            for (int j = 0; j < n; ++j) { double t = A[c][j]; A[c][j] = A[piv][j]; A[piv][j] = t; }
            for (int j = 0; j < nrhs; ++j) { double t = B[c][j]; B[c][j] = B[piv][j]; B[piv][j] = t; }
        }
        for (int r = c + 1; r < n; ++r) {
            const double f = A[r][c] / A[c][c];
            if (f == 0.0) continue;
            for (int j = c; j < n; ++j) A[r][j] -= f * A[c][j];
            for (int j = 0; j < nrhs; ++j) B[r][j] -= f * B[c][j];
        }
    }
    for (int c = n - 1; c >= 0; --c)
        for (int j = 0; j < nrhs; ++j) {
            double t = B[c][j];
            for (int m = c + 1; m < n; ++m) t -= A[c][m] * B[m][j];
            B[c][j] = t / A[c][c];
        }
}
/* x <- M^-1 x  (M = R->M[k]) */
static void soft_apply_minv(const resto_t *R, int k, double *x) {
    double A[NA][NA], Bv[NA][NA];
    memcpy(A, R->M[k], sizeof A);
    for (int i = 0; i < NA; ++i) Bv[i][0] = x[i];
    gauss_solve(NA, A, Bv, 1);
    for (int i = 0; i < NA; ++i) x[i] = Bv[i][0];
}
/* x <- M^-T x */
static void soft_apply_mtinv(const resto_t *R, int k, double *x) {
    double A[NA][NA], Bv[NA][NA];
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) A[i][j] = R->M[k][j][i];
    for (int i = 0; i < NA; ++i) Bv[i][0] = x[i];
    gauss_solve(NA, A, Bv, 1);
    for (int i = 0; i < NA; ++i) x[i] = Bv[i][0];
}
/* soft rows of node k with the Hessian shift delta: D, M = I + D P_k, P~_k = solve(M^T, P_k).  Returns
   0 if S = P_k(phys, phys) + D^-1 is not positive definite: eliminating the row slack w = D lam of the
   soft rows is then not a minimisation and the KKT matrix has the wrong inertia (the Riccati form of
   IPOPT's inertia test, next to Quu > 0) */
static int soft_node(const ctx_t *C, const double Pk[NA][NA], int k, double delta) {
    resto_t *R = C->R;
    for (int i = 0; i < NA; ++i) {
        const int r = NA * k + i;
        double D = 0.0;
        if (i < 8) {
            const double d = R->dsc[r];
            if (C->mode == 2) { R->Spd[r] = 1.0; R->Snd[r] = 1.0; }
            else { R->Spd[r] = R->zp[r] / R->pc[r] + delta; R->Snd[r] = R->zn[r] / R->nc[r] + delta; }
            D = (1.0 / R->Spd[r] + 1.0 / R->Snd[r]) / (d * d);
        }
        R->D[r] = D;
        for (int j = 0; j < NA; ++j) R->M[k][i][j] = (i == j) + D * Pk[i][j];
    }
    double A[NA][NA], Bm[NA][NA];
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) { A[i][j] = R->M[k][j][i]; Bm[i][j] = Pk[i][j]; }
    gauss_solve(NA, A, Bm, NA);
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) R->Pt[k][i][j] = 0.5 * (Bm[i][j] + Bm[j][i]);
    double L[8][8];     /* Cholesky of S */
    for (int i = 0; i < 8; ++i) for (int j = 0; j <= i; ++j) {
        double t = Pk[i][j] + (i == j ? 1.0 / R->D[NA * k + i] : 0.0);
        for (int m = 0; m < j; ++m) t -= L[i][m] * L[j][m];
        if (i == j) { if (!(t > 0.0)) return 0; L[i][i] = sqrt(t); }
        else L[i][j] = t / L[j][j];
    }
    return 1;
}

/* IPOPT ApplicationReturnStatus values (Infeasible_Problem_Detected = 2: the restoration problem converged to a
   point of local infeasibility; Restoration_Failed = -2: the restoration itself failed, or, with the phases
   off, the filter line search) */
enum { ST_SOLVED = 0, ST_ACCEPTABLE = 1, ST_INFEASIBLE = 2, ST_MAXITER = -1, ST_LS_FAIL = -2, ST_INERTIA_FAIL = -3,
       ST_BAD_INPUT = -10 };

static double g_relax = 1e-8;
void oracle_lmpc_set_relax(double r) { g_relax = r; }
/* second-order correction on/off (IPOPT default on; off mirrors the GPU kernel's line search) */
static int g_max_soc = 4;
void oracle_lmpc_set_soc(int max_soc) { g_max_soc = max_soc < 0 ? 0 : max_soc; }

static void stage_z(const double *X, const double *U, int k, double *z) {
    for (int i = 0; i < NA; ++i) z[i] = X[NA * k + i];
    z[NA] = U[NU * k]; z[NA + 1] = U[NU * k + 1];
}

/* cost :444-464: stage (x_k - t)^T Q (x_k - t) + [u; du]^T R [u; du], terminal Qt */
static double objective(const prob_t *P, const double *X, const double *U, const double *t) {
    double f = 0.0;
    for (int k = 0; k <= P->N; ++k) {
        const double *x = X + NA * k, *Q = k < P->N ? P->Q : P->Qt;
        for (int i = 0; i < 8; ++i) f += Q[i] * (x[i] - t[i]) * (x[i] - t[i]);
        if (k < P->N) {
            const double *u = U + NU * k;
            const double d0 = u[0] - x[8], d1 = u[1] - x[9];
            f += P->R[0] * u[0] * u[0] + P->R[1] * u[1] * u[1] + P->R[2] * d0 * d0 + P->R[3] * d1 * d1;
        }
    }
    return f;
}
static void cost_grad(const prob_t *P, const double *z, const double *t, int terminal, double *g) {
    const double *Q = terminal ? P->Qt : P->Q;
    for (int j = 0; j < NZ; ++j) g[j] = 0.0;
    for (int i = 0; i < 8; ++i) g[i] = 2 * Q[i] * (z[i] - t[i]);
    if (!terminal) {
        const double d0 = z[10] - z[8], d1 = z[11] - z[9];
        g[10] = 2 * P->R[0] * z[10] + 2 * P->R[2] * d0; g[11] = 2 * P->R[1] * z[11] + 2 * P->R[3] * d1;
        g[8] = -2 * P->R[2] * d0; g[9] = -2 * P->R[3] * d1;
    }
}

/* augmented defects (N+1 blocks of NA), unscaled; returns the scaled l1 norm (IPOPT's theta) */
static double residuals(const ctx_t *C, const work_t *W, const double *X, const double *U, double g[][NA]) {
    const prob_t *P = C->P; double th = 0.0;
    for (int i = 0; i < 8; ++i) g[0][i] = X[i] - C->x0[i];
    g[0][8] = X[8] - C->up0[0]; g[0][9] = X[9] - C->up0[1];
    for (int k = 0; k < P->N; ++k) {
        double xn[8];
        rk4_val(P, X + NA * k, U + NU * k, xn);
        for (int i = 0; i < 8; ++i) g[k + 1][i] = X[NA * (k + 1) + i] - xn[i];
        g[k + 1][8] = X[NA * (k + 1) + 8] - U[NU * k]; g[k + 1][9] = X[NA * (k + 1) + 9] - U[NU * k + 1];
    }
    for (int k = 0; k <= P->N; ++k) for (int i = 0; i < NA; ++i) th += W->dsc[NA * k + i] * fabs(g[k][i]);
    return th;
}

static double barrier_obj(const ctx_t *C, const double *X, const double *U) {
    const prob_t *P = C->P;
    double phi = C->sc * objective(P, X, U, C->tgt);
    for (int j = 0; j < NU * P->N; ++j) {
        double sl = U[j] - C->lo, su = C->hi - U[j];
        if (!(sl > 0) || !(su > 0)) return INFINITY;
        phi -= C->mu * (log(sl) + log(su));
    }
    return phi;
}

static int chol2(double a00, double a01, double a11, double L[3]) {
    if (!(a00 > 0)) return 0;
    double l00 = sqrt(a00), l10 = a01 / l00, d = a11 - l10 * l10;
    if (!(d > 0)) return 0;
    L[0] = l00; L[1] = l10; L[2] = sqrt(d);
    return 1;
}
static void chol2_solve(const double L[3], const double *b, double *x) {
    double y0 = b[0] / L[0], y1 = (b[1] - L[1] * y0) / L[2];
    x[1] = y1 / L[2]; x[0] = (y0 - L[1] * x[1]) / L[0];
}

static void stage_qp(const ctx_t *C, const work_t *W, int k, double delta, double Hq[NZ][NZ], double *gq) {
    const prob_t *P = C->P; const double sc = C->sc;
    double z[NZ];
    stage_z(W->X, W->U, k, z);
    if (C->mode) {
        /* restoration: the proximity term eta/2 ||D_R (x - x_R)||^2 on the reference NLP's variables
           (states and inputs, not the Delta-u copies), plus the lambda-weighted dynamics Hessian
           (mode 1); mode 2 (least-square multipliers): unit weights, gradient - z_L + z_U on u */
        const resto_t *R = C->R;
        for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) Hq[a][b] = C->mode == 1 ? W->Hs[k][a][b] : 0.0;
        for (int j = 0; j < NZ; ++j) gq[j] = 0.0;
        for (int i = 0; i < 8; ++i) {
            const int r = NA * k + i;
            const double w = R->eta * R->DRx[r] * R->DRx[r];
            Hq[i][i] += C->mode == 1 ? w : 1.0;
            gq[i] = w * (z[i] - R->XR[r]);
        }
        for (int a = 0; a < NU; ++a) {
            const int j = NU * k + a;
            const double w = R->eta * R->DRu[j] * R->DRu[j];
            double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
            gq[10 + a] = w * (z[10 + a] - R->UR[j]);
            if (C->mode == 1) {
                Hq[10 + a][10 + a] += w + W->zL[j] / sl + W->zU[j] / su;
                gq[10 + a] += -C->mu / sl + C->mu / su;
            } else {
                Hq[10 + a][10 + a] += 1.0;
                gq[10 + a] += -W->zL[j] + W->zU[j];
            }
        }
        if (C->mode == 1) for (int a = 0; a < NZ; ++a) Hq[a][a] += delta;
        if (R->ovr) for (int j = 0; j < NZ; ++j) gq[j] = R->gov[k][j];
        return;
    }
    for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) Hq[a][b] = W->Hs[k][a][b];
    for (int i = 0; i < 8; ++i) Hq[i][i] += sc * 2 * P->Q[i];
    for (int a = 0; a < 2; ++a) {
        Hq[10 + a][10 + a] += sc * 2 * (P->R[a] + P->R[2 + a]); Hq[8 + a][8 + a] += sc * 2 * P->R[2 + a];
        Hq[10 + a][8 + a] -= sc * 2 * P->R[2 + a]; Hq[8 + a][10 + a] -= sc * 2 * P->R[2 + a];
    }
    cost_grad(P, z, C->tgt, 0, gq);
    for (int j = 0; j < NZ; ++j) gq[j] *= sc;
    for (int a = 0; a < NU; ++a) {
        const int j = NU * k + a;
        double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
        Hq[10 + a][10 + a] += W->zL[j] / sl + W->zU[j] / su;
        gq[10 + a] += -C->mu / sl + C->mu / su;
    }
    for (int a = 0; a < NZ; ++a) Hq[a][a] += delta;
}

/* terminal value function (Hessian into Pn, gradient into pn) */
static void terminal_qp(const ctx_t *C, const work_t *W, double delta, double Pn[NA][NA], double *pn) {
    const prob_t *P = C->P; const int N = P->N;
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) Pn[i][j] = 0.0;
    if (C->mode) {
        const resto_t *R = C->R;
        for (int i = 0; i < NA; ++i) pn[i] = 0.0;
        for (int i = 0; i < 8; ++i) {
            const int r = NA * N + i;
            const double w = R->eta * R->DRx[r] * R->DRx[r];
            Pn[i][i] = C->mode == 1 ? w + delta : 1.0;
            pn[i] = w * (W->X[r] - R->XR[r]);
        }
        if (C->mode == 1) { Pn[8][8] = delta; Pn[9][9] = delta; }
        if (R->ovr) for (int i = 0; i < NA; ++i) pn[i] = R->gov[N][i];
        return;
    }
    double zN[NZ], gN[NZ];
    for (int i = 0; i < NA; ++i) zN[i] = W->X[NA * N + i];
    zN[10] = zN[11] = 0.0;
    cost_grad(P, zN, C->tgt, 1, gN);
    for (int i = 0; i < NA; ++i) pn[i] = C->sc * gN[i];
    for (int i = 0; i < 8; ++i) Pn[i][i] = C->sc * 2 * P->Qt[i];
    for (int i = 0; i < NA; ++i) Pn[i][i] += delta;
}

static int riccati_factor(const ctx_t *C, work_t *W, double delta) {
    const prob_t *P = C->P; const int N = P->N;
    double pn[NA];
    terminal_qp(C, W, delta, W->Pm[N], pn);
    for (int k = N - 1; k >= 0; --k) {
        double Hq[NZ][NZ], gq[NZ];
        stage_qp(C, W, k, delta, Hq, gq);
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = W->Pm[k + 1];
        if (C->R) {
            if (!soft_node(C, (const double (*)[NA])W->Pm[k + 1], k + 1, delta)) return 0;
            Pp = C->R->Pt[k + 1];
        }
        double PA[NA][NA], PB[NA][NU], Quu[NU][NU];
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) { double s = 0; for (int m = 0; m < NA; ++m) s += Pp[i][m] * A[m][j]; PA[i][j] = s; }
            for (int j = 0; j < NU; ++j) { double s = 0; for (int m = 0; m < NA; ++m) s += Pp[i][m] * Bm[m][j]; PB[i][j] = s; }
        }
        double Qxx[NA][NA];
        for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) {
            double s = Hq[i][j]; for (int m = 0; m < NA; ++m) s += A[m][i] * PA[m][j]; Qxx[i][j] = s;
        }
        for (int a = 0; a < NU; ++a) {
            for (int i = 0; i < NA; ++i) { double s = Hq[NA + a][i]; for (int m = 0; m < NA; ++m) s += Bm[m][a] * PA[m][i]; W->Qux[k][a][i] = s; }
            for (int b = 0; b < NU; ++b) { double s = Hq[NA + a][NA + b]; for (int m = 0; m < NA; ++m) s += Bm[m][a] * PB[m][b]; Quu[a][b] = s; }
        }
        if (!chol2(Quu[0][0], 0.5 * (Quu[0][1] + Quu[1][0]), Quu[1][1], W->Lq[k])) return 0;
        for (int i = 0; i < NA; ++i) {
            double b2[2] = {W->Qux[k][0][i], W->Qux[k][1][i]}, x2[2];
            chol2_solve(W->Lq[k], b2, x2); W->K[k][0][i] = -x2[0]; W->K[k][1][i] = -x2[1];
        }
        for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j)
            W->Pm[k][i][j] = Qxx[i][j] + W->Qux[k][0][i] * W->K[k][0][j] + W->Qux[k][1][i] * W->K[k][1][j];
        for (int i = 0; i < NA; ++i) for (int j = 0; j < i; ++j) { double s = 0.5 * (W->Pm[k][i][j] + W->Pm[k][j][i]); W->Pm[k][i][j] = W->Pm[k][j][i] = s; }
    }
    if (C->R) return soft_node(C, (const double (*)[NA])W->Pm[0], 0, delta);     /* the soft initial-state rows */
    return 1;
}

/* vector pass + forward sweep for defect RHS rg (J d = -rg; soft rows: J d - D lam+ = -rg) */
static void riccati_solve(const ctx_t *C, work_t *W, double rg[][NA]) {
    const prob_t *P = C->P; const int N = P->N;
    const resto_t *R = C->R;
    double Pdum[NA][NA];
    terminal_qp(C, W, 0.0, Pdum, W->pv[N]);
    for (int k = N - 1; k >= 0; --k) {
        double Hq[NZ][NZ], gq[NZ];
        stage_qp(C, W, k, 0.0, Hq, gq);   /* only the gradient is used */
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = W->Pm[k + 1], pp[NA];
        memcpy(pp, W->pv[k + 1], sizeof pp);
        if (R) { Pp = (double (*)[NA])R->Pt[k + 1]; soft_apply_mtinv(R, k + 1, pp); }
        double hh[NA], qx[NA], qu[NU], kf[2];
        for (int i = 0; i < NA; ++i) { double s = pp[i]; for (int m = 0; m < NA; ++m) s -= Pp[i][m] * rg[k + 1][m]; hh[i] = s; }
        for (int i = 0; i < NA; ++i) { double s = gq[i]; for (int m = 0; m < NA; ++m) s += A[m][i] * hh[m]; qx[i] = s; }
        for (int a = 0; a < NU; ++a) { double s = gq[NA + a]; for (int m = 0; m < NA; ++m) s += Bm[m][a] * hh[m]; qu[a] = s; }
        chol2_solve(W->Lq[k], qu, kf);
        W->kff[k][0] = -kf[0]; W->kff[k][1] = -kf[1];
        for (int i = 0; i < NA; ++i) W->pv[k][i] = qx[i] + W->Qux[k][0][i] * W->kff[k][0] + W->Qux[k][1][i] * W->kff[k][1];
    }
    for (int i = 0; i < NA; ++i) W->dX[i] = -rg[0][i] - (R ? R->D[i] * W->pv[0][i] : 0.0);
    if (R) soft_apply_minv(R, 0, W->dX);
    for (int k = 0; k < N; ++k) {
        double *dx = W->dX + NA * k, *du = W->dU + NU * k, *dn = W->dX + NA * (k + 1);
        for (int a = 0; a < NU; ++a) { double s = W->kff[k][a]; for (int i = 0; i < NA; ++i) s += W->K[k][a][i] * dx[i]; du[a] = s; }
        for (int i = 0; i < NA; ++i) {
            double s = -rg[k + 1][i];
            for (int m = 0; m < NA; ++m) s += W->A[k][i][m] * dx[m];
            for (int a = 0; a < NU; ++a) s += W->Bm[k][i][a] * du[a];
            if (R) s -= R->D[NA * (k + 1) + i] * W->pv[k + 1][i];
            dn[i] = s;
        }
        if (R) soft_apply_minv(R, k + 1, dn);
    }
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        double s = W->pv[k][i]; for (int m = 0; m < NA; ++m) s += W->Pm[k][i][m] * W->dX[NA * k + m];
        W->lamp[NA * k + i] = -s;
    }
}

static double frac_to_boundary(const ctx_t *C, const work_t *W, const double *dU, double tau) {
    double a = 1.0;
    for (int j = 0; j < NU * C->P->N; ++j) {
        double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
        if (dU[j] < 0) a = fmin(a, -tau * sl / dU[j]);
        if (dU[j] > 0) a = fmin(a, tau * su / dU[j]);
    }
    return a;
}

static void linearise(const prob_t *P, work_t *W) {
    for (int k = 0; k < P->N; ++k) {
        double xn[8], nl[8], J[8][NZ];
        for (int i = 0; i < 8; ++i) nl[i] = -W->lam[NA * (k + 1) + i];
        rk4_derivs(P, W->X + NA * k, W->U + NU * k, nl, xn, J, W->Hs[k]);
        for (int i = 0; i < NA; ++i) { for (int j = 0; j < NA; ++j) W->A[k][i][j] = 0.0; W->Bm[k][i][0] = W->Bm[k][i][1] = 0.0; }
        for (int i = 0; i < 8; ++i) {
            for (int j = 0; j < 8; ++j) W->A[k][i][j] = J[i][j];
            W->Bm[k][i][0] = J[i][NA]; W->Bm[k][i][1] = J[i][NA + 1];
        }
        W->Bm[k][8][0] = 1.0; W->Bm[k][9][1] = 1.0;
    }
}

/* IPOPT's least-square estimate of the starting equality multipliers (DefaultIterateInitializer::
 * least_square_mults -> LeastSquareMultipliers, constr_mult_init_max 1000): y = argmin ||r + J^T y||
 * over the columns of the reference NLP (x_k, u_k), r = scaled grad f - z_L + z_U.  In the augmented
 * formulation [x_k; u_{k-1}] the copy rows x~_{k+1} = u_k are not rows of the reference NLP; giving the
 * copy variables weight 0 in [W J^T; J 0] [d; y] = [-r; 0] makes their columns absorb the Delta-u
 * gradient exactly (y_copy = -r_copy) and leaves the defect multipliers IPOPT's.  An LQR with unit
 * weights on x and u, weight 0 on the copies, zero constraint right-hand side: y_k = -(P_k dx_k + p_k).
 * Uses W->A / W->Bm of the starting point; fills lam (unscaled rows), returns max |lam / dsc|
 * (IPOPT compares the scaled multipliers). */
static double ls_multipliers(const ctx_t *C, work_t *W) {
    const prob_t *P = C->P; const int N = P->N; const double sc = C->sc;
    static __thread double Ks[NMAX][NU][NA], ks[NMAX][NU], Ps[NMAX + 1][NA][NA], ps[NMAX + 1][NA];
    double zN[NZ], gN[NZ];
    for (int i = 0; i < NA; ++i) zN[i] = W->X[NA * N + i];
    zN[10] = zN[11] = 0.0;
    cost_grad(P, zN, C->tgt, 1, gN);
    for (int i = 0; i < NA; ++i) { for (int j = 0; j < NA; ++j) Ps[N][i][j] = (i == j && i < 8); ps[N][i] = sc * gN[i]; }
    for (int k = N - 1; k >= 0; --k) {
        double z[NZ], gq[NZ];
        stage_z(W->X, W->U, k, z);
        cost_grad(P, z, C->tgt, 0, gq);
        for (int j = 0; j < NZ; ++j) gq[j] *= sc;
        for (int a = 0; a < NU; ++a) gq[10 + a] += -W->zL[NU * k + a] + W->zU[NU * k + a];
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = Ps[k + 1];
        double PA[NA][NA], PB[NA][NU], Qxx[NA][NA], Qux[NU][NA], Quu[NU][NU], qx[NA], qu[NU], L[3] = {1, 0, 1}, x2[2];
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) { double t = 0; for (int m = 0; m < NA; ++m) t += Pp[i][m] * A[m][j]; PA[i][j] = t; }
            for (int j = 0; j < NU; ++j) { double t = 0; for (int m = 0; m < NA; ++m) t += Pp[i][m] * Bm[m][j]; PB[i][j] = t; }
        }
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) { double t = (i == j && i < 8); for (int m = 0; m < NA; ++m) t += A[m][i] * PA[m][j]; Qxx[i][j] = t; }
            double t = gq[i]; for (int m = 0; m < NA; ++m) t += A[m][i] * ps[k + 1][m]; qx[i] = t;
        }
        for (int a = 0; a < NU; ++a) {
            for (int i = 0; i < NA; ++i) { double t = 0; for (int m = 0; m < NA; ++m) t += Bm[m][a] * PA[m][i]; Qux[a][i] = t; }
            for (int c = 0; c < NU; ++c) { double t = (a == c); for (int m = 0; m < NA; ++m) t += Bm[m][a] * PB[m][c]; Quu[a][c] = t; }
            double t = gq[NA + a]; for (int m = 0; m < NA; ++m) t += Bm[m][a] * ps[k + 1][m]; qu[a] = t;
        }
        chol2(Quu[0][0], 0.5 * (Quu[0][1] + Quu[1][0]), Quu[1][1], L);      /* Quu >= I */
        chol2_solve(L, qu, x2); ks[k][0] = -x2[0]; ks[k][1] = -x2[1];
        for (int i = 0; i < NA; ++i) {
            double b2[2] = {Qux[0][i], Qux[1][i]};
            chol2_solve(L, b2, x2); Ks[k][0][i] = -x2[0]; Ks[k][1][i] = -x2[1];
        }
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) Ps[k][i][j] = Qxx[i][j] + Qux[0][i] * Ks[k][0][j] + Qux[1][i] * Ks[k][1][j];
            ps[k][i] = qx[i] + Qux[0][i] * ks[k][0] + Qux[1][i] * ks[k][1];
        }
        /* symmetric as riccati_factor keeps it: unsymmetrised rounding let the unit-weight recursion lose its
           positive definiteness on unstable dynamics (Quu < 0 at k = 16 of a C5 stress instance) and overflow,
           where the dense least-squares solution is moderate (max |y| 547) */
        for (int i = 0; i < NA; ++i) for (int j = 0; j < i; ++j) { const double t = 0.5 * (Ps[k][i][j] + Ps[k][j][i]); Ps[k][i][j] = Ps[k][j][i] = t; }
#ifdef ORACLE_DEBUG
        { double pm = 0, qm = 0; for (int i = 0; i < NA; ++i) { qm = fmax(qm, fabs(ps[k][i])); for (int j = 0; j < NA; ++j) pm = fmax(pm, fabs(Ps[k][i][j])); }
          fprintf(stderr, "  lsq k %2d max|P| %.3e max|p| %.3e Quu %.3e %.3e %.3e\n", k, pm, qm, Quu[0][0], Quu[0][1], Quu[1][1]); }
#endif
    }
    double dx[NA] = {0}, ymax = 0.0;
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < NA; ++i) {
            double t = ps[k][i]; for (int m = 0; m < NA; ++m) t += Ps[k][i][m] * dx[m];
            W->lam[NA * k + i] = -t;
            if (i < 8) ymax = fmax(ymax, fabs(t) / W->dsc[NA * k + i]);   /* the copy rows are not IPOPT's */
            if (!isfinite(t)) ymax = INFINITY;     /* the recursion overflowed: far above constr_mult_init_max */
        }
        if (k == N) break;
        double du[NU], dn[NA];
        for (int a = 0; a < NU; ++a) { double t = ks[k][a]; for (int i = 0; i < NA; ++i) t += Ks[k][a][i] * dx[i]; du[a] = t; }
        for (int i = 0; i < NA; ++i) {
            double t = 0; for (int m = 0; m < NA; ++m) t += W->A[k][i][m] * dx[m];
            for (int a = 0; a < NU; ++a) t += W->Bm[k][i][a] * du[a];
            dn[i] = t;
        }
        memcpy(dx, dn, sizeof dx);
    }
    return ymax;
}

/* KKT residual measures at the iterate held in W (A, Bm linearised there) with defects g: max norms
   of IPOPT's eq. 5 (dinf, scaled pinf, unscaled pinf_u, complementarity c0 with mu = 0), the sums of
   |y~| and |z| for s_d / s_c and, when pd != NULL, IPOPT's primal-dual system error at C->mu
   (IpoptCalculatedQuantities::curr_primal_dual_system_error: the l1 norms of the primal
   infeasibility, the dual infeasibility and the complementarity z s - mu, added) */
static void kkt_errors(const ctx_t *C, const work_t *W, double g[][NA], double *sum_l_, double *sum_z_,
                       double *dinf_, double *pinf_, double *pinf_u_, double *c0_, double *pd) {
    const prob_t *P = C->P; const int N = P->N, nA = NA * (N + 1);
    double sum_l = 0, sum_z = 0, dinf = 0, pinf = 0, pinf_u = 0, c0 = 0, l1p = 0, l1d = 0, l1c = 0;
    for (int i = 0; i < nA; ++i) sum_l += fabs(W->lam[i]) / W->dsc[i];
    for (int k = 0; k <= N; ++k) {
        double z[NZ], gc[NZ], gl[NZ];
        for (int i = 0; i < NA; ++i) z[i] = W->X[NA * k + i];
        z[10] = k < N ? W->U[NU * k] : 0.0; z[11] = k < N ? W->U[NU * k + 1] : 0.0;
        cost_grad(P, z, C->tgt, k == N, gc);
        for (int j = 0; j < NZ; ++j) gl[j] = C->sc * gc[j];
        for (int i = 0; i < NA; ++i) gl[i] += W->lam[NA * k + i];
        if (k < N) {
            for (int m = 0; m < NA; ++m) {
                double l = W->lam[NA * (k + 1) + m];
                for (int i = 0; i < NA; ++i) gl[i] -= W->A[k][m][i] * l;
                gl[10] -= W->Bm[k][m][0] * l; gl[11] -= W->Bm[k][m][1] * l;
            }
            gl[10] += -W->zL[NU * k] + W->zU[NU * k]; gl[11] += -W->zL[NU * k + 1] + W->zU[NU * k + 1];
            for (int j = 0; j < NZ; ++j) { dinf = fmax(dinf, fabs(gl[j])); l1d += fabs(gl[j]); }
            for (int a = 0; a < NU; ++a) {
                const int j = NU * k + a;
                const double cl = W->zL[j] * (W->U[j] - C->lo), cu = W->zU[j] * (C->hi - W->U[j]);
                c0 = fmax(c0, fmax(fabs(cl), fabs(cu)));
                l1c += fabs(cl - C->mu) + fabs(cu - C->mu);
                sum_z += W->zL[j] + W->zU[j];
            }
        } else {
            for (int i = 0; i < NA; ++i) { dinf = fmax(dinf, fabs(gl[i])); l1d += fabs(gl[i]); }
        }
        for (int i = 0; i < NA; ++i) {
            pinf = fmax(pinf, W->dsc[NA * k + i] * fabs(g[k][i]));
            pinf_u = fmax(pinf_u, fabs(g[k][i]));
            l1p += W->dsc[NA * k + i] * fabs(g[k][i]);
        }
    }
    *sum_l_ = sum_l; *sum_z_ = sum_z; *dinf_ = dinf; *pinf_ = pinf; *pinf_u_ = pinf_u; *c0_ = c0;
    if (pd) *pd = l1p + l1d + l1c;
}

static double g_mult_init_max = 1e3;   /* IPOPT constr_mult_init_max (default 1000; 0 = zero multipliers) */
void oracle_lmpc_set_mult_init_max(double m) { g_mult_init_max = m; }

/* IPOPT's soft restoration phase (BacktrackingLineSearch::TrySoftRestoStep, soft_resto_pderror_reduction_factor
 * 0.9999): the primal-dual step of the current direction, damped only by the fraction to the boundary
 * (one step length min(alpha_primal_max, alpha_dual_max) for x, y and z), is taken if the original filter
 * accepts it with alpha_primal_test = 0 (*orig = 1: the phase ends) or if it reduces the primal-dual system
 * error at the current mu by the factor.  Returns the step length (0: rejected); W is left unchanged. */
static double bound_dual_step(const ctx_t *C, work_t *W, int nU, double tau);
static int g_soft_resto = 1;
void oracle_lmpc_set_soft_resto(int on) { g_soft_resto = on; }

static double soft_resto_step(const ctx_t *C, work_t *W, int nfilt, double th, double phi, double th_max,
                              double tau, double curr_pd, double gt[][NA], double *th_t, double *ph_t, int *orig) {
    const prob_t *P = C->P; const int N = P->N, nU = NU * N, nA = NA * (N + 1);
    const double gam_th = 1e-5, gam_ph = 1e-8;
    const double a = fmin(frac_to_boundary(C, W, W->dU, tau), bound_dual_step(C, W, nU, tau));
    for (int i = 0; i < nA; ++i) W->Xt[i] = W->X[i] + a * W->dX[i];
    for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + a * W->dU[j];
    *th_t = residuals(C, W, W->Xt, W->Ut, gt);
    *ph_t = barrier_obj(C, W->Xt, W->Ut);
    *orig = 0;
    /* FilterLSAcceptor::CheckAcceptabilityOfTrialPoint(0): sufficient decrease against the current
       iterate (no Armijo branch at alpha 0), then the filter (which holds the current point) */
    int in_filter = !(*th_t < th_max) || !isfinite(*ph_t);
    for (int q = 0; q < nfilt && !in_filter; ++q) in_filter = *th_t >= W->filt_th[q] && *ph_t >= W->filt_ph[q];
    if (!in_filter && (LE(*th_t, (1 - gam_th) * th, th) || LE(*ph_t - phi, -gam_ph * th, phi))) { *orig = 1; return a; }
    if (!isfinite(*ph_t)) return 0.0;
    /* the primal-dual system error at the trial point (x, y, z all moved by a) */
    work_t *S = (work_t *)malloc(sizeof(work_t));
    memcpy(S, W, sizeof(work_t));
    memcpy(W->X, S->Xt, sizeof(double) * nA); memcpy(W->U, S->Ut, sizeof(double) * nU);
    for (int i = 0; i < nA; ++i) W->lam[i] = S->lam[i] + a * (S->lamp[i] - S->lam[i]);
    for (int j = 0; j < nU; ++j) { W->zL[j] = S->zL[j] + a * S->dzL[j]; W->zU[j] = S->zU[j] + a * S->dzU[j]; }
    linearise(P, W);
    double sl, sz, di, pi, pu, c0, pd;
    kkt_errors(C, W, gt, &sl, &sz, &di, &pi, &pu, &c0, &pd);
    memcpy(W, S, sizeof(work_t));
    free(S);
    return pd <= 0.9999 * curr_pd ? a : 0.0;
}

/* ---------------------------------------------------------------------------------------------
 * IPOPT's restoration phase (MinC_1NrmRestorationPhase::PerformRestoration with RestoIpoptNLP,
 * RestoIterateInitializer and RestoFilterConvergenceCheck; IPOPT 3.14 defaults, restated -- no IPOPT
 * source is in the image):
 *   - rho = resto_penalty_parameter 1000, eta(mu) = resto_proximity_weight 1 * sqrt(mu) of the
 *     restoration's current mu, D_R = diag(min(1, 1/|x_R|)), x_R = the current point;
 *   - start: mu_R = max(mu, ||d c||_inf); x = x_R; per row n = a + sqrt(a^2 + b), p = d c + n with
 *     a = mu_R/(2 rho) - d c/2, b = d c mu_R/(2 rho); z_p = mu_R/p, z_n = mu_R/n; the u-bound
 *     multipliers min(rho, z); equality multipliers by least squares (dropped above 1000);
 *   - the restoration problem is solved by the same algorithm (monotone mu, filter line search with
 *     second-order correction, inertia correction) with its own filter; its iterations count in the
 *     iteration counter and max_iter caps the total;
 *   - at every iteration after the first the original problem's progress is tested at the current
 *     point: theta_orig <= 0.9 theta_orig(start) (required_infeasibility_reduction) and acceptable
 *     to the original filter (which holds the start point) and to the start point; then the phase
 *     returns: the u-bound multipliers take the step (mu - z s_trial)/s that pretends the whole
 *     progress was one primal-dual Newton step, cut by the fraction to the boundary and reset to 1
 *     if any exceeds bound_mult_reset_threshold 1000; the equality multipliers restart at 0
 *     (constr_mult_reset_threshold 0);
 *   - the restoration problem converging (optimal or acceptable) means local infeasibility; a failed
 *     line search inside it is a restoration failure: the solve ends with status 2 (IPOPT's
 *     Infeasible_Problem_Detected) or -2 (Restoration_Failed).
 * Returns 1 with the new iterate in W (multipliers included) and *it set to the last restoration
 * iteration, 0 with *status set.
 * --------------------------------------------------------------------------------------------- */
static int g_resto = 1;
void oracle_lmpc_set_resto(int on) { g_resto = on; }

/* restoration residuals: p, n rows (rp, rn of the barrier Lagrangian gradient), soft-row right-hand
   sides rg = cres/d - (rn/Sn - rp/Sp)/d + D lam (physical rows) or g (copy rows) for constraint values
   cres (d g + n - p, or a second-order correction's c_soc) */
static void resto_rhs(const ctx_t *C, const work_t *W, double cres[][NA], double rg[][NA]) {
    const resto_t *R = C->R; const int N = C->P->N;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        const int r = NA * k + i;
        if (i < 8) {
            const double d = R->dsc[r];
            rg[k][i] = cres[k][i] / d - (R->rn[r] / R->Snd[r] - R->rp[r] / R->Spd[r]) / d + R->D[r] * W->lam[r];
        } else {
            rg[k][i] = cres[k][i];
        }
    }
}
/* constraint values of the restoration problem at (X, U, p, n): d g + n - p on the physical rows, g
   on the copy rows; returns its l1 norm (theta of the restoration problem) */
static double resto_cons(const ctx_t *C, work_t *W, const double *X, const double *U, const double *pc,
                         const double *nc, double g[][NA], double cres[][NA]) {
    const resto_t *R = C->R; const int N = C->P->N;
    residuals(C, W, X, U, g);
    double th = 0.0;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        const int r = NA * k + i;
        cres[k][i] = i < 8 ? R->dsc[r] * g[k][i] + nc[r] - pc[r] : g[k][i];
        th += fabs(cres[k][i]);
    }
    return th;
}
static double resto_barrier(const ctx_t *C, const double *X, const double *U, const double *pc, const double *nc) {
    const resto_t *R = C->R; const int N = C->P->N;
    double f = 0.0, lb = 0.0;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < 8; ++i) {
        const int r = NA * k + i;
        const double e = R->DRx[r] * (X[r] - R->XR[r]);
        f += R->rho * (pc[r] + nc[r]) + 0.5 * R->eta * e * e;
        if (!(pc[r] > 0) || !(nc[r] > 0)) return INFINITY;
        lb += log(pc[r]) + log(nc[r]);
    }
    for (int j = 0; j < NU * N; ++j) {
        const double e = R->DRu[j] * (U[j] - R->UR[j]);
        f += 0.5 * R->eta * e * e;
        double sl = U[j] - C->lo, su = C->hi - U[j];
        if (!(sl > 0) || !(su > 0)) return INFINITY;
        lb += log(sl) + log(su);
    }
    return f - C->mu * lb;
}
/* optimality-error measures of the restoration problem at the iterate in W (A, Bm there) */
static void resto_errors(const ctx_t *C, const work_t *W, double cres[][NA], double *dinf_, double *pinf_,
                         double *c0_, double *cmin_, double *sum_l_, double *sum_z_) {
    const resto_t *R = C->R; const int N = C->P->N;
    double dinf = 0, pinf = 0, c0 = 0, cmin = INFINITY, sum_l = 0, sum_z = 0;
    for (int k = 0; k <= N; ++k) {
        double gl[NZ];
        for (int j = 0; j < NZ; ++j) gl[j] = 0.0;
        for (int i = 0; i < 8; ++i) {
            const int r = NA * k + i;
            gl[i] = R->eta * R->DRx[r] * R->DRx[r] * (W->X[r] - R->XR[r]);
        }
        for (int i = 0; i < NA; ++i) gl[i] += W->lam[NA * k + i];
        if (k < N) {
            for (int a = 0; a < NU; ++a) {
                const int j = NU * k + a;
                gl[10 + a] = R->eta * R->DRu[j] * R->DRu[j] * (W->U[j] - R->UR[j]) - W->zL[j] + W->zU[j];
            }
            for (int m = 0; m < NA; ++m) {
                double l = W->lam[NA * (k + 1) + m];
                for (int i = 0; i < NA; ++i) gl[i] -= W->A[k][m][i] * l;
                gl[10] -= W->Bm[k][m][0] * l; gl[11] -= W->Bm[k][m][1] * l;
            }
            for (int j = 0; j < NZ; ++j) dinf = fmax(dinf, fabs(gl[j]));
            for (int a = 0; a < NU; ++a) {
                const int j = NU * k + a;
                const double cl = W->zL[j] * (W->U[j] - C->lo), cu = W->zU[j] * (C->hi - W->U[j]);
                c0 = fmax(c0, fmax(cl, cu)); cmin = fmin(cmin, fmin(cl, cu));
                sum_z += W->zL[j] + W->zU[j];
            }
        } else {
            for (int i = 0; i < NA; ++i) dinf = fmax(dinf, fabs(gl[i]));
        }
        for (int i = 0; i < NA; ++i) {
            const int r = NA * k + i;
            pinf = fmax(pinf, fabs(cres[k][i]));
            if (i < 8) {
                const double y = W->lam[r] / R->dsc[r];
                dinf = fmax(dinf, fmax(fabs(R->rho - R->zp[r] - y), fabs(R->rho - R->zn[r] + y)));
                const double cp = R->zp[r] * R->pc[r], cn = R->zn[r] * R->nc[r];
                c0 = fmax(c0, fmax(cp, cn)); cmin = fmin(cmin, fmin(cp, cn));
                sum_z += R->zp[r] + R->zn[r];
                sum_l += fabs(y);
            } else {
                sum_l += fabs(W->lam[r]);
            }
        }
    }
    *dinf_ = dinf; *pinf_ = pinf; *c0_ = c0; *cmin_ = cmin; *sum_l_ = sum_l; *sum_z_ = sum_z;
}

/* Iterative refinement of the restoration step (IPOPT refines every solve of its augmented system,
   PDFullSpaceSolver; the GPU kernel refines its restoration steps the same way): the residuals of the full
   Newton system at the step in V / R (stationarity of x and u, the scaled defect rows d J dx + dn - dp + c,
   the p / n rows) are solved for on the same factorisation when they exceed 1e-12 (1 + |step|) (lam = 0
   and the residuals in place of the gradients and right-hand sides), and the correction is added; at most
   g_resto_refine times per step.  Returns 1 if a correction was made. */
static int g_resto_refine = 3;
void oracle_lmpc_set_resto_refine(int n) { g_resto_refine = n < 0 ? 0 : n; }
static int resto_refine(const ctx_t *C, work_t *V, double cres[][NA], double rg[][NA]) {
    resto_t *R = C->R; const prob_t *P = C->P; const int N = P->N, nA = NA * (N + 1), nU = NU * N;
    double emax = 0.0, smax = 0.0;
#define EM(v) (emax = fmax(emax, fabs(v)))
#define SM(v) (smax = fmax(smax, fabs(v)))
    for (int k = 0; k < N; ++k) {
        double Hq[NZ][NZ], gq[NZ], dz[NZ];
        stage_qp(C, V, k, R->delta, Hq, gq);
        for (int a = 0; a < NA; ++a) dz[a] = V->dX[NA * k + a];
        dz[10] = V->dU[NU * k]; dz[11] = V->dU[NU * k + 1];
        for (int a = 0; a < NZ; ++a) { double t = gq[a]; for (int b = 0; b < NZ; ++b) t += Hq[a][b] * dz[b]; R->ex[k][a] = t; }
        for (int i = 0; i < NA; ++i) R->ex[k][i] += V->lamp[NA * k + i];
        for (int m = 0; m < NA; ++m) {
            const double l = V->lamp[NA * (k + 1) + m];
            for (int i = 0; i < NA; ++i) R->ex[k][i] -= V->A[k][m][i] * l;
            R->ex[k][10] -= V->Bm[k][m][0] * l; R->ex[k][11] -= V->Bm[k][m][1] * l;
        }
        for (int a = 0; a < NZ; ++a) EM(R->ex[k][a]);
    }
    {
        double Pn[NA][NA], pn[NA];
        terminal_qp(C, V, R->delta, Pn, pn);
        for (int i = 0; i < NZ; ++i) R->ex[N][i] = 0.0;
        for (int i = 0; i < NA; ++i) {
            double t = pn[i] + V->lamp[NA * N + i];
            for (int j = 0; j < NA; ++j) t += Pn[i][j] * V->dX[NA * N + j];
            R->ex[N][i] = t;
            EM(t);
        }
    }
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        const int r = NA * k + i;
        double jd = V->dX[r];
        if (k > 0) {
            for (int m = 0; m < NA; ++m) jd -= V->A[k - 1][i][m] * V->dX[NA * (k - 1) + m];
            for (int a = 0; a < NU; ++a) jd -= V->Bm[k - 1][i][a] * V->dU[NU * (k - 1) + a];
        }
        SM(V->dX[r]);
        if (i < 8) {
            const double d = R->dsc[r], dy = (V->lamp[r] - V->lam[r]) / d;
            R->ec[k][i] = d * jd + R->dnc[r] - R->dpc[r] + cres[k][i];
            R->ep[r] = R->Spd[r] * R->dpc[r] - dy + R->rp[r];
            R->en[r] = R->Snd[r] * R->dnc[r] + dy + R->rn[r];
            EM(R->ep[r]); EM(R->en[r]); SM(R->dpc[r]); SM(R->dnc[r]);
        } else {
            R->ec[k][i] = jd + cres[k][i];
        }
        EM(R->ec[k][i]);
    }
    for (int j = 0; j < nU; ++j) SM(V->dU[j]);
#undef EM
#undef SM
    if (!(emax > 1e-12 * (1.0 + smax))) return 0;
    work_t *Sv = (work_t *)malloc(sizeof(work_t));
    resto_t *SR = (resto_t *)malloc(sizeof(resto_t));
    memcpy(Sv, V, sizeof(work_t)); memcpy(SR, R, sizeof(resto_t));
    memset(V->lam, 0, sizeof(double) * nA);
    for (int i = 0; i < nA; ++i) { R->rp[i] = R->ep[i]; R->rn[i] = R->en[i]; }
    R->ovr = 1;
    memcpy(R->gov, R->ex, sizeof(double[NZ]) * (N + 1));
    resto_rhs(C, V, R->ec, rg);
    riccati_solve(C, V, rg);
    for (int i = 0; i < nA; ++i) {
        Sv->dX[i] += V->dX[i];
        Sv->lamp[i] += V->lamp[i];
        if ((i % NA) < 8) {
            const double dy = V->lamp[i] / R->dsc[i];
            SR->dpc[i] += (dy - R->ep[i]) / R->Spd[i];
            SR->dnc[i] += (-dy - R->en[i]) / R->Snd[i];
        }
    }
    for (int j = 0; j < nU; ++j) Sv->dU[j] += V->dU[j];
    memcpy(V, Sv, sizeof(work_t)); memcpy(R, SR, sizeof(resto_t));
    free(Sv); free(SR);
    return 1;
}

static int restoration(const ctx_t *C0, work_t *W, int *it_io, int max_iter, double tol, double acc_tol, int acc_iter,
                       double th0, double phi0, int nfilt0, double tau0, double g0[][NA], int *status) {
    const prob_t *P = C0->P; const int N = P->N, nU = NU * N, nA = NA * (N + 1), nrow = 8 * (N + 1);
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, gam_al = 0.05, kap_soc = 0.99;
    const double mu_min = tol / 10, s_max = 100.0;
    resto_t *R = (resto_t *)calloc(1, sizeof(resto_t));
    work_t *V = (work_t *)malloc(sizeof(work_t));
    memcpy(V, W, sizeof(work_t));
    double (*g)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*gt)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*cres)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*ct)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*csg)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*rg)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double *sv = (double *)malloc(sizeof(double) * (2 * nA + nU + 2 * nA));
    ctx_t C = *C0;
    C.R = R; C.mode = 1;
    R->rho = 1000.0; R->dsc = W->dsc;
    int ok_out = 0;
    /* RestoIpoptNLP: reference point and D_R */
    for (int r = 0; r < nA; ++r) { R->XR[r] = W->X[r]; R->DRx[r] = 1.0 / fmax(1.0, fabs(W->X[r])); }
    for (int j = 0; j < nU; ++j) { R->UR[j] = W->U[j]; R->DRu[j] = 1.0 / fmax(1.0, fabs(W->U[j])); }
    /* RestoIterateInitializer */
    double cmax = 0.0;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) cmax = fmax(cmax, W->dsc[NA * k + i] * fabs(g0[k][i]));
    C.mu = fmax(C0->mu, cmax);
    R->eta = sqrt(C.mu);
    for (int k = 0; k <= N; ++k) for (int i = 0; i < 8; ++i) {
        const int r = NA * k + i;
        const double c = W->dsc[r] * g0[k][i];
        const double a = C.mu / (2.0 * R->rho) - 0.5 * c, b = c * C.mu / (2.0 * R->rho);
        R->nc[r] = a + sqrt(a * a + b);
        R->pc[r] = c + R->nc[r];
        R->zp[r] = C.mu / R->pc[r]; R->zn[r] = C.mu / R->nc[r];
    }
    for (int j = 0; j < nU; ++j) { V->zL[j] = fmin(R->rho, W->zL[j]); V->zU[j] = fmin(R->rho, W->zU[j]); }
    /* least-square equality multipliers (LeastSquareMultipliers on the restoration problem: unit
       weights on x, u, p, n; the p / n columns make every physical row soft with D = 2/d^2) */
    linearise(P, V);
    {
        C.mode = 2;
        for (int r = 0; r < nA; ++r) { R->rp[r] = (r % NA) < 8 ? R->rho - R->zp[r] : 0.0; R->rn[r] = (r % NA) < 8 ? R->rho - R->zn[r] : 0.0; }
        riccati_factor(&C, V, 0.0);      /* unit weights: every Quu >= I */
        memset(V->lam, 0, sizeof(double) * nA);
        for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) cres[k][i] = 0.0;
        resto_rhs(&C, V, cres, rg);       /* rg = -(rn - rp)/d: D lam = 0, Sp = Sn = 1 */
        riccati_solve(&C, V, rg);
        double ym = 0.0;
        for (int r = 0; r < nA; ++r) {
            if ((r % NA) < 8) ym = fmax(ym, fabs(V->lamp[r]) / W->dsc[r]);
            if (!isfinite(V->lamp[r])) ym = INFINITY;
        }
        if (ym <= 1e3) memcpy(V->lam, V->lamp, sizeof(double) * nA);
        else memset(V->lam, 0, sizeof(double) * nA);
        C.mode = 1;
    }
    double th = resto_cons(&C, V, V->X, V->U, R->pc, R->nc, g, cres);
    const double th_max = 1e4 * fmax(1.0, th), th_min = 1e-4 * fmax(1.0, th);
    int nfilt = 0, rit = *it_io + 1, first = 1, acc_count = 0;
    double delta_last = 0.0;
    for (;; ++rit) {
        linearise(P, V);
        if (!first) {
            /* RestoConvergenceCheck: progress of the original problem at the current point */
            const double tho = residuals(C0, V, V->X, V->U, gt);
            if (tho <= 0.9 * th0) {
                const double pho = barrier_obj(C0, V->X, V->U);
                int acc = isfinite(pho);
                for (int q = 0; q < nfilt0 && acc; ++q) acc = !(tho >= W->filt_th[q] && pho >= W->filt_ph[q]);
                acc = acc && (LE(tho, (1 - gam_th) * th0, th0) || LE(pho - phi0, -gam_ph * th0, phi0));
                if (acc) { ok_out = 1; break; }
            }
        }
        first = 0;
        double dinf, pinf, c0, cmin, sum_l, sum_z;
        resto_errors(&C, V, cres, &dinf, &pinf, &c0, &cmin, &sum_l, &sum_z);
        const double nb = 2.0 * nU + 2.0 * nrow;
        const double s_d = fmax(s_max, (sum_l + sum_z) / (nA + nb)) / s_max;     /* rows + bound multipliers */
        const double s_c = fmax(s_max, sum_z / nb) / s_max;
        const double err = fmax(dinf / s_d, fmax(pinf, c0 / s_c));
        if (rit >= max_iter) { *status = ST_MAXITER; break; }
        if (err <= tol && dinf <= 1.0 && pinf <= 1e-4 && c0 <= 1e-4) { *status = ST_INFEASIBLE; break; }   /* local infeasibility */
        if (acc_iter > 0 && err <= acc_tol && pinf <= 1e-2 && c0 <= 1e-2) {
            if (++acc_count >= acc_iter) { *status = ST_INFEASIBLE; break; }
        } else {
            acc_count = 0;
        }
        for (;;) {
            const double cmu = fmax(c0 - C.mu, C.mu - cmin);
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * C.mu || C.mu <= mu_min) break;
            C.mu = fmax(mu_min, fmin(0.2 * C.mu, pow(C.mu, 1.5)));
            R->eta = sqrt(C.mu);
            nfilt = 0;
        }
        const double tau = fmax(0.99, 1.0 - C.mu);
        for (int r = 0; r < nA; ++r) if ((r % NA) < 8) {
            const double y = V->lam[r] / W->dsc[r];
            R->rp[r] = R->rho - C.mu / R->pc[r] - y;
            R->rn[r] = R->rho - C.mu / R->nc[r] + y;
        }
        double delta = 0.0;
        int ok = riccati_factor(&C, V, 0.0);
        for (int attempt = 0; !ok && attempt < 60; ++attempt) {
            delta = (attempt == 0) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            ok = riccati_factor(&C, V, delta);
        }
        if (!ok) { *status = ST_INERTIA_FAIL; break; }
        if (delta > 0) delta_last = delta;
        R->delta = delta;
        /* the step: Riccati for the soft rows, then p, n and every bound multiplier */
        double amax = 0, az = 0;
        #define RESTO_STEP(CV) do {                                                                   \
            resto_rhs(&C, V, CV, rg);                                                                 \
            riccati_solve(&C, V, rg);                                                                 \
            for (int r = 0; r < nA; ++r) if ((r % NA) < 8) {                                         \
                const double dy = (V->lamp[r] - V->lam[r]) / W->dsc[r];                               \
                R->dpc[r] = (dy - R->rp[r]) / R->Spd[r];                                              \
                R->dnc[r] = (-dy - R->rn[r]) / R->Snd[r];                                             \
            }                                                                                         \
            for (int rr_ = 0; rr_ < g_resto_refine && resto_refine(&C, V, CV, rg); ++rr_) {}          \
            amax = frac_to_boundary(&C, V, V->dU, tau); az = 1.0;                                     \
            for (int r = 0; r < nA; ++r) if ((r % NA) < 8) {                                         \
                R->dzp[r] = C.mu / R->pc[r] - R->zp[r] - R->zp[r] / R->pc[r] * R->dpc[r];             \
                R->dzn[r] = C.mu / R->nc[r] - R->zn[r] - R->zn[r] / R->nc[r] * R->dnc[r];             \
                if (R->dpc[r] < 0) amax = fmin(amax, -tau * R->pc[r] / R->dpc[r]);                    \
                if (R->dnc[r] < 0) amax = fmin(amax, -tau * R->nc[r] / R->dnc[r]);                    \
                if (R->dzp[r] < 0) az = fmin(az, -tau * R->zp[r] / R->dzp[r]);                        \
                if (R->dzn[r] < 0) az = fmin(az, -tau * R->zn[r] / R->dzn[r]);                        \
            }                                                                                         \
            az = fmin(az, bound_dual_step(&C, V, nU, tau));                                           \
        } while (0)
        RESTO_STEP(cres);
#ifdef ORACLE_DEBUG
        {   /* linearised restoration constraints: d J dx + dn - dp = -cres (physical rows), J dx = -g (copies);
               p-row stationarity: Sp dp - dy = -rp */
            double e1 = 0.0, e2 = 0.0;
            for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
                const int r = NA * k + i;
                double jd = V->dX[r];
                if (k > 0) {
                    for (int m = 0; m < NA; ++m) jd -= V->A[k - 1][i][m] * V->dX[NA * (k - 1) + m];
                    for (int a = 0; a < NU; ++a) jd -= V->Bm[k - 1][i][a] * V->dU[NU * (k - 1) + a];
                }
                if (i < 8) {
                    e1 = fmax(e1, fabs(W->dsc[r] * jd + R->dnc[r] - R->dpc[r] + cres[k][i]));
                    const double dy = (V->lamp[r] - V->lam[r]) / W->dsc[r];
                    e2 = fmax(e2, fabs(R->Spd[r] * R->dpc[r] - dy + R->rp[r]) + fabs(R->Snd[r] * R->dnc[r] + dy + R->rn[r]));
                } else e1 = fmax(e1, fabs(jd + cres[k][i]));
            }
            fprintf(stderr, "  resto step check: constraint %.2e  p/n rows %.2e\n", e1, e2);
        }
#endif
        const double phi = resto_barrier(&C, V->X, V->U, R->pc, R->nc);
        double gTd = 0.0;
        for (int k = 0; k <= N; ++k) for (int i = 0; i < 8; ++i) {
            const int r = NA * k + i;
            gTd += R->eta * R->DRx[r] * R->DRx[r] * (V->X[r] - R->XR[r]) * V->dX[r];
            gTd += (R->rho - C.mu / R->pc[r]) * R->dpc[r] + (R->rho - C.mu / R->nc[r]) * R->dnc[r];
        }
        for (int j = 0; j < nU; ++j)
            gTd += (R->eta * R->DRu[j] * R->DRu[j] * (V->U[j] - R->UR[j]) - C.mu / (V->U[j] - C.lo) + C.mu / (C.hi - V->U[j])) * V->dU[j];
        double amin = gam_th;
        if (gTd < 0) amin = fmin(gam_th, fmin(gam_ph * th / (-gTd), pow(th, s_th) / pow(-gTd, s_ph)));
        amin *= gam_al;
        double alpha = amax, th_t = 0, ph_t = 0;
        int accepted = 0, ftype = 0;
        #define RESTO_TRIAL(AL) do {                                                                  \
            for (int i = 0; i < nA; ++i) V->Xt[i] = V->X[i] + (AL) * V->dX[i];                       \
            for (int j = 0; j < nU; ++j) V->Ut[j] = V->U[j] + (AL) * V->dU[j];                       \
            for (int r = 0; r < nA; ++r) if ((r % NA) < 8) {                                         \
                R->pt_[r] = R->pc[r] + (AL) * R->dpc[r]; R->nt_[r] = R->nc[r] + (AL) * R->dnc[r];    \
            }                                                                                         \
            th_t = resto_cons(&C, V, V->Xt, V->Ut, R->pt_, R->nt_, gt, ct);                          \
            ph_t = resto_barrier(&C, V->Xt, V->Ut, R->pt_, R->nt_);                                  \
        } while (0)
        for (int ls = 0; ls < 80 && !accepted; ++ls) {
            if (alpha < amin && ls > 0) break;
            RESTO_TRIAL(alpha);
            /* the restoration problem's own filter (filter_accept reads W->filt_*: swap in R's) */
            {
                int in_f = !(th_t < th_max) || !isfinite(ph_t);
                for (int q = 0; q < nfilt && !in_f; ++q) in_f = th_t >= R->filt_th[q] && ph_t >= R->filt_ph[q];
                if (!in_f) {
                    const int sw = gTd < 0 && alpha * pow(-gTd, s_ph) > pow(th, s_th);
                    if (th <= th_min && sw) { if (LE(ph_t, phi + 1e-8 * alpha * gTd, phi)) { accepted = 1; ftype = 1; } }
                    else accepted = LE(th_t, (1 - gam_th) * th, th) || LE(ph_t - phi, -gam_ph * th, phi);
                }
            }
            if (!accepted && ls == 0 && !(th_t < th)) {
                /* second-order correction on the restoration problem's constraints */
                memcpy(sv, V->dX, sizeof(double) * nA); memcpy(sv + nA, V->lamp, sizeof(double) * nA);
                memcpy(sv + 2 * nA, V->dU, sizeof(double) * nU);
                memcpy(sv + 2 * nA + nU, R->dpc, sizeof(double) * nA); memcpy(sv + 3 * nA + nU, R->dnc, sizeof(double) * nA);
                double asoc = alpha, th_old = 0.0;
                for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) csg[k][i] = cres[k][i];
                for (int c = 0; c < 4; ++c) {
                    if (c > 0 && !(th_t <= kap_soc * th_old)) break;
                    th_old = th_t;
                    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) csg[k][i] = asoc * csg[k][i] + ct[k][i];
                    RESTO_STEP(csg);
                    asoc = amax;
                    RESTO_TRIAL(asoc);
                    int in_f = !(th_t < th_max) || !isfinite(ph_t);
                    for (int q = 0; q < nfilt && !in_f; ++q) in_f = th_t >= R->filt_th[q] && ph_t >= R->filt_ph[q];
                    int acc = 0;
                    if (!in_f) {
                        const int sw = gTd < 0 && alpha * pow(-gTd, s_ph) > pow(th, s_th);
                        if (th <= th_min && sw) { if (LE(ph_t, phi + 1e-8 * alpha * gTd, phi)) { acc = 1; ftype = 1; } }
                        else acc = LE(th_t, (1 - gam_th) * th, th) || LE(ph_t - phi, -gam_ph * th, phi);
                    }
                    if (acc) { accepted = 1; alpha = asoc; break; }
                }
                if (!accepted) {
                    memcpy(V->dX, sv, sizeof(double) * nA); memcpy(V->lamp, sv + nA, sizeof(double) * nA);
                    memcpy(V->dU, sv + 2 * nA, sizeof(double) * nU);
                    memcpy(R->dpc, sv + 2 * nA + nU, sizeof(double) * nA); memcpy(R->dnc, sv + 3 * nA + nU, sizeof(double) * nA);
                    /* the bound-multiplier steps of the plain direction back */
                    for (int r = 0; r < nA; ++r) if ((r % NA) < 8) {
                        R->dzp[r] = C.mu / R->pc[r] - R->zp[r] - R->zp[r] / R->pc[r] * R->dpc[r];
                        R->dzn[r] = C.mu / R->nc[r] - R->zn[r] - R->zn[r] / R->nc[r] * R->dnc[r];
                    }
                    az = 1.0;
                    for (int r = 0; r < nA; ++r) if ((r % NA) < 8) {
                        if (R->dzp[r] < 0) az = fmin(az, -tau * R->zp[r] / R->dzp[r]);
                        if (R->dzn[r] < 0) az = fmin(az, -tau * R->zn[r] / R->dzn[r]);
                    }
                    az = fmin(az, bound_dual_step(&C, V, nU, tau));
                }
            }
            if (!accepted) alpha *= 0.5;
        }
#ifdef ORACLE_DEBUG
        fprintf(stderr, "  resto it %3d mu %.2e err %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e th %.3e th_t %.3e phi %.6e ph_t %.6e gTd %.3e acc %d\n",
                rit, C.mu, err, dinf / s_d, pinf, c0 / s_c, delta, amax, alpha, th, th_t, phi, ph_t, gTd, accepted);
        {
            double sx = 0, sp_ = 0, su = 0, sl = 0, sz = 0, slam = 0;
            for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
                const int r = NA * k + i;
                sx += fabs(V->dX[r]); sl += fabs(V->lamp[r]); slam += fabs(V->lam[r]);
                if (i < 8) { sp_ += fabs(R->dpc[r]) + fabs(R->dnc[r]); sz += R->zp[r] + R->zn[r]; }
            }
            for (int j = 0; j < nU; ++j) su += fabs(V->dU[j]);
            fprintf(stderr, "   chk it %3d th %.12e phi %.12e gTd %.12e dx %.12e dpn %.12e du %.12e lamp %.12e lam %.12e zpn %.12e az %.12e\n",
                    rit, th, phi, gTd, sx, sp_, su, sl, slam, sz, az);
        }
#endif
        if (!accepted) { *status = ST_LS_FAIL; break; }     /* restoration failure */
        if (!ftype && nfilt < 256) { R->filt_th[nfilt] = (1 - gam_th) * th; R->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
        memcpy(V->X, V->Xt, sizeof(double) * nA);
        memcpy(V->U, V->Ut, sizeof(double) * nU);
        for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) cres[k][i] = ct[k][i];
        th = th_t;
        for (int i = 0; i < nA; ++i) V->lam[i] += alpha * (V->lamp[i] - V->lam[i]);
        for (int r = 0; r < nA; ++r) if ((r % NA) < 8) {
            R->pc[r] = R->pt_[r]; R->nc[r] = R->nt_[r];
            const double zp = R->zp[r] + az * R->dzp[r], zn = R->zn[r] + az * R->dzn[r];
            R->zp[r] = fmax(fmin(zp, 1e10 * C.mu / R->pc[r]), C.mu / (1e10 * R->pc[r]));
            R->zn[r] = fmax(fmin(zn, 1e10 * C.mu / R->nc[r]), C.mu / (1e10 * R->nc[r]));
        }
        for (int j = 0; j < nU; ++j) {
            double sl = V->U[j] - C.lo, su = C.hi - V->U[j];
            double zl = V->zL[j] + az * V->dzL[j], zu = V->zU[j] + az * V->dzU[j];
            V->zL[j] = fmax(fmin(zl, 1e10 * C.mu / sl), C.mu / (1e10 * sl));
            V->zU[j] = fmax(fmin(zu, 1e10 * C.mu / su), C.mu / (1e10 * su));
        }
        #undef RESTO_TRIAL
        #undef RESTO_STEP
    }
    if (ok_out) {
        /* back to the original problem: x from the restoration phase, u-bound multipliers by the
           pretended Newton step (mu - z s_trial)/s cut by the fraction to the boundary, reset to 1
           above 1000; equality multipliers 0 */
        const double mu0 = C0->mu;
        double az = 1.0, zmax = 0.0;
        for (int j = 0; j < nU; ++j) {
            const double sl = W->U[j] - C0->lo, su = C0->hi - W->U[j];
            const double slt = V->U[j] - C0->lo, sut = C0->hi - V->U[j];
            W->dzL[j] = (mu0 - W->zL[j] * slt) / sl;
            W->dzU[j] = (mu0 - W->zU[j] * sut) / su;
            if (W->dzL[j] < 0) az = fmin(az, -tau0 * W->zL[j] / W->dzL[j]);
            if (W->dzU[j] < 0) az = fmin(az, -tau0 * W->zU[j] / W->dzU[j]);
        }
        for (int j = 0; j < nU; ++j) {
            W->zL[j] += az * W->dzL[j]; W->zU[j] += az * W->dzU[j];
            zmax = fmax(zmax, fmax(W->zL[j], W->zU[j]));
        }
        if (zmax > 1e3) for (int j = 0; j < nU; ++j) { W->zL[j] = 1.0; W->zU[j] = 1.0; }
        memcpy(W->X, V->X, sizeof(double) * nA);
        memcpy(W->U, V->U, sizeof(double) * nU);
        memset(W->lam, 0, sizeof(double) * nA);
        for (int j = 0; j < nU; ++j) {      /* AcceptTrialPoint: kappa_sigma correction */
            const double sl = W->U[j] - C0->lo, su = C0->hi - W->U[j];
            W->zL[j] = fmax(fmin(W->zL[j], 1e10 * mu0 / sl), mu0 / (1e10 * sl));
            W->zU[j] = fmax(fmin(W->zU[j], 1e10 * mu0 / su), mu0 / (1e10 * su));
        }
        *it_io = rit - 1;
    } else {
        /* IPOPT copies the restoration phase's last iterate into the original problem's fields on failure */
        memcpy(W->X, V->X, sizeof(double) * nA);
        memcpy(W->U, V->U, sizeof(double) * nU);
        *it_io = rit;
    }
    free(g); free(gt); free(cres); free(ct); free(csg); free(rg); free(sv);
    free(V); free(R);
    return ok_out;
}

/* prm = [Q(8), Qt(8), R(4), u_lo, u_hi];  acc_tol / acc_iter: IPOPT acceptable_tol / acceptable_iter (0 = off) */
/* filter line-search acceptance of a trial (th_t, ph_t) for the step size alpha (IPOPT
   FilterLSAcceptor::CheckAcceptabilityOfTrialPoint with alpha_primal_test = alpha); *ftype is set
   when the Armijo (f-type) condition accepted it */
static int filter_accept(const work_t *W, int nfilt, double th_t, double ph_t, double th, double phi, double gTd,
                         double alpha, double th_max, double th_min, int *ftype) {
    const double gam_th = 1e-5, gam_ph = 1e-8, sw_delta = 1.0, s_th = 1.1, s_ph = 2.3, eta_ph = 1e-8;
    if (!(th_t < th_max) || !isfinite(ph_t)) return 0;
    for (int q = 0; q < nfilt; ++q) if (th_t >= W->filt_th[q] && ph_t >= W->filt_ph[q]) return 0;
    const int sw = gTd < 0 && alpha * pow(-gTd, s_ph) > sw_delta * pow(th, s_th);
    if (th <= th_min && sw) {
        if (LE(ph_t, phi + eta_ph * alpha * gTd, phi)) { *ftype = 1; return 1; }
        return 0;
    }
    return LE(th_t, (1 - gam_th) * th, th) || LE(ph_t - phi, -gam_ph * th, phi);
}

/* bound-multiplier directions of the primal step dU (the complementarity rows of the KKT system)
   and their fraction-to-the-boundary step */
static double bound_dual_step(const ctx_t *C, work_t *W, int nU, double tau) {
    double az = 1.0;
    for (int j = 0; j < nU; ++j) {
        double sl = W->U[j] - C->lo, su = C->hi - W->U[j], du = W->dU[j];
        W->dzL[j] = C->mu / sl - W->zL[j] - W->zL[j] / sl * du;
        W->dzU[j] = C->mu / su - W->zU[j] + W->zU[j] / su * du;
        if (W->dzL[j] < 0) az = fmin(az, -tau * W->zL[j] / W->dzL[j]);
        if (W->dzU[j] < 0) az = fmin(az, -tau * W->zU[j] / W->dzU[j]);
    }
    return az;
}

#ifdef ORACLE_RICCATI_PROBE
static void riccati_probe(const ctx_t *C, work_t *W);
#endif
int oracle_lmpc_solve(int N, double Ts, const double *state, const double *u_prev, const double *pvec,
                      const double *target, const double *prm, const double *w_init, int max_iter, double tol,
                      double acc_tol, int acc_iter, double *u0, double *fval, double *w_out, int32_t *iters_out) {
    if (N < 1 || N > NMAX || !(Ts > 0) || !(prm[21] > prm[20])) return ST_BAD_INPUT;
    work_t *W = (work_t *)calloc(1, sizeof(work_t));
    if (!W) return ST_BAD_INPUT;
    prob_t P;
    memset(&P, 0, sizeof P);
    P.N = N; P.Ts = Ts;
    memcpy(P.Q, prm, sizeof(double) * 8); memcpy(P.Qt, prm + 8, sizeof(double) * 8); memcpy(P.R, prm + 16, sizeof(double) * 4);
    P.ulo = prm[20]; P.uhi = prm[21];
    unpack_params(pvec, &P.M);
    const double lo = P.ulo - g_relax * fmax(1.0, fabs(P.ulo)), hi = P.uhi + g_relax * fmax(1.0, fabs(P.uhi));
    const double mu_min = tol / 10, kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, s_max = 100.0;
    const double gam_th = 1e-5, gam_ph = 1e-8, sw_delta = 1.0, s_th = 1.1, s_ph = 2.3, gam_al = 0.05, kap_soc = 0.99;
    const int nU = NU * N, nA = NA * (N + 1);
    ctx_t C;
    memset(&C, 0, sizeof C);
    C.P = &P; C.x0 = state; C.up0 = u_prev; C.tgt = target; C.mu = 0.1; C.lo = lo; C.hi = hi; C.R = NULL; C.mode = 0;
    /* initial point: w_init (the worker's warm start, zeros on the first solve :492) */
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < 8; ++i) W->X[NA * k + i] = w_init ? w_init[8 * k + i] : 0.0;
    for (int j = 0; j < nU; ++j) {
        double u = w_init ? w_init[8 * (N + 1) + j] : 0.0;
        double pl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo)), pu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
        if (u < lo + pl) u = lo + pl;
        if (u > hi - pu) u = hi - pu;
        W->U[j] = u; W->zL[j] = 1.0; W->zU[j] = 1.0;
    }
    W->X[8] = u_prev[0]; W->X[9] = u_prev[1];
    for (int k = 1; k <= N; ++k) { W->X[NA * k + 8] = W->U[NU * (k - 1)]; W->X[NA * k + 9] = W->U[NU * (k - 1) + 1]; }
    /* gradient-based scaling of the objective and of every constraint row at the start point */
    double gmax = 0.0;
    for (int k = 0; k <= N; ++k) {
        double z[NZ], g[NZ];
        for (int i = 0; i < NA; ++i) z[i] = W->X[NA * k + i];
        z[10] = k < N ? W->U[NU * k] : 0.0; z[11] = k < N ? W->U[NU * k + 1] : 0.0;
        cost_grad(&P, z, target, k == N, g);
        for (int j = 0; j < NZ; ++j) gmax = fmax(gmax, fabs(g[j]));
    }
    C.sc = gmax > 100.0 ? 100.0 / gmax : 1.0;
    linearise(&P, W);
    for (int i = 0; i < NA; ++i) W->dsc[i] = 1.0;
    for (int k = 0; k < N; ++k) for (int i = 0; i < NA; ++i) {
        double m = 1.0;   /* d/dx_{k+1} */
        for (int j = 0; j < NA; ++j) m = fmax(m, fabs(W->A[k][i][j]));
        m = fmax(m, fmax(fabs(W->Bm[k][i][0]), fabs(W->Bm[k][i][1])));
        W->dsc[NA * (k + 1) + i] = m > 100.0 ? 100.0 / m : 1.0;
    }

    if (g_mult_init_max > 0.0) {
        const double ym = ls_multipliers(&C, W);
#ifdef ORACLE_DEBUG
        fprintf(stderr, "least-square multipliers: max |y| %.6e (constr_mult_init_max %.0f)\n", ym, g_mult_init_max);
#endif
        if (!(ym <= g_mult_init_max)) memset(W->lam, 0, sizeof(double) * nA);
        linearise(&P, W);      /* the Lagrangian Hessian of iteration 0 with these multipliers */
    }
    double (*g)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*gt)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*csg)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double th = residuals(&C, W, W->X, W->U, g);
    const double th_max = 1e4 * fmax(1.0, th), th_min = 1e-4 * fmax(1.0, th);
    int nfilt = 0, status = ST_MAXITER, it, acc_count = 0, in_soft = 0, soft_count = 0;
    double delta_last = 0.0;
    for (it = 0;; ++it) {
        if (it > 0) linearise(&P, W);
        /* optimality error (IPOPT eq. 5) with scaled rows: y~ = lam / d */
        double sum_l, sum_z, dinf, pinf, pinf_u, c0;
        kkt_errors(&C, W, g, &sum_l, &sum_z, &dinf, &pinf, &pinf_u, &c0, NULL);
        const int nb = 2 * nU;
        const double s_d = fmax(s_max, (sum_l + sum_z) / (nA + nb)) / s_max;
        const double s_c = fmax(s_max, sum_z / nb) / s_max;
        const double err = fmax(dinf / s_d, fmax(pinf, c0 / s_c));
        /* IPOPT OptimalityErrorConvergenceCheck: optimal, then acceptable, then the iteration cap */
        if (err <= tol && dinf / C.sc <= 1.0 && pinf_u <= 1e-4 && c0 / C.sc <= 1e-4) { status = ST_SOLVED; break; }
        if (acc_iter > 0 && err <= acc_tol && pinf_u <= 1e-2 && c0 / C.sc <= 1e-2) {
            if (++acc_count >= acc_iter) { status = ST_ACCEPTABLE; break; }
        } else {
            acc_count = 0;
        }
        if (it >= max_iter) { status = ST_MAXITER; break; }
        for (;;) {
            double cmu = 0;
            for (int j = 0; j < nU; ++j)
                cmu = fmax(cmu, fmax(fabs(W->zL[j] * (W->U[j] - lo) - C.mu), fabs(W->zU[j] * (hi - W->U[j]) - C.mu)));
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > kappa_eps * C.mu || C.mu <= mu_min) break;
            C.mu = fmax(mu_min, fmin(kappa_mu * C.mu, pow(C.mu, theta_mu)));
            nfilt = 0; in_soft = 0;      /* BacktrackingLineSearch::Reset: the filter and the soft phase */
        }
        const double tau = fmax(0.99, 1.0 - C.mu);
#ifdef ORACLE_RICCATI_PROBE
        if (it == 0) riccati_probe(&C, W);      /* diagnostic build (tools/lmpc_riccati_probe.c) */
#endif
        double delta = 0.0;
        int ok = riccati_factor(&C, W, 0.0);
        for (int attempt = 0; !ok && attempt < 60; ++attempt) {
            delta = (attempt == 0) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))   /* perturb_dec_fact 1/3 */
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            ok = riccati_factor(&C, W, delta);
        }
        if (!ok) { status = ST_INERTIA_FAIL; break; }
        if (delta > 0) delta_last = delta;
        riccati_solve(&C, W, g);
        double az = bound_dual_step(&C, W, nU, tau);
        double amax = frac_to_boundary(&C, W, W->dU, tau);
        const double phi = barrier_obj(&C, W->X, W->U);
        double gTd = 0.0;
        for (int k = 0; k <= N; ++k) {
            double z[NZ], gc[NZ];
            for (int i = 0; i < NA; ++i) z[i] = W->X[NA * k + i];
            z[10] = k < N ? W->U[NU * k] : 0.0; z[11] = k < N ? W->U[NU * k + 1] : 0.0;
            cost_grad(&P, z, target, k == N, gc);
            for (int i = 0; i < NA; ++i) gTd += C.sc * gc[i] * W->dX[NA * k + i];
            if (k < N)
                for (int a = 0; a < NU; ++a) {
                    const int j = NU * k + a;
                    gTd += (C.sc * gc[10 + a] - C.mu / (W->U[j] - lo) + C.mu / (hi - W->U[j])) * W->dU[j];
                }
        }
        double amin = gam_th;
        if (gTd < 0) amin = fmin(gam_th, fmin(gam_ph * th / (-gTd), sw_delta * pow(th, s_th) / pow(-gTd, s_ph)));
        if (th == 0.0 && gTd < 0) amin = 0.0;
        amin *= gam_al;
        double alpha = amax, th_t = 0, ph_t = 0;
        int accepted = 0, ftype = 0;
        double tn = 0.0;
        for (int i = 0; i < nA; ++i) tn = fmax(tn, fabs(W->dX[i]) / (1.0 + fabs(W->X[i])));
        for (int j = 0; j < nU; ++j) tn = fmax(tn, fabs(W->dU[j]) / (1.0 + fabs(W->U[j])));
        const int tiny = tn < 10.0 * 2.220446049250313e-16;
        for (int ls = 0; ls < 80 && !accepted && !in_soft; ++ls) {
            if (alpha < amin && ls > 0) break;
            for (int i = 0; i < nA; ++i) W->Xt[i] = W->X[i] + alpha * W->dX[i];
            for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + alpha * W->dU[j];
            th_t = residuals(&C, W, W->Xt, W->Ut, gt);
            ph_t = barrier_obj(&C, W->Xt, W->Ut);
            if (tiny) { accepted = 1; ftype = 1; break; }
            accepted = filter_accept(W, nfilt, th_t, ph_t, th, phi, gTd, alpha, th_max, th_min, &ftype);
            if (!accepted && ls == 0 && !(th_t < th) && g_max_soc > 0) {
                /* IPOPT FilterLSAcceptor::TrySecondOrderCorrection: c_soc <- a_soc c_soc + c(trial),
                   starting from c(x) with a_soc = alpha; the corrected step re-uses the factorisation;
                   at most max_soc passes, continued while theta(trial) <= kappa_soc theta(previous) */
                double *sv = (double *)malloc(sizeof(double) * (2 * nA + nU));
                memcpy(sv, W->dX, sizeof(double) * nA); memcpy(sv + nA, W->lamp, sizeof(double) * nA);
                memcpy(sv + 2 * nA, W->dU, sizeof(double) * nU);
                double asoc = alpha, th_old = 0.0;
                for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) csg[k][i] = g[k][i];
                for (int c = 0; c < g_max_soc; ++c) {
                    if (c > 0 && !(th_t <= kap_soc * th_old)) break;
                    th_old = th_t;
                    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) csg[k][i] = asoc * csg[k][i] + gt[k][i];
                    riccati_solve(&C, W, csg);
                    asoc = frac_to_boundary(&C, W, W->dU, tau);
                    for (int i = 0; i < nA; ++i) W->Xt[i] = W->X[i] + asoc * W->dX[i];
                    for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + asoc * W->dU[j];
                    th_t = residuals(&C, W, W->Xt, W->Ut, gt);
                    ph_t = barrier_obj(&C, W->Xt, W->Ut);
                    if (filter_accept(W, nfilt, th_t, ph_t, th, phi, gTd, alpha, th_max, th_min, &ftype)) {
                        /* IPOPT takes the SOC solve as the whole step: its bound-multiplier
                           directions and their fraction to the boundary follow the corrected dU */
                        accepted = 1; alpha = asoc; az = bound_dual_step(&C, W, nU, tau);
                        break;
                    }
                }
                if (!accepted) {    /* back to the plain direction */
                    memcpy(W->dX, sv, sizeof(double) * nA); memcpy(W->lamp, sv + nA, sizeof(double) * nA);
                    memcpy(W->dU, sv + 2 * nA, sizeof(double) * nU);
                }
                free(sv);
            }
            if (!accepted) alpha *= 0.5;
        }
        int soft = 0;
        if (!accepted && g_soft_resto) {
            /* the line search failed (or the soft restoration phase is on): IPOPT's soft restoration
               phase, at most max_soft_resto_iters = 10 steps; on entry PrepareRestoPhaseStart puts the
               current point into the filter */
            if (!in_soft) {
                if (nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
                soft_count = 0;
            }
            if (!(in_soft && ++soft_count > 10)) {
                double sl_, sz_, di_, pi_, pu_, c0_, pd;
                kkt_errors(&C, W, g, &sl_, &sz_, &di_, &pi_, &pu_, &c0_, &pd);
                int orig = 0;
                const double a = soft_resto_step(&C, W, nfilt, th, phi, th_max, tau, pd, gt, &th_t, &ph_t, &orig);
                if (a > 0.0) {
                    accepted = 1; soft = 1; alpha = a; az = a;
                    in_soft = !orig;
                    if (orig) soft_count = 0;
                }
            }
        }
#ifdef ORACLE_DEBUG
        fprintf(stderr, "it %3d soft %d mu %.2e err %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e th %.3e th_t %.3e phi %.6e ph_t %.6e gTd %.3e acc %d\n",
                it, in_soft, C.mu, err, dinf / s_d, pinf, c0 / s_c, delta, amax, alpha, th, th_t, phi, ph_t, gTd, accepted);
#endif
        if (!accepted && g_resto) {
            /* IPOPT's restoration phase (the start point entered the filter with the soft phase above,
               or enters it here when that phase is off) */
            if (!g_soft_resto && nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
            int rst = ST_LS_FAIL;
            if (!restoration(&C, W, &it, max_iter, tol, acc_tol, acc_iter, th, phi, nfilt, tau, g, &rst)) {
                status = rst;
                break;
            }
            th = residuals(&C, W, W->X, W->U, g);
            in_soft = 0; soft_count = 0;
            continue;
        }
        if (!accepted) { status = ST_LS_FAIL; break; }
        if (!soft && !ftype && nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
        memcpy(W->X, W->Xt, sizeof(double) * nA);
        memcpy(W->U, W->Ut, sizeof(double) * nU);
        memcpy(g, gt, sizeof(double) * NA * (N + 1));
        th = th_t;
        for (int i = 0; i < nA; ++i) W->lam[i] += alpha * (W->lamp[i] - W->lam[i]);
        for (int j = 0; j < nU; ++j) {
            double sl = W->U[j] - lo, su = hi - W->U[j];
            double zl = W->zL[j] + az * W->dzL[j], zu = W->zU[j] + az * W->dzU[j];
            W->zL[j] = fmax(fmin(zl, 1e10 * C.mu / sl), C.mu / (1e10 * sl));
            W->zU[j] = fmax(fmin(zu, 1e10 * C.mu / su), C.mu / (1e10 * su));
        }
    }
    if (iters_out) *iters_out = it;
    if (u0) { u0[0] = W->U[0]; u0[1] = W->U[1]; }
    if (fval) *fval = objective(&P, W->X, W->U, target);
    if (w_out) {
        for (int k = 0; k <= N; ++k) for (int i = 0; i < 8; ++i) w_out[8 * k + i] = W->X[NA * k + i];
        memcpy(w_out + 8 * (N + 1), W->U, sizeof(double) * nU);
    }
    free(g); free(gt); free(csg);
    free(W);
    return status;
}

/* batched driver: state rows of 8, u_prev rows of 2, pvec rows of 34, target rows of 8, prm rows of 22,
 * w rows of 8(N+1)+2N */
int oracle_lmpc_solve_batch(int B, int N, double Ts, const double *state, const double *u_prev, const double *pvec,
                            const double *target, const double *prm, const double *w_init, int max_iter, double tol,
                            double acc_tol, int acc_iter, int nthreads, double *u0, double *f, double *w_out,
                            int32_t *status, int32_t *iters) {
    const int nw = 8 * (N + 1) + 2 * N;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int b = 0; b < B; ++b) {
        int32_t itb = 0;
        status[b] = oracle_lmpc_solve(N, Ts, state + 8 * b, u_prev + 2 * b, pvec + NPV * b, target + 8 * b, prm + 22 * b,
                                      w_init ? w_init + (size_t)nw * b : NULL, max_iter, tol, acc_tol, acc_iter,
                                      u0 + 2 * b, f + b, w_out ? w_out + (size_t)nw * b : NULL, &itb);
        iters[b] = itb;
    }
    (void)nthreads;
    return 0;
}

/* one RK4 step (:431-436) for B states: the dynamics KAT hook */
void oracle_lmpc_rk4(int B, double Ts, const double *x, const double *u, const double *pvec, double *xn) {
    for (int b = 0; b < B; ++b) {
        prob_t P;
        memset(&P, 0, sizeof P);
        P.Ts = Ts;
        unpack_params(pvec + NPV * b, &P.M);
        rk4_val(&P, x + 8 * b, u + 2 * b, xn + 8 * b);
    }
}
