/*
 * rmpc_ipm.c -- CPU oracle for the RMPC regressor NMPC solve (+ RLS update).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker / timed CPU baseline.  Never
 * linked into the shipped solver.
 *
 * Restates (RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py):
 *   RLS.update :10-30; _phi/_dyn_regressor/_rk4 :171-193; NLP :35-168
 *   (defects :109-112, du rows :114-121, velocity caps :123-127, cost :129-140,
 *   U box :146-154); solve with warm start :212-222; IPOPT options
 *   print_level 0, sb yes, max_iter 200 (:158-162), everything else default.
 * IPOPT's algorithm as in pmpc_ipm.c (monotone mu, least-square starting
 * multipliers, filter line search with second-order correction, inertia
 * correction, bound_relax 1e-8, gradient scaling), with IPOPT's slack
 * formulation for the inequality rows
 * g(w) - s = 0, g_L <= s <= g_U.  The KKT system is solved by a Riccati
 * recursion on the augmented state [x_k; u_{k-1}] (the Delta-u rows couple
 * consecutive controls); slacks and their multipliers are eliminated per stage.
 * A failed filter line search goes through IPOPT's soft restoration phase and then
 * its restoration phase (MinC_1NrmRestorationPhase, as restated in lmpc_ipm.c, with
 * the inequality rows' p / n in series with their slacks, and iterative refinement of
 * the restoration step): status 2 (Infeasible_Problem_Detected) when the restoration
 * problem converges, e.g. for a measured |v| above vmax at the pinned node 0.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* IPOPT Compare_le: lhs <= rhs up to 10 machine epsilons of |base| */
#define LE(l, r, b) ((l) - (r) <= 10.0 * 2.220446049250313e-16 * fabs(b))
#ifdef ORACLE_DEBUG
#include <stdio.h>
#endif

#define NXS 4           /* physical states px vx py vy */
#define NA 6            /* augmented state [x; u_prev] */
#define NU 2
#define NZ 8            /* jet variables [x(4) up(2) u(2)] (up unused by the dynamics) */
#define NH 36
#define NMAX 64
#define NIQ 6           /* inequality rows per stage: du_x du_y, vx-vmax, -vx-vmax, vy-vmax, -vy-vmax */

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
static inline jet jscale(jet a, double s) { return jaxpy(jconst(0.0), s, a); }
static inline jet jsin(jet a) {
    double s = sin(a.v), c = cos(a.v); jet r; r.v = s;
    for (int i = 0; i < NZ; ++i) r.d[i] = c * a.d[i];
    for (int i = 0; i < NZ; ++i) for (int j = 0; j <= i; ++j) r.h[hx(i, j)] = c * a.h[hx(i, j)] - s * a.d[i] * a.d[j];
    return r;
}
static inline jet jtanh(jet a) {
    double t = tanh(a.v), d1 = 1.0 - t * t, d2 = -2.0 * t * d1; jet r; r.v = t;
    for (int i = 0; i < NZ; ++i) r.d[i] = d1 * a.d[i];
    for (int i = 0; i < NZ; ++i) for (int j = 0; j <= i; ++j) r.h[hx(i, j)] = d1 * a.h[hx(i, j)] + d2 * a.d[i] * a.d[j];
    return r;
}

typedef struct {
    int N; double Ts, gz, Qp, Qv, Ru, Rdu, ulo, uhi, dulo, duhi, vmax, veps;
    double th[14];
} prob_t;

/* R4 on jets: xdot = [vx, gz sin(a) + phi.thx, vy, gz sin(b) + phi.thy] (:178-186) */
static void dyn_jet(const prob_t *P, const jet *x, const jet *u, jet *xd) {
    jet ph[7];
    ph[0] = x[0]; ph[1] = x[1]; ph[2] = x[2]; ph[3] = x[3];
    ph[4] = jtanh(jscale(x[1], 1.0 / P->veps)); ph[5] = jtanh(jscale(x[3], 1.0 / P->veps)); ph[6] = jconst(1.0);
    jet ax = jscale(jsin(u[0]), P->gz), ay = jscale(jsin(u[1]), P->gz);
    for (int i = 0; i < 7; ++i) { ax = jaxpy(ax, P->th[i], ph[i]); ay = jaxpy(ay, P->th[7 + i], ph[i]); }
    xd[0] = x[1]; xd[1] = ax; xd[2] = x[3]; xd[3] = ay;
}
static void dyn_val(const prob_t *P, const double *x, const double *u, double *xd) {
    double ph[7] = {x[0], x[1], x[2], x[3], tanh(x[1] / P->veps), tanh(x[3] / P->veps), 1.0};
    double ax = P->gz * sin(u[0]), ay = P->gz * sin(u[1]);
    for (int i = 0; i < 7; ++i) { ax += ph[i] * P->th[i]; ay += ph[i] * P->th[7 + i]; }
    xd[0] = x[1]; xd[1] = ax; xd[2] = x[3]; xd[3] = ay;
}
/* R4 RK4 (:188-193) */
static void rk4_val(const prob_t *P, const double *x, const double *u, double *xn) {
    double k1[4], k2[4], k3[4], k4[4], y[4], h = P->Ts;
    dyn_val(P, x, u, k1);
    for (int i = 0; i < 4; ++i) y[i] = x[i] + h / 2 * k1[i];
    dyn_val(P, y, u, k2);
    for (int i = 0; i < 4; ++i) y[i] = x[i] + h / 2 * k2[i];
    dyn_val(P, y, u, k3);
    for (int i = 0; i < 4; ++i) y[i] = x[i] + h * k3[i];
    dyn_val(P, y, u, k4);
    for (int i = 0; i < 4; ++i) xn[i] = x[i] + h / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
}
/* RK4 on jets over z = [x(4), up(2), u(2)]: value, Jacobian rows and -lam-contracted Hessian */
static void rk4_derivs(const prob_t *P, const double *x, const double *u, const double *nlam,
                       double *xn, double J[4][NZ], double H[NZ][NZ]) {
    jet xj[4], uj[2], k1[4], k2[4], k3[4], k4[4], y[4];
    double h = P->Ts;
    for (int i = 0; i < 4; ++i) xj[i] = jvar(x[i], i);
    for (int i = 0; i < 2; ++i) uj[i] = jvar(u[i], NA + i);
    dyn_jet(P, xj, uj, k1);
    for (int i = 0; i < 4; ++i) y[i] = jaxpy(xj[i], h / 2, k1[i]);
    dyn_jet(P, y, uj, k2);
    for (int i = 0; i < 4; ++i) y[i] = jaxpy(xj[i], h / 2, k2[i]);
    dyn_jet(P, y, uj, k3);
    for (int i = 0; i < 4; ++i) y[i] = jaxpy(xj[i], h, k3[i]);
    dyn_jet(P, y, uj, k4);
    for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) H[a][b] = 0.0;
    for (int i = 0; i < 4; ++i) {
        jet s = jaxpy(jaxpy(jaxpy(k1[i], 2.0, k2[i]), 2.0, k3[i]), 1.0, k4[i]);
        jet r = jaxpy(xj[i], h / 6, s);
        xn[i] = r.v;
        for (int j = 0; j < NZ; ++j) J[i][j] = r.d[j];
        for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) H[a][b] += nlam[i] * r.h[hx(a, b)];
    }
}

/* inequality row i at a stage: value C z with z = [x(4), up(2), u(2)] */
static double iq_val(const prob_t *P, int i, const double *z) {
    switch (i) {
        case 0: return z[6] - z[4];
        case 1: return z[7] - z[5];
        case 2: return z[1] - P->vmax;
        case 3: return -z[1] - P->vmax;
        case 4: return z[3] - P->vmax;
        default: return -z[3] - P->vmax;
    }
}
static void iq_row(int i, double *c) {
    for (int j = 0; j < NZ; ++j) c[j] = 0.0;
    switch (i) {
        case 0: c[6] = 1; c[4] = -1; break;
        case 1: c[7] = 1; c[5] = -1; break;
        case 2: c[1] = 1; break;
        case 3: c[1] = -1; break;
        case 4: c[3] = 1; break;
        default: c[3] = -1; break;
    }
}

typedef struct {
    double X[NA * (NMAX + 1)], U[NU * NMAX];            /* augmented states, controls */
    double lam[NA * (NMAX + 1)];                        /* defect multipliers (incl. x_0 = [x0; u_prev]) */
    double zL[NU * NMAX], zU[NU * NMAX];                /* U box multipliers */
    double S[NMAX][NIQ], y[NMAX][NIQ], vL[NMAX][NIQ], vU[NMAX][NIQ];   /* slacks + multipliers */
    double A[NMAX][NA][NA], Bm[NMAX][NA][NU], Hs[NMAX][NZ][NZ], c[NMAX][NA];
    double Lq[NMAX][3], Qux[NMAX][NU][NA], K[NMAX][NU][NA], Pm[NMAX + 1][NA][NA];
    double kff[NMAX][NU], pv[NMAX + 1][NA], grad[NMAX + 1][NZ];
    double dX[NA * (NMAX + 1)], dU[NU * NMAX], lamp[NA * (NMAX + 1)], dzL[NU * NMAX], dzU[NU * NMAX];
    double dS[NMAX][NIQ], dy[NMAX][NIQ], dvL[NMAX][NIQ], dvU[NMAX][NIQ];
    double Xt[NA * (NMAX + 1)], Ut[NU * NMAX], St[NMAX][NIQ];
    double filt_th[256], filt_ph[256];
} work_t;

struct resto_s;
typedef struct {
    const prob_t *P; const double *x0, *up0, *R; double sc, mu, lo, hi;
    double sL[NIQ], sU[NIQ];                            /* relaxed slack bounds (+-inf as +-1e300) */
    struct resto_s *Rs;     /* restoration phase data (NULL: the original problem) */
    int mode;               /* 0 original problem, 1 restoration Newton step, 2 restoration least-square multipliers */
    double ds_shift;        /* inertia shift of the slack block in the original problem's step (slack_shift) */
} ctx_t;

/* IPOPT ApplicationReturnStatus values (Infeasible_Problem_Detected = 2: the restoration problem converged to a
   point of local infeasibility; Restoration_Failed = -2: the restoration itself failed, or, with the phases
   off, the filter line search) */
enum { ST_SOLVED = 0, ST_INFEASIBLE = 2, ST_MAXITER = -1, ST_LS_FAIL = -2, ST_INERTIA_FAIL = -3, ST_BAD_INPUT = -10 };

/* IPOPT's restoration phase for this NLP (MinC_1NrmRestorationPhase, RestoIpoptNLP; restated as in
 * lmpc_ipm.c, which has the full commentary):
 *   min rho sum(p + n) + eta/2 ||D_R (x - x_R)||^2
 *   s.t. c(x) + n_c - p_c = 0 (the physical defect rows, x_0 pinning included),
 *        d(x) - s + n_d - p_d = 0 with the slack bounds kept (the Delta-u and velocity-cap rows),
 *        p, n >= 0, the U box,
 * over the reference NLP's variables x = [X; U] (the u_{k-1} copy rows of the augmented state are not
 * rows of the reference NLP and stay hard; the row scaling is 1 here: no constraint gradient exceeds 100).
 * In the Newton system the defect rows become soft rows J dx - D dlam = rhs with D = 1/S_p + 1/S_n,
 * absorbed by the Riccati recursion as in lmpc_ipm.c; an inequality row keeps its stage-local
 * elimination with the slack, p and n in series: y + dy = sig (C dz + r) + off with
 * 1/sig = 1/S_s + 1/S_p + 1/S_n (the S_* are the primal-dual barrier Hessians plus the inertia shift). */
typedef struct resto_s {
    double pc[NA * (NMAX + 1)], nc[NA * (NMAX + 1)], zp[NA * (NMAX + 1)], zn[NA * (NMAX + 1)];
    double dpc[NA * (NMAX + 1)], dnc[NA * (NMAX + 1)], dzp[NA * (NMAX + 1)], dzn[NA * (NMAX + 1)];
    double rp[NA * (NMAX + 1)], rn[NA * (NMAX + 1)];
    double D[NA * (NMAX + 1)], Spd[NA * (NMAX + 1)], Snd[NA * (NMAX + 1)];
    double pt_[NA * (NMAX + 1)], nt_[NA * (NMAX + 1)];
    double qp[NMAX][NIQ], qn[NMAX][NIQ], zqp[NMAX][NIQ], zqn[NMAX][NIQ];         /* p, n of the inequality rows */
    double dqp[NMAX][NIQ], dqn[NMAX][NIQ], dzqp[NMAX][NIQ], dzqn[NMAX][NIQ];
    double rqp[NMAX][NIQ], rqn[NMAX][NIQ], qpt[NMAX][NIQ], qnt[NMAX][NIQ];
    double Ssd[NMAX][NIQ], Sqp[NMAX][NIQ], Sqn[NMAX][NIQ], sig[NMAX][NIQ], off[NMAX][NIQ], psi[NMAX][NIQ];
    double XR[NA * (NMAX + 1)], UR[NU * NMAX], DRx[NA * (NMAX + 1)], DRu[NU * NMAX];
    double M[NMAX + 1][NA][NA], Pt[NMAX + 1][NA][NA];
    double filt_th[256], filt_ph[256];
    double rho, eta, delta;
    /* iterative refinement: residuals of the full Newton system, gradient override of the correction solve */
    int ovr;
    double gov[NMAX + 1][NZ];
    double ex[NMAX + 1][NZ], ec[NMAX + 1][NA], eq[NMAX][NIQ], ep[NA * (NMAX + 1)], en[NA * (NMAX + 1)];
    double eqp[NMAX][NIQ], eqn[NMAX][NIQ], es[NMAX][NIQ];
} resto_t;

/* A X = B by Gaussian elimination with partial pivoting (n x n, nrhs columns); A and B are overwritten */
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
/* x <- M_k^-1 x, x <- M_k^-T x */
static void soft_apply(const resto_t *R, int k, int trans, double *x) {
    double A[NA][NA], Bv[NA][NA];
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) A[i][j] = trans ? R->M[k][j][i] : R->M[k][i][j];
    for (int i = 0; i < NA; ++i) Bv[i][0] = x[i];
    gauss_solve(NA, A, Bv, 1);
    for (int i = 0; i < NA; ++i) x[i] = Bv[i][0];
}
/* soft defect rows of node k (shift delta): D, M = I + D P_k, P~_k = M^-T P_k; 0 when S = P_k(phys, phys) + D^-1
   is not positive definite (wrong inertia, lmpc_ipm.c soft_node) */
static int soft_node(const ctx_t *C, const double Pk[NA][NA], int k, double delta) {
    resto_t *R = C->Rs;
    for (int i = 0; i < NA; ++i) {
        const int r = NA * k + i;
        double D = 0.0;
        if (i < NXS) {
            if (C->mode == 2) { R->Spd[r] = 1.0; R->Snd[r] = 1.0; }
            else { R->Spd[r] = R->zp[r] / R->pc[r] + delta; R->Snd[r] = R->zn[r] / R->nc[r] + delta; }
            D = 1.0 / R->Spd[r] + 1.0 / R->Snd[r];
        }
        R->D[r] = D;
        for (int j = 0; j < NA; ++j) R->M[k][i][j] = (i == j) + D * Pk[i][j];
    }
    double A[NA][NA], Bm[NA][NA];
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) { A[i][j] = R->M[k][j][i]; Bm[i][j] = Pk[i][j]; }
    gauss_solve(NA, A, Bm, NA);
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) R->Pt[k][i][j] = 0.5 * (Bm[i][j] + Bm[j][i]);
    double L[NXS][NXS];
    for (int i = 0; i < NXS; ++i) for (int j = 0; j <= i; ++j) {
        double t = Pk[i][j] + (i == j ? 1.0 / R->D[NA * k + i] : 0.0);
        for (int m = 0; m < j; ++m) t -= L[i][m] * L[j][m];
        if (i == j) { if (!(t > 0.0)) return 0; L[i][i] = sqrt(t); }
        else L[i][j] = t / L[j][j];
    }
    return 1;
}

/* IPOPT bound_relax_factor (1e-8 default); the golden generator sets 0 to solve the exact NLP */
static double g_relax = 1e-8;
void oracle_rmpc_set_relax(double r) { g_relax = r; }
/* second-order correction on/off (IPOPT default on; off mirrors the GPU kernel's line search) */
static int g_max_soc = 4;      /* IPOPT max_soc (second-order corrections per line search; the restoration
                                  phase's line search reads the same option) */
void oracle_rmpc_set_soc(int max_soc) { g_max_soc = max_soc < 0 ? 0 : max_soc; }
/* IPOPT shifts the slack block of its KKT system by the same inertia perturbation as the x block
   (delta_s = delta_x, PDPerturbationHandler).  Off by default here and in the kernel: the original problem's
   inertia correction never engages on the RMPC workloads (C3 and its 2x / 3x / 6x velocity spreads), and
   tests/test_oracle_rmpc.py checks that turning the shift on leaves every solve bit-identical.  The
   restoration phase always shifts its slack, p and n blocks (resto_iq_terms). */
static int g_slack_shift = 0;
void oracle_rmpc_set_slack_shift(int on) { g_slack_shift = on; }

static void stage_z(const double *X, const double *U, int k, double *z) {
    for (int i = 0; i < NA; ++i) z[i] = X[NA * k + i];
    z[6] = U[NU * k]; z[7] = U[NU * k + 1];
}

/* objective (:129-140) and its gradient per stage over z (terminal: x only) */
static double objective(const prob_t *P, const double *X, const double *U, const double *R) {
    double f = 0.0;
    for (int k = 0; k <= P->N; ++k) {
        const double *x = X + NA * k, *r = R + 4 * k;
        f += P->Qp * ((x[0] - r[0]) * (x[0] - r[0]) + (x[2] - r[2]) * (x[2] - r[2]))
           + P->Qv * ((x[1] - r[1]) * (x[1] - r[1]) + (x[3] - r[3]) * (x[3] - r[3]));
        if (k < P->N) {
            const double *u = U + NU * k;
            double d0 = u[0] - x[4], d1 = u[1] - x[5];
            f += P->Ru * (u[0] * u[0] + u[1] * u[1]) + P->Rdu * (d0 * d0 + d1 * d1);
        }
    }
    return f;
}
static void cost_grad(const prob_t *P, const double *z, const double *r, int terminal, double *g) {
    for (int j = 0; j < NZ; ++j) g[j] = 0.0;
    g[0] = 2 * P->Qp * (z[0] - r[0]); g[1] = 2 * P->Qv * (z[1] - r[1]);
    g[2] = 2 * P->Qp * (z[2] - r[2]); g[3] = 2 * P->Qv * (z[3] - r[3]);
    if (!terminal) {
        double d0 = z[6] - z[4], d1 = z[7] - z[5];
        g[6] = 2 * P->Ru * z[6] + 2 * P->Rdu * d0; g[7] = 2 * P->Ru * z[7] + 2 * P->Rdu * d1;
        g[4] = -2 * P->Rdu * d0; g[5] = -2 * P->Rdu * d1;
    }
}

/* constraint residuals: augmented defects (N+1 blocks of 6) and inequality residuals C z - s; returns l1 norm */
static double residuals(const ctx_t *C, const double *X, const double *U, double S[][NIQ],
                        double g[][NA], double r[][NIQ]) {
    const prob_t *P = C->P; double th = 0.0;
    for (int i = 0; i < 4; ++i) g[0][i] = X[i] - C->x0[i];
    g[0][4] = X[4] - C->up0[0]; g[0][5] = X[5] - C->up0[1];
    for (int i = 0; i < NA; ++i) th += fabs(g[0][i]);
    for (int k = 0; k < P->N; ++k) {
        double xn[4], z[NZ];
        rk4_val(P, X + NA * k, U + NU * k, xn);
        for (int i = 0; i < 4; ++i) g[k + 1][i] = X[NA * (k + 1) + i] - xn[i];
        g[k + 1][4] = X[NA * (k + 1) + 4] - U[NU * k]; g[k + 1][5] = X[NA * (k + 1) + 5] - U[NU * k + 1];
        for (int i = 0; i < NA; ++i) th += fabs(g[k + 1][i]);
        stage_z(X, U, k, z);
        for (int i = 0; i < NIQ; ++i) { r[k][i] = iq_val(P, i, z) - S[k][i]; th += fabs(r[k][i]); }
    }
    return th;
}

static double barrier_obj(const ctx_t *C, const double *X, const double *U, double S[][NIQ]) {
    const prob_t *P = C->P;
    double phi = C->sc * objective(P, X, U, C->R);
    for (int j = 0; j < NU * P->N; ++j) {
        double sl = U[j] - C->lo, su = C->hi - U[j];
        if (!(sl > 0) || !(su > 0)) return INFINITY;
        phi -= C->mu * (log(sl) + log(su));
    }
    for (int k = 0; k < P->N; ++k) for (int i = 0; i < NIQ; ++i) {
        double s = S[k][i];
        if (C->sL[i] > -1e299) { if (!(s - C->sL[i] > 0)) return INFINITY; phi -= C->mu * log(s - C->sL[i]); }
        if (C->sU[i] < 1e299) { if (!(C->sU[i] - s > 0)) return INFINITY; phi -= C->mu * log(C->sU[i] - s); }
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

/* slack barrier Sigma and psi for stage k row i (one-sided rows have no lower part) */
static void slack_terms(const ctx_t *C, const work_t *W, int k, int i, double *sig, double *psi) {
    double s = W->S[k][i], sg = 0.0, ps = 0.0;
    if (C->sL[i] > -1e299) { double d = s - C->sL[i]; sg += W->vL[k][i] / d; ps -= C->mu / d; }
    if (C->sU[i] < 1e299) { double d = C->sU[i] - s; sg += W->vU[k][i] / d; ps += C->mu / d; }
    *sig = sg; *psi = ps;
}

/* restoration: inequality row i of stage k with its slack, p and n eliminated (shift delta):
   y + dy = sig (C dz + r) + off.  Mode 2 (least-square multipliers): unit weights, the slack's
   gradient -v_L + v_U, p / n gradients rho - z, y = 0. */
static void resto_iq_terms(const ctx_t *C, const work_t *W, int k, double delta) {
    resto_t *R = C->Rs;
    for (int i = 0; i < NIQ; ++i) {
        double Ss, ps, Sp, Sn, rp, rn, yv;
        if (C->mode == 2) {
            Ss = Sp = Sn = 1.0; ps = -W->vL[k][i] + W->vU[k][i];
            rp = R->rho - R->zqp[k][i]; rn = R->rho - R->zqn[k][i]; yv = 0.0;
        } else {
            slack_terms(C, W, k, i, &Ss, &ps);
            Ss += delta;
            Sp = R->zqp[k][i] / R->qp[k][i] + delta; Sn = R->zqn[k][i] / R->qn[k][i] + delta;
            rp = R->rqp[k][i]; rn = R->rqn[k][i]; yv = W->y[k][i];
        }
        const double sg = 1.0 / (1.0 / Ss + 1.0 / Sp + 1.0 / Sn);
        R->Ssd[k][i] = Ss; R->Sqp[k][i] = Sp; R->Sqn[k][i] = Sn; R->sig[k][i] = sg; R->psi[k][i] = ps;
        R->off[k][i] = sg * (ps / Ss + yv * (1.0 / Sp + 1.0 / Sn) - rn / Sn + rp / Sp);
    }
}

/* Stage Hessian (8x8 over z) incl. slack elimination C^T Sigma C and box Sigma; gradient incl. C^T(Sigma r + psi) */
static void stage_qp(const ctx_t *C, const work_t *W, int k, double rr[NIQ], double delta, double Hq[NZ][NZ], double *gq) {
    const prob_t *P = C->P; const double sc = C->sc;
    double z[NZ];
    stage_z(W->X, W->U, k, z);
    if (C->mode) {
        /* restoration: proximity term on the reference NLP's variables (states, inputs; not the copies),
           the lambda-weighted dynamics Hessian (mode 1), the inequality rows through resto_iq_terms;
           mode 2: unit weights, gradient - z_L + z_U on u */
        const resto_t *R = C->Rs;
        const int m1 = C->mode != 2;         /* mode 3: the mode-1 rows without the eliminated inequality rows */
        for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) Hq[a][b] = m1 ? W->Hs[k][a][b] : 0.0;
        for (int j = 0; j < NZ; ++j) gq[j] = 0.0;
        for (int i = 0; i < NXS; ++i) {
            const int r = NA * k + i;
            const double w = R->eta * R->DRx[r] * R->DRx[r];
            Hq[i][i] += m1 ? w : 1.0;
            gq[i] = w * (z[i] - R->XR[r]);
        }
        for (int a = 0; a < NU; ++a) {
            const int j = NU * k + a;
            const double w = R->eta * R->DRu[j] * R->DRu[j];
            double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
            gq[NA + a] = w * (z[NA + a] - R->UR[j]);
            if (m1) {
                Hq[NA + a][NA + a] += w + W->zL[j] / sl + W->zU[j] / su;
                gq[NA + a] += -C->mu / sl + C->mu / su;
            } else {
                Hq[NA + a][NA + a] += 1.0;
                gq[NA + a] += -W->zL[j] + W->zU[j];
            }
        }
        if (R->ovr) for (int j = 0; j < NZ; ++j) gq[j] = R->gov[k][j];
        for (int i = 0; i < NIQ && C->mode != 3; ++i) {
            double cr[NZ];
            iq_row(i, cr);
            const double sg = R->sig[k][i], o = R->off[k][i];
            for (int a = 0; a < NZ; ++a) {
                if (cr[a] == 0.0) continue;
                for (int b = 0; b < NZ; ++b) Hq[a][b] += sg * cr[a] * cr[b];
                gq[a] += cr[a] * (sg * rr[i] + o);
            }
        }
        if (m1) for (int a = 0; a < NZ; ++a) Hq[a][a] += delta;
        return;
    }
    for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) Hq[a][b] = W->Hs[k][a][b];
    Hq[0][0] += sc * 2 * P->Qp; Hq[2][2] += sc * 2 * P->Qp; Hq[1][1] += sc * 2 * P->Qv; Hq[3][3] += sc * 2 * P->Qv;
    for (int a = 0; a < 2; ++a) {
        Hq[6 + a][6 + a] += sc * 2 * (P->Ru + P->Rdu); Hq[4 + a][4 + a] += sc * 2 * P->Rdu;
        Hq[6 + a][4 + a] -= sc * 2 * P->Rdu; Hq[4 + a][6 + a] -= sc * 2 * P->Rdu;
    }
    cost_grad(P, z, C->R + 4 * k, 0, gq);
    for (int j = 0; j < NZ; ++j) gq[j] *= sc;
    for (int a = 0; a < NU; ++a) {
        const int j = NU * k + a;
        double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
        Hq[6 + a][6 + a] += W->zL[j] / sl + W->zU[j] / su;
        gq[6 + a] += -C->mu / sl + C->mu / su;
    }
    for (int i = 0; i < NIQ; ++i) {
        double cr[NZ], sig, psi;
        iq_row(i, cr);
        slack_terms(C, W, k, i, &sig, &psi);
        sig += C->ds_shift;
        for (int a = 0; a < NZ; ++a) {
            if (cr[a] == 0.0) continue;
            for (int b = 0; b < NZ; ++b) Hq[a][b] += sig * cr[a] * cr[b];
            gq[a] += cr[a] * (sig * rr[i] + psi);
        }
    }
    for (int a = 0; a < NZ; ++a) Hq[a][a] += delta;
}

/* terminal value-function gradient (restoration: the proximity term of the physical states) */
static void terminal_grad(const ctx_t *C, const work_t *W, double *pn) {
    const prob_t *P = C->P; const int N = P->N;
    if (C->mode) {
        const resto_t *R = C->Rs;
        for (int i = 0; i < NA; ++i) pn[i] = R->ovr ? R->gov[N][i] : 0.0;
        for (int i = 0; i < NXS && !R->ovr; ++i) {
            const int r = NA * N + i;
            pn[i] = R->eta * R->DRx[r] * R->DRx[r] * (W->X[r] - R->XR[r]);
        }
        return;
    }
    double zN[NZ], gN[NZ];
    stage_z(W->X, W->U, N, zN);   /* U beyond N unused for terminal */
    cost_grad(P, zN, C->R + 4 * N, 1, gN);
    for (int i = 0; i < NA; ++i) pn[i] = C->sc * gN[i];
}

static int riccati_factor(const ctx_t *C, work_t *W, double r[][NIQ], double delta) {
    const prob_t *P = C->P; const int N = P->N; const double sc = C->sc;
    double (*Pn)[NA] = W->Pm[N];
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) Pn[i][j] = 0.0;
    if (C->mode) {
        for (int i = 0; i < NXS; ++i) {
            const int rr = NA * N + i;
            Pn[i][i] = C->mode == 1 ? C->Rs->eta * C->Rs->DRx[rr] * C->Rs->DRx[rr] : 1.0;
        }
        if (C->mode == 1) for (int i = 0; i < NA; ++i) Pn[i][i] += delta;
    } else {
        Pn[0][0] = Pn[2][2] = sc * 2 * P->Qp; Pn[1][1] = Pn[3][3] = sc * 2 * P->Qv;
        for (int i = 0; i < NA; ++i) Pn[i][i] += delta;
    }
    for (int k = N - 1; k >= 0; --k) {
        double Hq[NZ][NZ], gq[NZ];
        if (C->Rs) resto_iq_terms(C, W, k, delta);
        stage_qp(C, W, k, r[k], delta, Hq, gq);
        for (int j = 0; j < NZ; ++j) W->grad[k][j] = gq[j];
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = W->Pm[k + 1];
        if (C->Rs) {
            if (!soft_node(C, (const double (*)[NA])W->Pm[k + 1], k + 1, delta)) return 0;
            Pp = C->Rs->Pt[k + 1];
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
    if (C->Rs) return soft_node(C, (const double (*)[NA])W->Pm[0], 0, delta);     /* the soft initial-state rows */
    return 1;
}

/* vector pass + forward sweep for defect RHS rg (J d = -rg; restoration: soft rows J d - D lam+ = -rg)
   and inequality residuals r */
static void riccati_solve(const ctx_t *C, work_t *W, double rg[][NA], double r[][NIQ]) {
    const prob_t *P = C->P; const int N = P->N;
    const resto_t *R = C->Rs;
    terminal_grad(C, W, W->pv[N]);
    for (int k = N - 1; k >= 0; --k) {
        double Hq[NZ][NZ], gq[NZ];
        stage_qp(C, W, k, r[k], 0.0, Hq, gq);   /* only the gradient is used */
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = W->Pm[k + 1], *pp = W->pv[k + 1], ppt[NA];
        if (R) {
            memcpy(ppt, pp, sizeof ppt); soft_apply(R, k + 1, 1, ppt);
            pp = ppt; Pp = (double (*)[NA])R->Pt[k + 1];
        }
        double hh[NA], qx[NA], qu[NU], kf[2];
        for (int i = 0; i < NA; ++i) { double s = pp[i]; for (int m = 0; m < NA; ++m) s -= Pp[i][m] * rg[k + 1][m]; hh[i] = s; }
        for (int i = 0; i < NA; ++i) { double s = gq[i]; for (int m = 0; m < NA; ++m) s += A[m][i] * hh[m]; qx[i] = s; }
        for (int a = 0; a < NU; ++a) { double s = gq[NA + a]; for (int m = 0; m < NA; ++m) s += Bm[m][a] * hh[m]; qu[a] = s; }
        chol2_solve(W->Lq[k], qu, kf);
        W->kff[k][0] = -kf[0]; W->kff[k][1] = -kf[1];
        for (int i = 0; i < NA; ++i) W->pv[k][i] = qx[i] + W->Qux[k][0][i] * W->kff[k][0] + W->Qux[k][1][i] * W->kff[k][1];
    }
    for (int i = 0; i < NA; ++i) W->dX[i] = -rg[0][i] - (R ? R->D[i] * W->pv[0][i] : 0.0);
    if (R) soft_apply(R, 0, 0, W->dX);
    for (int k = 0; k < N; ++k) {
        double *dx = W->dX + NA * k, *du = W->dU + NU * k;
        for (int a = 0; a < NU; ++a) { double s = W->kff[k][a]; for (int i = 0; i < NA; ++i) s += W->K[k][a][i] * dx[i]; du[a] = s; }
        for (int i = 0; i < NA; ++i) {
            double s = -rg[k + 1][i];
            for (int m = 0; m < NA; ++m) s += W->A[k][i][m] * dx[m];
            for (int a = 0; a < NU; ++a) s += W->Bm[k][i][a] * du[a];
            if (R) s -= R->D[NA * (k + 1) + i] * W->pv[k + 1][i];
            W->dX[NA * (k + 1) + i] = s;
        }
        if (R) soft_apply(R, k + 1, 0, W->dX + NA * (k + 1));
    }
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        double s = W->pv[k][i]; for (int m = 0; m < NA; ++m) s += W->Pm[k][i][m] * W->dX[NA * k + m];
        W->lamp[NA * k + i] = -s;
    }
    /* slack steps ds = C dz + r, multiplier steps; restoration: y + dy from the eliminated row, then the
       slack, p and n steps of the stationarity rows -y + psi + S_s ds = 0, rho -+ y - mu/(p|n) */
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        double cr[NZ], dz[NZ], sig, psi, cdz = 0.0;
        iq_row(i, cr);
        for (int a = 0; a < NA; ++a) dz[a] = W->dX[NA * k + a];
        dz[6] = W->dU[NU * k]; dz[7] = W->dU[NU * k + 1];
        for (int a = 0; a < NZ; ++a) cdz += cr[a] * dz[a];
        if (R) {
            resto_t *Rw = C->Rs;
            const double yn = R->sig[k][i] * (cdz + r[k][i]) + R->off[k][i], dy = yn - W->y[k][i];
            W->dy[k][i] = dy;
            W->dS[k][i] = (yn - R->psi[k][i]) / R->Ssd[k][i];
            Rw->dqp[k][i] = (dy - R->rqp[k][i]) / R->Sqp[k][i];
            Rw->dqn[k][i] = (-dy - R->rqn[k][i]) / R->Sqn[k][i];
            continue;
        }
        slack_terms(C, W, k, i, &sig, &psi);
        W->dS[k][i] = cdz + r[k][i];
        (void)psi;
    }
}

static double frac_to_boundary(const ctx_t *C, const work_t *W, const double *dU, double dS[][NIQ], double tau) {
    double a = 1.0;
    for (int j = 0; j < NU * C->P->N; ++j) {
        double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
        if (dU[j] < 0) a = fmin(a, -tau * sl / dU[j]);
        if (dU[j] > 0) a = fmin(a, tau * su / dU[j]);
    }
    for (int k = 0; k < C->P->N; ++k) for (int i = 0; i < NIQ; ++i) {
        double s = W->S[k][i], d = dS[k][i];
        if (C->sL[i] > -1e299 && d < 0) a = fmin(a, -tau * (s - C->sL[i]) / d);
        if (C->sU[i] < 1e299 && d > 0) a = fmin(a, tau * (C->sU[i] - s) / d);
    }
    return a;
}

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

/* dual directions of the primal step (dU, dS): box multipliers, slack-row multipliers y from
   the eliminated system, slack-bound multipliers; returns their fraction-to-the-boundary step */
static double dual_steps(const ctx_t *C, work_t *W, int nU, double tau) {
    double az = 1.0;
    for (int j = 0; j < nU; ++j) {
        double sl = W->U[j] - C->lo, su = C->hi - W->U[j], du = W->dU[j];
        W->dzL[j] = C->mu / sl - W->zL[j] - W->zL[j] / sl * du;
        W->dzU[j] = C->mu / su - W->zU[j] + W->zU[j] / su * du;
        if (W->dzL[j] < 0) az = fmin(az, -tau * W->zL[j] / W->dzL[j]);
        if (W->dzU[j] < 0) az = fmin(az, -tau * W->zU[j] / W->dzU[j]);
    }
    for (int k = 0; k < C->P->N; ++k) for (int i = 0; i < NIQ; ++i) {
        double s = W->S[k][i], ds = W->dS[k][i], sig, psi;
        slack_terms(C, W, k, i, &sig, &psi);
        /* dy from the eliminated system: y + dy = Sigma*ds + psi' with psi' = -mu/(s-sL)+mu/(sU-s)
           (the restoration's riccati_solve has set it from the soft row) */
        if (!C->Rs) W->dy[k][i] = (sig + C->ds_shift) * ds + psi - W->y[k][i];
        if (C->sL[i] > -1e299) {
            double d = s - C->sL[i];
            W->dvL[k][i] = C->mu / d - W->vL[k][i] - W->vL[k][i] / d * ds;
            if (W->dvL[k][i] < 0) az = fmin(az, -tau * W->vL[k][i] / W->dvL[k][i]);
        } else W->dvL[k][i] = 0.0;
        double d = C->sU[i] - s;
        W->dvU[k][i] = C->mu / d - W->vU[k][i] + W->vU[k][i] / d * ds;
        if (W->dvU[k][i] < 0) az = fmin(az, -tau * W->vU[k][i] / W->dvU[k][i]);
    }
    return az;
}

/* IPOPT's least-square estimate of the starting multipliers (DefaultIterateInitializer::least_square_mults
 * -> LeastSquareMultipliers, constr_mult_init_max 1000): [I J^T; J 0] [d; y] = [-r; 0] over the columns of
 * x, u and the slacks s of the inequality rows d(x) - s = 0, with r_x = scaled grad f - z_L + z_U and
 * r_s = -v_L + v_U.  Eliminating d_s = J_d d_x gives per stage the Hessian I + C^T C (the u_{k-1} copies of
 * the augmented state weighted 0: they are not variables of the reference NLP, see lmpc_ipm.c) and the
 * gradient r + C^T r_s; y_c = -(P_k dx_k + p_k), y_d = C dz + r_s.  Fills W->lam and W->y at the starting
 * point (W->A / W->Bm set); returns max(|y_c|, |y_d|) over the rows of the reference NLP. */
static double ls_multipliers(const ctx_t *C, work_t *W) {
    const prob_t *P = C->P; const int N = P->N; const double sc = C->sc;
    static __thread double Ks[NMAX][NU][NA], ks[NMAX][NU], Ps[NMAX + 1][NA][NA], ps[NMAX + 1][NA];
    static __thread double Hs[NMAX][NZ][NZ], gs[NMAX][NZ];
    double zN[NZ], gN[NZ];
    stage_z(W->X, W->U, N, zN);
    cost_grad(P, zN, C->R + 4 * N, 1, gN);
    for (int i = 0; i < NA; ++i) { for (int j = 0; j < NA; ++j) Ps[N][i][j] = (i == j && i < 4); ps[N][i] = sc * gN[i]; }
    for (int k = N - 1; k >= 0; --k) {
        double z[NZ], (*Hq)[NZ] = Hs[k], *gq = gs[k];
        stage_z(W->X, W->U, k, z);
        cost_grad(P, z, C->R + 4 * k, 0, gq);
        for (int a = 0; a < NZ; ++a) { gq[a] *= sc; for (int b2 = 0; b2 < NZ; ++b2) Hq[a][b2] = (a == b2 && (a < 4 || a >= NA)); }
        for (int a = 0; a < NU; ++a) gq[NA + a] += -W->zL[NU * k + a] + W->zU[NU * k + a];
        for (int i = 0; i < NIQ; ++i) {
            double cr[NZ];
            iq_row(i, cr);
            const double rs = -W->vL[k][i] + W->vU[k][i];
            for (int a = 0; a < NZ; ++a) {
                if (cr[a] == 0.0) continue;
                for (int b2 = 0; b2 < NZ; ++b2) Hq[a][b2] += cr[a] * cr[b2];
                gq[a] += cr[a] * rs;
            }
        }
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = Ps[k + 1];
        double PA[NA][NA], PB[NA][NU], Qxx[NA][NA], Qux[NU][NA], Quu[NU][NU], qx[NA], qu[NU], L[3] = {1, 0, 1}, x2[2];
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) { double t = 0; for (int m = 0; m < NA; ++m) t += Pp[i][m] * A[m][j]; PA[i][j] = t; }
            for (int j = 0; j < NU; ++j) { double t = 0; for (int m = 0; m < NA; ++m) t += Pp[i][m] * Bm[m][j]; PB[i][j] = t; }
        }
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) { double t = Hq[i][j]; for (int m = 0; m < NA; ++m) t += A[m][i] * PA[m][j]; Qxx[i][j] = t; }
            double t = gq[i]; for (int m = 0; m < NA; ++m) t += A[m][i] * ps[k + 1][m]; qx[i] = t;
        }
        for (int a = 0; a < NU; ++a) {
            for (int i = 0; i < NA; ++i) { double t = Hq[NA + a][i]; for (int m = 0; m < NA; ++m) t += Bm[m][a] * PA[m][i]; Qux[a][i] = t; }
            for (int c = 0; c < NU; ++c) { double t = Hq[NA + a][NA + c]; for (int m = 0; m < NA; ++m) t += Bm[m][a] * PB[m][c]; Quu[a][c] = t; }
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
        for (int i = 0; i < NA; ++i) for (int j = 0; j < i; ++j) { const double t = 0.5 * (Ps[k][i][j] + Ps[k][j][i]); Ps[k][i][j] = Ps[k][j][i] = t; }
    }
    double dx[NA] = {0}, ymax = 0.0;
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < NA; ++i) {
            double t = ps[k][i]; for (int m = 0; m < NA; ++m) t += Ps[k][i][m] * dx[m];
            W->lam[NA * k + i] = -t;
            if (i < 4) ymax = fmax(ymax, fabs(t));      /* the copy rows are not IPOPT's */
        }
        if (k == N) break;
        double du[NU], dn[NA], dz[NZ];
        for (int a = 0; a < NU; ++a) { double t = ks[k][a]; for (int i = 0; i < NA; ++i) t += Ks[k][a][i] * dx[i]; du[a] = t; }
        for (int i = 0; i < NA; ++i) dz[i] = dx[i];
        dz[NA] = du[0]; dz[NA + 1] = du[1];
        for (int i = 0; i < NIQ; ++i) {
            double cr[NZ], cdz = 0.0;
            iq_row(i, cr);
            for (int a = 0; a < NZ; ++a) cdz += cr[a] * dz[a];
            W->y[k][i] = cdz - W->vL[k][i] + W->vU[k][i];
            ymax = fmax(ymax, fabs(W->y[k][i]));
        }
        for (int i = 0; i < NA; ++i) {
            double t = 0; for (int m = 0; m < NA; ++m) t += W->A[k][i][m] * dx[m];
            for (int a = 0; a < NU; ++a) t += W->Bm[k][i][a] * du[a];
            dn[i] = t;
        }
        memcpy(dx, dn, sizeof dx);
    }
    return ymax;
}

static double g_mult_init_max = 1e3;   /* IPOPT constr_mult_init_max (default 1000; 0 = zero multipliers) */
void oracle_rmpc_set_mult_init_max(double m) { g_mult_init_max = m; }
/* IPOPT's soft restoration and restoration phases on / off (off: a failed line search ends at -2) */
static int g_soft_resto = 1, g_resto = 1;
void oracle_rmpc_set_resto(int on) { g_soft_resto = on; g_resto = on; }

/* the dynamics Jacobians (A, Bm) and the -lambda-weighted RK4 Hessians at the iterate in W */
static void linearise(const prob_t *P, work_t *W) {
    for (int k = 0; k < P->N; ++k) {
        double xn[4], nl[4], J[4][NZ];
        for (int i = 0; i < 4; ++i) nl[i] = -W->lam[NA * (k + 1) + i];
        rk4_derivs(P, W->X + NA * k, W->U + NU * k, nl, xn, J, W->Hs[k]);
        for (int i = 0; i < NA; ++i) { for (int j = 0; j < NA; ++j) W->A[k][i][j] = 0.0; W->Bm[k][i][0] = W->Bm[k][i][1] = 0.0; }
        for (int i = 0; i < 4; ++i) { for (int j = 0; j < 4; ++j) W->A[k][i][j] = J[i][j]; W->Bm[k][i][0] = J[i][6]; W->Bm[k][i][1] = J[i][7]; }
        W->Bm[k][4][0] = 1.0; W->Bm[k][5][1] = 1.0;
    }
}

/* IPOPT's primal-dual system error at C->mu (IpoptCalculatedQuantities::curr_primal_dual_system_error):
   l1 norms of the primal infeasibility (defects g, inequality residuals r), of the dual infeasibility
   (x, u and slack rows) and of the complementarity z s - mu of the U box and the slack bounds, added */
static double pd_error(const ctx_t *C, const work_t *W, double g[][NA], double r[][NIQ]) {
    const prob_t *P = C->P; const int N = P->N;
    double l1 = 0.0;
    for (int k = 0; k <= N; ++k) {
        double z[NZ], gc[NZ], gl[NZ];
        stage_z(W->X, W->U, k < N ? k : N - 1, z);
        if (k == N) for (int i = 0; i < NA; ++i) z[i] = W->X[NA * N + i];
        cost_grad(P, z, C->R + 4 * k, k == N, gc);
        for (int j = 0; j < NZ; ++j) gl[j] = C->sc * gc[j];
        for (int i = 0; i < NA; ++i) gl[i] += W->lam[NA * k + i];
        if (k < N) {
            for (int m = 0; m < NA; ++m) {
                double l = W->lam[NA * (k + 1) + m];
                for (int i = 0; i < NA; ++i) gl[i] -= W->A[k][m][i] * l;
                gl[6] -= W->Bm[k][m][0] * l; gl[7] -= W->Bm[k][m][1] * l;
            }
            for (int i = 0; i < NIQ; ++i) { double cr[NZ]; iq_row(i, cr); for (int j = 0; j < NZ; ++j) gl[j] += cr[j] * W->y[k][i]; }
            gl[6] += -W->zL[NU * k] + W->zU[NU * k]; gl[7] += -W->zL[NU * k + 1] + W->zU[NU * k + 1];
            for (int j = 0; j < NZ; ++j) l1 += fabs(gl[j]);
            for (int i = 0; i < NIQ; ++i) {
                l1 += fabs(-W->y[k][i] - W->vL[k][i] + W->vU[k][i]) + fabs(r[k][i]);
                if (C->sL[i] > -1e299) l1 += fabs(W->vL[k][i] * (W->S[k][i] - C->sL[i]) - C->mu);
                l1 += fabs(W->vU[k][i] * (C->sU[i] - W->S[k][i]) - C->mu);
            }
            for (int a = 0; a < NU; ++a) {
                const int j = NU * k + a;
                l1 += fabs(W->zL[j] * (W->U[j] - C->lo) - C->mu) + fabs(W->zU[j] * (C->hi - W->U[j]) - C->mu);
            }
        } else {
            for (int i = 0; i < NA; ++i) l1 += fabs(gl[i]);
        }
        for (int i = 0; i < NA; ++i) l1 += fabs(g[k][i]);
    }
    return l1;
}

/* IPOPT's soft restoration phase (BacktrackingLineSearch::TrySoftRestoStep, soft_resto_pderror_reduction_factor
   0.9999; lmpc_ipm.c soft_resto_step): the primal-dual step of the current direction, damped only by the
   fraction to the boundary (one step length for x, s, y, z, v), taken if the original filter accepts it
   with alpha_primal_test = 0 (*orig = 1) or if it reduces the primal-dual system error by the factor.
   Returns the step length (0: rejected); the trial point is left in Xt / Ut / St, gt / rt. */
static double soft_resto_step(const ctx_t *C, work_t *W, int nfilt, double th, double phi, double th_max,
                              double tau, double curr_pd, double gt[][NA], double rt[][NIQ], double *th_t,
                              double *ph_t, int *orig) {
    const prob_t *P = C->P; const int N = P->N, nU = NU * N, nA = NA * (N + 1);
    const double gam_th = 1e-5, gam_ph = 1e-8;
    const double a = fmin(frac_to_boundary(C, W, W->dU, W->dS, tau), dual_steps(C, W, nU, tau));
    for (int i = 0; i < nA; ++i) W->Xt[i] = W->X[i] + a * W->dX[i];
    for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + a * W->dU[j];
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) W->St[k][i] = W->S[k][i] + a * W->dS[k][i];
    *th_t = residuals(C, W->Xt, W->Ut, W->St, gt, rt);
    *ph_t = barrier_obj(C, W->Xt, W->Ut, W->St);
    *orig = 0;
    int in_filter = !(*th_t < th_max) || !isfinite(*ph_t);
    for (int q = 0; q < nfilt && !in_filter; ++q) in_filter = *th_t >= W->filt_th[q] && *ph_t >= W->filt_ph[q];
    if (!in_filter && (LE(*th_t, (1 - gam_th) * th, th) || LE(*ph_t - phi, -gam_ph * th, phi))) { *orig = 1; return a; }
    if (!isfinite(*ph_t)) return 0.0;
    work_t *S = (work_t *)malloc(sizeof(work_t));
    memcpy(S, W, sizeof(work_t));
    memcpy(W->X, S->Xt, sizeof(double) * nA); memcpy(W->U, S->Ut, sizeof(double) * nU);
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        W->S[k][i] = S->St[k][i];
        W->y[k][i] = S->y[k][i] + a * S->dy[k][i];
        W->vL[k][i] = S->vL[k][i] + a * S->dvL[k][i]; W->vU[k][i] = S->vU[k][i] + a * S->dvU[k][i];
    }
    for (int i = 0; i < nA; ++i) W->lam[i] = S->lam[i] + a * (S->lamp[i] - S->lam[i]);
    for (int j = 0; j < nU; ++j) { W->zL[j] = S->zL[j] + a * S->dzL[j]; W->zU[j] = S->zU[j] + a * S->dzU[j]; }
    linearise(P, W);
    const double pd = pd_error(C, W, gt, rt);
    memcpy(W, S, sizeof(work_t));
    free(S);
    return pd <= 0.9999 * curr_pd ? a : 0.0;
}

/* ---------------------------------------------------------------------------------------------
 * IPOPT's restoration phase (MinC_1NrmRestorationPhase::PerformRestoration; lmpc_ipm.c restoration()
 * has the commentary, the same choices are made here): rho 1000, eta = sqrt(mu_R), D_R = min(1, 1/|x_R|),
 * mu_R = max(mu, ||(c, d - s)||_inf), p / n per row from the closed form of RestoIterateInitializer,
 * bound multipliers (U box, slack bounds) min(rho, z), equality multipliers by least squares (dropped
 * above 1000); the restoration problem is solved by the same algorithm with its own filter; the
 * original problem is re-entered once theta_orig <= 0.9 theta_orig(start) at a point the original
 * filter accepts (bound multipliers by the pretended Newton step, reset to 1 above 1000; equality
 * multipliers 0); the restoration problem converging means local infeasibility (status 2), its line
 * search failing a restoration failure (-2).
 * --------------------------------------------------------------------------------------------- */
/* constraint values of the restoration problem at (X, U, S, p, n) into cg / cr; returns their l1 norm */
static double resto_cons(const ctx_t *C, const double *X, const double *U, double S[][NIQ], const double *pc,
                         const double *nc, double qp[][NIQ], double qn[][NIQ], double g[][NA], double r[][NIQ],
                         double cg[][NA], double cr[][NIQ]) {
    const int N = C->P->N;
    residuals(C, X, U, S, g, r);
    double th = 0.0;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        const int rr = NA * k + i;
        cg[k][i] = i < NXS ? g[k][i] + nc[rr] - pc[rr] : g[k][i];
        th += fabs(cg[k][i]);
    }
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) { cr[k][i] = r[k][i] + qn[k][i] - qp[k][i]; th += fabs(cr[k][i]); }
    return th;
}
/* soft-row right-hand sides of the defect rows: rg = c - (rn/S_n - rp/S_p) + D lam (physical rows), c (copies) */
static void resto_rhs(const ctx_t *C, const work_t *W, double cg[][NA], double rg[][NA]) {
    const resto_t *R = C->Rs; const int N = C->P->N;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        const int r = NA * k + i;
        rg[k][i] = i < NXS ? cg[k][i] - (R->rn[r] / R->Snd[r] - R->rp[r] / R->Spd[r]) + R->D[r] * W->lam[r] : cg[k][i];
    }
}
static double resto_barrier(const ctx_t *C, const double *X, const double *U, double S[][NIQ], const double *pc,
                            const double *nc, double qp[][NIQ], double qn[][NIQ]) {
    const resto_t *R = C->Rs; const int N = C->P->N;
    double f = 0.0, lb = 0.0;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NXS; ++i) {
        const int r = NA * k + i;
        const double e = R->DRx[r] * (X[r] - R->XR[r]);
        f += R->rho * (pc[r] + nc[r]) + 0.5 * R->eta * e * e;
        if (!(pc[r] > 0) || !(nc[r] > 0)) return INFINITY;
        lb += log(pc[r]) + log(nc[r]);
    }
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        f += R->rho * (qp[k][i] + qn[k][i]);
        if (!(qp[k][i] > 0) || !(qn[k][i] > 0)) return INFINITY;
        lb += log(qp[k][i]) + log(qn[k][i]);
        if (C->sL[i] > -1e299) { if (!(S[k][i] - C->sL[i] > 0)) return INFINITY; lb += log(S[k][i] - C->sL[i]); }
        if (!(C->sU[i] - S[k][i] > 0)) return INFINITY;
        lb += log(C->sU[i] - S[k][i]);
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
static void resto_errors(const ctx_t *C, const work_t *W, double cg[][NA], double cr[][NIQ], double *dinf_,
                         double *pinf_, double *c0_, double *cmin_, double *sum_l_, double *sum_z_, int *nb_) {
    const resto_t *R = C->Rs; const int N = C->P->N;
    double dinf = 0, pinf = 0, c0 = 0, cmin = INFINITY, sum_l = 0, sum_z = 0;
    int nb = 0;
#define CMPL(v) do { const double cv_ = (v); c0 = fmax(c0, cv_); cmin = fmin(cmin, cv_); ++nb; } while (0)
    for (int k = 0; k <= N; ++k) {
        double gl[NZ];
        for (int j = 0; j < NZ; ++j) gl[j] = 0.0;
        for (int i = 0; i < NXS; ++i) {
            const int r = NA * k + i;
            gl[i] = R->eta * R->DRx[r] * R->DRx[r] * (W->X[r] - R->XR[r]);
        }
        for (int i = 0; i < NA; ++i) gl[i] += W->lam[NA * k + i];
        if (k < N) {
            for (int a = 0; a < NU; ++a) {
                const int j = NU * k + a;
                gl[NA + a] = R->eta * R->DRu[j] * R->DRu[j] * (W->U[j] - R->UR[j]) - W->zL[j] + W->zU[j];
            }
            for (int m = 0; m < NA; ++m) {
                const double l = W->lam[NA * (k + 1) + m];
                for (int i = 0; i < NA; ++i) gl[i] -= W->A[k][m][i] * l;
                gl[6] -= W->Bm[k][m][0] * l; gl[7] -= W->Bm[k][m][1] * l;
            }
            for (int i = 0; i < NIQ; ++i) { double c[NZ]; iq_row(i, c); for (int j = 0; j < NZ; ++j) gl[j] += c[j] * W->y[k][i]; }
            for (int j = 0; j < NZ; ++j) dinf = fmax(dinf, fabs(gl[j]));
#ifdef ORACLE_DEBUG
            for (int j = 0; j < NZ; ++j) if (fabs(gl[j]) > 1e-7) fprintf(stderr, "    dinf x k %d j %d %.3e\n", k, j, gl[j]);
            for (int i = 0; i < NIQ; ++i) { const double y = W->y[k][i];
                double a1 = fabs(-y - W->vL[k][i] + W->vU[k][i]), a2 = fabs(R->rho - R->zqp[k][i] - y), a3 = fabs(R->rho - R->zqn[k][i] + y);
                if (fmax(a1, fmax(a2, a3)) > 1e-7) fprintf(stderr, "    dinf iq k %d i %d s %.3e p %.3e n %.3e y %.6e\n", k, i, a1, a2, a3, y); }
#endif
            for (int a = 0; a < NU; ++a) {
                const int j = NU * k + a;
                CMPL(W->zL[j] * (W->U[j] - C->lo)); CMPL(W->zU[j] * (C->hi - W->U[j]));
                sum_z += W->zL[j] + W->zU[j];
            }
            for (int i = 0; i < NIQ; ++i) {
                const double y = W->y[k][i];
                dinf = fmax(dinf, fabs(-y - W->vL[k][i] + W->vU[k][i]));
                dinf = fmax(dinf, fmax(fabs(R->rho - R->zqp[k][i] - y), fabs(R->rho - R->zqn[k][i] + y)));
                pinf = fmax(pinf, fabs(cr[k][i]));
                if (C->sL[i] > -1e299) { CMPL(W->vL[k][i] * (W->S[k][i] - C->sL[i])); sum_z += W->vL[k][i]; }
                CMPL(W->vU[k][i] * (C->sU[i] - W->S[k][i])); sum_z += W->vU[k][i];
                CMPL(R->zqp[k][i] * R->qp[k][i]); CMPL(R->zqn[k][i] * R->qn[k][i]);
                sum_z += R->zqp[k][i] + R->zqn[k][i];
                sum_l += fabs(y);
            }
        } else {
            for (int i = 0; i < NA; ++i) dinf = fmax(dinf, fabs(gl[i]));
#ifdef ORACLE_DEBUG
            for (int i = 0; i < NA; ++i) if (fabs(gl[i]) > 1e-7) fprintf(stderr, "    dinf xN i %d %.3e\n", i, gl[i]);
#endif
        }
        for (int i = 0; i < NA; ++i) {
            const int r = NA * k + i;
            pinf = fmax(pinf, fabs(cg[k][i]));
            sum_l += fabs(W->lam[r]);
            if (i < NXS) {
#ifdef ORACLE_DEBUG
                if (fmax(fabs(R->rho - R->zp[r] - W->lam[r]), fabs(R->rho - R->zn[r] + W->lam[r])) > 1e-7)
                    fprintf(stderr, "    dinf def k %d i %d p %.3e n %.3e lam %.9e zp %.3e zn %.3e pc %.3e nc %.3e\n", k, i, R->rho - R->zp[r] - W->lam[r], R->rho - R->zn[r] + W->lam[r], W->lam[r], R->zp[r], R->zn[r], R->pc[r], R->nc[r]);
#endif
                dinf = fmax(dinf, fmax(fabs(R->rho - R->zp[r] - W->lam[r]), fabs(R->rho - R->zn[r] + W->lam[r])));
                CMPL(R->zp[r] * R->pc[r]); CMPL(R->zn[r] * R->nc[r]);
                sum_z += R->zp[r] + R->zn[r];
            }
        }
    }
#undef CMPL
    *dinf_ = dinf; *pinf_ = pinf; *c0_ = c0; *cmin_ = cmin; *sum_l_ = sum_l; *sum_z_ = sum_z; *nb_ = nb;
}

/* Iterative refinement of the restoration step.  With a p or n at the l1 kink (rho -+ y ~ mu/p) the soft
   rows reach D ~ 1e6 and D lam+ ~ 1e9, and the eliminated solve meets the Newton rows only to ~1e-7, above
   tol; IPOPT refines every solve of its augmented system (PDFullSpaceSolver).  The residuals of the full
   system at the step in V / R (stationarity of x and u, defect rows, inequality rows, the p / n rows of both
   kinds, the slack rows) are solved for on the same factorisation when they exceed 1e-12 (1 + |step|)
   (lam = y = 0 and the residuals in place of the gradients and right-hand sides), and the correction is
   added.  Returns 1 if a correction was made. */
static int resto_refine(const ctx_t *Cm, work_t *V, double cg[][NA], double cr[][NIQ], double rg[][NA]) {
    resto_t *R = Cm->Rs; const prob_t *P = Cm->P; const int N = P->N, nA = NA * (N + 1), nU = NU * N;
    ctx_t C3 = *Cm;
    C3.mode = 3;
    double emax = 0.0, smax = 0.0;
#define EM(v) (emax = fmax(emax, fabs(v)))
#define SM(v) (smax = fmax(smax, fabs(v)))
    for (int k = 0; k < N; ++k) {
        double Hq[NZ][NZ], gq[NZ], dz[NZ], zero[NIQ] = {0};
        stage_qp(&C3, V, k, zero, R->delta, Hq, gq);
        for (int a = 0; a < NA; ++a) dz[a] = V->dX[NA * k + a];
        dz[6] = V->dU[NU * k]; dz[7] = V->dU[NU * k + 1];
        for (int a = 0; a < NZ; ++a) { double t = gq[a]; for (int b = 0; b < NZ; ++b) t += Hq[a][b] * dz[b]; R->ex[k][a] = t; }
        for (int i = 0; i < NA; ++i) R->ex[k][i] += V->lamp[NA * k + i];
        for (int m = 0; m < NA; ++m) {
            const double l = V->lamp[NA * (k + 1) + m];
            for (int i = 0; i < NA; ++i) R->ex[k][i] -= V->A[k][m][i] * l;
            R->ex[k][6] -= V->Bm[k][m][0] * l; R->ex[k][7] -= V->Bm[k][m][1] * l;
        }
        for (int i = 0; i < NIQ; ++i) {
            double c[NZ];
            iq_row(i, c);
            const double yn = V->y[k][i] + V->dy[k][i];
            for (int a = 0; a < NZ; ++a) R->ex[k][a] += c[a] * yn;
        }
        for (int a = 0; a < NZ; ++a) EM(R->ex[k][a]);
    }
    {
        double pn[NA];
        terminal_grad(Cm, V, pn);
        for (int i = 0; i < NZ; ++i) R->ex[N][i] = 0.0;
        for (int i = 0; i < NA; ++i) {
            const int r = NA * N + i;
            const double h = (i < NXS ? R->eta * R->DRx[r] * R->DRx[r] : 0.0) + R->delta;
            R->ex[N][i] = h * V->dX[r] + pn[i] + V->lamp[r];
            EM(R->ex[N][i]);
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
        if (i < NXS) {
            const double dl = V->lamp[r] - V->lam[r];
            R->ec[k][i] = jd + R->dnc[r] - R->dpc[r] + cg[k][i];
            R->ep[r] = R->Spd[r] * R->dpc[r] - dl + R->rp[r];
            R->en[r] = R->Snd[r] * R->dnc[r] + dl + R->rn[r];
            EM(R->ep[r]); EM(R->en[r]); SM(R->dpc[r]); SM(R->dnc[r]);
        } else {
            R->ec[k][i] = jd + cg[k][i];
        }
        EM(R->ec[k][i]);
    }
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        double c[NZ], dz[NZ], cdz = 0.0;
        iq_row(i, c);
        for (int a = 0; a < NA; ++a) dz[a] = V->dX[NA * k + a];
        dz[6] = V->dU[NU * k]; dz[7] = V->dU[NU * k + 1];
        for (int a = 0; a < NZ; ++a) cdz += c[a] * dz[a];
        const double dy = V->dy[k][i];
        R->eq[k][i] = cdz - V->dS[k][i] + R->dqn[k][i] - R->dqp[k][i] + cr[k][i];
        R->eqp[k][i] = R->Sqp[k][i] * R->dqp[k][i] - dy + R->rqp[k][i];
        R->eqn[k][i] = R->Sqn[k][i] * R->dqn[k][i] + dy + R->rqn[k][i];
        R->es[k][i] = R->Ssd[k][i] * V->dS[k][i] - (V->y[k][i] + dy) + R->psi[k][i];
        EM(R->eq[k][i]); EM(R->eqp[k][i]); EM(R->eqn[k][i]); EM(R->es[k][i]);
        SM(V->dS[k][i]); SM(R->dqp[k][i]); SM(R->dqn[k][i]);
    }
    for (int j = 0; j < nU; ++j) SM(V->dU[j]);
#undef EM
#undef SM
    if (!(emax > 1e-12 * (1.0 + smax))) return 0;
    /* the correction solve on the same factorisation */
    work_t *Sv = (work_t *)malloc(sizeof(work_t));
    resto_t *SR = (resto_t *)malloc(sizeof(resto_t));
    memcpy(Sv, V, sizeof(work_t)); memcpy(SR, R, sizeof(resto_t));
    memset(V->lam, 0, sizeof(double) * nA);
    for (int i = 0; i < nA; ++i) { R->rp[i] = R->ep[i]; R->rn[i] = R->en[i]; }
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        V->y[k][i] = 0.0;
        R->rqp[k][i] = R->eqp[k][i]; R->rqn[k][i] = R->eqn[k][i]; R->psi[k][i] = R->es[k][i];
        R->off[k][i] = R->sig[k][i] * (R->psi[k][i] / R->Ssd[k][i] - R->rqn[k][i] / R->Sqn[k][i] + R->rqp[k][i] / R->Sqp[k][i]);
    }
    R->ovr = 1;
    memcpy(R->gov, R->ex, sizeof(double[NZ]) * (N + 1));
    resto_rhs(Cm, V, R->ec, rg);
    riccati_solve(Cm, V, rg, R->eq);
    /* V / R now hold the correction; add it to the saved step */
    for (int i = 0; i < nA; ++i) {
        Sv->dX[i] += V->dX[i];
        Sv->lamp[i] += V->lamp[i];
        if ((i % NA) < NXS) {
            SR->dpc[i] += (V->lamp[i] - R->ep[i]) / R->Spd[i];
            SR->dnc[i] += (-V->lamp[i] - R->en[i]) / R->Snd[i];
        }
    }
    for (int j = 0; j < nU; ++j) Sv->dU[j] += V->dU[j];
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        Sv->dy[k][i] += V->dy[k][i]; Sv->dS[k][i] += V->dS[k][i];
        SR->dqp[k][i] += R->dqp[k][i]; SR->dqn[k][i] += R->dqn[k][i];
    }
    memcpy(V, Sv, sizeof(work_t)); memcpy(R, SR, sizeof(resto_t));
    free(Sv); free(SR);
    return 1;
}

static int restoration(const ctx_t *C0, work_t *W, int *it_io, int max_iter, double tol, double th0, double phi0,
                       int nfilt0, double tau0, double g0[][NA], double r0[][NIQ], int *status) {
    const prob_t *P = C0->P; const int N = P->N, nU = NU * N, nA = NA * (N + 1), nI = NIQ * N;
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, gam_al = 0.05, kap_soc = 0.99;
    const double mu_min = tol / 10, s_max = 100.0;
    resto_t *R = (resto_t *)calloc(1, sizeof(resto_t));
    work_t *V = (work_t *)malloc(sizeof(work_t));
    work_t *Sv = (work_t *)malloc(sizeof(work_t));
    resto_t *SR = (resto_t *)malloc(sizeof(resto_t));
    memcpy(V, W, sizeof(work_t));
    const size_t szg = sizeof(double[NA]) * (N + 1), szr = sizeof(double[NIQ]) * N;
    double (*g)[NA] = calloc(N + 1, sizeof(double[NA])), (*gt)[NA] = calloc(N + 1, sizeof(double[NA]));
    double (*cg)[NA] = calloc(N + 1, sizeof(double[NA])), (*cgt)[NA] = calloc(N + 1, sizeof(double[NA]));
    double (*csg)[NA] = calloc(N + 1, sizeof(double[NA])), (*rg)[NA] = calloc(N + 1, sizeof(double[NA]));
    double (*r)[NIQ] = calloc(N, sizeof(double[NIQ])), (*rt)[NIQ] = calloc(N, sizeof(double[NIQ]));
    double (*cr)[NIQ] = calloc(N, sizeof(double[NIQ])), (*crt)[NIQ] = calloc(N, sizeof(double[NIQ]));
    double (*csr)[NIQ] = calloc(N, sizeof(double[NIQ]));
    ctx_t C = *C0;
    C.Rs = R; C.mode = 1; C.ds_shift = 0.0;
    R->rho = 1000.0;
    int ok_out = 0;
    /* RestoIpoptNLP: reference point and D_R */
    for (int i = 0; i < nA; ++i) { R->XR[i] = W->X[i]; R->DRx[i] = 1.0 / fmax(1.0, fabs(W->X[i])); }
    for (int j = 0; j < nU; ++j) { R->UR[j] = W->U[j]; R->DRu[j] = 1.0 / fmax(1.0, fabs(W->U[j])); }
    /* RestoIterateInitializer */
    double cmax = 0.0;
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) cmax = fmax(cmax, fabs(g0[k][i]));
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) cmax = fmax(cmax, fabs(r0[k][i]));
    C.mu = fmax(C0->mu, cmax);
    R->eta = sqrt(C.mu);
#define PN_INIT(c, p, n) do {                                                                        \
        const double a_ = C.mu / (2.0 * R->rho) - 0.5 * (c), b_ = (c) * C.mu / (2.0 * R->rho);        \
        (n) = a_ + sqrt(a_ * a_ + b_); (p) = (c) + (n);                                               \
    } while (0)
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NXS; ++i) {
        const int rr = NA * k + i;
        PN_INIT(g0[k][i], R->pc[rr], R->nc[rr]);
        R->zp[rr] = C.mu / R->pc[rr]; R->zn[rr] = C.mu / R->nc[rr];
    }
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        PN_INIT(r0[k][i], R->qp[k][i], R->qn[k][i]);
        R->zqp[k][i] = C.mu / R->qp[k][i]; R->zqn[k][i] = C.mu / R->qn[k][i];
        V->vL[k][i] = fmin(R->rho, W->vL[k][i]); V->vU[k][i] = fmin(R->rho, W->vU[k][i]);
    }
#undef PN_INIT
    for (int j = 0; j < nU; ++j) { V->zL[j] = fmin(R->rho, W->zL[j]); V->zU[j] = fmin(R->rho, W->zU[j]); }
    /* least-square equality multipliers of the restoration problem (unit weights on x, u, s, p, n) */
    linearise(P, V);
    {
        C.mode = 2;
        for (int i = 0; i < nA; ++i) { R->rp[i] = (i % NA) < NXS ? R->rho - R->zp[i] : 0.0; R->rn[i] = (i % NA) < NXS ? R->rho - R->zn[i] : 0.0; }
        memset(V->lam, 0, sizeof(double) * nA);
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) V->y[k][i] = 0.0;
        riccati_factor(&C, V, cr, 0.0);          /* cr = 0: unit weights, every Quu >= I */
        resto_rhs(&C, V, cg, rg);                /* cg = 0 */
        riccati_solve(&C, V, rg, cr);
        double ym = 0.0;
        for (int i = 0; i < nA; ++i) {
            if ((i % NA) < NXS) ym = fmax(ym, fabs(V->lamp[i]));
            if (!isfinite(V->lamp[i])) ym = INFINITY;
        }
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            ym = fmax(ym, fabs(V->dy[k][i]));
            if (!isfinite(V->dy[k][i])) ym = INFINITY;
        }
        if (ym <= 1e3) {
            memcpy(V->lam, V->lamp, sizeof(double) * nA);
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) V->y[k][i] = V->dy[k][i];
        }
        C.mode = 1;
    }
    double th = resto_cons(&C, V->X, V->U, V->S, R->pc, R->nc, R->qp, R->qn, g, r, cg, cr);
    const double th_max = 1e4 * fmax(1.0, th), th_min = 1e-4 * fmax(1.0, th);
    int nfilt = 0, rit = *it_io + 1, first = 1;
    double delta_last = 0.0;
    for (;; ++rit) {
        linearise(P, V);
        if (!first) {
            /* the original problem's progress at the current point */
            const double tho = residuals(C0, V->X, V->U, V->S, gt, rt);
            if (tho <= 0.9 * th0) {
                const double pho = barrier_obj(C0, V->X, V->U, V->S);
                int acc = isfinite(pho);
                for (int q = 0; q < nfilt0 && acc; ++q) acc = !(tho >= W->filt_th[q] && pho >= W->filt_ph[q]);
                acc = acc && (LE(tho, (1 - gam_th) * th0, th0) || LE(pho - phi0, -gam_ph * th0, phi0));
                if (acc) { ok_out = 1; break; }
            }
        }
        first = 0;
        double dinf, pinf, c0, cmin, sum_l, sum_z;
        int nb;
        resto_errors(&C, V, cg, cr, &dinf, &pinf, &c0, &cmin, &sum_l, &sum_z, &nb);
        const double s_d = fmax(s_max, (sum_l + sum_z) / (nA + nI + nb)) / s_max;
        const double s_c = fmax(s_max, sum_z / nb) / s_max;
        const double err = fmax(dinf / s_d, fmax(pinf, c0 / s_c));
        if (rit >= max_iter) { *status = ST_MAXITER; break; }
        if (err <= tol && dinf <= 1.0 && pinf <= 1e-4 && c0 <= 1e-4) { *status = ST_INFEASIBLE; break; }   /* local infeasibility */
        for (;;) {
            const double cmu = fmax(c0 - C.mu, C.mu - cmin);
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * C.mu || C.mu <= mu_min) break;
            C.mu = fmax(mu_min, fmin(0.2 * C.mu, pow(C.mu, 1.5)));
            R->eta = sqrt(C.mu);
            nfilt = 0;
        }
        const double tau = fmax(0.99, 1.0 - C.mu);
        for (int i = 0; i < nA; ++i) if ((i % NA) < NXS) {
            R->rp[i] = R->rho - C.mu / R->pc[i] - V->lam[i];
            R->rn[i] = R->rho - C.mu / R->nc[i] + V->lam[i];
        }
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            R->rqp[k][i] = R->rho - C.mu / R->qp[k][i] - V->y[k][i];
            R->rqn[k][i] = R->rho - C.mu / R->qn[k][i] + V->y[k][i];
        }
        double delta = 0.0;
        int ok = riccati_factor(&C, V, cr, 0.0);
        for (int attempt = 0; !ok && attempt < 60; ++attempt) {
            delta = (attempt == 0) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            ok = riccati_factor(&C, V, cr, delta);
        }
        if (!ok) { *status = ST_INERTIA_FAIL; break; }
        if (delta > 0) delta_last = delta;
        R->delta = delta;
        double amax = 0, az = 0;
        /* bound-multiplier steps of p, n (both row kinds), the U box and the slack bounds, their fractions */
#define PN_DUALS() do {                                                                                 \
            az = dual_steps(&C, V, nU, tau);                                                            \
            for (int i = 0; i < nA; ++i) if ((i % NA) < NXS) {                                          \
                R->dzp[i] = C.mu / R->pc[i] - R->zp[i] - R->zp[i] / R->pc[i] * R->dpc[i];               \
                R->dzn[i] = C.mu / R->nc[i] - R->zn[i] - R->zn[i] / R->nc[i] * R->dnc[i];               \
                if (R->dzp[i] < 0) az = fmin(az, -tau * R->zp[i] / R->dzp[i]);                          \
                if (R->dzn[i] < 0) az = fmin(az, -tau * R->zn[i] / R->dzn[i]);                          \
            }                                                                                           \
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {                                 \
                R->dzqp[k][i] = C.mu / R->qp[k][i] - R->zqp[k][i] - R->zqp[k][i] / R->qp[k][i] * R->dqp[k][i]; \
                R->dzqn[k][i] = C.mu / R->qn[k][i] - R->zqn[k][i] - R->zqn[k][i] / R->qn[k][i] * R->dqn[k][i]; \
                if (R->dzqp[k][i] < 0) az = fmin(az, -tau * R->zqp[k][i] / R->dzqp[k][i]);              \
                if (R->dzqn[k][i] < 0) az = fmin(az, -tau * R->zqn[k][i] / R->dzqn[k][i]);              \
            }                                                                                           \
        } while (0)
#define RESTO_STEP(CG, CR) do {                                                                         \
            resto_rhs(&C, V, CG, rg);                                                                   \
            riccati_solve(&C, V, rg, CR);                                                               \
            for (int i = 0; i < nA; ++i) if ((i % NA) < NXS) {                                          \
                const double dy_ = V->lamp[i] - V->lam[i];                                              \
                R->dpc[i] = (dy_ - R->rp[i]) / R->Spd[i];                                               \
                R->dnc[i] = (-dy_ - R->rn[i]) / R->Snd[i];                                              \
            }                                                                                           \
            for (int rr_ = 0; rr_ < 3 && resto_refine(&C, V, CG, CR, rg); ++rr_) {}                     \
            amax = frac_to_boundary(&C, V, V->dU, V->dS, tau);                                          \
            for (int i = 0; i < nA; ++i) if ((i % NA) < NXS) {                                          \
                if (R->dpc[i] < 0) amax = fmin(amax, -tau * R->pc[i] / R->dpc[i]);                      \
                if (R->dnc[i] < 0) amax = fmin(amax, -tau * R->nc[i] / R->dnc[i]);                      \
            }                                                                                           \
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {                                 \
                if (R->dqp[k][i] < 0) amax = fmin(amax, -tau * R->qp[k][i] / R->dqp[k][i]);             \
                if (R->dqn[k][i] < 0) amax = fmin(amax, -tau * R->qn[k][i] / R->dqn[k][i]);             \
            }                                                                                           \
            PN_DUALS();                                                                                 \
        } while (0)
        RESTO_STEP(cg, cr);
        const double phi = resto_barrier(&C, V->X, V->U, V->S, R->pc, R->nc, R->qp, R->qn);
        double gTd = 0.0;
        for (int k = 0; k <= N; ++k) for (int i = 0; i < NXS; ++i) {
            const int rr = NA * k + i;
            gTd += R->eta * R->DRx[rr] * R->DRx[rr] * (V->X[rr] - R->XR[rr]) * V->dX[rr];
            gTd += (R->rho - C.mu / R->pc[rr]) * R->dpc[rr] + (R->rho - C.mu / R->nc[rr]) * R->dnc[rr];
        }
        for (int j = 0; j < nU; ++j)
            gTd += (R->eta * R->DRu[j] * R->DRu[j] * (V->U[j] - R->UR[j]) - C.mu / (V->U[j] - C.lo) + C.mu / (C.hi - V->U[j])) * V->dU[j];
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            double sg, ps;
            slack_terms(&C, V, k, i, &sg, &ps);
            gTd += (R->rho - C.mu / R->qp[k][i]) * R->dqp[k][i] + (R->rho - C.mu / R->qn[k][i]) * R->dqn[k][i] + ps * V->dS[k][i];
        }
        double amin = gam_th;
        if (gTd < 0) amin = fmin(gam_th, fmin(gam_ph * th / (-gTd), pow(th, s_th) / pow(-gTd, s_ph)));
        amin *= gam_al;
        double alpha = amax, th_t = 0, ph_t = 0;
        int accepted = 0, ftype = 0;
#define RESTO_TRIAL(AL) do {                                                                            \
            for (int i = 0; i < nA; ++i) V->Xt[i] = V->X[i] + (AL) * V->dX[i];                         \
            for (int j = 0; j < nU; ++j) V->Ut[j] = V->U[j] + (AL) * V->dU[j];                         \
            for (int i = 0; i < nA; ++i) if ((i % NA) < NXS) {                                          \
                R->pt_[i] = R->pc[i] + (AL) * R->dpc[i]; R->nt_[i] = R->nc[i] + (AL) * R->dnc[i];       \
            }                                                                                           \
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {                                 \
                V->St[k][i] = V->S[k][i] + (AL) * V->dS[k][i];                                          \
                R->qpt[k][i] = R->qp[k][i] + (AL) * R->dqp[k][i]; R->qnt[k][i] = R->qn[k][i] + (AL) * R->dqn[k][i]; \
            }                                                                                           \
            th_t = resto_cons(&C, V->Xt, V->Ut, V->St, R->pt_, R->nt_, R->qpt, R->qnt, gt, rt, cgt, crt); \
            ph_t = resto_barrier(&C, V->Xt, V->Ut, V->St, R->pt_, R->nt_, R->qpt, R->qnt);               \
        } while (0)
#define RESTO_ACCEPT(AL, ACC) do {                                                                      \
            int in_f_ = !(th_t < th_max) || !isfinite(ph_t);                                            \
            for (int q = 0; q < nfilt && !in_f_; ++q) in_f_ = th_t >= R->filt_th[q] && ph_t >= R->filt_ph[q]; \
            (ACC) = 0;                                                                                  \
            if (!in_f_) {                                                                               \
                const int sw_ = gTd < 0 && (AL) * pow(-gTd, s_ph) > pow(th, s_th);                      \
                if (th <= th_min && sw_) { if (LE(ph_t, phi + 1e-8 * (AL) * gTd, phi)) { (ACC) = 1; ftype = 1; } } \
                else (ACC) = LE(th_t, (1 - gam_th) * th, th) || LE(ph_t - phi, -gam_ph * th, phi);     \
            }                                                                                           \
        } while (0)
        for (int ls = 0; ls < 80 && !accepted; ++ls) {
            if (alpha < amin && ls > 0) break;
            RESTO_TRIAL(alpha);
            RESTO_ACCEPT(alpha, accepted);
            if (!accepted && ls == 0 && !(th_t < th) && g_max_soc > 0) {
                /* second-order correction on the restoration problem's constraints */
                memcpy(Sv, V, sizeof(work_t)); memcpy(SR, R, sizeof(resto_t));
                double asoc = alpha, th_old = 0.0;
                memcpy(csg, cg, szg); memcpy(csr, cr, szr);
                for (int c = 0; c < g_max_soc; ++c) {
                    if (c > 0 && !(th_t <= kap_soc * th_old)) break;
                    th_old = th_t;
                    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) csg[k][i] = asoc * csg[k][i] + cgt[k][i];
                    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) csr[k][i] = asoc * csr[k][i] + crt[k][i];
                    RESTO_STEP(csg, csr);
                    asoc = amax;
                    RESTO_TRIAL(asoc);
                    int acc;
                    RESTO_ACCEPT(alpha, acc);
                    if (acc) { accepted = 1; alpha = asoc; break; }
                }
                if (!accepted) {    /* back to the plain direction and its multiplier steps */
                    memcpy(V, Sv, sizeof(work_t)); memcpy(R, SR, sizeof(resto_t));
                    PN_DUALS();
                }
            }
            if (!accepted) alpha *= 0.5;
        }
#ifdef ORACLE_DEBUG
        fprintf(stderr, "  resto it %3d mu %.2e err %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e th %.3e th_t %.3e acc %d\n",
                rit, C.mu, err, dinf / s_d, pinf, c0 / s_c, delta, amax, alpha, th, th_t, accepted);
#endif
        if (!accepted) { *status = ST_LS_FAIL; break; }     /* restoration failure */
        if (!ftype && nfilt < 256) { R->filt_th[nfilt] = (1 - gam_th) * th; R->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
        memcpy(V->X, V->Xt, sizeof(double) * nA);
        memcpy(V->U, V->Ut, sizeof(double) * nU);
        memcpy(cg, cgt, szg); memcpy(cr, crt, szr);
        th = th_t;
        for (int i = 0; i < nA; ++i) V->lam[i] += alpha * (V->lamp[i] - V->lam[i]);
#define KSIG(z, s, m) fmax(fmin((z), 1e10 * (m) / (s)), (m) / (1e10 * (s)))
        for (int i = 0; i < nA; ++i) if ((i % NA) < NXS) {
            R->pc[i] = R->pt_[i]; R->nc[i] = R->nt_[i];
            R->zp[i] = KSIG(R->zp[i] + az * R->dzp[i], R->pc[i], C.mu);
            R->zn[i] = KSIG(R->zn[i] + az * R->dzn[i], R->nc[i], C.mu);
        }
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            V->S[k][i] = V->St[k][i];
            V->y[k][i] += alpha * V->dy[k][i];
            R->qp[k][i] = R->qpt[k][i]; R->qn[k][i] = R->qnt[k][i];
            R->zqp[k][i] = KSIG(R->zqp[k][i] + az * R->dzqp[k][i], R->qp[k][i], C.mu);
            R->zqn[k][i] = KSIG(R->zqn[k][i] + az * R->dzqn[k][i], R->qn[k][i], C.mu);
            if (C.sL[i] > -1e299) V->vL[k][i] = KSIG(V->vL[k][i] + az * V->dvL[k][i], V->S[k][i] - C.sL[i], C.mu);
            V->vU[k][i] = KSIG(V->vU[k][i] + az * V->dvU[k][i], C.sU[i] - V->S[k][i], C.mu);
        }
        for (int j = 0; j < nU; ++j) {
            V->zL[j] = KSIG(V->zL[j] + az * V->dzL[j], V->U[j] - C.lo, C.mu);
            V->zU[j] = KSIG(V->zU[j] + az * V->dzU[j], C.hi - V->U[j], C.mu);
        }
#undef RESTO_ACCEPT
#undef RESTO_TRIAL
#undef RESTO_STEP
#undef PN_DUALS
    }
    if (ok_out) {
        /* back to the original problem: bound multipliers by the pretended Newton step (mu - z s_trial)/s cut
           by the fraction to the boundary, all reset to 1 above 1000; equality multipliers 0 */
        const double mu0 = C0->mu;
        double az = 1.0, zmax = 0.0;
#define PRETEND(z, dz, s, st) do { (dz) = (mu0 - (z) * (st)) / (s); if ((dz) < 0) az = fmin(az, -tau0 * (z) / (dz)); } while (0)
        for (int j = 0; j < nU; ++j) {
            PRETEND(W->zL[j], W->dzL[j], W->U[j] - C0->lo, V->U[j] - C0->lo);
            PRETEND(W->zU[j], W->dzU[j], C0->hi - W->U[j], C0->hi - V->U[j]);
        }
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            if (C0->sL[i] > -1e299) PRETEND(W->vL[k][i], W->dvL[k][i], W->S[k][i] - C0->sL[i], V->S[k][i] - C0->sL[i]);
            else W->dvL[k][i] = 0.0;
            PRETEND(W->vU[k][i], W->dvU[k][i], C0->sU[i] - W->S[k][i], C0->sU[i] - V->S[k][i]);
        }
#undef PRETEND
        for (int j = 0; j < nU; ++j) {
            W->zL[j] += az * W->dzL[j]; W->zU[j] += az * W->dzU[j];
            zmax = fmax(zmax, fmax(W->zL[j], W->zU[j]));
        }
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            W->vL[k][i] += az * W->dvL[k][i]; W->vU[k][i] += az * W->dvU[k][i];
            zmax = fmax(zmax, fmax(W->vL[k][i], W->vU[k][i]));
        }
        if (zmax > 1e3) {
            for (int j = 0; j < nU; ++j) { W->zL[j] = 1.0; W->zU[j] = 1.0; }
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) { W->vL[k][i] = C0->sL[i] > -1e299 ? 1.0 : 0.0; W->vU[k][i] = 1.0; }
        }
        memcpy(W->X, V->X, sizeof(double) * nA);
        memcpy(W->U, V->U, sizeof(double) * nU);
        memset(W->lam, 0, sizeof(double) * nA);
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            W->S[k][i] = V->S[k][i]; W->y[k][i] = 0.0;
            if (C0->sL[i] > -1e299) W->vL[k][i] = KSIG(W->vL[k][i], W->S[k][i] - C0->sL[i], mu0);
            W->vU[k][i] = KSIG(W->vU[k][i], C0->sU[i] - W->S[k][i], mu0);
        }
        for (int j = 0; j < nU; ++j) {      /* AcceptTrialPoint: kappa_sigma correction */
            W->zL[j] = KSIG(W->zL[j], W->U[j] - C0->lo, mu0);
            W->zU[j] = KSIG(W->zU[j], C0->hi - W->U[j], mu0);
        }
        *it_io = rit - 1;
    } else {
        /* IPOPT copies the restoration phase's last iterate into the original problem's fields on failure */
        memcpy(W->X, V->X, sizeof(double) * nA);
        memcpy(W->U, V->U, sizeof(double) * nU);
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) W->S[k][i] = V->S[k][i];
        *it_io = rit;
    }
#undef KSIG
    free(g); free(gt); free(cg); free(cgt); free(csg); free(rg); free(r); free(rt); free(cr); free(crt); free(csr);
    free(V); free(Sv); free(SR); free(R);
    return ok_out;
}

int oracle_rmpc_solve(int N, double Ts, const double *x0, const double *u_prev, const double *theta,
                      const double *Rref, const double *prm, const double *w_init, int max_iter, double tol,
                      double *u0, double *fval, double *w_out, int32_t *iters_out) {
    /* prm = [Qp, Qv, Ru, Rdu, u_lo, u_hi, du_lo, du_hi, vmax, v_eps] */
    if (N < 1 || N > NMAX || !(Ts > 0) || !(prm[5] > prm[4]) || !(prm[7] > prm[6])) return ST_BAD_INPUT;
    work_t *W = (work_t *)calloc(1, sizeof(work_t));
    if (!W) return ST_BAD_INPUT;
    prob_t P = {N, Ts, -9.81, prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], prm[8], prm[9], {0}};
    memcpy(P.th, theta, sizeof(double) * 14);
    const double lo = P.ulo - g_relax * fmax(1.0, fabs(P.ulo)), hi = P.uhi + g_relax * fmax(1.0, fabs(P.uhi));
    const double mu_min = tol / 10, kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, s_max = 100.0;
    const double gam_th = 1e-5, gam_ph = 1e-8, sw_delta = 1.0, s_th = 1.1, s_ph = 2.3, gam_al = 0.05, kap_soc = 0.99;
    const int nU = NU * N, nA = NA * (N + 1), nI = NIQ * N;
    ctx_t C;
    memset(&C, 0, sizeof C);
    C.P = &P; C.x0 = x0; C.up0 = u_prev; C.R = Rref; C.mu = 0.1; C.lo = lo; C.hi = hi;
    for (int i = 0; i < NIQ; ++i) {
        double gl = i < 2 ? P.dulo : -1e300, gu = i < 2 ? P.duhi : 0.0;
        C.sL[i] = gl > -1e299 ? gl - g_relax * fmax(1.0, fabs(gl)) : -1e300;     /* bound_relax_factor */
        C.sU[i] = gu + g_relax * fmax(1.0, fabs(gu));
    }
    /* initial point: w_init (reference warm start, zeros on the first call :168) */
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 4; ++i) W->X[NA * k + i] = w_init ? w_init[4 * k + i] : 0.0;
    }
    for (int j = 0; j < nU; ++j) {
        double u = w_init ? w_init[4 * (N + 1) + j] : 0.0;
        double pl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo)), pu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
        if (u < lo + pl) u = lo + pl;
        if (u > hi - pu) u = hi - pu;
        W->U[j] = u; W->zL[j] = 1.0; W->zU[j] = 1.0;
    }
    /* auxiliary copies u_{k-1} */
    W->X[4] = u_prev[0]; W->X[5] = u_prev[1];
    for (int k = 1; k <= N; ++k) { W->X[NA * k + 4] = W->U[NU * (k - 1)]; W->X[NA * k + 5] = W->U[NU * (k - 1) + 1]; }
    /* slacks: s = g(w) pushed into the relaxed bounds */
    for (int k = 0; k < N; ++k) {
        double z[NZ]; stage_z(W->X, W->U, k, z);
        for (int i = 0; i < NIQ; ++i) {
            double s = iq_val(&P, i, z), sl = C.sL[i], su = C.sU[i];
            if (sl > -1e299) {
                double pl = fmin(1e-2 * fmax(1.0, fabs(sl)), 1e-2 * (su - sl)), pu = fmin(1e-2 * fmax(1.0, fabs(su)), 1e-2 * (su - sl));
                s = fmin(fmax(s, sl + pl), su - pu);
            } else {
                s = fmin(s, su - 1e-2 * fmax(1.0, fabs(su)));
            }
            W->S[k][i] = s; W->vL[k][i] = sl > -1e299 ? 1.0 : 0.0; W->vU[k][i] = 1.0; W->y[k][i] = 0.0;
        }
    }
    /* gradient-based objective scaling */
    double gmax = 0.0;
    for (int k = 0; k <= N; ++k) {
        double z[NZ], g[NZ]; stage_z(W->X, W->U, k < N ? k : 0, z);
        if (k == N) for (int i = 0; i < NA; ++i) z[i] = W->X[NA * N + i];
        cost_grad(&P, z, Rref + 4 * k, k == N, g);
        for (int j = 0; j < NZ; ++j) gmax = fmax(gmax, fabs(g[j]));
    }
    C.sc = gmax > 100.0 ? 100.0 / gmax : 1.0;

    if (g_mult_init_max > 0.0) {
        for (int k = 0; k < N; ++k) {        /* the Jacobian at the starting point */
            double xn[4], nl[4] = {0, 0, 0, 0}, J[4][NZ];
            rk4_derivs(&P, W->X + NA * k, W->U + NU * k, nl, xn, J, W->Hs[k]);
            for (int i = 0; i < NA; ++i) { for (int j = 0; j < NA; ++j) W->A[k][i][j] = 0.0; W->Bm[k][i][0] = W->Bm[k][i][1] = 0.0; }
            for (int i = 0; i < 4; ++i) { for (int j = 0; j < 4; ++j) W->A[k][i][j] = J[i][j]; W->Bm[k][i][0] = J[i][6]; W->Bm[k][i][1] = J[i][7]; }
            W->Bm[k][4][0] = 1.0; W->Bm[k][5][1] = 1.0;
        }
        if (!(ls_multipliers(&C, W) <= g_mult_init_max)) {
            memset(W->lam, 0, sizeof W->lam);
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) W->y[k][i] = 0.0;
        }
    }
    double (*g)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*r)[NIQ] = (double (*)[NIQ])calloc(N, sizeof(double[NIQ]));
    double (*gt)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*rt)[NIQ] = (double (*)[NIQ])calloc(N, sizeof(double[NIQ]));
    double (*csg)[NA] = (double (*)[NA])calloc(N + 1, sizeof(double[NA]));
    double (*csr)[NIQ] = (double (*)[NIQ])calloc(N, sizeof(double[NIQ]));
    double th = residuals(&C, W->X, W->U, W->S, g, r);
    const double th_max = 1e4 * fmax(1.0, th), th_min = 1e-4 * fmax(1.0, th);
    int nfilt = 0, status = ST_MAXITER, it, in_soft = 0, soft_count = 0;
    double delta_last = 0.0;
    for (it = 0; it < max_iter; ++it) {
        linearise(&P, W);
        /* optimality error (IPOPT eq. 5): x rows, u rows, slack rows; complementarity of box and slack bounds */
        double sum_l = 0, sum_z = 0, dinf = 0, pinf = 0, c0 = 0; int nb = 0;
        for (int i = 0; i < nA; ++i) sum_l += fabs(W->lam[i]);
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) sum_l += fabs(W->y[k][i]);
        for (int k = 0; k <= N; ++k) {
            double z[NZ], gc[NZ];
            stage_z(W->X, W->U, k < N ? k : N - 1, z);
            if (k == N) { for (int i = 0; i < NA; ++i) z[i] = W->X[NA * N + i]; }
            cost_grad(&P, z, Rref + 4 * k, k == N, gc);
            double gl[NZ];
            for (int j = 0; j < NZ; ++j) gl[j] = C.sc * gc[j];
            for (int i = 0; i < NA; ++i) gl[i] += W->lam[NA * k + i];
            if (k < N) {
                for (int m = 0; m < NA; ++m) {
                    double l = W->lam[NA * (k + 1) + m];
                    for (int i = 0; i < NA; ++i) gl[i] -= W->A[k][m][i] * l;
                    gl[6] -= W->Bm[k][m][0] * l; gl[7] -= W->Bm[k][m][1] * l;
                }
                for (int i = 0; i < NIQ; ++i) { double cr[NZ]; iq_row(i, cr); for (int j = 0; j < NZ; ++j) gl[j] += cr[j] * W->y[k][i]; }
                gl[6] += -W->zL[NU * k] + W->zU[NU * k]; gl[7] += -W->zL[NU * k + 1] + W->zU[NU * k + 1];
                for (int j = 0; j < NZ; ++j) dinf = fmax(dinf, fabs(gl[j]));
                for (int i = 0; i < NIQ; ++i) {
                    dinf = fmax(dinf, fabs(-W->y[k][i] - W->vL[k][i] + W->vU[k][i]));
                    pinf = fmax(pinf, fabs(r[k][i]));
                    if (C.sL[i] > -1e299) { c0 = fmax(c0, fabs(W->vL[k][i] * (W->S[k][i] - C.sL[i]))); sum_z += W->vL[k][i]; ++nb; }
                    c0 = fmax(c0, fabs(W->vU[k][i] * (C.sU[i] - W->S[k][i]))); sum_z += W->vU[k][i]; ++nb;
                }
                for (int a = 0; a < NU; ++a) {
                    const int j = NU * k + a;
                    c0 = fmax(c0, fmax(fabs(W->zL[j] * (W->U[j] - lo)), fabs(W->zU[j] * (hi - W->U[j]))));
                    sum_z += W->zL[j] + W->zU[j]; nb += 2;
                }
            } else {
                for (int i = 0; i < NA; ++i) dinf = fmax(dinf, fabs(gl[i]));
            }
            for (int i = 0; i < NA; ++i) pinf = fmax(pinf, fabs(g[k][i]));
        }
        const double s_d = fmax(s_max, (sum_l + sum_z) / (nA + nI + nb)) / s_max;
        const double s_c = fmax(s_max, sum_z / nb) / s_max;
        if (fmax(dinf / s_d, fmax(pinf, c0 / s_c)) <= tol) { status = ST_SOLVED; break; }
        for (;;) {
            double cmu = 0;
            for (int j = 0; j < nU; ++j)
                cmu = fmax(cmu, fmax(fabs(W->zL[j] * (W->U[j] - lo) - C.mu), fabs(W->zU[j] * (hi - W->U[j]) - C.mu)));
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
                if (C.sL[i] > -1e299) cmu = fmax(cmu, fabs(W->vL[k][i] * (W->S[k][i] - C.sL[i]) - C.mu));
                cmu = fmax(cmu, fabs(W->vU[k][i] * (C.sU[i] - W->S[k][i]) - C.mu));
            }
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > kappa_eps * C.mu || C.mu <= mu_min) break;
            C.mu = fmax(mu_min, fmin(kappa_mu * C.mu, pow(C.mu, theta_mu)));
            nfilt = 0; in_soft = 0;      /* BacktrackingLineSearch::Reset: the filter and the soft phase */
        }
        const double tau = fmax(0.99, 1.0 - C.mu);
        double delta = 0.0;
        C.ds_shift = 0.0;
        int ok = riccati_factor(&C, W, r, 0.0);
        for (int attempt = 0; !ok && attempt < 60; ++attempt) {
            delta = (attempt == 0) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))   /* perturb_dec_fact 1/3 */
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            C.ds_shift = g_slack_shift ? delta : 0.0;
            ok = riccati_factor(&C, W, r, delta);
        }
        if (!ok) { status = ST_INERTIA_FAIL; break; }
        if (delta > 0) delta_last = delta;
        riccati_solve(&C, W, g, r);
        double az = dual_steps(&C, W, nU, tau);
        double amax = frac_to_boundary(&C, W, W->dU, W->dS, tau);
        /* filter line search with second-order correction */
        const double phi = barrier_obj(&C, W->X, W->U, W->S);
        double gTd = 0.0;
        for (int k = 0; k <= N; ++k) {
            double z[NZ], gc[NZ];
            stage_z(W->X, W->U, k < N ? k : N - 1, z);
            if (k == N) for (int i = 0; i < NA; ++i) z[i] = W->X[NA * N + i];
            cost_grad(&P, z, Rref + 4 * k, k == N, gc);
            for (int i = 0; i < NA; ++i) gTd += C.sc * gc[i] * W->dX[NA * k + i];
            if (k < N) {
                for (int a = 0; a < NU; ++a) {
                    const int j = NU * k + a;
                    gTd += (C.sc * gc[6 + a] - C.mu / (W->U[j] - lo) + C.mu / (hi - W->U[j])) * W->dU[j];
                }
                for (int i = 0; i < NIQ; ++i) {
                    double sig, psi; slack_terms(&C, W, k, i, &sig, &psi);
                    gTd += psi * W->dS[k][i];
                }
            }
        }
        double amin = gam_th;
        if (gTd < 0) amin = fmin(gam_th, fmin(gam_ph * th / (-gTd), sw_delta * pow(th, s_th) / pow(-gTd, s_ph)));
        if (th == 0.0 && gTd < 0) amin = 0.0;
        amin *= gam_al;
        double alpha = amax, th_t = 0, ph_t = 0;
        int accepted = 0, ftype = 0;
        /* IPOPT tiny-step test: max |d|/(1+|x|) < 10 eps_mach -> accept the full step, unfiltered */
        double tn = 0.0;
        for (int i = 0; i < nA; ++i) tn = fmax(tn, fabs(W->dX[i]) / (1.0 + fabs(W->X[i])));
        for (int j = 0; j < nU; ++j) tn = fmax(tn, fabs(W->dU[j]) / (1.0 + fabs(W->U[j])));
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) tn = fmax(tn, fabs(W->dS[k][i]) / (1.0 + fabs(W->S[k][i])));
        const int tiny = tn < 10.0 * 2.220446049250313e-16;
        for (int ls = 0; ls < 80 && !accepted && !in_soft; ++ls) {
            if (alpha < amin && ls > 0) break;
            for (int i = 0; i < nA; ++i) W->Xt[i] = W->X[i] + alpha * W->dX[i];
            for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + alpha * W->dU[j];
            for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) W->St[k][i] = W->S[k][i] + alpha * W->dS[k][i];
            th_t = residuals(&C, W->Xt, W->Ut, W->St, gt, rt);
            ph_t = barrier_obj(&C, W->Xt, W->Ut, W->St);
            if (tiny) { accepted = 1; ftype = 1; break; }
            accepted = filter_accept(W, nfilt, th_t, ph_t, th, phi, gTd, alpha, th_max, th_min, &ftype);
            if (!accepted && ls == 0 && !(th_t < th) && g_max_soc > 0) {
                /* IPOPT FilterLSAcceptor::TrySecondOrderCorrection: c_soc <- a_soc c_soc + c(trial)
                   (defects and slack rows d(x) - s), starting from c(x) with a_soc = alpha; the
                   corrected step re-uses the factorisation (dual RHS unchanged); at most max_soc
                   passes, continued while theta(trial) <= kappa_soc theta(previous) */
                work_t *Sv = (work_t *)malloc(sizeof(work_t));
                memcpy(Sv, W, sizeof(work_t));
                double asoc = alpha, th_old = 0.0;
                for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) csg[k][i] = g[k][i];
                for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) csr[k][i] = r[k][i];
                for (int c = 0; c < g_max_soc; ++c) {
                    if (c > 0 && !(th_t <= kap_soc * th_old)) break;
                    th_old = th_t;
                    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) csg[k][i] = asoc * csg[k][i] + gt[k][i];
                    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) csr[k][i] = asoc * csr[k][i] + rt[k][i];
                    riccati_solve(&C, W, csg, csr);
                    asoc = frac_to_boundary(&C, W, W->dU, W->dS, tau);
                    for (int i = 0; i < nA; ++i) W->Xt[i] = W->X[i] + asoc * W->dX[i];
                    for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + asoc * W->dU[j];
                    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) W->St[k][i] = W->S[k][i] + asoc * W->dS[k][i];
                    th_t = residuals(&C, W->Xt, W->Ut, W->St, gt, rt);
                    ph_t = barrier_obj(&C, W->Xt, W->Ut, W->St);
                    if (filter_accept(W, nfilt, th_t, ph_t, th, phi, gTd, alpha, th_max, th_min, &ftype)) {
                        /* IPOPT takes the SOC solve as the whole step: the slack-row multipliers, the
                           bound-multiplier directions and their fraction to the boundary follow it */
                        accepted = 1; alpha = asoc; az = dual_steps(&C, W, nU, tau);
                        break;
                    }
                }
                if (!accepted) {    /* back to the plain direction */
                    memcpy(W->dX, Sv->dX, sizeof W->dX); memcpy(W->dU, Sv->dU, sizeof W->dU);
                    memcpy(W->lamp, Sv->lamp, sizeof W->lamp); memcpy(W->dS, Sv->dS, sizeof W->dS);
                }
                free(Sv);
            }
            if (!accepted) alpha *= 0.5;
        }
#ifdef ORACLE_DEBUG
        fprintf(stderr, "it %3d mu %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e az %.3e th %.2e\n",
                it, C.mu, dinf / s_d, pinf, c0 / s_c, delta, amax, alpha, az, th);
#endif
        int soft = 0;
        if (!accepted && g_soft_resto) {
            /* IPOPT's soft restoration phase (lmpc_ipm.c): at most 10 steps; on entry the current point
               goes into the filter */
            if (!in_soft) {
                if (nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
                soft_count = 0;
            }
            if (!(in_soft && ++soft_count > 10)) {
                int orig = 0;
                const double a = soft_resto_step(&C, W, nfilt, th, phi, th_max, tau, pd_error(&C, W, g, r), gt, rt,
                                                 &th_t, &ph_t, &orig);
                if (a > 0.0) {
                    accepted = 1; soft = 1; alpha = a; az = a;
                    in_soft = !orig;
                    if (orig) soft_count = 0;
                }
            }
        }
        if (!accepted && g_resto) {
            /* IPOPT's restoration phase (the start point entered the filter with the soft phase above,
               or enters it here when that phase is off) */
            if (!g_soft_resto && nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
            int rst = ST_LS_FAIL;
            if (!restoration(&C, W, &it, max_iter, tol, th, phi, nfilt, tau, g, r, &rst)) { status = rst; break; }
            th = residuals(&C, W->X, W->U, W->S, g, r);
            in_soft = 0; soft_count = 0;
            continue;
        }
        if (!accepted) { status = ST_LS_FAIL; break; }
        if (!soft && !ftype && nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
        memcpy(W->X, W->Xt, sizeof(double) * nA);
        memcpy(W->U, W->Ut, sizeof(double) * nU);
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) W->S[k][i] = W->St[k][i];
        memcpy(g, gt, sizeof(double) * NA * (N + 1));
        memcpy(r, rt, sizeof(double) * NIQ * N);
        th = th_t;
        for (int i = 0; i < nA; ++i) W->lam[i] += alpha * (W->lamp[i] - W->lam[i]);
        for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
            W->y[k][i] += alpha * W->dy[k][i];
            double s = W->S[k][i];
            if (C.sL[i] > -1e299) {
                double d = s - C.sL[i], v = W->vL[k][i] + az * W->dvL[k][i];
                W->vL[k][i] = fmax(fmin(v, 1e10 * C.mu / d), C.mu / (1e10 * d));
            }
            double d = C.sU[i] - s, v = W->vU[k][i] + az * W->dvU[k][i];
            W->vU[k][i] = fmax(fmin(v, 1e10 * C.mu / d), C.mu / (1e10 * d));
        }
        for (int j = 0; j < nU; ++j) {
            double sl = W->U[j] - lo, su = hi - W->U[j];
            double zl = W->zL[j] + az * W->dzL[j], zu = W->zU[j] + az * W->dzU[j];
            W->zL[j] = fmax(fmin(zl, 1e10 * C.mu / sl), C.mu / (1e10 * sl));
            W->zU[j] = fmax(fmin(zu, 1e10 * C.mu / su), C.mu / (1e10 * su));
        }
    }
    if (iters_out) *iters_out = it;
    if (u0) { u0[0] = W->U[0]; u0[1] = W->U[1]; }
    if (fval) *fval = objective(&P, W->X, W->U, Rref);
    if (w_out) {
        for (int k = 0; k <= N; ++k) for (int i = 0; i < 4; ++i) w_out[4 * k + i] = W->X[NA * k + i];
        memcpy(w_out + 4 * (N + 1), W->U, sizeof(double) * nU);
    }
    free(g); free(r); free(gt); free(rt); free(csg); free(csr);
    free(W);
    return status;
}

/* RLS.update (np_mpc...:17-27) for one axis, p = 7: theta[7], P[7x7] updated in place */
void oracle_rls_update(double *theta, double *P, const double *phi, double y, double lam) {
    double Pphi[7], denom = lam, err = y;
    for (int i = 0; i < 7; ++i) { double s = 0; for (int j = 0; j < 7; ++j) s += P[7 * i + j] * phi[j]; Pphi[i] = s; }
    for (int i = 0; i < 7; ++i) denom += phi[i] * Pphi[i];
    double K[7];
    for (int i = 0; i < 7; ++i) { K[i] = Pphi[i] / denom; err -= phi[i] * theta[i]; }
    for (int i = 0; i < 7; ++i) theta[i] += K[i] * err;
    double phiP[7];
    for (int j = 0; j < 7; ++j) { double s = 0; for (int i = 0; i < 7; ++i) s += phi[i] * P[7 * i + j]; phiP[j] = s; }
    for (int i = 0; i < 7; ++i) for (int j = 0; j < 7; ++j) P[7 * i + j] = (P[7 * i + j] - K[i] * phiP[j]) / lam;
}

/* batched driver (prm rows of 10, theta rows of 14, Rref rows of 4(N+1), w_init rows of 4(N+1)+2N) */
int oracle_rmpc_solve_batch(int B, int N, double Ts, const double *x0, const double *u_prev, const double *theta,
                            const double *Rref, const double *prm, const double *w_init, int max_iter, double tol,
                            int nthreads, double *u0, double *f, double *w_out, int32_t *status, int32_t *iters) {
    const int nw = 4 * (N + 1) + 2 * N;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int b = 0; b < B; ++b) {
        int32_t itb = 0;
        status[b] = oracle_rmpc_solve(N, Ts, x0 + 4 * b, u_prev + 2 * b, theta + 14 * b, Rref + 4 * (N + 1) * b,
                                      prm + 10 * b, w_init ? w_init + (size_t)nw * b : NULL, max_iter, tol,
                                      u0 + 2 * b, f + b, w_out ? w_out + (size_t)nw * b : NULL, &itb);
        iters[b] = itb;
    }
    (void)nthreads;
    return 0;
}
