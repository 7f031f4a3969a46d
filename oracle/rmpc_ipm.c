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

typedef struct {
    const prob_t *P; const double *x0, *up0, *R; double sc, mu, lo, hi;
    double sL[NIQ], sU[NIQ];                            /* relaxed slack bounds (+-inf as +-1e300) */
} ctx_t;

enum { ST_SOLVED = 0, ST_MAXITER = -1, ST_LS_FAIL = -2, ST_INERTIA_FAIL = -3, ST_BAD_INPUT = -10 };

/* IPOPT bound_relax_factor (1e-8 default); the golden generator sets 0 to solve the exact NLP */
static double g_relax = 1e-8;
void oracle_rmpc_set_relax(double r) { g_relax = r; }
/* second-order correction on/off (IPOPT default on; off mirrors the GPU kernel's line search) */
static int g_max_soc = 4;      /* IPOPT max_soc (second-order corrections per line search) */
void oracle_rmpc_set_soc(int max_soc) { g_max_soc = max_soc < 0 ? 0 : max_soc; }

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

/* Stage Hessian (8x8 over z) incl. slack elimination C^T Sigma C and box Sigma; gradient incl. C^T(Sigma r + psi) */
static void stage_qp(const ctx_t *C, const work_t *W, int k, double rr[NIQ], double delta, double Hq[NZ][NZ], double *gq) {
    const prob_t *P = C->P; const double sc = C->sc;
    double z[NZ];
    stage_z(W->X, W->U, k, z);
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
        for (int a = 0; a < NZ; ++a) {
            if (cr[a] == 0.0) continue;
            for (int b = 0; b < NZ; ++b) Hq[a][b] += sig * cr[a] * cr[b];
            gq[a] += cr[a] * (sig * rr[i] + psi);
        }
    }
    for (int a = 0; a < NZ; ++a) Hq[a][a] += delta;
}

static int riccati_factor(const ctx_t *C, work_t *W, double r[][NIQ], double delta) {
    const prob_t *P = C->P; const int N = P->N; const double sc = C->sc;
    double (*Pn)[NA] = W->Pm[N];
    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) Pn[i][j] = 0.0;
    Pn[0][0] = Pn[2][2] = sc * 2 * P->Qp; Pn[1][1] = Pn[3][3] = sc * 2 * P->Qv;
    for (int i = 0; i < NA; ++i) Pn[i][i] += delta;
    for (int k = N - 1; k >= 0; --k) {
        double Hq[NZ][NZ], gq[NZ];
        stage_qp(C, W, k, r[k], delta, Hq, gq);
        for (int j = 0; j < NZ; ++j) W->grad[k][j] = gq[j];
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = W->Pm[k + 1];
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
    return 1;
}

/* vector pass + forward sweep for defect RHS rg (J d = -rg) and inequality residuals r */
static void riccati_solve(const ctx_t *C, work_t *W, double rg[][NA], double r[][NIQ]) {
    const prob_t *P = C->P; const int N = P->N;
    double zN[NZ], gN[NZ];
    stage_z(W->X, W->U, N, zN);   /* U beyond N unused for terminal */
    cost_grad(P, zN, C->R + 4 * N, 1, gN);
    for (int i = 0; i < NA; ++i) W->pv[N][i] = C->sc * gN[i];
    for (int k = N - 1; k >= 0; --k) {
        double Hq[NZ][NZ], gq[NZ];
        stage_qp(C, W, k, r[k], 0.0, Hq, gq);   /* only the gradient is used */
        double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = W->Pm[k + 1], *pp = W->pv[k + 1];
        double hh[NA], qx[NA], qu[NU], kf[2];
        for (int i = 0; i < NA; ++i) { double s = pp[i]; for (int m = 0; m < NA; ++m) s -= Pp[i][m] * rg[k + 1][m]; hh[i] = s; }
        for (int i = 0; i < NA; ++i) { double s = gq[i]; for (int m = 0; m < NA; ++m) s += A[m][i] * hh[m]; qx[i] = s; }
        for (int a = 0; a < NU; ++a) { double s = gq[NA + a]; for (int m = 0; m < NA; ++m) s += Bm[m][a] * hh[m]; qu[a] = s; }
        chol2_solve(W->Lq[k], qu, kf);
        W->kff[k][0] = -kf[0]; W->kff[k][1] = -kf[1];
        for (int i = 0; i < NA; ++i) W->pv[k][i] = qx[i] + W->Qux[k][0][i] * W->kff[k][0] + W->Qux[k][1][i] * W->kff[k][1];
    }
    for (int i = 0; i < NA; ++i) W->dX[i] = -rg[0][i];
    for (int k = 0; k < N; ++k) {
        double *dx = W->dX + NA * k, *du = W->dU + NU * k;
        for (int a = 0; a < NU; ++a) { double s = W->kff[k][a]; for (int i = 0; i < NA; ++i) s += W->K[k][a][i] * dx[i]; du[a] = s; }
        for (int i = 0; i < NA; ++i) {
            double s = -rg[k + 1][i];
            for (int m = 0; m < NA; ++m) s += W->A[k][i][m] * dx[m];
            for (int a = 0; a < NU; ++a) s += W->Bm[k][i][a] * du[a];
            W->dX[NA * (k + 1) + i] = s;
        }
    }
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NA; ++i) {
        double s = W->pv[k][i]; for (int m = 0; m < NA; ++m) s += W->Pm[k][i][m] * W->dX[NA * k + m];
        W->lamp[NA * k + i] = -s;
    }
    /* slack steps ds = C dz + r, multiplier steps */
    for (int k = 0; k < N; ++k) for (int i = 0; i < NIQ; ++i) {
        double cr[NZ], dz[NZ], sig, psi, cdz = 0.0;
        iq_row(i, cr);
        for (int a = 0; a < NA; ++a) dz[a] = W->dX[NA * k + a];
        dz[6] = W->dU[NU * k]; dz[7] = W->dU[NU * k + 1];
        for (int a = 0; a < NZ; ++a) cdz += cr[a] * dz[a];
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
        /* dy from the eliminated system: y + dy = Sigma*ds + psi' with psi' = -mu/(s-sL)+mu/(sU-s) */
        W->dy[k][i] = sig * ds + psi - W->y[k][i];
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
    int nfilt = 0, status = ST_MAXITER, it;
    double delta_last = 0.0;
    for (it = 0; it < max_iter; ++it) {
        for (int k = 0; k < N; ++k) {
            double xn[4], nl[4], J[4][NZ];
            for (int i = 0; i < 4; ++i) nl[i] = -W->lam[NA * (k + 1) + i];
            rk4_derivs(&P, W->X + NA * k, W->U + NU * k, nl, xn, J, W->Hs[k]);
            for (int i = 0; i < NA; ++i) { for (int j = 0; j < NA; ++j) W->A[k][i][j] = 0.0; W->Bm[k][i][0] = W->Bm[k][i][1] = 0.0; }
            for (int i = 0; i < 4; ++i) { for (int j = 0; j < 4; ++j) W->A[k][i][j] = J[i][j]; W->Bm[k][i][0] = J[i][6]; W->Bm[k][i][1] = J[i][7]; }
            W->Bm[k][4][0] = 1.0; W->Bm[k][5][1] = 1.0;
        }
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
            nfilt = 0;
        }
        const double tau = fmax(0.99, 1.0 - C.mu);
        double delta = 0.0;
        int ok = riccati_factor(&C, W, r, 0.0);
        for (int attempt = 0; !ok && attempt < 60; ++attempt) {
            delta = (attempt == 0) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))   /* perturb_dec_fact 1/3 */
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
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
        for (int ls = 0; ls < 80 && !accepted; ++ls) {
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
        if (!accepted) { status = ST_LS_FAIL; break; }
        if (!ftype && nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
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
