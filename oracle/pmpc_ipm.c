/*
 * pmpc_ipm.c -- CPU oracle for the PMPC tray-tilt NMPC solve.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load the library built from this file, and
 * only as the checker / the timed CPU baseline ("kind": "port").  The shipped
 * solver (dart-dual-arm-non-prehensile-manipulation_amd/csrc) never links it.
 *
 * What it restates (paths relative to the reference root):
 *   - the NLP of PMPC/src/controller/mpc_3d.py:28-85 (dynamics :87-97, RK4
 *     :99-104, multiple-shooting defects :37,:48, cost :44-46,:63-66,
 *     box bounds :71-79), on the FULL 6-state model (x, y and z sub-states);
 *   - the cold start of PMPC.solve (:123) and its outputs (:133-138);
 *   - IPOPT's primal-dual barrier method as configured by mpc_3d.py:82
 *     (all options at IPOPT defaults): monotone mu (mu_init 0.1, kappa_mu 0.2,
 *     theta_mu 1.5, kappa_eps 10), fraction-to-boundary tau = max(0.99, 1-mu),
 *     bound_relax_factor 1e-8, bound multipliers initialised to 1, equality
 *     multipliers initialised to IPOPT's least-square estimate
 *     (constr_mult_init_max 1000), gradient-based objective scaling
 *     (nlp_scaling_max_gradient 100), exact Lagrangian Hessian, inertia
 *     correction (delta_w first 1e-4, x100 first time / x8 afterwards, reuse
 *     last/3), the filter line search of Waechter & Biegler 2006 (Alg. A,
 *     IPOPT's constants) with the second-order correction (max_soc 4).
 *   Deviations (documented in DESIGN.md): the KKT system is solved by an
 *   exact stage-wise Riccati recursion instead of MUMPS (same Newton step up
 *   to rounding); no restoration phase (status -2 where IPOPT would enter it).
 *
 * Exact first/second derivatives of the RK4 map are taken with second-order
 * forward "jets" (value, gradient, Hessian in the 8 stage variables x,u).
 *
 * Parity status: CasADi/IPOPT cannot run in this image, so this oracle is
 * pinned against committed golden fixtures produced by two independent
 * solvers (tests/golden/make_goldens.py) and the numpy KKT certificate.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* IPOPT Compare_le: lhs <= rhs up to 10 machine epsilons of |base| */
#define LE(l, r, b) ((l) - (r) <= 10.0 * 2.220446049250313e-16 * fabs(b))

/* second-order correction on/off (IPOPT default on; the GPU kernel mirrors the off path) */
static int g_max_soc = 4;      /* IPOPT max_soc (second-order corrections per line search) */
void oracle_pmpc_set_soc(int max_soc) { g_max_soc = max_soc < 0 ? 0 : max_soc; }
#ifdef ORACLE_DEBUG
#include <stdio.h>
#endif
#ifdef _OPENMP
#include <omp.h>
#endif

#define NX 6
#define NU 2
#define NZ 8
#define NH 36
#define NMAX 128

typedef struct { double v, d[NZ], h[NH]; } jet;

static inline int hx(int i, int j) { if (i < j) { int t = i; i = j; j = t; } return i * (i + 1) / 2 + j; }

static inline jet jconst(double c) { jet r; memset(&r, 0, sizeof r); r.v = c; return r; }
static inline jet jvar(double v, int i) { jet r = jconst(v); r.d[i] = 1.0; return r; }
static inline jet jaxpy(jet a, double s, jet b) {           /* a + s*b */
    jet r; r.v = a.v + s * b.v;
    for (int i = 0; i < NZ; ++i) r.d[i] = a.d[i] + s * b.d[i];
    for (int i = 0; i < NH; ++i) r.h[i] = a.h[i] + s * b.h[i];
    return r;
}
static inline jet jscale(jet a, double s) { jet r; r.v = s * a.v;
    for (int i = 0; i < NZ; ++i) r.d[i] = s * a.d[i];
    for (int i = 0; i < NH; ++i) r.h[i] = s * a.h[i];
    return r; }
static inline jet jsin(jet a) {
    double s = sin(a.v), c = cos(a.v); jet r; r.v = s;
    for (int i = 0; i < NZ; ++i) r.d[i] = c * a.d[i];
    for (int i = 0; i < NZ; ++i) for (int j = 0; j <= i; ++j) r.h[hx(i, j)] = c * a.h[hx(i, j)] - s * a.d[i] * a.d[j];
    return r;
}
static inline jet jsq(jet a) {
    jet r; r.v = a.v * a.v;
    for (int i = 0; i < NZ; ++i) r.d[i] = 2 * a.v * a.d[i];
    for (int i = 0; i < NZ; ++i) for (int j = 0; j <= i; ++j) r.h[hx(i, j)] = 2 * a.v * a.h[hx(i, j)] + 2 * a.d[i] * a.d[j];
    return r;
}

typedef struct { int N; double Ts, g, mu, Qp, Qv, R, ulo, uhi; } prob_t;

/* P1  mpc_3d.py:87-97 on jets */
static void dyn_jet(const prob_t *P, const jet *x, const jet *u, jet *xd) {
    jet ax = jaxpy(jscale(jsin(u[0]), P->g), -P->mu, x[1]);           /* :91 */
    jet ay = jaxpy(jscale(jsin(u[1]), P->g), -P->mu, x[3]);           /* :92 */
    jet vzn = jscale(jaxpy(jsq(u[0]), 1.0, jsq(u[1])), -P->g);         /* :93 */
    jet az = jscale(jaxpy(vzn, -1.0, x[5]), 1.0 / P->Ts);              /* :95 */
    xd[0] = x[1]; xd[1] = ax; xd[2] = x[3]; xd[3] = ay; xd[4] = vzn; xd[5] = az;   /* :97 */
}

/* P1 values only */
static void dyn_val(const prob_t *P, const double *x, const double *u, double *xd) {
    double ax = P->g * sin(u[0]) - P->mu * x[1];
    double ay = P->g * sin(u[1]) - P->mu * x[3];
    double vzn = -P->g * (u[0] * u[0] + u[1] * u[1]);
    double az = (vzn - x[5]) / P->Ts;
    xd[0] = x[1]; xd[1] = ax; xd[2] = x[3]; xd[3] = ay; xd[4] = vzn; xd[5] = az;
}

/* P2  mpc_3d.py:99-104 */
static void rk4_val(const prob_t *P, const double *x, const double *u, double *xn) {
    double k1[NX], k2[NX], k3[NX], k4[NX], y[NX], h = P->Ts;
    dyn_val(P, x, u, k1);
    for (int i = 0; i < NX; ++i) y[i] = x[i] + h / 2 * k1[i];
    dyn_val(P, y, u, k2);
    for (int i = 0; i < NX; ++i) y[i] = x[i] + h / 2 * k2[i];
    dyn_val(P, y, u, k3);
    for (int i = 0; i < NX; ++i) y[i] = x[i] + h * k3[i];
    dyn_val(P, y, u, k4);
    for (int i = 0; i < NX; ++i) xn[i] = x[i] + h / 6 * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
}

/* RK4 on jets: value, Jacobian [A|B] and lam-contracted Hessian (8x8) of sum_i lam_i xn_i */
static void rk4_derivs(const prob_t *P, const double *x, const double *u, const double *lam,
                       double *xn, double A[NX][NX], double Bm[NX][NU], double H[NZ][NZ]) {
    jet xj[NX], uj[NU], k1[NX], k2[NX], k3[NX], k4[NX], y[NX];
    double h = P->Ts;
    for (int i = 0; i < NX; ++i) xj[i] = jvar(x[i], i);
    for (int i = 0; i < NU; ++i) uj[i] = jvar(u[i], NX + i);
    dyn_jet(P, xj, uj, k1);
    for (int i = 0; i < NX; ++i) y[i] = jaxpy(xj[i], h / 2, k1[i]);
    dyn_jet(P, y, uj, k2);
    for (int i = 0; i < NX; ++i) y[i] = jaxpy(xj[i], h / 2, k2[i]);
    dyn_jet(P, y, uj, k3);
    for (int i = 0; i < NX; ++i) y[i] = jaxpy(xj[i], h, k3[i]);
    dyn_jet(P, y, uj, k4);
    for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) H[a][b] = 0.0;
    for (int i = 0; i < NX; ++i) {
        jet s = jaxpy(jaxpy(jaxpy(k1[i], 2.0, k2[i]), 2.0, k3[i]), 1.0, k4[i]);
        jet r = jaxpy(xj[i], h / 6, s);
        xn[i] = r.v;
        for (int j = 0; j < NX; ++j) A[i][j] = r.d[j];
        for (int j = 0; j < NU; ++j) Bm[i][j] = r.d[NX + j];
        if (lam) for (int a = 0; a < NZ; ++a) for (int b = 0; b < NZ; ++b) H[a][b] += lam[i] * r.h[hx(a, b)];
    }
}

/* stage cost gradient (mpc_3d.py:44-46; terminal :63-66 has the same state weights) */
static void cost_grad_x(const prob_t *P, const double *x, const double *ref, double *gx) {
    gx[0] = 2 * P->Qp * (x[0] - ref[0]); gx[1] = 2 * P->Qv * (x[1] - ref[1]);
    gx[2] = 2 * P->Qp * (x[2] - ref[2]); gx[3] = 2 * P->Qv * (x[3] - ref[3]);
    gx[4] = 0.0; gx[5] = 0.0;
}
static double objective(const prob_t *P, const double *X, const double *U, const double *ref) {
    double f = 0.0;
    for (int k = 0; k <= P->N; ++k) {
        const double *x = X + NX * k;
        double ep = (x[0] - ref[0]) * (x[0] - ref[0]) + (x[2] - ref[2]) * (x[2] - ref[2]);
        double ev = (x[1] - ref[1]) * (x[1] - ref[1]) + (x[3] - ref[3]) * (x[3] - ref[3]);
        f += P->Qp * ep + P->Qv * ev;
        if (k < P->N) f += P->R * (U[NU * k] * U[NU * k] + U[NU * k + 1] * U[NU * k + 1]);
    }
    return f;
}

/* small dense helpers */
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

typedef struct {
    double X[NX * (NMAX + 1)], U[NU * NMAX], lam[NX * (NMAX + 1)], zL[NU * NMAX], zU[NU * NMAX];
    double A[NMAX][NX][NX], Bm[NMAX][NX][NU], H[NMAX][NZ][NZ], c[NMAX][NX];
    /* Riccati factorisation */
    double Lq[NMAX][3], Qux[NMAX][NU][NX], K[NMAX][NU][NX], Pm[NMAX + 1][NX][NX];
    /* step */
    double kff[NMAX][NU], pv[NMAX + 1][NX];
    double dX[NX * (NMAX + 1)], dU[NU * NMAX], lamp[NX * (NMAX + 1)], dzL[NU * NMAX], dzU[NU * NMAX];
    double Xt[NX * (NMAX + 1)], Ut[NU * NMAX], csoc[NMAX + 1][NX], gt[NMAX + 1][NX];
    double filt_th[256], filt_ph[256];
} work_t;

enum { ST_SOLVED = 0, ST_MAXITER = -1, ST_LS_FAIL = -2, ST_INERTIA_FAIL = -3, ST_BAD_INPUT = -10 };

typedef struct {
    const prob_t *P; const double *state, *ref; double sc, mu, lo, hi; int N;
} ctx_t;

/* constraint residuals g (N+1 blocks) at (X,U); returns l1 norm */
static double constraints(const ctx_t *C, const double *X, const double *U, double g[][NX]) {
    double th = 0.0;
    for (int i = 0; i < NX; ++i) { g[0][i] = X[i] - C->state[i]; th += fabs(g[0][i]); }     /* mpc_3d.py:37 */
    for (int k = 0; k < C->N; ++k) {
        double xn[NX];
        rk4_val(C->P, X + NX * k, U + NU * k, xn);
        for (int i = 0; i < NX; ++i) { g[k + 1][i] = X[NX * (k + 1) + i] - xn[i]; th += fabs(g[k + 1][i]); }  /* :48 */
    }
    return th;
}

/* barrier objective phi_mu (scaled); +inf outside the box */
static double barrier_obj(const ctx_t *C, const double *X, const double *U) {
    double phi = C->sc * objective(C->P, X, U, C->ref);
    for (int j = 0; j < NU * C->N; ++j) {
        double sl = U[j] - C->lo, su = C->hi - U[j];
        if (!(sl > 0) || !(su > 0)) return INFINITY;
        phi -= C->mu * (log(sl) + log(su));
    }
    return phi;
}

/* Riccati factorisation of the KKT matrix (Hessian blocks + delta*I).  Returns 0 on wrong inertia. */
static int riccati_factor(const ctx_t *C, work_t *W, double delta) {
    const prob_t *P = C->P; const int N = C->N; const double sc = C->sc;
    double (*Pn)[NX] = W->Pm[N];
    for (int i = 0; i < NX; ++i) for (int j = 0; j < NX; ++j) Pn[i][j] = 0.0;
    Pn[0][0] = Pn[2][2] = sc * 2 * P->Qp; Pn[1][1] = Pn[3][3] = sc * 2 * P->Qv;
    for (int i = 0; i < NX; ++i) Pn[i][i] += delta;
    for (int k = N - 1; k >= 0; --k) {
        double (*A)[NX] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Hk)[NZ] = W->H[k];
        double (*Pp)[NX] = W->Pm[k + 1];
        double PA[NX][NX], PB[NX][NU], Qxx[NX][NX], Quu[NU][NU];
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) { double s = 0; for (int m = 0; m < NX; ++m) s += Pp[i][m] * A[m][j]; PA[i][j] = s; }
            for (int j = 0; j < NU; ++j) { double s = 0; for (int m = 0; m < NX; ++m) s += Pp[i][m] * Bm[m][j]; PB[i][j] = s; }
        }
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) { double s = Hk[i][j]; for (int m = 0; m < NX; ++m) s += A[m][i] * PA[m][j]; Qxx[i][j] = s; }
            Qxx[i][i] += delta;
        }
        Qxx[0][0] += sc * 2 * P->Qp; Qxx[2][2] += sc * 2 * P->Qp; Qxx[1][1] += sc * 2 * P->Qv; Qxx[3][3] += sc * 2 * P->Qv;
        for (int a = 0; a < NU; ++a) {
            const int j = NU * k + a;
            double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
            for (int i = 0; i < NX; ++i) { double s = Hk[NX + a][i]; for (int m = 0; m < NX; ++m) s += Bm[m][a] * PA[m][i]; W->Qux[k][a][i] = s; }
            for (int b = 0; b < NU; ++b) { double s = Hk[NX + a][NX + b]; for (int m = 0; m < NX; ++m) s += Bm[m][a] * PB[m][b]; Quu[a][b] = s; }
            Quu[a][a] += sc * 2 * P->R + W->zL[j] / sl + W->zU[j] / su + delta;
        }
        if (!chol2(Quu[0][0], 0.5 * (Quu[0][1] + Quu[1][0]), Quu[1][1], W->Lq[k])) return 0;
        for (int i = 0; i < NX; ++i) {
            double b[2] = {W->Qux[k][0][i], W->Qux[k][1][i]}, x[2];
            chol2_solve(W->Lq[k], b, x); W->K[k][0][i] = -x[0]; W->K[k][1][i] = -x[1];
        }
        for (int i = 0; i < NX; ++i) for (int j = 0; j < NX; ++j)
            W->Pm[k][i][j] = Qxx[i][j] + W->Qux[k][0][i] * W->K[k][0][j] + W->Qux[k][1][i] * W->K[k][1][j];
        for (int i = 0; i < NX; ++i) for (int j = 0; j < i; ++j) { double s = 0.5 * (W->Pm[k][i][j] + W->Pm[k][j][i]); W->Pm[k][i][j] = W->Pm[k][j][i] = s; }
    }
    return 1;
}

/* Solve the factorised KKT system for constraint RHS rg (the linearised constraints read
 * J d = -rg) and the barrier-gradient RHS at the current point.  Fills dX, dU, lamp. */
static void riccati_solve(const ctx_t *C, work_t *W, double rg[][NX]) {
    const prob_t *P = C->P; const int N = C->N; const double sc = C->sc, mu = C->mu;
    double gx[NX];
    cost_grad_x(P, W->X + NX * N, C->ref, gx);
    for (int i = 0; i < NX; ++i) W->pv[N][i] = sc * gx[i];
    for (int k = N - 1; k >= 0; --k) {
        double (*A)[NX] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NX] = W->Pm[k + 1], *pp = W->pv[k + 1];
        double h[NX], qx[NX], qu[NU], kf[2];
        for (int i = 0; i < NX; ++i) { double s = pp[i]; for (int m = 0; m < NX; ++m) s -= Pp[i][m] * rg[k + 1][m]; h[i] = s; }
        cost_grad_x(P, W->X + NX * k, C->ref, gx);
        for (int i = 0; i < NX; ++i) { double s = sc * gx[i]; for (int m = 0; m < NX; ++m) s += A[m][i] * h[m]; qx[i] = s; }
        for (int a = 0; a < NU; ++a) {
            const int j = NU * k + a;
            double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
            double s = sc * 2 * P->R * W->U[j] - mu / sl + mu / su;
            for (int m = 0; m < NX; ++m) s += Bm[m][a] * h[m];
            qu[a] = s;
        }
        chol2_solve(W->Lq[k], qu, kf);
        W->kff[k][0] = -kf[0]; W->kff[k][1] = -kf[1];
        for (int i = 0; i < NX; ++i) W->pv[k][i] = qx[i] + W->Qux[k][0][i] * W->kff[k][0] + W->Qux[k][1][i] * W->kff[k][1];
    }
    for (int i = 0; i < NX; ++i) W->dX[i] = -rg[0][i];
    for (int k = 0; k < N; ++k) {
        double *dx = W->dX + NX * k, *du = W->dU + NU * k;
        for (int a = 0; a < NU; ++a) { double s = W->kff[k][a]; for (int i = 0; i < NX; ++i) s += W->K[k][a][i] * dx[i]; du[a] = s; }
        for (int i = 0; i < NX; ++i) {
            double s = -rg[k + 1][i];
            for (int m = 0; m < NX; ++m) s += W->A[k][i][m] * dx[m];
            for (int a = 0; a < NU; ++a) s += W->Bm[k][i][a] * du[a];
            W->dX[NX * (k + 1) + i] = s;
        }
    }
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NX; ++i) {
        double s = W->pv[k][i]; for (int m = 0; m < NX; ++m) s += W->Pm[k][i][m] * W->dX[NX * k + m];
        W->lamp[NX * k + i] = -s;
    }
}

/* largest alpha in (0,1] keeping U + alpha dU strictly inside by fraction tau */
static double frac_to_boundary(const ctx_t *C, const work_t *W, const double *dU, double tau) {
    double a = 1.0;
    for (int j = 0; j < NU * C->N; ++j) {
        double sl = W->U[j] - C->lo, su = C->hi - W->U[j];
        if (dU[j] < 0) a = fmin(a, -tau * sl / dU[j]);
        if (dU[j] > 0) a = fmin(a, tau * su / dU[j]);
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

/* IPOPT's least-square estimate of the equality multipliers at the starting point
 * (DefaultIterateInitializer::least_square_mults -> LeastSquareMultipliers::CalculateMultipliers, on by
 * default with constr_mult_init_max = 1000): the augmented system [I J^T; J 0] [d; y] = [-r; 0] with
 * r = grad f (scaled) - z_L + z_U, i.e. y minimises ||r + J^T y||.  With the stage structure of the
 * shooting defects (J d = 0: d_x0 = 0, d_x(k+1) = A_k d_xk + B_k d_uk) it is an LQR with unit weights:
 * y_k = -(P_k dx_k + p_k).  Uses W->A, W->Bm of the starting point; returns max |y|. */
static double ls_multipliers(const ctx_t *C, work_t *W, double *y) {
    const prob_t *P = C->P; const int N = C->N; const double sc = C->sc;
    double Pm[NX][NX], pv[NX], gx[NX];
    static __thread double Ks[NMAX][NU][NX], ks[NMAX][NU], Ps[NMAX + 1][NX][NX], ps[NMAX + 1][NX];
    cost_grad_x(P, W->X + NX * N, C->ref, gx);
    for (int i = 0; i < NX; ++i) { for (int j = 0; j < NX; ++j) Pm[i][j] = (i == j); pv[i] = sc * gx[i]; }
    memcpy(Ps[N], Pm, sizeof Pm); memcpy(ps[N], pv, sizeof pv);
    for (int k = N - 1; k >= 0; --k) {
        double (*A)[NX] = W->A[k], (*Bm)[NU] = W->Bm[k];
        double PA[NX][NX], PB[NX][NU], Qxx[NX][NX], Qux[NU][NX], Quu[NU][NU], qx[NX], qu[NU], L[3] = {1, 0, 1};
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) { double t = 0; for (int m = 0; m < NX; ++m) t += Ps[k + 1][i][m] * A[m][j]; PA[i][j] = t; }
            for (int j = 0; j < NU; ++j) { double t = 0; for (int m = 0; m < NX; ++m) t += Ps[k + 1][i][m] * Bm[m][j]; PB[i][j] = t; }
        }
        cost_grad_x(P, W->X + NX * k, C->ref, gx);
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) { double t = (i == j); for (int m = 0; m < NX; ++m) t += A[m][i] * PA[m][j]; Qxx[i][j] = t; }
            double t = sc * gx[i]; for (int m = 0; m < NX; ++m) t += A[m][i] * ps[k + 1][m]; qx[i] = t;
        }
        for (int a = 0; a < NU; ++a) {
            const int j = NU * k + a;
            for (int i = 0; i < NX; ++i) { double t = 0; for (int m = 0; m < NX; ++m) t += Bm[m][a] * PA[m][i]; Qux[a][i] = t; }
            for (int c = 0; c < NU; ++c) { double t = (a == c); for (int m = 0; m < NX; ++m) t += Bm[m][a] * PB[m][c]; Quu[a][c] = t; }
            double t = sc * 2 * P->R * W->U[j] - W->zL[j] + W->zU[j];
            for (int m = 0; m < NX; ++m) t += Bm[m][a] * ps[k + 1][m];
            qu[a] = t;
        }
        chol2(Quu[0][0], 0.5 * (Quu[0][1] + Quu[1][0]), Quu[1][1], L);      /* Quu >= I: positive definite */
        double x2[2];
        chol2_solve(L, qu, x2); ks[k][0] = -x2[0]; ks[k][1] = -x2[1];
        for (int i = 0; i < NX; ++i) {
            double b2[2] = {Qux[0][i], Qux[1][i]};
            chol2_solve(L, b2, x2); Ks[k][0][i] = -x2[0]; Ks[k][1][i] = -x2[1];
        }
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) Ps[k][i][j] = Qxx[i][j] + Qux[0][i] * Ks[k][0][j] + Qux[1][i] * Ks[k][1][j];
            ps[k][i] = qx[i] + Qux[0][i] * ks[k][0] + Qux[1][i] * ks[k][1];
        }
        for (int i = 0; i < NX; ++i) for (int j = 0; j < i; ++j) { const double t = 0.5 * (Ps[k][i][j] + Ps[k][j][i]); Ps[k][i][j] = Ps[k][j][i] = t; }
    }
    double dx[NX] = {0}, ymax = 0.0;
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < NX; ++i) {
            double t = ps[k][i]; for (int m = 0; m < NX; ++m) t += Ps[k][i][m] * dx[m];
            y[NX * k + i] = -t; ymax = fmax(ymax, fabs(t));
        }
        if (k == N) break;
        double du[NU], dn[NX];
        for (int a = 0; a < NU; ++a) { double t = ks[k][a]; for (int i = 0; i < NX; ++i) t += Ks[k][a][i] * dx[i]; du[a] = t; }
        for (int i = 0; i < NX; ++i) {
            double t = 0; for (int m = 0; m < NX; ++m) t += W->A[k][i][m] * dx[m];
            for (int a = 0; a < NU; ++a) t += W->Bm[k][i][a] * du[a];
            dn[i] = t;
        }
        memcpy(dx, dn, sizeof dx);
    }
    return ymax;
}

static double g_mult_init_max = 1e3;   /* IPOPT constr_mult_init_max (default 1000; 0 = zero multipliers) */
void oracle_pmpc_set_mult_init_max(double m) { g_mult_init_max = m; }

int oracle_pmpc_solve(int N, double Ts, const double *state, const double *target, const double *prm,
                      const double *w_init, int max_iter, double tol,
                      double *u0, double *fval, double *w_out, int32_t *iters_out) {
    if (N < 1 || N > NMAX || !(Ts > 0) || !(prm[5] > prm[4])) return ST_BAD_INPUT;
    work_t *W = (work_t *)calloc(1, sizeof(work_t));
    if (!W) return ST_BAD_INPUT;
    prob_t P = {N, Ts, -9.81, prm[0], prm[1], prm[2], prm[3], prm[4], prm[5]};
    /* IPOPT bound_relax_factor = 1e-8 */
    const double lo = P.ulo - 1e-8 * fmax(1.0, fabs(P.ulo)), hi = P.uhi + 1e-8 * fmax(1.0, fabs(P.uhi));
    const double mu_min = tol / 10, kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, s_max = 100.0;
    /* filter line-search constants (IPOPT defaults) */
    const double gam_th = 1e-5, gam_ph = 1e-8, sw_delta = 1.0, s_th = 1.1, s_ph = 2.3, gam_al = 0.05, kap_soc = 0.99;
    const int nU = NU * N, ng = NX * (N + 1);

    /* initial point: cold start (mpc_3d.py:123) or caller warm start; bound push kappa_1 = kappa_2 = 1e-2 */
    for (int k = 0; k <= N; ++k) for (int i = 0; i < NX; ++i) W->X[NX * k + i] = w_init ? w_init[NX * k + i] : state[i];
    for (int j = 0; j < nU; ++j) {
        double u = w_init ? w_init[NX * (N + 1) + j] : 0.0;
        double pl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo)), pu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
        if (u < lo + pl) u = lo + pl;
        if (u > hi - pu) u = hi - pu;
        W->U[j] = u; W->zL[j] = 1.0; W->zU[j] = 1.0;
    }
    /* gradient-based objective scaling (nlp_scaling_max_gradient = 100) */
    double gmax = 0.0;
    for (int k = 0; k <= N; ++k) {
        double gx[NX]; cost_grad_x(&P, W->X + NX * k, target, gx);
        for (int i = 0; i < NX; ++i) gmax = fmax(gmax, fabs(gx[i]));
        if (k < N) for (int j = 0; j < NU; ++j) gmax = fmax(gmax, fabs(2 * P.R * W->U[NU * k + j]));
    }
    ctx_t C = {&P, state, target, gmax > 100.0 ? 100.0 / gmax : 1.0, 0.1, lo, hi, N};
    double (*g)[NX] = (double (*)[NX])calloc(N + 1, sizeof(double[NX]));

    if (g_mult_init_max > 0.0) {
        for (int k = 0; k < N; ++k) {
            double xn[NX], nl[NX] = {0};
            rk4_derivs(&P, W->X + NX * k, W->U + NU * k, nl, xn, W->A[k], W->Bm[k], W->H[k]);
        }
        const double ymax = ls_multipliers(&C, W, W->lam);
        if (!(ymax <= g_mult_init_max)) memset(W->lam, 0, sizeof(double) * ng);     /* constr_mult_init_max */
    }
    double th = constraints(&C, W->X, W->U, g);
    const double th_max = 1e4 * fmax(1.0, th), th_min = 1e-4 * fmax(1.0, th);
    int nfilt = 0, status = ST_MAXITER, it;
    double delta_last = 0.0;
    for (it = 0; it < max_iter; ++it) {
        /* ---- derivatives at the current point ------------------------------- */
        for (int k = 0; k < N; ++k) {
            double xn[NX], nl[NX];
            for (int i = 0; i < NX; ++i) nl[i] = -W->lam[NX * (k + 1) + i];   /* d2(lam^T g), g = x+ - f */
            rk4_derivs(&P, W->X + NX * k, W->U + NU * k, nl, xn, W->A[k], W->Bm[k], W->H[k]);
        }
        /* ---- optimality error, IPOPT eq. (5) ---------------------------------- */
        double sum_l = 0, sum_z = 0, dinf = 0, pinf = 0, c0 = 0;
        for (int i = 0; i < ng; ++i) sum_l += fabs(W->lam[i]);
        for (int j = 0; j < nU; ++j) sum_z += W->zL[j] + W->zU[j];
        for (int k = 0; k <= N; ++k) {
            double gx[NX]; cost_grad_x(&P, W->X + NX * k, target, gx);
            for (int i = 0; i < NX; ++i) {
                pinf = fmax(pinf, fabs(g[k][i]));
                double r = C.sc * gx[i] + W->lam[NX * k + i];
                if (k < N) for (int m = 0; m < NX; ++m) r -= W->A[k][m][i] * W->lam[NX * (k + 1) + m];
                dinf = fmax(dinf, fabs(r));
            }
            if (k < N) for (int a = 0; a < NU; ++a) {
                const int j = NU * k + a;
                double r = C.sc * 2 * P.R * W->U[j] - W->zL[j] + W->zU[j];
                for (int m = 0; m < NX; ++m) r -= W->Bm[k][m][a] * W->lam[NX * (k + 1) + m];
                dinf = fmax(dinf, fabs(r));
                c0 = fmax(c0, fmax(fabs(W->zL[j] * (W->U[j] - lo)), fabs(W->zU[j] * (hi - W->U[j]))));
            }
        }
        const double s_d = fmax(s_max, (sum_l + sum_z) / (ng + 2 * nU)) / s_max;
        const double s_c = fmax(s_max, sum_z / (2 * nU)) / s_max;
        if (fmax(dinf / s_d, fmax(pinf, c0 / s_c)) <= tol) { status = ST_SOLVED; break; }
        /* ---- monotone barrier update (possibly several times) --------------- */
        for (;;) {
            double cmu = 0;
            for (int j = 0; j < nU; ++j)
                cmu = fmax(cmu, fmax(fabs(W->zL[j] * (W->U[j] - lo) - C.mu), fabs(W->zU[j] * (hi - W->U[j]) - C.mu)));
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > kappa_eps * C.mu || C.mu <= mu_min) break;
            C.mu = fmax(mu_min, fmin(kappa_mu * C.mu, pow(C.mu, theta_mu)));
            nfilt = 0;                                     /* filter reset on barrier update */
        }
        const double tau = fmax(0.99, 1.0 - C.mu);

        /* ---- Newton step: Riccati with inertia correction ------------------- */
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

        double amax = frac_to_boundary(&C, W, W->dU, tau), az = bound_dual_step(&C, W, nU, tau);
        /* ---- filter line search with second-order correction (W&B 2006, Alg. A) */
        const double phi = barrier_obj(&C, W->X, W->U);
        double gTd = 0.0;
        for (int k = 0; k <= N; ++k) {
            double gx[NX]; cost_grad_x(&P, W->X + NX * k, target, gx);
            for (int i = 0; i < NX; ++i) gTd += C.sc * gx[i] * W->dX[NX * k + i];
        }
        for (int j = 0; j < nU; ++j)
            gTd += (C.sc * 2 * P.R * W->U[j] - C.mu / (W->U[j] - lo) + C.mu / (hi - W->U[j])) * W->dU[j];
        double amin = gam_th;
        if (gTd < 0) amin = fmin(gam_th, fmin(gam_ph * th / (-gTd), sw_delta * pow(th, s_th) / pow(-gTd, s_ph)));
        if (th == 0.0 && gTd < 0) amin = 0.0;
        amin *= gam_al;
        double alpha = amax, th_t = 0, ph_t = 0;
        int accepted = 0, ftype = 0, used_soc = 0;
        /* IPOPT tiny-step test: max |d|/(1+|x|) < 10 eps_mach -> accept the full step, unfiltered */
        double tn = 0.0;
        for (int i = 0; i < ng; ++i) tn = fmax(tn, fabs(W->dX[i]) / (1.0 + fabs(W->X[i])));
        for (int j = 0; j < nU; ++j) tn = fmax(tn, fabs(W->dU[j]) / (1.0 + fabs(W->U[j])));
        const int tiny = tn < 10.0 * 2.220446049250313e-16;
        for (int ls = 0; ls < 80 && !accepted; ++ls) {
            if (alpha < amin && ls > 0) break;
            for (int i = 0; i < ng; ++i) W->Xt[i] = W->X[i] + alpha * W->dX[i];
            for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + alpha * W->dU[j];
            th_t = constraints(&C, W->Xt, W->Ut, W->gt);
            ph_t = barrier_obj(&C, W->Xt, W->Ut);
            if (tiny) { accepted = 1; ftype = 1; break; }
            accepted = filter_accept(W, nfilt, th_t, ph_t, th, phi, gTd, alpha, th_max, th_min, &ftype);
            if (!accepted && ls == 0 && !(th_t < th) && g_max_soc > 0) {
                /* IPOPT FilterLSAcceptor::TrySecondOrderCorrection: c_soc <- a_soc c_soc + c(trial),
                   starting from c(x) with a_soc = alpha; the corrected step re-uses the factorisation;
                   at most max_soc passes, continued while theta(trial) <= kappa_soc theta(previous) */
                double save_dU[NU * NMAX], save_dX[NX * (NMAX + 1)], save_lp[NX * (NMAX + 1)];
                memcpy(save_dU, W->dU, sizeof(double) * nU); memcpy(save_dX, W->dX, sizeof(double) * ng); memcpy(save_lp, W->lamp, sizeof(double) * ng);
                double asoc = alpha, th_old = 0.0;
                for (int k = 0; k <= N; ++k) for (int i = 0; i < NX; ++i) W->csoc[k][i] = g[k][i];
                for (int c = 0; c < g_max_soc; ++c) {
                    if (c > 0 && !(th_t <= kap_soc * th_old)) break;
                    th_old = th_t;
                    for (int k = 0; k <= N; ++k) for (int i = 0; i < NX; ++i) W->csoc[k][i] = asoc * W->csoc[k][i] + W->gt[k][i];
                    riccati_solve(&C, W, W->csoc);
                    asoc = frac_to_boundary(&C, W, W->dU, tau);
                    for (int i = 0; i < ng; ++i) W->Xt[i] = W->X[i] + asoc * W->dX[i];
                    for (int j = 0; j < nU; ++j) W->Ut[j] = W->U[j] + asoc * W->dU[j];
                    th_t = constraints(&C, W->Xt, W->Ut, W->gt);
                    ph_t = barrier_obj(&C, W->Xt, W->Ut);
                    if (filter_accept(W, nfilt, th_t, ph_t, th, phi, gTd, alpha, th_max, th_min, &ftype)) {
                        /* IPOPT takes the SOC solve as the whole step: its bound-multiplier
                           directions and their fraction to the boundary follow the corrected dU */
                        accepted = 1; used_soc = 1; alpha = asoc; az = bound_dual_step(&C, W, nU, tau);
                        break;
                    }
                }
                if (!accepted) {    /* back to the plain direction */
                    memcpy(W->dU, save_dU, sizeof(double) * nU); memcpy(W->dX, save_dX, sizeof(double) * ng); memcpy(W->lamp, save_lp, sizeof(double) * ng);
                }
            }
            if (!accepted) {
                alpha *= 0.5;
            }
        }
#ifdef ORACLE_DEBUG
        fprintf(stderr, "it %3d mu %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e az %.3e soc %d th %.2e\n",
                it, C.mu, dinf / s_d, pinf, c0 / s_c, delta, amax, alpha, az, used_soc, th);
#endif
        (void)used_soc;
        if (!accepted) { status = ST_LS_FAIL; break; }   /* IPOPT would enter restoration here */
        if (!ftype && nfilt < 256) { W->filt_th[nfilt] = (1 - gam_th) * th; W->filt_ph[nfilt] = phi - gam_ph * th; ++nfilt; }
        memcpy(W->X, W->Xt, sizeof(double) * ng);
        memcpy(W->U, W->Ut, sizeof(double) * nU);
        memcpy(g, W->gt, sizeof(double) * ng);
        th = th_t;
        for (int i = 0; i < ng; ++i) W->lam[i] += alpha * (W->lamp[i] - W->lam[i]);
        for (int j = 0; j < nU; ++j) {
            double sl = W->U[j] - lo, su = hi - W->U[j];
            double zl = W->zL[j] + az * W->dzL[j], zu = W->zU[j] + az * W->dzU[j];
            zl = fmax(fmin(zl, 1e10 * C.mu / sl), C.mu / (1e10 * sl));   /* kappa_sigma = 1e10 */
            zu = fmax(fmin(zu, 1e10 * C.mu / su), C.mu / (1e10 * su));
            W->zL[j] = zl; W->zU[j] = zu;
        }
    }
    if (iters_out) *iters_out = it;
    if (u0) { u0[0] = W->U[0]; u0[1] = W->U[1]; }
    if (fval) *fval = objective(&P, W->X, W->U, target);
    if (w_out) { memcpy(w_out, W->X, sizeof(double) * ng); memcpy(w_out + ng, W->U, sizeof(double) * nU); }
    free(g);
    free(W);
    return status;
}


/* batched driver over instances (OpenMP when nthreads > 1) */
int oracle_pmpc_solve_batch(int B, int N, double Ts, const double *states, const double *targets, const double *prm,
                            int max_iter, double tol, int nthreads,
                            double *u0, double *f, double *w_out, int32_t *status, int32_t *iters) {
    const int nw = NX * (N + 1) + NU * N;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int b = 0; b < B; ++b) {
        int32_t itb = 0;
        int st = oracle_pmpc_solve(N, Ts, states + 6 * b, targets + 6 * b, prm + 6 * b, NULL, max_iter, tol,
                                   u0 + 2 * b, f + b, w_out ? w_out + (size_t)nw * b : NULL, &itb);
        status[b] = st;
        iters[b] = itb;
    }
    return 0;
}

/* single RK4 step (values), exported for known-answer tests of the restatement */
void oracle_pmpc_rk4(double Ts, double mu, const double *x, const double *u, double *xn) {
    prob_t P = {1, Ts, -9.81, mu, 0, 0, 0, 0, 0};
    rk4_val(&P, x, u, xn);
}

/* exported for known-answer tests: RK4 Jacobian and lam-contracted Hessian */
void oracle_pmpc_rk4_derivs(double Ts, double mu, const double *x, const double *u, const double *lam,
                            double *xn, double *A, double *Bm, double *H) {
    prob_t P = {1, Ts, -9.81, mu, 0, 0, 0, 0, 0};
    double a[NX][NX], b[NX][NU], h[NZ][NZ];
    rk4_derivs(&P, x, u, lam, xn, a, b, h);
    memcpy(A, a, sizeof a); memcpy(Bm, b, sizeof b); memcpy(H, h, sizeof h);
}
