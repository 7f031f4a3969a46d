// pmpc_ipm.hip -- batched PMPC interior-point solve for gfx950 (MI355X / CDNA4).
//
// Replaces the per-timestep `ca.nlpsol('solver','ipopt',...)` call of
// PMPC.solve (PMPC/src/controller/mpc_3d.py:115-138) for a whole batch of
// independent tray-tilt NMPC instances.
//
// Structure exploited: the reference NLP (mpc_3d.py:28-85)
// splits into two independent scalar-input optimal-control problems -- the x
// axis (px, vx; theta_x) and the y axis (py, vy; theta_y) -- plus the cost-free
// z sub-state (pz, vz), which only follows the controls (its multipliers are
// zero at every KKT point).  Each axis is linear in its state with input
// sin(theta):  x+ = Phi x + Gamma sin(theta), Phi/Gamma being exactly the RK4
// map of mpc_3d.py:99-104 applied to :91-92.  The kernel runs IPOPT's
// primal-dual barrier method on the (x, y) problem in lock-step (one mu, one
// step length, one filter, as IPOPT does on the full NLP) and rebuilds the z
// trajectory by the reference's own RK4 once the controls are final.
//
// Mapping: one wave64 per instance, lane k <-> shooting node k (0..N, N <= 63).
// Everything per node lives in VGPRs; the stage-coupled recursions (Riccati
// backward sweep, forward state sweep, z rollout) pass 2x2 blocks between
// neighbouring lanes with cross-lane shifts; norms and inner products are
// wave reductions.  No LDS, no global traffic inside the iteration loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pmpc_ipm.h"

namespace dartmpc {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// wave primitives
// ---------------------------------------------------------------------------
__device__ __forceinline__ double uniform(double x) {   // lane 0's value in every lane (SGPR broadcast)
    unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(b & 0xffffffffu));
    unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double wsum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return uniform(x);
}
__device__ __forceinline__ double wmax(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o));
    return uniform(x);
}
__device__ __forceinline__ double wmin(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o));
    return uniform(x);
}
__device__ __forceinline__ double from_next(double x) { return __shfl_down(x, 1); }  // lane k <- lane k+1
__device__ __forceinline__ double from_prev(double x) { return __shfl_up(x, 1); }    // lane k <- lane k-1
__device__ __forceinline__ bool wany(bool p) { return __ballot(p) != 0ull; }

// ---------------------------------------------------------------------------
// model pieces
// ---------------------------------------------------------------------------
// mpc_3d.py:87-97, one axis:  pdot = v,  vdot = g sin(theta) - mu v
__device__ __forceinline__ void axis_rhs(double g, double mu, double s, double p, double v, double& dp, double& dv) {
    (void)p;
    dp = v;
    dv = g * s - mu * v;
}
// mpc_3d.py:99-104 on one axis with s = sin(theta) held constant
__device__ __forceinline__ void axis_rk4(double h, double g, double mu, double s, double p, double v, double& pn, double& vn) {
    double k1p, k1v, k2p, k2v, k3p, k3v, k4p, k4v;
    axis_rhs(g, mu, s, p, v, k1p, k1v);
    axis_rhs(g, mu, s, p + h / 2 * k1p, v + h / 2 * k1v, k2p, k2v);
    axis_rhs(g, mu, s, p + h / 2 * k2p, v + h / 2 * k2v, k3p, k3v);
    axis_rhs(g, mu, s, p + h * k3p, v + h * k3v, k4p, k4v);
    pn = p + h / 6 * (k1p + 2 * k2p + 2 * k3p + k4p);
    vn = v + h / 6 * (k1v + 2 * k2v + 2 * k3v + k4v);
}
// z sub-state (mpc_3d.py:93-97): pzdot = vz_new, vzdot = (vz_new - vz)/Ts, literal RK4
__device__ __forceinline__ void z_rk4(double h, double w, double pz, double vz, double& pzn, double& vzn) {
    double k1v = (w - vz) / h;
    double k2v = (w - (vz + h / 2 * k1v)) / h;
    double k3v = (w - (vz + h / 2 * k2v)) / h;
    double k4v = (w - (vz + h * k3v)) / h;
    pzn = pz + h / 6 * (w + 2 * w + 2 * w + w);
    vzn = vz + h / 6 * (k1v + 2 * k2v + 2 * k3v + k4v);
}

struct Model {        // per-instance constants (wave-uniform)
    double a12, a22, b1, b2;      // x+ = [[1,a12],[0,a22]] x + [b1,b2] sin(theta)
    double qp2, qv2, r2;          // scaled 2*Qp, 2*Qv, 2*R
    double Qp, Qv, R, sc;
    double lo, hi;                // relaxed box
};

// per-node, per-axis iterate and work registers
struct Axis {
    double sp, sv, rp, rv;        // initial state, reference (uniform)
    double p, v, th;              // primal
    double lp, lv;                // multipliers of the constraint that defines x_k
    double zl, zu;                // bound multipliers (k < N)
    double s, c;                  // sin, cos theta
    double g1, g2;                // defect g_k
    double K1, K2, kff, iQ, U1, U2;
    double P11, P12, P22, p1, p2;
    double dp, dv, dth, dlp, dlv, dzl, dzu;
};

// defect g_k = x_k - f(x_{k-1}, u_{k-1}) (mpc_3d.py:48), g_0 = x_0 - state (:37)
__device__ __forceinline__ void defects(const Model& M, int k, double sp, double sv, double p, double v, double s,
                                        double& g1, double& g2) {
    double fp = p + M.a12 * v + M.b1 * s;
    double fv = M.a22 * v + M.b2 * s;
    double ip = from_prev(fp), iv = from_prev(fv);
    g1 = (k == 0) ? p - sp : p - ip;
    g2 = (k == 0) ? v - sv : v - iv;
}

// ---------------------------------------------------------------------------
// the kernel: one wave64 = one instance
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kWave) void pmpc_ipm_kernel(PmpcArgs a) {
    const int b = blockIdx.x;
    const int k = threadIdx.x;
    const int N = a.N;
    const bool xon = k <= N, uon = k < N;
    const double h = a.Ts;

    const double* st = a.x0 + 6 * b;
    const double* rf = a.ref + 6 * b;
    const double* pr = a.prm + 6 * b;
    const double mu_f = pr[0], Qp = pr[1], Qv = pr[2], R = pr[3], ulo = pr[4], uhi = pr[5];

    Model M;
    {   // RK4 map of the linear axis model applied to the basis: exact Phi, Gamma
        double pn, vn;
        axis_rk4(h, a.g, mu_f, 0.0, 0.0, 1.0, pn, vn); M.a12 = pn; M.a22 = vn;
        axis_rk4(h, a.g, mu_f, 1.0, 0.0, 0.0, pn, vn); M.b1 = pn; M.b2 = vn;
    }
    M.Qp = Qp; M.Qv = Qv; M.R = R;
    M.lo = ulo - 1e-8 * fmax(1.0, fabs(ulo));       // IPOPT bound_relax_factor = 1e-8
    M.hi = uhi + 1e-8 * fmax(1.0, fabs(uhi));
    const double lo = M.lo, hi = M.hi;

    Axis X[2];
    const int nw = 6 * (N + 1) + 2 * N;
    const double* ww = a.w_warm ? a.w_warm + (size_t)nw * b : nullptr;
    const double pushl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo));
    const double pushu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
    double gmax = 0.0;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        Axis& A = X[ax];
        A.sp = st[2 * ax]; A.sv = st[2 * ax + 1];
        A.rp = rf[2 * ax]; A.rv = rf[2 * ax + 1];
        A.p = xon ? (ww ? ww[6 * k + 2 * ax] : A.sp) : 0.0;       // cold start: tile(state) (mpc_3d.py:123)
        A.v = xon ? (ww ? ww[6 * k + 2 * ax + 1] : A.sv) : 0.0;
        double th = uon ? (ww ? ww[6 * (N + 1) + 2 * k + ax] : 0.0) : 0.0;
        if (uon) th = fmin(fmax(th, lo + pushl), hi - pushu);
        A.th = th;
        A.lp = 0.0; A.lv = 0.0;
        A.zl = uon ? 1.0 : 0.0; A.zu = uon ? 1.0 : 0.0;   // bound_mult_init_val = 1
        if (xon) gmax = fmax(gmax, fmax(fabs(2 * Qp * (A.p - A.rp)), fabs(2 * Qv * (A.v - A.rv))));
        if (uon) gmax = fmax(gmax, fabs(2 * R * A.th));
    }
    gmax = wmax(gmax);
    const double sc = gmax > 100.0 ? 100.0 / gmax : 1.0;     // nlp_scaling_max_gradient = 100
    M.sc = sc; M.qp2 = sc * 2 * Qp; M.qv2 = sc * 2 * Qv; M.r2 = sc * 2 * R;

    const double tol = a.tol, mu_min = tol / 10;
    const double n_eq = 6.0 * (N + 1), n_b = 4.0 * N;       // IPOPT counts on the full NLP
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, eta_ph = 1e-8, gam_al = 0.05;

    // constraint violation at the start (filter bounds)
    double th0 = 0.0;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        Axis& A = X[ax];
        A.s = uon ? sin(A.th) : 0.0;
        defects(M, k, A.sp, A.sv, A.p, A.v, A.s, A.g1, A.g2);
        if (xon) th0 += fabs(A.g1) + fabs(A.g2);
    }
    double theta = wsum(th0);
    const double th_max = 1e4 * fmax(1.0, theta), th_min = 1e-4 * fmax(1.0, theta);

    double fth = 0.0, fph = 0.0;      // filter entry held by lane (slot = lane id)
    int nfilt = 0;
    double mu = 0.1, delta_last = 0.0;
    int status = -1, it = 0;

    for (it = 0; it < a.max_iter; ++it) {
        // -------- point quantities ------------------------------------------
        double dinf = 0.0, pinf = 0.0, c0 = 0.0, suml = 0.0, sumz = 0.0;
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) {
            Axis& A = X[ax];
            double s = 0.0, c = 1.0;
            if (uon) sincos(A.th, &s, &c);
            A.s = s; A.c = c;
            defects(M, k, A.sp, A.sv, A.p, A.v, A.s, A.g1, A.g2);
            double lpn = from_next(A.lp), lvn = from_next(A.lv);
            if (xon) {
                double r1 = M.qp2 * (A.p - A.rp) + A.lp - (uon ? lpn : 0.0);
                double r2 = M.qv2 * (A.v - A.rv) + A.lv - (uon ? M.a12 * lpn + M.a22 * lvn : 0.0);
                dinf = fmax(dinf, fmax(fabs(r1), fabs(r2)));
                pinf = fmax(pinf, fmax(fabs(A.g1), fabs(A.g2)));
                suml += fabs(A.lp) + fabs(A.lv);
            }
            if (uon) {
                double sl = A.th - lo, su = hi - A.th;
                double ru = M.r2 * A.th - c * (M.b1 * lpn + M.b2 * lvn) - A.zl + A.zu;
                dinf = fmax(dinf, fabs(ru));
                c0 = fmax(c0, fmax(A.zl * sl, A.zu * su));
                sumz += A.zl + A.zu;
                // keep next-lane multipliers for the Hessian term
                A.dlp = lpn; A.dlv = lvn;
            } else {
                A.dlp = 0.0; A.dlv = 0.0;
            }
        }
        dinf = wmax(dinf); pinf = wmax(pinf); c0 = wmax(c0);
        suml = wsum(suml); sumz = wsum(sumz);
        const double s_d = fmax(100.0, (suml + sumz) / (n_eq + n_b)) / 100.0;
        const double s_c = fmax(100.0, sumz / n_b) / 100.0;
        if (fmax(dinf / s_d, fmax(pinf, c0 / s_c)) <= tol) { status = 0; break; }
        // -------- monotone barrier update -----------------------------------
        for (;;) {
            double cmu = 0.0;
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) {
                const Axis& A = X[ax];
                if (uon) cmu = fmax(cmu, fmax(fabs(A.zl * (A.th - lo) - mu), fabs(A.zu * (hi - A.th) - mu)));
            }
            cmu = wmax(cmu);
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * mu || mu <= mu_min) break;
            mu = fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu)));
            nfilt = 0;
        }
        const double tau = fmax(0.99, 1.0 - mu);

        // -------- Newton step: Riccati recursion + inertia correction ---------
        double delta = 0.0;
        bool ok = false;
        for (int attempt = 0; attempt < 60 && !ok; ++attempt) {
            if (attempt > 0)
                delta = (attempt == 1) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last / 3.0))
                                       : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            bool bad = false;
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) {
                Axis& A = X[ax];
                // terminal value function in every lane; lanes k < N are overwritten by the sweep
                A.P11 = M.qp2 + delta; A.P12 = 0.0; A.P22 = M.qv2 + delta;
                A.p1 = M.qp2 * (A.p - A.rp); A.p2 = M.qv2 * (A.v - A.rv);
            }
            const double gn[2][2] = {{from_next(X[0].g1), from_next(X[0].g2)}, {from_next(X[1].g1), from_next(X[1].g2)}};
            double Quu[2] = {1.0, 1.0};
            for (int step = 0; step < N; ++step) {
#pragma unroll
                for (int ax = 0; ax < 2; ++ax) {
                    Axis& A = X[ax];
                    const double P11 = from_next(A.P11), P12 = from_next(A.P12), P22 = from_next(A.P22);
                    const double pn1 = from_next(A.p1), pn2 = from_next(A.p2);
                    if (uon) {
                        const double a12 = M.a12, a22 = M.a22;
                        const double be1 = M.b1 * A.c, be2 = M.b2 * A.c;
                        const double sl = A.th - lo, su = hi - A.th;
                        // Hessian of the Lagrangian in theta: 2R + lam_{k+1}^T Gamma sin(theta) + Sigma + delta
                        const double Rt = M.r2 + A.s * (M.b1 * A.dlp + M.b2 * A.dlv) + A.zl / sl + A.zu / su + delta;
                        const double rt = M.r2 * A.th - mu / sl + mu / su;
                        const double q1 = M.qp2 * (A.p - A.rp), q2 = M.qv2 * (A.v - A.rv);
                        // Phi^T P Phi with Phi = [[1,a12],[0,a22]]
                        const double t12 = P11 * a12 + P12 * a22;
                        const double t22 = P12 * a12 + P22 * a22;
                        const double X11 = P11 + M.qp2 + delta;
                        const double X12 = t12;
                        const double X22 = a12 * t12 + a22 * t22 + M.qv2 + delta;
                        const double PB1 = P11 * be1 + P12 * be2, PB2 = P12 * be1 + P22 * be2;
                        const double Q = Rt + be1 * PB1 + be2 * PB2;
                        const double U1 = PB1, U2 = PB1 * a12 + PB2 * a22;
                        const double h1 = pn1 - (P11 * gn[ax][0] + P12 * gn[ax][1]);
                        const double h2 = pn2 - (P12 * gn[ax][0] + P22 * gn[ax][1]);
                        const double qx1 = q1 + h1, qx2 = q2 + a12 * h1 + a22 * h2;
                        const double qu = rt + be1 * h1 + be2 * h2;
                        const double iQ = 1.0 / Q;
                        A.iQ = iQ; A.U1 = U1; A.U2 = U2;
                        A.K1 = -iQ * U1; A.K2 = -iQ * U2; A.kff = -iQ * qu;
                        A.P11 = X11 - iQ * U1 * U1;
                        A.P12 = X12 - iQ * U1 * U2;
                        A.P22 = X22 - iQ * U2 * U2;
                        A.p1 = qx1 + U1 * A.kff;
                        A.p2 = qx2 + U2 * A.kff;
                        Quu[ax] = Q;
                    }
                }
            }
            if (uon) bad = !(Quu[0] > 0.0) || !(Quu[1] > 0.0) || !isfinite(Quu[0]) || !isfinite(Quu[1]);
            ok = !wany(bad);
        }
        if (!ok) { status = -3; break; }
        if (delta > 0.0) delta_last = delta;

        // -------- forward sweep of the state step ------------------------------
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) { X[ax].dp = -X[ax].g1; X[ax].dv = -X[ax].g2; }
        for (int step = 0; step < N; ++step) {
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) {
                Axis& A = X[ax];
                const double dth = A.K1 * A.dp + A.K2 * A.dv + A.kff;
                const double op = A.dp + M.a12 * A.dv + M.b1 * A.c * dth;
                const double ov = M.a22 * A.dv + M.b2 * A.c * dth;
                const double ip = from_prev(op), iv = from_prev(ov);
                if (k >= 1) { A.dp = ip - A.g1; A.dv = iv - A.g2; }
            }
        }
        double amax = 1.0, az = 1.0;
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) {
            Axis& A = X[ax];
            A.dth = uon ? A.K1 * A.dp + A.K2 * A.dv + A.kff : 0.0;
            // new multipliers lam+ = -(P dx + p), step = lam+ - lam
            A.dlp = xon ? -(A.P11 * A.dp + A.P12 * A.dv + A.p1) - A.lp : 0.0;
            A.dlv = xon ? -(A.P12 * A.dp + A.P22 * A.dv + A.p2) - A.lv : 0.0;
            if (uon) {
                const double sl = A.th - lo, su = hi - A.th;
                A.dzl = mu / sl - A.zl - A.zl / sl * A.dth;
                A.dzu = mu / su - A.zu + A.zu / su * A.dth;
                if (A.dth < 0) amax = fmin(amax, -tau * sl / A.dth);
                if (A.dth > 0) amax = fmin(amax, tau * su / A.dth);
                if (A.dzl < 0) az = fmin(az, -tau * A.zl / A.dzl);
                if (A.dzu < 0) az = fmin(az, -tau * A.zu / A.dzu);
            } else {
                A.dzl = 0.0; A.dzu = 0.0;
            }
        }
        amax = wmin(amax); az = wmin(az);

        // -------- filter line search (Waechter & Biegler 2006, Alg. A) ----------
        double phil = 0.0, gtdl = 0.0;
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) {
            const Axis& A = X[ax];
            if (xon) {
                const double ep = A.p - A.rp, ev = A.v - A.rv;
                phil += sc * (Qp * ep * ep + Qv * ev * ev);
                gtdl += M.qp2 * ep * A.dp + M.qv2 * ev * A.dv;
            }
            if (uon) {
                const double sl = A.th - lo, su = hi - A.th;
                phil += sc * R * A.th * A.th - mu * (log(sl) + log(su));
                gtdl += (M.r2 * A.th - mu / sl + mu / su) * A.dth;
            }
        }
        const double phi = wsum(phil), gTd = wsum(gtdl);
        double amin = gam_th;
        if (gTd < 0.0) amin = fmin(gam_th, fmin(gam_ph * theta / (-gTd), pow(theta, s_th) / pow(-gTd, s_ph)));
        amin *= gam_al;
        double alpha = amax, th_t = 0.0, ph_t = 0.0;
        bool accepted = false, ftype = false;
        for (int ls = 0; ls < 80; ++ls) {
            double thl = 0.0, phl = 0.0;
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) {
                const Axis& A = X[ax];
                const double pt = A.p + alpha * A.dp, vt = A.v + alpha * A.dv, tt = A.th + alpha * A.dth;
                const double s = uon ? sin(tt) : 0.0;
                double g1, g2;
                defects(M, k, A.sp, A.sv, pt, vt, s, g1, g2);
                if (xon) {
                    thl += fabs(g1) + fabs(g2);
                    const double ep = pt - A.rp, ev = vt - A.rv;
                    phl += sc * (Qp * ep * ep + Qv * ev * ev);
                }
                if (uon) phl += sc * R * tt * tt - mu * (log(tt - lo) + log(hi - tt));
            }
            th_t = wsum(thl); ph_t = wsum(phl);
            bool in_filter = !(th_t < th_max) || !isfinite(ph_t);
            in_filter = in_filter || wany(k < nfilt && th_t >= fth && ph_t >= fph);
            if (!in_filter) {
                const bool sw = gTd < 0.0 && alpha * pow(-gTd, s_ph) > pow(theta, s_th);
                if (theta <= th_min && sw) {
                    if (ph_t <= phi + eta_ph * alpha * gTd) { accepted = true; ftype = true; }
                } else if (th_t <= (1 - gam_th) * theta || ph_t <= phi - gam_ph * theta) {
                    accepted = true;
                }
            }
            if (accepted) break;
            alpha *= 0.5;
            if (alpha < amin) break;
        }
        if (!accepted) { status = -2; break; }   // IPOPT would enter its restoration phase here
        if (!ftype && nfilt < kWave) {
            if (k == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
            ++nfilt;
        }
        // -------- accept the step ------------------------------------------------
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) {
            Axis& A = X[ax];
            if (xon) {
                A.p += alpha * A.dp; A.v += alpha * A.dv;
                A.lp += alpha * A.dlp; A.lv += alpha * A.dlv;
            }
            if (uon) {
                A.th += alpha * A.dth;
                const double sl = A.th - lo, su = hi - A.th;
                double zl = A.zl + az * A.dzl, zu = A.zu + az * A.dzu;
                zl = fmax(fmin(zl, 1e10 * mu / sl), mu / (1e10 * sl));      // kappa_sigma = 1e10
                zu = fmax(fmin(zu, 1e10 * mu / su), mu / (1e10 * su));
                A.zl = zl; A.zu = zu;
            }
        }
        theta = th_t;
    }

    // -------- outputs ---------------------------------------------------------
    // objective (mpc_3d.py:44-46, :63-66), unscaled
    double fl = 0.0;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        const Axis& A = X[ax];
        if (xon) { const double ep = A.p - A.rp, ev = A.v - A.rv; fl += Qp * ep * ep + Qv * ev * ev; }
        if (uon) fl += R * A.th * A.th;
    }
    const double fval = wsum(fl);
    if (k == 0) {
        a.u0[2 * b] = X[0].th;
        a.u0[2 * b + 1] = X[1].th;
        a.f[b] = fval;
        a.status[b] = status;
        a.iters[b] = it;
    }
    if (a.w_out) {
        // z sub-state follows the final controls through the reference RK4 (mpc_3d.py:93-97, :99-104)
        const double w = uon ? -a.g * (X[0].th * X[0].th + X[1].th * X[1].th) : 0.0;
        double pz = st[4], vz = st[5];
        for (int step = 0; step < N; ++step) {
            double pzn, vzn;
            z_rk4(h, w, pz, vz, pzn, vzn);
            const double ip = from_prev(pzn), iv = from_prev(vzn);
            if (k >= 1) { pz = ip; vz = iv; }
        }
        double* wo = a.w_out + (size_t)nw * b;
        if (xon) {
            wo[6 * k + 0] = X[0].p; wo[6 * k + 1] = X[0].v;
            wo[6 * k + 2] = X[1].p; wo[6 * k + 3] = X[1].v;
            wo[6 * k + 4] = pz;     wo[6 * k + 5] = vz;
        }
        if (uon) { wo[6 * (N + 1) + 2 * k] = X[0].th; wo[6 * (N + 1) + 2 * k + 1] = X[1].th; }
    }
}

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_pmpc(const dartmpc::PmpcArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    hipLaunchKernelGGL(dartmpc::pmpc_ipm_kernel, dim3(args->B), dim3(dartmpc::kWave), 0, stream, *args);
    return hipGetLastError();
}
