// lmpc_ipm.hip -- batched LMPC interior-point solve (8-state Stribeck / rolling model), gfx950.
//
// Replaces the solve of RLMPC._solver_worker (LMPC/src/controller/rlmpc2.py:229-533): the NLP
// :239-491 with the model safe_dynamics :260-429 (index map :301-344), RK4 :431-436, cost
// :444-464 (Q, Qt on the state error, R on [u; Delta u]), U box, and IPOPT's options
// (:480-489: max_iter, tol, acceptable_tol, acceptable_iter; the 0.05 s wall-clock cap is not
// reproduced: the solve is deterministic here).  The 34-vector pvec is an input.
//
// Method: IPOPT's primal-dual barrier method as in pmpc_ipm.hip / rmpc_ipm.hip (monotone mu,
// filter line search, inertia correction, bound_relax 1e-8, gradient-based scaling of the
// objective and of the constraint rows) with IPOPT's optimal / acceptable termination tests.
// The Delta-u cost couples consecutive controls: the Riccati recursion runs on the augmented
// state x~_k = [x_k; u_{k-1}] (nx~ = 10), three LDS phases per node (ocp_wave.h, OcpLds3).
// Exact RK4 Jacobians (forward mode, 10 directions, two at a time over LDS-staged stage
// derivatives); the dynamics part of the Lagrangian Hessian is the RK-weighted
// Ts * sum_s w_s lambda^T f''(y_s) (error O(Ts^2) relative; it changes the Newton path only,
// never the KKT point).
//
// Mapping: one wave64 per instance, lane k = shooting node k (N <= 31) for node-local work;
// the node-coupled Riccati / forward sweeps run through LDS (ocp_wave.h).  The LDS image
// (~135 KB) is dynamic shared memory: one instance per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lmpc_ipm.h"
#include "ocp_wave.h"
#include "stamps.h"
#include "wave.h"

namespace dartmpc {

constexpr int LM_NMAXS = 32;      // max shooting nodes (N <= 31)
constexpr int LM_NSC = 10;        // stage-dependent tangent coefficients per RK stage
constexpr double LM_G = 9.81;     // rlmpc2.py:354
using LmLds = OcpLds3<10, LM_NMAXS>;

#ifdef DART_STAMPS
__device__ unsigned long long g_stamp_lm[16];
#endif

struct Strb {           // stribeck_fric parameters (rlmpc2.py:372-376)
    double Fc, dF, B, ivs, ieps;    // dF = F_s - F_c, ivs = 1 / (v_s + 1e-12), ieps = 1 / eps
};

struct LmModel {
    double im_x, im_y, m_x, m_y, c_x, c_y, k_x, k_y;
    Strb sx, sy, srx, sry;
    double iIx, iIy, r_x, r_y, c_rx, c_ry, tqx, tqy;   // tq = m g h_com (toppling torque scale)
    double h;                                         // Ts
};

struct LmShared {
    LmLds ocp;
    double SC[kWave][4][LM_NSC];      // per lane, per RK stage: d f / d y coefficients (tangent pass)
    double JL[kWave][12];             // per lane: J^T lambda_{k+1} staging, primal residual maxima
    LmModel model;                    // uniform problem data, read at the use sites (keeps VGPRs free)
    double Q[8], Qt[8], tgt[8];
};

__device__ __forceinline__ double sq(double p) { return fabs(p) + 1e-6; }   // squash_param :296-298

__device__ __forceinline__ Strb make_strb(double Fs, double Fc, double B, double vs, double eps) {
    Strb s;
    s.Fc = Fc; s.dF = Fs - Fc; s.B = B; s.ivs = 1.0 / (vs + 1e-12); s.ieps = 1.0 / eps;
    return s;
}

// value of the friction law: tanh(v/eps) (F_c + (F_s - F_c) exp(-|v|/(v_s + 1e-12))) + B v
__device__ __forceinline__ double strb(const Strb& p, double v) {
    const double e = exp_fast(-fabs(v) * p.ivs);
    const double T = tanh_fast(v * p.ieps);
    return fma(T, fma(p.dF, e, p.Fc), p.B * v);
}
// value, first and second derivative (d|v|/dv = sign(v), sign(0) = 0, as CasADi)
__device__ __forceinline__ void strb_d(const Strb& p, double v, double& S, double& S1, double& S2) {
    const double sg = (v > 0.0) ? 1.0 : ((v < 0.0) ? -1.0 : 0.0);
    const double e = exp_fast(-fabs(v) * p.ivs);
    const double T = tanh_fast(v * p.ieps);
    const double C = fma(p.dF, e, p.Fc);
    const double T1 = (1.0 - T * T) * p.ieps, C1 = -p.dF * e * sg * p.ivs;
    const double T2 = -2.0 * T * T1 * p.ieps, C2 = p.dF * e * (sg * sg) * p.ivs * p.ivs;
    S = fma(T, C, p.B * v);
    S1 = fma(T1, C, fma(T, C1, p.B));
    S2 = fma(T2, C, fma(2.0 * T1, C1, T * C2));
}

__device__ __forceinline__ double sin_any(double x) {
    double s, c;
    if (fabs(x) <= 1.0) sincos_small(x, s, c);
    else s = sin(x);
    return s;
}
__device__ __forceinline__ void sincos_any(double x, double& s, double& c) {
    if (fabs(x) <= 1.0) sincos_small(x, s, c);
    else sincos(x, &s, &c);
}

// safe_dynamics (:260-429): xdot of state y for tilt sines sa, sb
__device__ __forceinline__ void lm_f(const LmModel& m, const double* y, double sa, double sb, double* f) {
    const double Ffx = strb(m.sx, y[1]);
    const double Frx = strb(m.sx, fma(-m.r_x, y[7], y[1]));          // slip vx - r_x om_y
    const double Ffy = strb(m.sy, y[3]);
    const double Fry = strb(m.sy, fma(m.r_y, y[5], y[3]));           // slip vy - (-r_y om_x)
    const double Tnx = strb(m.srx, y[5]);
    const double Tny = strb(m.sry, y[7]);
    const double tx = -m.r_y * Fry - Tnx - m.c_rx * y[5] - m.tqx * sin_any(y[4]);
    const double ty = -m.r_x * Frx - Tny - m.c_ry * y[7] - m.tqy * sin_any(y[6]);
    const double rx = m.m_x * (LM_G * sa) - m.c_x * y[1] - m.k_x * y[0] - Ffx - Frx;
    const double ry = m.m_y * (LM_G * sb) - m.c_y * y[3] - m.k_y * y[2] - Ffy - Fry;
    f[0] = y[1]; f[1] = rx * m.im_x; f[2] = y[3]; f[3] = ry * m.im_y;
    f[4] = y[5]; f[5] = tx * m.iIx; f[6] = y[7]; f[7] = ty * m.iIy;
}

__device__ __forceinline__ void lm_rk4(const LmModel& m, const double* x, double sa, double sb, double* xn) {
    double k[8], y[8], acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { y[i] = x[i]; acc[i] = 0.0; }
#pragma unroll 1
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        lm_f(m, y, sa, sb, k);
#pragma unroll
        for (int i = 0; i < 8; ++i) { acc[i] = fma(wts, k[i], acc[i]); y[i] = fma(cst * m.h, k[i], x[i]); }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) xn[i] = fma(m.h / 6.0, acc[i], x[i]);
}

// Value pass of RK4 that also stores the tangent coefficients of every stage in sc[4][10] and
// accumulates the RK-weighted curvature -Ts sum_s w_s/6 lamn^T f''(y_s) (lamn = lambda_{k+1}).
// hd = [vxvx, vxwy, wywy, vyvy, vywx, wxwx, txtx, tyty, aa, bb] (state indices 1,7 / 3,5 / 4 / 6, u).
__device__ __forceinline__ void lm_rk4_lin(const LmModel& m, const double* x, double sa, double sb,
                                           const double* lamn, double* xn, double (*sc)[LM_NSC], double* hd) {
    const double nl[8] = {0.0, -lamn[1], 0.0, -lamn[3], 0.0, -lamn[5], 0.0, -lamn[7]};
    double y[8], acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { y[i] = x[i]; acc[i] = 0.0; }
#pragma unroll
    for (int i = 0; i < 10; ++i) hd[i] = 0.0;
#pragma unroll 1
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        double Sfx, Sfx1, Sfx2, Srx, Srx1, Srx2, Sfy, Sfy1, Sfy2, Sry, Sry1, Sry2, Snx, Snx1, Snx2, Sny, Sny1, Sny2;
        strb_d(m.sx, y[1], Sfx, Sfx1, Sfx2);
        strb_d(m.sx, fma(-m.r_x, y[7], y[1]), Srx, Srx1, Srx2);
        strb_d(m.sy, y[3], Sfy, Sfy1, Sfy2);
        strb_d(m.sy, fma(m.r_y, y[5], y[3]), Sry, Sry1, Sry2);
        strb_d(m.srx, y[5], Snx, Snx1, Snx2);
        strb_d(m.sry, y[7], Sny, Sny1, Sny2);
        double stx, ctx, sty, cty;
        sincos_any(y[4], stx, ctx);
        sincos_any(y[6], sty, cty);
        double k[8];
        k[0] = y[1]; k[2] = y[3]; k[4] = y[5]; k[6] = y[7];
        k[1] = (m.m_x * (LM_G * sa) - m.c_x * y[1] - m.k_x * y[0] - Sfx - Srx) * m.im_x;
        k[3] = (m.m_y * (LM_G * sb) - m.c_y * y[3] - m.k_y * y[2] - Sfy - Sry) * m.im_y;
        k[5] = (-m.r_y * Sry - Snx - m.c_rx * y[5] - m.tqx * stx) * m.iIx;
        k[7] = (-m.r_x * Srx - Sny - m.c_ry * y[7] - m.tqy * sty) * m.iIy;
        // tangent coefficients: d f1/d vx, d f1/d om_y, d f3/d vy, d f3/d om_x, d f5/d vy, d f5/d om_x,
        // d f5/d th_x, d f7/d vx, d f7/d om_y, d f7/d th_y
        sc[s][0] = (-m.c_x - Sfx1 - Srx1) * m.im_x;
        sc[s][1] = m.r_x * Srx1 * m.im_x;
        sc[s][2] = (-m.c_y - Sfy1 - Sry1) * m.im_y;
        sc[s][3] = -m.r_y * Sry1 * m.im_y;
        sc[s][4] = -m.r_y * Sry1 * m.iIx;
        sc[s][5] = (-m.r_y * m.r_y * Sry1 - Snx1 - m.c_rx) * m.iIx;
        sc[s][6] = -m.tqx * ctx * m.iIx;
        sc[s][7] = -m.r_x * Srx1 * m.iIy;
        sc[s][8] = (m.r_x * m.r_x * Srx1 - Sny1 - m.c_ry) * m.iIy;
        sc[s][9] = -m.tqy * cty * m.iIy;
        // curvature of nl^T f at y_s
        const double W = m.h * wts / 6.0;
        const double c_vx = nl[1] * (-Sfx2 * m.im_x);
        const double c_sx = nl[1] * (-Srx2 * m.im_x) + nl[7] * (-m.r_x * Srx2 * m.iIy);
        const double c_vy = nl[3] * (-Sfy2 * m.im_y);
        const double c_sy = nl[3] * (-Sry2 * m.im_y) + nl[5] * (-m.r_y * Sry2 * m.iIx);
        const double c_ox = nl[5] * (-Snx2 * m.iIx);
        const double c_oy = nl[7] * (-Sny2 * m.iIy);
        hd[0] = fma(W, c_vx + c_sx, hd[0]);
        hd[1] = fma(W, -m.r_x * c_sx, hd[1]);
        hd[2] = fma(W, fma(m.r_x * m.r_x, c_sx, c_oy), hd[2]);
        hd[3] = fma(W, c_vy + c_sy, hd[3]);
        hd[4] = fma(W, m.r_y * c_sy, hd[4]);
        hd[5] = fma(W, fma(m.r_y * m.r_y, c_sy, c_ox), hd[5]);
        hd[6] = fma(W, nl[5] * m.tqx * stx * m.iIx, hd[6]);
        hd[7] = fma(W, nl[7] * m.tqy * sty * m.iIy, hd[7]);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fma(wts, k[i], acc[i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = fma(cst * m.h, k[i], x[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) xn[i] = fma(m.h / 6.0, acc[i], x[i]);
    hd[8] = m.h * nl[1] * (-LM_G * sa);
    hd[9] = m.h * nl[3] * (-LM_G * sb);
}

// Tangent of RK4 along direction d (0..7 state, 8..9 tilt) from the stored stage coefficients:
// column d of the step Jacobian J = d x+ / d [x; u], written to column jc(d) of the node's M~;
// returns col . lamn (the J^T lambda term of the dual residual).
__device__ __forceinline__ double lm_column(const LmModel& m, const double (*sc)[LM_NSC], double gca, double gcb,
                                            int d, const double* lamn, double* Mk) {
    double yd[8], acc[8], e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { e[i] = (i == d) ? 1.0 : 0.0; yd[i] = e[i]; acc[i] = 0.0; }
    const double fa = d == 8 ? gca : 0.0, fb = d == 9 ? gcb : 0.0;
    const double kx1 = -m.k_x * m.im_x, ky3 = -m.k_y * m.im_y;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        const double* c = sc[s];
        double k[8];
        k[0] = yd[1]; k[2] = yd[3]; k[4] = yd[5]; k[6] = yd[7];
        k[1] = fma(kx1, yd[0], fma(c[0], yd[1], fma(c[1], yd[7], fa)));
        k[3] = fma(ky3, yd[2], fma(c[2], yd[3], fma(c[3], yd[5], fb)));
        k[5] = fma(c[4], yd[3], fma(c[5], yd[5], c[6] * yd[4]));
        k[7] = fma(c[7], yd[1], fma(c[8], yd[7], c[9] * yd[6]));
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fma(wts, k[i], acc[i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) yd[i] = fma(cst * m.h, k[i], e[i]);
    }
    const int jc = d < 8 ? d : d + 2;
    double dot = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double col = fma(m.h / 6.0, acc[i], e[i]);
        Mk[jc * LmLds::NC + i] = col;
        dot = fma(col, lamn[i], dot);
    }
    return dot;
}

// all ten columns, one direction at a time; J^T lambda_{k+1} into jl[10]
__device__ __forceinline__ void lm_columns(const LmModel& m, const double (*sc)[LM_NSC], double gca, double gcb,
                                           const double* lamn, double* Mk, double* jl, double* jl_lds) {
#pragma unroll 1
    for (int d = 0; d < 10; ++d) jl_lds[d] = lm_column(m, sc, gca, gcb, d, lamn, Mk);
#pragma unroll
    for (int d = 0; d < 10; ++d) jl[d] = jl_lds[d];
}

__global__ __launch_bounds__(kWave) void lmpc_ipm_kernel(LmpcArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LmShared& SH = *reinterpret_cast<LmShared*>(smem);
    LmLds* S = &SH.ocp;
    const Riccati3Roles<LmLds> RR = riccati3_roles<LmLds>();
    STAMP_DECL
    const int b = blockIdx.x;
    const int k = threadIdx.x;
    const int N = a.N;
    const bool xon = k <= N, uon = k < N;
    constexpr int NC = LmLds::NC;

    // ---------------- model parameters (uniform, staged in LDS) -------------------------------
    if (k == 0) {
        LmModel& m = SH.model;
        const double* p = a.pvec + LM_NPV * b;
        m.m_x = sq(p[0]); m.m_y = sq(p[1]); m.im_x = 1.0 / m.m_x; m.im_y = 1.0 / m.m_y;
        m.c_x = sq(p[2]); m.c_y = sq(p[3]); m.k_x = sq(p[4]); m.k_y = sq(p[5]);
        m.sx = make_strb(p[6], p[7], p[8], sq(p[9]), sq(p[10]));
        m.sy = make_strb(p[11], p[12], p[13], sq(p[14]), sq(p[15]));
        m.iIx = 1.0 / (sq(p[16]) + 1e-12); m.iIy = 1.0 / (sq(p[17]) + 1e-12);
        m.r_x = sq(p[18]); m.r_y = sq(p[19]); m.c_rx = sq(p[20]); m.c_ry = sq(p[21]);
        m.srx = make_strb(p[22], p[23], p[24], sq(p[25]), sq(p[26]));
        m.sry = make_strb(p[27], p[28], p[29], sq(p[30]), sq(p[31]));
        m.tqx = m.m_y * LM_G * sq(p[32]); m.tqy = m.m_x * LM_G * sq(p[33]);
        m.h = a.Ts;
        for (int i = 0; i < 8; ++i) {
            SH.Q[i] = a.prm[LM_NPRM * b + i]; SH.Qt[i] = a.prm[LM_NPRM * b + 8 + i]; SH.tgt[i] = a.target[8 * b + i];
        }
    }
    __syncthreads();
    const LmModel& m = SH.model;
    const double* Q = SH.Q;
    const double* tgt = SH.tgt;
    const double* Wq = k < N ? SH.Q : SH.Qt;     // stage or terminal weights (lane N is the terminal node)
    const double* Qt = SH.Qt;
    const double* pr = a.prm + LM_NPRM * b;
    const double R0 = pr[16], R1 = pr[17], R2 = pr[18], R3 = pr[19];
    const double ulo = pr[20], uhi = pr[21];

    const double lo = ulo - 1e-8 * fmax(1.0, fabs(ulo)), hi = uhi + 1e-8 * fmax(1.0, fabs(uhi));
    const bool poly = fmax(fabs(lo), fabs(hi)) <= 1.0;

    // ---------------- constant structure of the stage blocks ------------------------------------
    double* Mk = &S->M[xon ? k : 0][0][0];
    double* Hk = S->H[xon ? k : 0];
    if (uon) {
        for (int e = 0; e < LmLds::ND * NC; ++e) Mk[e] = 0.0;
        for (int e = 0; e < LmLds::NTP; ++e) Hk[e] = 0.0;
        Mk[10 * NC + 8] = 1.0; Mk[11 * NC + 9] = 1.0;     // up+ = u
        Mk[12 * NC + 10] = 1.0;                            // homogeneous coordinate
    }

    // ---------------- initial point (lane k = node k) --------------------------------------------
    const double* st0 = a.state + 8 * b;
    const double* upv = a.u_prev + 2 * b;
    const int nw = 8 * (N + 1) + 2 * N;
    const double* ww = a.w_warm ? a.w_warm + (size_t)nw * b : nullptr;
    double x[8], up[2], u[2], lam[10], zl[2], zu[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = xon && ww ? ww[8 * k + i] : 0.0;   // warm start w0 (zeros first, :492)
    const double pushl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo));
    const double pushu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const double t = uon && ww ? ww[8 * (N + 1) + 2 * k + j] : 0.0;
        u[j] = uon ? fmin(fmax(t, lo + pushl), hi - pushu) : 0.0;
        zl[j] = uon ? 1.0 : 0.0; zu[j] = uon ? 1.0 : 0.0;
    }
    {
        const double p0 = from_prev(u[0]), p1 = from_prev(u[1]);
        up[0] = k == 0 ? upv[0] : p0;
        up[1] = k == 0 ? upv[1] : p1;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) lam[i] = 0.0;

    auto cost_grad = [&](const double* xx, const double* uu, const double* pp, double* g) {
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] = 2.0 * Wq[i] * (xx[i] - tgt[i]);
        const double d0 = uu[0] - pp[0], d1 = uu[1] - pp[1];
        g[8] = uon ? -2.0 * R2 * d0 : 0.0; g[9] = uon ? -2.0 * R3 * d1 : 0.0;
        g[10] = uon ? fma(2.0 * R0, uu[0], 2.0 * R2 * d0) : 0.0;
        g[11] = uon ? fma(2.0 * R1, uu[1], 2.0 * R3 * d1) : 0.0;
    };
    auto cost_val = [&](const double* xx, const double* uu, const double* pp) {
        double f = 0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i) f = fma(Wq[i] * (xx[i] - tgt[i]), xx[i] - tgt[i], f);
        const double d0 = uu[0] - pp[0], d1 = uu[1] - pp[1];
        const double fu = R0 * uu[0] * uu[0] + R1 * uu[1] * uu[1] + R2 * d0 * d0 + R3 * d1 * d1;
        return xon ? f + (uon ? fu : 0.0) : 0.0;
    };
    // incoming augmented defect g_k of node k for a trial point (value-only RK4 of lane k-1)
    auto defects = [&](const double* xx, const double* pp, const double* uu, double* g) {
        double sa, ca, sb, cb, xn[8];
        tilt_sincos(poly, uu[0], sa, ca);
        tilt_sincos(poly, uu[1], sb, cb);
        lm_rk4(m, xx, sa, sb, xn);
        double f[10];
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = from_prev(xn[i]);
        f[8] = from_prev(uu[0]); f[9] = from_prev(uu[1]);
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] = k == 0 ? xx[i] - st0[i] : xx[i] - f[i];
        g[8] = k == 0 ? pp[0] - upv[0] : pp[0] - f[8];
        g[9] = k == 0 ? pp[1] - upv[1] : pp[1] - f[9];
    };

    // objective scaling (max |grad f| at the start point), constraint-row scaling (max |grad g_i|)
    double gmax = 0.0;
    {
        double g[12];
        cost_grad(x, u, up, g);
#pragma unroll
        for (int i = 0; i < 12; ++i) gmax = fmax(gmax, xon ? fabs(g[i]) : 0.0);
    }
    gmax = wmax(gmax);
    const double sc = gmax > 100.0 ? 100.0 / gmax : 1.0;

    double dsc[8];          // scaling of the incoming physical defect rows of node k (up rows: 1)
    {
        double sa, ca, sb, cb, xn[8], hd[10], nl0[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) nl0[i] = 0.0;
        tilt_sincos(poly, u[0], sa, ca);
        tilt_sincos(poly, u[1], sb, cb);
        lm_rk4_lin(m, x, sa, sb, nl0, xn, SH.SC[k], hd);
        double* Mt = &S->M[xon ? k : 0][0][0];
        const double lz[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        const double (*scs)[LM_NSC] = SH.SC[k];
        const double gca = LM_G * ca, gcb = LM_G * cb;
        if (uon) {
            double jl0[10];
            lm_columns(m, scs, gca, gcb, lz, Mt, jl0, SH.JL[k]);
        }
        double rs[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            double mx = 1.0;
#pragma unroll
            for (int j = 0; j < 8; ++j) mx = fmax(mx, fabs(Mt[j * NC + i]));
            mx = fmax(mx, fmax(fabs(Mt[10 * NC + i]), fabs(Mt[11 * NC + i])));
            rs[i] = uon ? (mx > 100.0 ? 100.0 / mx : 1.0) : 1.0;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) { const double t = from_prev(rs[i]); dsc[i] = k == 0 ? 1.0 : t; }
    }

    const double tol = a.tol, mu_min = tol / 10;
    const double nA = 10.0 * (N + 1), nb = 4.0 * N;
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, eta_ph = 1e-8, gam_al = 0.05;

    auto theta_of = [&](const double* g) {
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i) t = fma(dsc[i], fabs(g[i]), t);
        return xon ? t + fabs(g[8]) + fabs(g[9]) : 0.0;
    };
    double theta;
    {
        double g0[10];
        defects(x, up, u, g0);
        theta = wsum(theta_of(g0));
    }
    const double th_max = 1e4 * fmax(1.0, theta), th_min = 1e-4 * fmax(1.0, theta);
    double fth = 0.0, fph = 0.0;
    int nfilt = 0, acc_count = 0;
    double mu = 0.1, delta_last = 0.0;
    int status = -1, it = 0;

    STAMP(0);
    for (it = 0;; ++it) {
        // ---------------- derivatives, residuals, optimality error ---------------------------
        // The stage data go to LDS as soon as they exist (H without its gradient row, the
        // columns of M~, the defect column, dx~_0) to keep the register working set small.
        const double isl0 = uon ? frcp(u[0] - lo) : 0.0, isl1 = uon ? frcp(u[1] - lo) : 0.0;
        const double isu0 = uon ? frcp(hi - u[0]) : 0.0, isu1 = uon ? frcp(hi - u[1]) : 0.0;
        double lamn[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) { const double t = from_next(lam[i]); lamn[i] = uon ? t : 0.0; }
        double jl[10];      // J^T lambda_{k+1} (x columns 0..7, tilt 8..9)
        {
            double sa, ca, sb, cb;
            tilt_sincos(poly, u[0], sa, ca);
            tilt_sincos(poly, u[1], sb, cb);
            double xn[8];
            {
                double hd[10];
                lm_rk4_lin(m, x, sa, sb, lamn, xn, SH.SC[k], hd);
                if (uon) {   // z = [x(8), up(2), u(2), 1]: packed Hessian (gradient row later)
#pragma unroll
                    for (int i = 0; i < 8; ++i) Hk[hp(i, i)] = sc * 2.0 * Q[i];
                    Hk[hp(1, 1)] += hd[0]; Hk[hp(7, 1)] = hd[1]; Hk[hp(7, 7)] += hd[2];
                    Hk[hp(3, 3)] += hd[3]; Hk[hp(5, 3)] = hd[4]; Hk[hp(5, 5)] += hd[5];
                    Hk[hp(4, 4)] += hd[6]; Hk[hp(6, 6)] += hd[7];
                    Hk[hp(8, 8)] = sc * 2.0 * R2; Hk[hp(9, 9)] = sc * 2.0 * R3;
                    Hk[hp(10, 10)] = sc * 2.0 * (R0 + R2) + hd[8] + zl[0] * isl0 + zu[0] * isu0;
                    Hk[hp(11, 11)] = sc * 2.0 * (R1 + R3) + hd[9] + zl[1] * isl1 + zu[1] * isu1;
                    Hk[hp(10, 8)] = -sc * 2.0 * R2; Hk[hp(11, 9)] = -sc * 2.0 * R3;
                }
            }
            if (uon) {
                lm_columns(m, SH.SC[k], LM_G * ca, LM_G * cb, lamn, Mk, jl, SH.JL[k]);
            } else {
#pragma unroll
                for (int i = 0; i < 10; ++i) jl[i] = 0.0;
            }
            // outgoing augmented defect c_k = [F(z_k); u_k] - x~_{k+1} -> defect column of M~
            double cdef[10];
#pragma unroll
            for (int i = 0; i < 8; ++i) { const double t = from_next(x[i]); cdef[i] = xn[i] - t; }
            { const double t0 = from_next(up[0]), t1 = from_next(up[1]); cdef[8] = u[0] - t0; cdef[9] = u[1] - t1; }
            if (uon) {
#pragma unroll
                for (int r = 0; r < 10; ++r) Mk[12 * NC + r] = cdef[r];
            }
            // incoming defect g_k: primal residuals now, -g_0 = dx~_0 for the forward sweep
            double pl = 0.0, plu = 0.0;
#pragma unroll
            for (int i = 0; i < 10; ++i) {
                const double t = from_prev(cdef[i]);
                double gi = -t;
                if (k == 0) gi = i < 8 ? x[i] - st0[i] : up[i - 8] - upv[i - 8];
                const double d = i < 8 ? dsc[i] : 1.0;
                pl = fmax(pl, xon ? d * fabs(gi) : 0.0);
                plu = fmax(plu, xon ? fabs(gi) : 0.0);
                if (k == 0) S->dx0[i] = -gi;
            }
            SH.JL[k][10] = pl; SH.JL[k][11] = plu;      // primal residual maxima (LDS: frees registers)
        }
        double dinf = 0.0, c0 = 0.0, cmin = 1e300, suml = 0.0, sumz = 0.0;
        double pinf = SH.JL[k][10], pinf_u = SH.JL[k][11];
        {
            double gl[12];
            cost_grad(x, u, up, gl);
#pragma unroll
            for (int j = 0; j < 12; ++j) gl[j] *= sc;
#pragma unroll
            for (int i = 0; i < 10; ++i) gl[i] += lam[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) gl[j] -= jl[j];
            gl[10] -= jl[8] + lamn[8] + zl[0] - zu[0];
            gl[11] -= jl[9] + lamn[9] + zl[1] - zu[1];
#pragma unroll
            for (int j = 0; j < 12; ++j) dinf = fmax(dinf, (j < 10 ? xon : uon) ? fabs(gl[j]) : 0.0);
#pragma unroll
            for (int i = 0; i < 10; ++i) suml += xon ? fabs(lam[i]) / (i < 8 ? dsc[i] : 1.0) : 0.0;
#pragma unroll
            for (int j = 0; j < 2; ++j) if (uon) {
                const double cl = zl[j] * (u[j] - lo), cu = zu[j] * (hi - u[j]);
                c0 = fmax(c0, fmax(cl, cu)); cmin = fmin(cmin, fmin(cl, cu)); sumz += zl[j] + zu[j];
            }
        }
        dinf = wmaxf((float)dinf); pinf = wmaxf((float)pinf); pinf_u = wmaxf((float)pinf_u); c0 = wmaxf((float)c0);
        const double cminw = wminf((float)cmin);
        suml = wsumf((float)suml); sumz = wsumf((float)sumz);
        const double s_d = fmax(100.0, (suml + sumz) / (nA + nb)) / 100.0;
        const double s_c = fmax(100.0, sumz / nb) / 100.0;
        const double err = fmax(dinf / s_d, fmax(pinf, c0 / s_c));
        // IPOPT OptimalityErrorConvergenceCheck: optimal, then acceptable, then the iteration cap
        if (err <= tol && dinf <= sc && pinf_u <= 1e-4 && c0 <= 1e-4 * sc) { status = 0; break; }
        if (a.acc_iter > 0 && err <= a.acc_tol && pinf_u <= 1e-2 && c0 <= 1e-2 * sc) {
            if (++acc_count >= a.acc_iter) { status = 1; break; }
        } else {
            acc_count = 0;
        }
        if (it >= a.max_iter) { status = -1; break; }
        for (;;) {
            const double cmu = fmax(c0 - mu, mu - cminw);
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * mu || mu <= mu_min) break;
            mu = fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu)));
            nfilt = 0;
        }
        const double tau = fmax(0.99, 1.0 - mu);
        STAMP(1);

        // ---------------- gradient rows (they depend on mu) ------------------------------------
        {
            double gq[12];
            cost_grad(x, u, up, gq);
#pragma unroll
            for (int j = 0; j < 12; ++j) gq[j] *= sc;
            if (uon) {
                gq[10] += -mu * isl0 + mu * isu0; gq[11] += -mu * isl1 + mu * isu1;
#pragma unroll
                for (int j = 0; j < 12; ++j) Hk[hp(12, j)] = gq[j];
            }
            if (k == N) {   // terminal value function [[2 Qt, q_N], [q_N^T, 0]] on x~ (packed, NP = 11)
                double* PN = S->PK[N];
                for (int e = 0; e < LmLds::NPT; ++e) PN[e] = 0.0;
#pragma unroll
                for (int i = 0; i < 8; ++i) PN[hp(i, i)] = sc * 2.0 * Qt[i];
#pragma unroll
                for (int j = 0; j < 10; ++j) PN[hp(10, j)] = gq[j];
            }
        }
        __syncthreads();
        STAMP(2);

        // ---------------- Newton step: Riccati with inertia correction -----------------------
        double delta = 0.0, dapplied = 0.0;
        bool ok = riccati3_sweep(S, N, RR);
        int attempt = 1;
        for (; attempt < 60 && !ok; ++attempt) {
            delta = (attempt == 1) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last / 3.0))
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            const double dd = delta - dapplied;
            if (uon) {
#pragma unroll
                for (int j = 0; j < 12; ++j) Hk[hp(j, j)] += dd;
            }
            if (k == N) {
#pragma unroll
                for (int j = 0; j < 10; ++j) S->PK[N][hp(j, j)] += dd;
            }
            dapplied = delta;
            __syncthreads();
            ok = riccati3_sweep(S, N, RR);
        }
        STAMP_ADD(9, attempt);
        STAMP(3);
        if (!ok) { status = -3; break; }
        if (delta > 0.0) delta_last = delta;
        closed_loop3(S, N);
        double dx[10], dU[2], lamp[10];
        forward_sweep(S, N, k, dx);
        asm volatile("" ::: "memory");     // keep the K / Pt reads below after the sweep (register pressure)
        {
            const int kk = xon ? k : 0;
            const double* K0 = S->PK[uon ? k : 0] + LmLds::NPT;
            const double* K1 = K0 + LmLds::NP;
            double d0 = K0[10], d1 = K1[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) { d0 = fma(K0[j], dx[j], d0); d1 = fma(K1[j], dx[j], d1); }
            dU[0] = uon ? d0 : 0.0; dU[1] = uon ? d1 : 0.0;
            node_multiplier3(S, kk, dx, lamp);
        }
        STAMP(4);
        double dzl[2], dzu[2];
        dzl[0] = uon ? mu * isl0 - zl[0] - zl[0] * isl0 * dU[0] : 0.0;
        dzl[1] = uon ? mu * isl1 - zl[1] - zl[1] * isl1 * dU[1] : 0.0;
        dzu[0] = uon ? mu * isu0 - zu[0] + zu[0] * isu0 * dU[0] : 0.0;
        dzu[1] = uon ? mu * isu1 - zu[1] + zu[1] * isu1 * dU[1] : 0.0;
        double amax = 1.0, az = 1.0;
        if (uon) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (dU[j] < 0) amax = fmin(amax, -tau * (u[j] - lo) / dU[j]);
                if (dU[j] > 0) amax = fmin(amax, tau * (hi - u[j]) / dU[j]);
                if (dzl[j] < 0) az = fmin(az, -tau * zl[j] / dzl[j]);
                if (dzu[j] < 0) az = fmin(az, -tau * zu[j] / dzu[j]);
            }
        }
        amax = (double)wminf((float)amax) * (1.0 - 1.0 / 1048576.0);
        az = (double)wminf((float)az) * (1.0 - 1.0 / 1048576.0);
        STAMP(5);

        // ---------------- filter line search -------------------------------------------------
        double phil = sc * cost_val(x, u, up), gtdl = 0.0;
        if (uon) phil -= mu * log((u[0] - lo) * (hi - u[0]) * (u[1] - lo) * (hi - u[1]));
        {
            double gz_[12];
            cost_grad(x, u, up, gz_);
#pragma unroll
            for (int i = 0; i < 10; ++i) gtdl += xon ? sc * gz_[i] * dx[i] : 0.0;
            if (uon) gtdl += (sc * gz_[10] - mu * isl0 + mu * isu0) * dU[0] + (sc * gz_[11] - mu * isl1 + mu * isu1) * dU[1];
        }
        const double phi = wsum(phil), gTd = wsum(gtdl);
        const float lg_th = theta > 0.0 ? lg2(theta) : -3.0e38f;
        const float lg_gd = gTd < 0.0 ? lg2(-gTd) : 3.0e38f;
        const float lg_sw = (float)s_th * lg_th - (float)s_ph * lg_gd;
        double amin = gam_th;
        if (gTd < 0.0) amin = fmin(gam_th, fmin(gam_ph * theta / (-gTd), (double)__builtin_amdgcn_exp2f(fmaxf(lg_sw, -126.0f))));
        amin *= gam_al;
        double alpha = amax, th_t = 0.0, ph_t = 0.0;
        bool accepted = false, ftype = false;
        float tnl = 0.0f;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const double xi = i < 8 ? x[i] : up[i - 8];
            tnl = fmaxf(tnl, xon ? fabsf((float)dx[i]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)xi)) : 0.0f);
        }
        if (uon) {
#pragma unroll
            for (int j = 0; j < 2; ++j) tnl = fmaxf(tnl, fabsf((float)dU[j]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)u[j])));
        }
        const bool tiny = wmaxf(tnl) < 2.2e-15f;
        STAMP(6);
        int ls = 0;
        for (; ls < 80; ++ls) {
            double xt[8], pt[2], ut[2], gt[10];
#pragma unroll
            for (int i = 0; i < 8; ++i) xt[i] = fma(alpha, dx[i], x[i]);
            pt[0] = fma(alpha, dx[8], up[0]); pt[1] = fma(alpha, dx[9], up[1]);
            ut[0] = fma(alpha, dU[0], u[0]); ut[1] = fma(alpha, dU[1], u[1]);
            defects(xt, pt, ut, gt);
            double phl = sc * cost_val(xt, ut, pt);
            if (uon) phl -= mu * log((ut[0] - lo) * (hi - ut[0]) * (ut[1] - lo) * (hi - ut[1]));
            th_t = wsum(theta_of(gt)); ph_t = wsum(phl);
            if (tiny) { accepted = true; ftype = true; break; }
            bool in_filter = !(th_t < th_max) || !isfinite(ph_t);
            in_filter = in_filter || wany(k < nfilt && th_t >= fth && ph_t >= fph);
            if (!in_filter) {
                const bool sw = gTd < 0.0 && lg2(alpha) > lg_sw;
                if (theta <= th_min && sw) {
                    if (cmp_le(ph_t, phi + eta_ph * alpha * gTd, phi)) { accepted = true; ftype = true; }
                } else if (cmp_le(th_t, (1 - gam_th) * theta, theta) || cmp_le(ph_t - phi, -gam_ph * theta, phi)) {
                    accepted = true;
                }
            }
            if (accepted) break;
            alpha *= 0.5;
            if (alpha < amin) break;
        }
        STAMP_ADD(10, ls + 1);
        STAMP(7);
        if (!accepted) { status = -2; break; }
        if (!ftype && nfilt < kWave) {
            if (k == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
            ++nfilt;
        }
        // ---------------- accept ------------------------------------------------------------
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = xon ? fma(alpha, dx[i], x[i]) : x[i];
        up[0] = xon ? fma(alpha, dx[8], up[0]) : up[0];
        up[1] = xon ? fma(alpha, dx[9], up[1]) : up[1];
#pragma unroll
        for (int i = 0; i < 10; ++i) lam[i] = xon ? fma(alpha, lamp[i] - lam[i], lam[i]) : 0.0;
        if (uon) {
            u[0] = fma(alpha, dU[0], u[0]); u[1] = fma(alpha, dU[1], u[1]);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double il = frcp(u[j] - lo), iu = frcp(hi - u[j]);
                zl[j] = fmax(fmin(fma(az, dzl[j], zl[j]), 1e10 * mu * il), 1e-10 * mu * il);
                zu[j] = fmax(fmin(fma(az, dzu[j], zu[j]), 1e10 * mu * iu), 1e-10 * mu * iu);
            }
        }
        theta = th_t;
        STAMP(8);
    }

    // ---------------- outputs -------------------------------------------------------------
    const double fval = wsum(cost_val(x, u, up));
    if (k == 0) {
        a.u0[2 * b] = u[0]; a.u0[2 * b + 1] = u[1];
        a.f[b] = fval; a.status[b] = status; a.iters[b] = it;
    }
    if (a.w_out) {
        double* wo = a.w_out + (size_t)nw * b;
        if (xon) {
#pragma unroll
            for (int i = 0; i < 8; ++i) wo[8 * k + i] = x[i];
        }
        if (uon) { wo[8 * (N + 1) + 2 * k] = u[0]; wo[8 * (N + 1) + 2 * k + 1] = u[1]; }
    }
    STAMP_FLUSH_TO(g_stamp_lm, b);
}

}  // namespace dartmpc

extern "C" size_t dartmpc_lmpc_lds_bytes(void) { return sizeof(dartmpc::LmShared); }

extern "C" hipError_t dartmpc_launch_lmpc(const dartmpc::LmpcArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    if (args->N < 1 || args->N >= dartmpc::LM_NMAXS) return hipErrorInvalidValue;
    static bool attr_set = false;
    const size_t lds = sizeof(dartmpc::LmShared);
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)dartmpc::lmpc_ipm_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(dartmpc::lmpc_ipm_kernel, dim3(args->B), dim3(dartmpc::kWave), lds, stream, *args);
    return hipGetLastError();
}

#ifdef DART_STAMPS
extern "C" hipError_t dartmpc_read_stamps_lmpc(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_lm), sizeof(unsigned long long) * 12, 0,
                               hipMemcpyDeviceToHost);
}
#endif
