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
// Exact derivatives as IPOPT gets them from CasADi: per direction of z = [x; u], the RK4 tangent
// (a column of the step Jacobian) and a second-order adjoint sweep back through the four stages
// (a column of the exact Hessian of lambda^T x+), from per-stage derivative data staged in LDS.
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
    // per node (row 32: scratch of the idle lanes), per RK stage: d f / d y coefficients, and the
    // second-derivative data turned into adjoint-weighted curvature coefficients
    NodeArr<double[4][LM_NSC], LM_NMAXS + 1> SC;
    NodeArr<double[4][8], LM_NMAXS + 1> SD;
    NodeArr<double[12], LM_NMAXS + 1> JL;      // J^T lambda_{k+1} staging, primal residual maxima
    NodeArr<double[14], LM_NMAXS + 1> DL;      // per node: lambda_{k+1}, tilt curvature, g cos(u) for the mirror lanes
    NodeArr<double[10], LM_NMAXS + 1> CS;      // second-order correction: c_soc rows of node k (incoming defect)
    NodeArr<double[22], LM_NMAXS + 1> SV;      // second-order correction: the plain step (dx~, lambda+, du) of node k
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

__device__ __forceinline__ void lm_rk4(const LmModel& mlds, const double* x, double sa, double sb, double* xn) {
    const LmModel m = mlds;     // model to registers once (LDS round trips off the stage chains)
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

// Value pass of RK4 that also stores, per stage s, the tangent coefficients sc[s][10] (the
// nonzero entries of d f / d y at y_s) and the second-derivative data sd[s][8] = [S''(vx),
// S''(slip x), S''(vy), S''(slip y), S''(om_x), S''(om_y), sin th_x, sin th_y].
__device__ __forceinline__ void lm_rk4_lin(const LmModel& mlds, const double* x, double sa, double sb, double* xn,
                                           double (*sc)[LM_NSC], double (*sd)[8]) {
    const LmModel m = mlds;     // model to registers once: the stage loop reads every field ~4 times
    double y[8], acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { y[i] = x[i]; acc[i] = 0.0; }
#pragma unroll 1
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        // each friction term's value / slope / curvature goes into k, sc, sd as soon as it exists
        // (short live ranges: this pass runs under heavy register pressure)
        double k[8];
        k[0] = y[1]; k[2] = y[3]; k[4] = y[5]; k[6] = y[7];
        {
            double Sfx, Sfx1, Sfx2, Srx, Srx1, Srx2;
            strb_d(m.sx, y[1], Sfx, Sfx1, Sfx2);
            strb_d(m.sx, fma(-m.r_x, y[7], y[1]), Srx, Srx1, Srx2);
            sd[s][0] = Sfx2; sd[s][1] = Srx2;
            sc[s][0] = (-m.c_x - Sfx1 - Srx1) * m.im_x;
            sc[s][1] = m.r_x * Srx1 * m.im_x;
            sc[s][7] = -m.r_x * Srx1 * m.iIy;
            k[1] = (m.m_x * (LM_G * sa) - m.c_x * y[1] - m.k_x * y[0] - Sfx - Srx) * m.im_x;
            k[7] = -m.r_x * Srx;                                   // completed below
            double Sny, Sny1, Sny2, sty, cty;
            strb_d(m.sry, y[7], Sny, Sny1, Sny2);
            sincos_any(y[6], sty, cty);
            sd[s][5] = Sny2; sd[s][7] = sty;
            sc[s][8] = (m.r_x * m.r_x * Srx1 - Sny1 - m.c_ry) * m.iIy;
            sc[s][9] = -m.tqy * cty * m.iIy;
            k[7] = (k[7] - Sny - m.c_ry * y[7] - m.tqy * sty) * m.iIy;
        }
        {
            double Sfy, Sfy1, Sfy2, Sry, Sry1, Sry2;
            strb_d(m.sy, y[3], Sfy, Sfy1, Sfy2);
            strb_d(m.sy, fma(m.r_y, y[5], y[3]), Sry, Sry1, Sry2);
            sd[s][2] = Sfy2; sd[s][3] = Sry2;
            sc[s][2] = (-m.c_y - Sfy1 - Sry1) * m.im_y;
            sc[s][3] = -m.r_y * Sry1 * m.im_y;
            sc[s][4] = -m.r_y * Sry1 * m.iIx;
            k[3] = (m.m_y * (LM_G * sb) - m.c_y * y[3] - m.k_y * y[2] - Sfy - Sry) * m.im_y;
            k[5] = -m.r_y * Sry;                                   // completed below
            double Snx, Snx1, Snx2, stx, ctx;
            strb_d(m.srx, y[5], Snx, Snx1, Snx2);
            sincos_any(y[4], stx, ctx);
            sd[s][4] = Snx2; sd[s][6] = stx;
            sc[s][5] = (-m.r_y * m.r_y * Sry1 - Snx1 - m.c_rx) * m.iIx;
            sc[s][6] = -m.tqx * ctx * m.iIx;
            k[5] = (k[5] - Snx - m.c_rx * y[5] - m.tqx * stx) * m.iIx;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fma(wts, k[i], acc[i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = fma(cst * m.h, k[i], x[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) xn[i] = fma(m.h / 6.0, acc[i], x[i]);
}

// q = (d f / d y at stage s)^T v from the stage's tangent coefficients
__device__ __forceinline__ void lm_jtv(const LmModel& m, const double* c, const double* v, double* q) {
    const double kx1 = -m.k_x * m.im_x, ky3 = -m.k_y * m.im_y;
    q[0] = kx1 * v[1];
    q[1] = fma(c[0], v[1], fma(c[7], v[7], v[0]));
    q[2] = ky3 * v[3];
    q[3] = fma(c[2], v[3], fma(c[4], v[5], v[2]));
    q[4] = c[6] * v[5];
    q[5] = fma(c[3], v[3], fma(c[5], v[5], v[4]));
    q[6] = c[9] * v[7];
    q[7] = fma(c[1], v[1], fma(c[8], v[7], v[6]));
}

// First-order adjoint of L = nl^T x+ (nl = -lambda_{k+1}) through the four RK4 stages; converts the
// stage second-derivative data sd[s] in place into the curvature coefficients of kb_s^T f'' at y_s:
// [A1, A2, A3, B1, B2, B3, C1, C2] with (vx, om_y) block [[A1, A2], [A2, A3]], (vy, om_x) block
// [[B1, B2], [B2, B3]], th_x: C1, th_y: C2; returns the tilt curvature huu[2] = sum_s kb_s^T f_uu.
__device__ __forceinline__ void lm_adjoint_curv(const LmModel& m, const double (*sc)[LM_NSC], double (*sd)[8],
                                                const double* lamn, double sa, double sb, double* huu) {
    double kb[8], yb[8];
    const double h = m.h;
#pragma unroll
    for (int i = 0; i < 8; ++i) kb[i] = -(h / 6.0) * lamn[i];        // kb_4
    huu[0] = 0.0; huu[1] = 0.0;
#pragma unroll 1
    for (int s = 3; s >= 0; --s) {
        double* d = sd[s];
        const double c_vx = kb[1] * (-d[0] * m.im_x);
        const double c_sx = kb[1] * (-d[1] * m.im_x) + kb[7] * (-m.r_x * d[1] * m.iIy);
        const double c_vy = kb[3] * (-d[2] * m.im_y);
        const double c_sy = kb[3] * (-d[3] * m.im_y) + kb[5] * (-m.r_y * d[3] * m.iIx);
        const double c_ox = kb[5] * (-d[4] * m.iIx);
        const double c_oy = kb[7] * (-d[5] * m.iIy);
        const double c_tx = kb[5] * (m.tqx * d[6] * m.iIx);
        const double c_ty = kb[7] * (m.tqy * d[7] * m.iIy);
        d[0] = c_vx + c_sx; d[1] = -m.r_x * c_sx; d[2] = fma(m.r_x * m.r_x, c_sx, c_oy);
        d[3] = c_vy + c_sy; d[4] = m.r_y * c_sy; d[5] = fma(m.r_y * m.r_y, c_sy, c_ox);
        d[6] = c_tx; d[7] = c_ty;
        huu[0] = fma(kb[1], -LM_G * sa, huu[0]);
        huu[1] = fma(kb[3], -LM_G * sb, huu[1]);
        if (s > 0) {      // kb_{s-1} = w_{s-1} h/6 nl + c_s h J_s^T kb_s  (c = 1, 1/2, 1/2 for s = 3, 2, 1)
            lm_jtv(m, sc[s], kb, yb);
            const double cs = s == 3 ? h : 0.5 * h, ws = (s == 1 ? 1.0 : 2.0) * h / 6.0;
#pragma unroll
            for (int i = 0; i < 8; ++i) kb[i] = fma(cs, yb[i], -ws * lamn[i]);
        }
    }
}

// Direction d (0..7 state, 8..9 tilt): tangent of RK4 -> column d of the step Jacobian (written to
// column jc(d) of M~, returns col . lamn), then the second-order adjoint sweep back through the
// stages -> column d of the exact Hessian of -lambda^T x+ over z = [x; u], written to the packed
// stage Hessian (rows i >= d).
__device__ __forceinline__ double lm_direction(const LmModel& m, const double (*sc)[LM_NSC], const double (*cv)[8],
                                               const double* huu, double gca, double gcb, int d, const double* lamn,
                                               double* Mk, double* Hk) {
    double yd[4][8], acc[8], e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { e[i] = (i == d) ? 1.0 : 0.0; yd[0][i] = e[i]; acc[i] = 0.0; }
    const double fa = d == 8 ? gca : 0.0, fb = d == 9 ? gcb : 0.0;
    const double kx1 = -m.k_x * m.im_x, ky3 = -m.k_y * m.im_y;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        const double* c = sc[s];
        const double* y = yd[s];
        double k[8];
        k[0] = y[1]; k[2] = y[3]; k[4] = y[5]; k[6] = y[7];
        k[1] = fma(kx1, y[0], fma(c[0], y[1], fma(c[1], y[7], fa)));
        k[3] = fma(ky3, y[2], fma(c[2], y[3], fma(c[3], y[5], fb)));
        k[5] = fma(c[4], y[3], fma(c[5], y[5], c[6] * y[4]));
        k[7] = fma(c[7], y[1], fma(c[8], y[7], c[9] * y[6]));
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fma(wts, k[i], acc[i]);
        if (s < 3) {
#pragma unroll
            for (int i = 0; i < 8; ++i) yd[s + 1][i] = fma(cst * m.h, k[i], e[i]);
        }
    }
    const int jc = d < 8 ? d : d + 2;
    double dot = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double col = fma(m.h / 6.0, acc[i], e[i]);
        Mk[jc * LmLds::NC + i] = col;
        dot = fma(col, lamn[i], dot);
    }
    // second-order adjoint: kbd_s = d/dd kb_s, ybd_s = J_s^T kbd_s + (kb_s^T f'')_s yd_s
    double kbd[8], hx[8], hu0 = d == 8 ? huu[0] : 0.0, hu1 = d == 9 ? huu[1] : 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) { kbd[i] = 0.0; hx[i] = 0.0; }
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        const double* cc = cv[s];
        const double* y = yd[s];
        double q[8];
        lm_jtv(m, sc[s], kbd, q);
        q[1] = fma(cc[0], y[1], fma(cc[1], y[7], q[1]));
        q[7] = fma(cc[1], y[1], fma(cc[2], y[7], q[7]));
        q[3] = fma(cc[3], y[3], fma(cc[4], y[5], q[3]));
        q[5] = fma(cc[4], y[3], fma(cc[5], y[5], q[5]));
        q[4] = fma(cc[6], y[4], q[4]);
        q[6] = fma(cc[7], y[6], q[6]);
        hu0 = fma(gca, kbd[1], hu0);
        hu1 = fma(gcb, kbd[3], hu1);
#pragma unroll
        for (int i = 0; i < 8; ++i) hx[i] += q[i];
        const double cs = s == 3 ? m.h : 0.5 * m.h;
#pragma unroll
        for (int i = 0; i < 8; ++i) kbd[i] = cs * q[i];
    }
    // rows i >= d of column d (z indices: x 0..7, tilt 10, 11)
    const int zd = jc;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (i >= d) Hk[hp(i, zd)] = hx[i];
    Hk[hp(10, zd)] = hu0;
    Hk[hp(11, zd)] = hu1;
    return dot;
}

// all ten directions, one at a time; J^T lambda_{k+1} into jl[10]
__device__ __forceinline__ void lm_directions(const LmModel& m, const double (*sc)[LM_NSC], const double (*cv)[8],
                                              const double* huu, double gca, double gcb, const double* lamn, double* Mk,
                                              double* Hk, double* jl, double* jl_lds) {
#pragma unroll 1
    for (int d = 0; d < 10; ++d) jl_lds[d] = lm_direction(m, sc, cv, huu, gca, gcb, d, lamn, Mk, Hk);
#pragma unroll
    for (int d = 0; d < 10; ++d) jl[d] = jl_lds[d];
}

// directions d0 .. d0+4 of one node (the two half-waves of the wave split the ten directions);
// per-node inputs from LDS: dl = [lambda_{k+1}(10), huu(2), g cos a, g cos b]
__device__ __forceinline__ void lm_directions_half(const LmModel& m, const double (*sc)[LM_NSC], const double (*cv)[8],
                                                   const double* dl, int d0, double* Mk, double* Hk, double* jl_lds) {
    double lamn[10], huu[2];
#pragma unroll
    for (int i = 0; i < 10; ++i) lamn[i] = dl[i];
    huu[0] = dl[10]; huu[1] = dl[11];
    const double gca = dl[12], gcb = dl[13];
    const LmModel mr = m;       // model to registers once for the five directions
#pragma unroll 1
    for (int d = d0; d < d0 + 5; ++d) jl_lds[d] = lm_direction(mr, sc, cv, huu, gca, gcb, d, lamn, Mk, Hk);
}

__global__ __launch_bounds__(kWave) void lmpc_ipm_kernel(LmpcArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LmShared& SH = *reinterpret_cast<LmShared*>(smem);
    LmLds* S = &SH.ocp;
    const Riccati3Roles<LmLds> RR = riccati3_roles<LmLds>();
    STAMP_DECL
    if (blockIdx.x % a.pack) return;          // small batches packed onto one XCD (launcher)
    const int b = blockIdx.x / a.pack;
    const int k = threadIdx.x;
    const int N = a.N;
    const bool xon = k <= N, uon = k < N;
    const int sr = xon ? k : LM_NMAXS;        // per-node LDS scratch row (idle lanes share row 32)
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
        double sa, ca, sb, cb, xn[8], huu[2];
        const double lz[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        tilt_sincos(poly, u[0], sa, ca);
        tilt_sincos(poly, u[1], sb, cb);
        lm_rk4_lin(m, x, sa, sb, xn, SH.SC[sr], SH.SD[sr]);
        lm_adjoint_curv(m, SH.SC[sr], SH.SD[sr], lz, sa, sb, huu);
        double* Mt = &S->M[xon ? k : 0][0][0];
        if (uon) {
            double jl0[10];
            lm_directions(m, SH.SC[sr], SH.SD[sr], huu, LM_G * ca, LM_G * cb, lz, Mt, Hk, jl0, SH.JL[sr]);
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
            lm_rk4_lin(m, x, sa, sb, xn, SH.SC[sr], SH.SD[sr]);
            {
                double huu[2];
                lm_adjoint_curv(m, SH.SC[sr], SH.SD[sr], lamn, sa, sb, huu);
                if (k < 32) {
#pragma unroll
                    for (int i = 0; i < 10; ++i) SH.DL[k][i] = lamn[i];
                    SH.DL[k][10] = huu[0]; SH.DL[k][11] = huu[1]; SH.DL[k][12] = LM_G * ca; SH.DL[k][13] = LM_G * cb;
                }
                __syncthreads();
                STAMP(13);
                {   // exact dynamics Hessian (x, u blocks) and the Jacobian columns: lanes k and k + 32 take
                    // directions 0..4 and 5..9 of node k
                    const int kn = k & 31;
                    if (kn < N)
                        lm_directions_half(m, SH.SC[kn], SH.SD[kn], SH.DL[kn], k < 32 ? 0 : 5, &S->M[kn][0][0], S->H[kn],
                                           SH.JL[kn]);
                }
                __syncthreads();
                STAMP(14);
                if (uon) {
                    // the cost / barrier terms: z = [x(8), up(2), u(2), 1], gradient row later
#pragma unroll
                    for (int i = 0; i < 10; ++i) jl[i] = SH.JL[sr][i];
#pragma unroll
                    for (int i = 0; i < 8; ++i) Hk[hp(i, i)] += sc * 2.0 * Q[i];
                    Hk[hp(8, 8)] = sc * 2.0 * R2; Hk[hp(9, 9)] = sc * 2.0 * R3;
                    Hk[hp(10, 10)] += sc * 2.0 * (R0 + R2) + zl[0] * isl0 + zu[0] * isu0;
                    Hk[hp(11, 11)] += sc * 2.0 * (R1 + R3) + zl[1] * isl1 + zu[1] * isu1;
                    Hk[hp(10, 8)] = -sc * 2.0 * R2; Hk[hp(11, 9)] = -sc * 2.0 * R3;
                } else {
#pragma unroll
                    for (int i = 0; i < 10; ++i) jl[i] = 0.0;
                }
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
                SH.CS[sr][i] = gi;       // c(x) for a second-order correction
            }
            SH.JL[sr][10] = pl; SH.JL[sr][11] = plu;    // primal residual maxima (LDS: frees registers)
        }
        double dinf = 0.0, c0 = 0.0, cmin = 1e300, suml = 0.0, sumz = 0.0;
        double pinf = SH.JL[sr][10], pinf_u = SH.JL[sr][11];
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

        // ---------------- Newton step and filter line search ----------------------------------
        // One copy of the Riccati solve serves the plain Newton step (with inertia correction) and
        // IPOPT's second-order correction passes (FilterLSAcceptor::TrySecondOrderCorrection; max_soc,
        // kappa_soc 0.99): a rejected full step with theta(trial) >= theta re-solves the system with
        // c_soc <- alpha_soc c_soc + c(x_trial) (from c(x), alpha_soc = alpha) in the defect column of
        // M~ and dx~_0 (H~, incl. the inertia shift, is unchanged) and tries x + alpha_soc d_soc.
        double dx[10], dU[2], lamp[10], gt[10], dzl[2], dzu[2];
        double amax = 1.0, az = 1.0, phi = 0.0, gTd = 0.0, amin = 0.0, alpha = 1.0, th_t = 0.0, ph_t = 0.0;
        double th_prev = 0.0;
        float lg_sw = 0.0f;
        bool accepted = false, ftype = false, tiny = false, ok = true;
        int ls = 0, soc = -1;        // soc: -1 plain step, >= 0 second-order-correction pass
        // the Newton step from the factorised value functions: forward sweep, du = K [dx~; 1], lambda+
        auto recover_step = [&]() {
            forward_sweep(S, N, k, dx);
            STAMP(12);
            asm volatile("" ::: "memory");     // keep the K / Pt reads below after the sweep (register pressure)
            const int kk = xon ? k : 0;
            const double* K0 = S->PK[uon ? k : 0] + LmLds::NPT;
            const double* K1 = K0 + LmLds::NP;
            double d0 = K0[10], d1 = K1[10];
#pragma unroll
            for (int j = 0; j < 10; ++j) { d0 = fma(K0[j], dx[j], d0); d1 = fma(K1[j], dx[j], d1); }
            dU[0] = uon ? d0 : 0.0; dU[1] = uon ? d1 : 0.0;
            node_multiplier3(S, kk, dx, lamp);
        };
        // primal fraction to the boundary of dU (wave-uniform)
        auto primal_ftb = [&]() {
            double am = 1.0;
            if (uon) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (dU[j] < 0) am = fmin(am, -tau * (u[j] - lo) / dU[j]);
                    if (dU[j] > 0) am = fmin(am, tau * (hi - u[j]) / dU[j]);
                }
            }
            return (double)wminf((float)am) * (1.0 - 1.0 / 1048576.0);
        };
        // bound-multiplier directions of dU and their fraction to the boundary (wave-uniform)
        auto dual_step = [&]() {
            dzl[0] = uon ? mu * isl0 - zl[0] - zl[0] * isl0 * dU[0] : 0.0;
            dzl[1] = uon ? mu * isl1 - zl[1] - zl[1] * isl1 * dU[1] : 0.0;
            dzu[0] = uon ? mu * isu0 - zu[0] + zu[0] * isu0 * dU[0] : 0.0;
            dzu[1] = uon ? mu * isu1 - zu[1] + zu[1] * isu1 * dU[1] : 0.0;
            double az_ = 1.0;
            if (uon) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (dzl[j] < 0) az_ = fmin(az_, -tau * zl[j] / dzl[j]);
                    if (dzu[j] < 0) az_ = fmin(az_, -tau * zu[j] / dzu[j]);
                }
            }
            return (double)wminf((float)az_) * (1.0 - 1.0 / 1048576.0);
        };
        // trial point x + al d: incoming defects gt of node k, wave-summed theta and barrier objective
        auto trial = [&](double al) {
            double xt[8], pt[2], ut[2];
#pragma unroll
            for (int i = 0; i < 8; ++i) xt[i] = fma(al, dx[i], x[i]);
            pt[0] = fma(al, dx[8], up[0]); pt[1] = fma(al, dx[9], up[1]);
            ut[0] = fma(al, dU[0], u[0]); ut[1] = fma(al, dU[1], u[1]);
            defects(xt, pt, ut, gt);
            double phl = sc * cost_val(xt, ut, pt);
            if (uon) phl -= mu * log((ut[0] - lo) * (hi - ut[0]) * (ut[1] - lo) * (hi - ut[1]));
            th_t = wsum(theta_of(gt)); ph_t = wsum(phl);
        };
        // filter acceptance of (th_t, ph_t) for the step size al_test (IPOPT alpha_primal_test)
        auto acceptable = [&](double al_test, bool& ft) {
            bool in_filter = !(th_t < th_max) || !isfinite(ph_t);
            in_filter = in_filter || wany(k < nfilt && th_t >= fth && ph_t >= fph);
            if (in_filter) return false;
            const bool sw = gTd < 0.0 && lg2(al_test) > lg_sw;
            if (theta <= th_min && sw) {
                if (cmp_le(ph_t, phi + eta_ph * al_test * gTd, phi)) { ft = true; return true; }
                return false;
            }
            return cmp_le(th_t, (1 - gam_th) * theta, theta) || cmp_le(ph_t - phi, -gam_ph * theta, phi);
        };
        for (;;) {
            // Riccati (one call site): plain step with inertia correction, or a second-order
            // correction with the same factorisation and the defects c_soc
            if (soc >= 0) {
                double cs[10];
#pragma unroll
                for (int i = 0; i < 10; ++i) cs[i] = xon ? SH.CS[sr][i] : 0.0;
#pragma unroll
                for (int r = 0; r < 10; ++r) {
                    const double t = from_next(cs[r]);
                    if (uon) Mk[12 * NC + r] = -t;
                    if (k == 0) S->dx0[r] = -cs[r];
                }
                __syncthreads();
                STAMP_ADD(15, 1);
            }
            {
                double delta = 0.0, dapplied = 0.0;
                int attempt = 0;
                for (;;) {
                    ok = riccati3_sweep(S, N, RR);
                    if (ok || soc >= 0 || ++attempt >= 60) break;
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
                }
                STAMP_ADD(9, attempt + 1);
                if (soc >= 0) ok = true;
                else if (ok && delta > 0.0) delta_last = delta;
            }
            STAMP(3);
            if (!ok) break;
            closed_loop3(S, N);
            STAMP(11);
            recover_step();
            STAMP(4);
            double al_try;
            if (soc < 0) {
                amax = primal_ftb();
                az = dual_step();
                STAMP(5);
                double phil = sc * cost_val(x, u, up), gtdl = 0.0;
                if (uon) phil -= mu * log((u[0] - lo) * (hi - u[0]) * (u[1] - lo) * (hi - u[1]));
                {
                    double gz_[12];
                    cost_grad(x, u, up, gz_);
#pragma unroll
                    for (int i = 0; i < 10; ++i) gtdl += xon ? sc * gz_[i] * dx[i] : 0.0;
                    if (uon) gtdl += (sc * gz_[10] - mu * isl0 + mu * isu0) * dU[0] + (sc * gz_[11] - mu * isl1 + mu * isu1) * dU[1];
                }
                phi = wsum(phil); gTd = wsum(gtdl);
                const float lg_th = theta > 0.0 ? lg2(theta) : -3.0e38f;
                const float lg_gd = gTd < 0.0 ? lg2(-gTd) : 3.0e38f;
                lg_sw = (float)s_th * lg_th - (float)s_ph * lg_gd;
                amin = gam_th;
                if (gTd < 0.0) amin = fmin(gam_th, fmin(gam_ph * theta / (-gTd), (double)__builtin_amdgcn_exp2f(fmaxf(lg_sw, -126.0f))));
                amin *= gam_al;
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
                tiny = wmaxf(tnl) < 2.2e-15f;
                alpha = amax;
                al_try = alpha;
                STAMP(6);
            } else {
                al_try = primal_ftb();
            }
            bool resolve = false;
            for (;;) {
                trial(al_try);
                if (soc < 0) {
                    if (tiny) { accepted = true; ftype = true; break; }
                    if (acceptable(alpha, ftype)) { accepted = true; break; }
                    if (ls == 0 && a.max_soc > 0 && !(th_t < theta)) {
                        if (xon) {      // c_soc = alpha c(x) + c(x_trial); keep the plain step
#pragma unroll
                            for (int i = 0; i < 10; ++i) {
                                SH.CS[sr][i] = fma(alpha, SH.CS[sr][i], gt[i]);
                                SH.SV[sr][i] = dx[i]; SH.SV[sr][10 + i] = lamp[i];
                            }
                            SH.SV[sr][20] = dU[0]; SH.SV[sr][21] = dU[1];
                        }
                        th_prev = th_t; soc = 0; resolve = true;
                        break;
                    }
                } else {
                    bool ft = false;
                    if (acceptable(alpha, ft)) {
                        accepted = true; ftype = ft; alpha = al_try;
                        az = dual_step();      // IPOPT takes the corrected solve as the whole step
                        break;
                    }
                    if (soc + 1 < a.max_soc && th_t <= 0.99 * th_prev) {
                        if (xon) {      // c_soc <- alpha_soc c_soc + c(x_soc trial)
#pragma unroll
                            for (int i = 0; i < 10; ++i) SH.CS[sr][i] = fma(al_try, SH.CS[sr][i], gt[i]);
                        }
                        th_prev = th_t; ++soc; resolve = true;
                        break;
                    }
                    if (xon) {      // corrections failed: back to the plain step, backtrack
#pragma unroll
                        for (int i = 0; i < 10; ++i) { dx[i] = SH.SV[sr][i]; lamp[i] = SH.SV[sr][10 + i]; }
                        dU[0] = SH.SV[sr][20]; dU[1] = SH.SV[sr][21];
                    }
                    soc = -1;
                }
                ++ls;
                alpha *= 0.5;
                if (alpha < amin || ls >= 80) break;
                al_try = alpha;
            }
            if (!resolve) break;
        }
        if (!ok) { status = -3; break; }
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
    dartmpc::LmpcArgs a = *args;
    a.pack = (a.B <= 32) ? 8 : 1;            // one XCD (and its L2) for the code of a small batch
    hipLaunchKernelGGL(dartmpc::lmpc_ipm_kernel, dim3(a.B * a.pack), dim3(dartmpc::kWave), lds, stream, a);
    return hipGetLastError();
}

#ifdef DART_STAMPS
extern "C" hipError_t dartmpc_read_stamps_lmpc(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_lm), sizeof(unsigned long long) * 16, 0,
                               hipMemcpyDeviceToHost);
}
#endif
