// rmpc_ipm.hip -- batched RMPC (regressor NMPC + fused RLS update) interior-point solve, gfx950.
//
// Replaces AdaptiveNPMPCSmooth.solve (RMPC/dev_dual/controller/
// np_mpc_adaptive_with_linear_regressor.py:212-222, NLP :35-168) and the per-step RLS
// update of the driver (RMPC/dev_dual/rob_ctrl.py:335-343, RLS :10-30) for a batch of
// independent instances.
//
// Model (np_mpc...:171-193): x = [px, vx, py, vy], u = [alpha, beta],
//   ax = gz sin(alpha) + phi(x).theta_x,  ay = gz sin(beta) + phi(x).theta_y,
//   phi = [px, vx, py, vy, tanh(vx/v_eps), tanh(vy/v_eps), 1],  RK4 with step Ts.
// NLP rows (:103-127): defects; Delta-u in [du_lo, du_hi] (u_{-1} = u_prev); velocity caps
// |vx|,|vy| <= vmax on nodes 0..N-1.  Cost (:129-140): staged reference, Ru |u|^2, Rdu |Du|^2.
//
// Method: IPOPT's primal-dual barrier method as in pmpc_ipm.hip (monotone mu, filter line search,
// inertia correction, bound_relax 1e-8, gradient scaling), with IPOPT's slack formulation of the
// inequality rows (g(w) - s = 0, bounds on s) eliminated per stage.  The Delta-u coupling is
// carried by the augmented state x~_k = [x_k; u_{k-1}] (nx~ = 6).  Exact derivatives as IPOPT
// gets them from CasADi: per direction the RK4 tangent (a Jacobian column) and a second-order
// adjoint sweep through the four stages (a column of the exact Hessian of lambda^T x+).
//
// Mapping: one wave64 per instance; lane k and its mirror lane k + 32 own shooting node k (N <= 31):
// both run the node-local work (model evaluation, multipliers, line search) and they split the six
// slack rows of the node three and three (slacks, slack multipliers, their steps and barrier terms);
// the node-coupled Riccati and forward sweeps run through LDS with the lanes sharing each node's dense
// algebra (ocp_wave.h).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ocp_wave.h"
#include "rmpc_ipm.h"
#include "stamps.h"
#include "wave.h"

// this kernel runs at the register limit: its double sums use the readlane cross-row step (wsum_rl)

namespace dartmpc {

constexpr int RM_NMAXS = 32;      // max shooting nodes (N <= 31)
constexpr int RM_NIQ = 6;         // inequality rows per node: du_x, du_y, vx-vmax, -vx-vmax, vy-vmax, -vy-vmax
constexpr int RM_NQ = 3;          // of them per lane: rows 0..2 on lane k, rows 3..5 on its mirror lane k + 32
static_assert(2 * RM_NQ == RM_NIQ, "the node and mirror lanes split the rows evenly");
using RmLds = OcpLds<6, RM_NMAXS>;

#ifdef DART_STAMPS
__device__ unsigned long long g_stamp_rm[16];
#endif

struct RmModel {
    double th[14];
    double gz, h, ie;             // gravity, Ts, 1/v_eps
};

struct RmShared {
    RmLds ocp;
    double theta[14];
    double rls_Pphi[2][7], rls_phiP[2][7];
    RmModel model;                            // uniform, read at the use sites (keeps VGPRs free)
    NodeArr<double[8], RM_NMAXS + 1> JL;      // J^T lambda staging, primal residual maxima
};

// continuous model (np_mpc...:178-186); also returns d f / d vx|vy of rows 1, 3 and tanh values
// (the node lane k evaluates tanh(vx / v_eps), its mirror lane k + 32 tanh(vy / v_eps) of the same node,
// and the pair exchange both: one tanh per lane instead of two, the same bits; EXEC must be full)
__device__ __forceinline__ void rm_f(const RmModel& m, const double* y, double sa, double sb, double* f,
                                     double& j1vx, double& j1vy, double& j3vx, double& j3vy, double& tx, double& ty,
                                     bool mir) {
    half_pair(tanh_econ((mir ? y[3] : y[1]) * m.ie), tx, ty);
    const double* a = m.th;
    const double* c = m.th + 7;
    f[0] = y[1];
    f[2] = y[3];
    f[1] = m.gz * sa + a[0] * y[0] + a[1] * y[1] + a[2] * y[2] + a[3] * y[3] + a[4] * tx + a[5] * ty + a[6];
    f[3] = m.gz * sb + c[0] * y[0] + c[1] * y[1] + c[2] * y[2] + c[3] * y[3] + c[4] * tx + c[5] * ty + c[6];
    const double dtx = (1.0 - tx * tx) * m.ie, dty = (1.0 - ty * ty) * m.ie;
    j1vx = a[1] + a[4] * dtx; j1vy = a[3] + a[5] * dty;
    j3vx = c[1] + c[4] * dtx; j3vy = c[3] + c[5] * dty;
}

// RK4 value (np_mpc...:188-193)
__device__ __forceinline__ void rm_rk4(const RmModel& mlds, const double* x, double sa, double sb, double* xn, bool mir) {
    const RmModel m = mlds;     // model to registers once (LDS round trips off the stage chains)
    double k[4], y[4], acc[4], d0, d1, d2, d3, tx, ty;
    rm_f(m, x, sa, sb, k, d0, d1, d2, d3, tx, ty, mir);
#pragma unroll
    for (int i = 0; i < 4; ++i) { acc[i] = k[i]; y[i] = x[i] + m.h / 2 * k[i]; }
    rm_f(m, y, sa, sb, k, d0, d1, d2, d3, tx, ty, mir);
#pragma unroll
    for (int i = 0; i < 4; ++i) { acc[i] += 2 * k[i]; y[i] = x[i] + m.h / 2 * k[i]; }
    rm_f(m, y, sa, sb, k, d0, d1, d2, d3, tx, ty, mir);
#pragma unroll
    for (int i = 0; i < 4; ++i) { acc[i] += 2 * k[i]; y[i] = x[i] + m.h * k[i]; }
    rm_f(m, y, sa, sb, k, d0, d1, d2, d3, tx, ty, mir);
#pragma unroll
    for (int i = 0; i < 4; ++i) xn[i] = x[i] + m.h / 6 * (acc[i] + k[i]);
}

// Value pass of RK4 storing per stage s the tangent coefficients sc[s] = [d f1/d vx, d f1/d vy,
// d f3/d vx, d f3/d vy] and the tanh curvature sd[s] = [T''(vx), T''(vy)] (T = tanh(v / v_eps)).
__device__ __forceinline__ void rm_rk4_lin(const RmModel& mlds, const double* x, double sa, double sb, double* xn,
                                           double (*sc)[4], double (*sd)[2], bool mir) {
    const RmModel m = mlds;     // model to registers once
    double y[4], acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { y[i] = x[i]; acc[i] = 0.0; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        double k[4], j1vx, j1vy, j3vx, j3vy, tx, ty;
        rm_f(m, y, sa, sb, k, j1vx, j1vy, j3vx, j3vy, tx, ty, mir);
        sc[s][0] = j1vx; sc[s][1] = j1vy; sc[s][2] = j3vx; sc[s][3] = j3vy;
        sd[s][0] = -2.0 * tx * (1.0 - tx * tx) * m.ie * m.ie;
        sd[s][1] = -2.0 * ty * (1.0 - ty * ty) * m.ie * m.ie;
#pragma unroll
        for (int i = 0; i < 4; ++i) { acc[i] = fma(wts, k[i], acc[i]); y[i] = fma(cst * m.h, k[i], x[i]); }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) xn[i] = fma(m.h / 6.0, acc[i], x[i]);
}

// q = (d f / d y at stage s)^T v
__device__ __forceinline__ void rm_jtv(const RmModel& m, const double* c, const double* v, double* q) {
    q[0] = fma(m.th[0], v[1], m.th[7] * v[3]);
    q[1] = fma(c[0], v[1], fma(c[2], v[3], v[0]));
    q[2] = fma(m.th[2], v[1], m.th[9] * v[3]);
    q[3] = fma(c[1], v[1], fma(c[3], v[3], v[2]));
}

// First-order adjoint of nl^T x+ (nl = -lambda_{k+1}) through the RK4 stages; turns sd[s] into the
// curvature coefficients of kb_s^T f'' at y_s ((vx, vx) and (vy, vy)); returns the tilt curvature.
__device__ __forceinline__ void rm_adjoint_curv(const RmModel& mlds, const double (*sc)[4], double (*sd)[2],
                                                const double* lamn, double sa, double sb, double* huu) {
    const RmModel m = mlds;
    double kb[4], yb[4];
    const double h = m.h;
#pragma unroll
    for (int i = 0; i < 4; ++i) kb[i] = -(h / 6.0) * lamn[i];
    huu[0] = 0.0; huu[1] = 0.0;
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        sd[s][0] = fma(kb[1], m.th[4], kb[3] * m.th[11]) * sd[s][0];
        sd[s][1] = fma(kb[1], m.th[5], kb[3] * m.th[12]) * sd[s][1];
        huu[0] = fma(kb[1], -m.gz * sa, huu[0]);
        huu[1] = fma(kb[3], -m.gz * sb, huu[1]);
        if (s > 0) {
            rm_jtv(m, sc[s], kb, yb);
            const double cs = s == 3 ? h : 0.5 * h, ws = (s == 1 ? 1.0 : 2.0) * h / 6.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) kb[i] = fma(cs, yb[i], -ws * lamn[i]);
        }
    }
}

// Direction d (0..3 state, 4..5 tilt): RK4 tangent -> Jacobian column (into M~, returns col . lamn),
// then the second-order adjoint sweep -> column d of the exact Hessian of -lambda^T x+ (rows >= d,
// z indices x 0..3, tilt 6..7).
__device__ __forceinline__ double rm_direction(const RmModel& m, const double (*sc)[4], const double (*cv)[2],
                                               const double* huu, double gca, double gcb, int d, const double* lamn,
                                               double* Mk, double* Hk) {
    double yd[4][4], acc[4], e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { e[i] = (i == d) ? 1.0 : 0.0; yd[0][i] = e[i]; acc[i] = 0.0; }
    const double fa = d == 4 ? gca : 0.0, fb = d == 5 ? gcb : 0.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        const double* c = sc[s];
        const double* y = yd[s];
        double k[4];
        k[0] = y[1]; k[2] = y[3];
        k[1] = fma(m.th[0], y[0], fma(c[0], y[1], fma(m.th[2], y[2], fma(c[1], y[3], fa))));
        k[3] = fma(m.th[7], y[0], fma(c[2], y[1], fma(m.th[9], y[2], fma(c[3], y[3], fb))));
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = fma(wts, k[i], acc[i]);
        if (s < 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) yd[s + 1][i] = fma(cst * m.h, k[i], e[i]);
        }
    }
    const int jc = d < 4 ? d : d + 2;
    double dot = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double col = fma(m.h / 6.0, acc[i], e[i]);
        Mk[jc * RmLds::NC + i] = col;
        dot = fma(col, lamn[i], dot);
    }
    double kbd[4], hx[4], hu0 = d == 4 ? huu[0] : 0.0, hu1 = d == 5 ? huu[1] : 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) { kbd[i] = 0.0; hx[i] = 0.0; }
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        double q[4];
        rm_jtv(m, sc[s], kbd, q);
        q[1] = fma(cv[s][0], yd[s][1], q[1]);
        q[3] = fma(cv[s][1], yd[s][3], q[3]);
        hu0 = fma(gca, kbd[1], hu0);
        hu1 = fma(gcb, kbd[3], hu1);
#pragma unroll
        for (int i = 0; i < 4; ++i) hx[i] += q[i];
        const double cs = s == 3 ? m.h : 0.5 * m.h;
#pragma unroll
        for (int i = 0; i < 4; ++i) kbd[i] = cs * q[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i >= d) Hk[hp(i, jc)] = hx[i];
    Hk[hp(6, jc)] = hu0;
    Hk[hp(7, jc)] = hu1;
    return dot;
}

// directions d0 .. d0+2 of one node (the node and mirror lanes split the six directions), from the
// stage data of this lane's RK4 pass
__device__ __forceinline__ void rm_directions(const RmModel& m, const double (*scr)[4], const double (*cvr)[2],
                                              const double* lamn, const double* huu, double gca, double gcb, int d0,
                                              double* Mk, double* Hk, double* jl_lds) {
    RmModel mr;
#pragma unroll
    for (int i = 0; i < 14; ++i) mr.th[i] = m.th[i];
    mr.gz = m.gz; mr.h = m.h; mr.ie = m.ie;
#pragma unroll
    for (int d = d0; d < d0 + 3; ++d) jl_lds[d] = rm_direction(mr, scr, cvr, huu, gca, gcb, d, lamn, Mk, Hk);
}

// z = [px vx py vy upx upy ux uy]: the inequality row values C z (np_mpc...:114-127) of one lane's three
// rows: du_x, du_y, vx - vmax on the node lane; -vx - vmax, vy - vmax, -vy - vmax on the mirror lane
__device__ __forceinline__ void rm_iq3(const double* z, double vmax, bool mir, double* c) {
    c[0] = mir ? -z[1] - vmax : z[6] - z[4];
    c[1] = mir ? z[3] - vmax : z[7] - z[5];
    c[2] = mir ? -z[3] - vmax : z[1] - vmax;
}

__global__ __launch_bounds__(kWave) void rmpc_ipm_kernel(RmpcArgs a) {
    __shared__ RmShared SH;
    RmLds* S = &SH.ocp;
    STAMP_DECL
    if (blockIdx.x % a.pack) return;          // small batches packed onto one XCD (launcher)
    const int b = blockIdx.x / a.pack;
    // lane k and its mirror lane k + 32 both own node k: the node work runs on both, the slack rows are
    // split (rm_iq3), and sums over the wave count the node terms on the node lanes only
    const int lane = threadIdx.x;
    const int k = lane & 31;
    const bool mir = lane >= 32, nod = !mir;
    const int N = a.N;
    const bool xon = k <= N, uon = k < N;
    const double* pr = a.prm + 10 * b;
    const double Qp = pr[0], Qv = pr[1], Ru = pr[2], Rdu = pr[3];
    const double ulo = pr[4], uhi = pr[5], dulo = pr[6], duhi = pr[7], vmax = pr[8], veps = pr[9];

    // ---------------- fused RLS update (np_mpc...:17-27, rob_ctrl.py:340-343) -----------------
    if (a.rls_P) {
        double* Pg = a.rls_P + 98 * b;
        const double* ph = a.rls_phi + 7 * b;
        const double lamr = a.rls_lambda;
        if (lane < 28) {
            const int ax = (lane % 14) / 7, i = lane % 7;
            double s = 0.0;
            if (lane < 14) { for (int j = 0; j < 7; ++j) s = fma(Pg[49 * ax + 7 * i + j], ph[j], s); SH.rls_Pphi[ax][i] = s; }
            else { for (int j = 0; j < 7; ++j) s = fma(ph[j], Pg[49 * ax + 7 * j + i], s); SH.rls_phiP[ax][i] = s; }
        }
        __syncthreads();
        double den[2], err[2];
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) {
            double dn = lamr, e = a.rls_y[2 * b + ax];
            for (int i = 0; i < 7; ++i) { dn = fma(ph[i], SH.rls_Pphi[ax][i], dn); e = fma(-ph[i], a.theta[14 * b + 7 * ax + i], e); }
            den[ax] = dn; err[ax] = e;
        }
        double pnew[2];
        int idx[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int e = lane + 64 * r;
            idx[r] = e;
            if (e < 98) {
                const int ax = e / 49, i = (e % 49) / 7, j = e % 7;
                const double Ki = SH.rls_Pphi[ax][i] / den[ax];
                pnew[r] = (Pg[e] - Ki * SH.rls_phiP[ax][j]) / lamr;
            }
        }
        double thn = 0.0;
        if (lane < 14) {
            const int ax = lane / 7, i = lane % 7;
            thn = a.theta[14 * b + lane] + SH.rls_Pphi[ax][i] / den[ax] * err[ax];
        }
        __syncthreads();          // every lane has read P, theta before anyone writes
#pragma unroll
        for (int r = 0; r < 2; ++r) if (idx[r] < 98) Pg[idx[r]] = pnew[r];
        if (lane < 14) { a.theta[14 * b + lane] = thn; SH.theta[lane] = thn; }
    } else if (lane < 14) {
        SH.theta[lane] = a.theta[14 * b + lane];
    }
    __syncthreads();

    if (lane < 14) SH.model.th[lane] = SH.theta[lane];
    if (lane == 0) { SH.model.gz = a.g; SH.model.h = a.Ts; SH.model.ie = 1.0 / veps; }
    __syncthreads();
    const RmModel& m = SH.model;
    const int sr = xon ? k : RM_NMAXS;        // per-node LDS scratch row (idle lanes share row 32)
    double* Mk = &S->M[xon ? k : 0][0][0];
    double* Hk = S->H[xon ? k : 0];
    if (uon) {       // constant structure: zero once, then only the variable entries are written
        for (int e = 0; e < RmLds::ND * RmLds::NC; ++e) Mk[e] = 0.0;
        for (int e = 0; e < tri(9); ++e) Hk[e] = 0.0;
        Mk[6 * RmLds::NC + 4] = 1.0; Mk[7 * RmLds::NC + 5] = 1.0;     // up+ = u
        Mk[8 * RmLds::NC + 6] = 1.0;                                  // homogeneous coordinate
    }

    const double lo = ulo - 1e-8 * fmax(1.0, fabs(ulo)), hi = uhi + 1e-8 * fmax(1.0, fabs(uhi));
    // relaxed bounds of this lane's slack rows: lower bounds only on the du rows (slots 0, 1 of the node lanes)
    double sL[RM_NQ], sU[RM_NQ];
    bool tw[RM_NQ];
#pragma unroll
    for (int i = 0; i < RM_NQ; ++i) {
        tw[i] = nod && i < 2;
        sL[i] = tw[i] ? dulo - 1e-8 * fmax(1.0, fabs(dulo)) : -1e300;
        sU[i] = tw[i] ? duhi + 1e-8 * fmax(1.0, fabs(duhi)) : 1e-8;
    }
    const bool poly = fmax(fabs(lo), fabs(hi)) <= 1.0;

    // ---------------- iterate (lanes k and k + 32 = node k) ---------------------------------------
    const double* x0 = a.x0 + 4 * b;
    const double* upv = a.u_prev + 2 * b;
    const double* rr = a.Rref + 4 * (N + 1) * b + 4 * (xon ? k : 0);
    const double r0 = rr[0], r1 = rr[1], r2 = rr[2], r3 = rr[3];
    const int nw = 4 * (N + 1) + 2 * N;
    const double* ww = a.w_warm ? a.w_warm + (size_t)nw * b : nullptr;
    double x[4], up[2], u[2], lam[6], zl[2], zu[2], s[RM_NQ], yq[RM_NQ], vl[RM_NQ], vu[RM_NQ];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = xon && ww ? ww[4 * k + i] : 0.0;   // reference warm start, zeros first call (:168)
    const double pushl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo));
    const double pushu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        double t = uon && ww ? ww[4 * (N + 1) + 2 * k + j] : 0.0;
        u[j] = uon ? fmin(fmax(t, lo + pushl), hi - pushu) : 0.0;
        zl[j] = uon ? 1.0 : 0.0; zu[j] = uon ? 1.0 : 0.0;
    }
    {   // auxiliary copies up_k = u_{k-1}, up_0 = u_prev
        const double p0 = from_prev(u[0]), p1 = from_prev(u[1]);
        up[0] = k == 0 ? upv[0] : p0;
        up[1] = k == 0 ? upv[1] : p1;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) lam[i] = 0.0;
    {   // slacks: s = C z pushed into the relaxed bounds; multipliers 1
        double z[8] = {x[0], x[1], x[2], x[3], up[0], up[1], u[0], u[1]}, c[RM_NQ];
        rm_iq3(z, vmax, mir, c);
#pragma unroll
        for (int i = 0; i < RM_NQ; ++i) {
            double v = fmin(c[i], sU[i] - 1e-2 * fmax(1.0, fabs(sU[i])));
            if (i < 2) {
                const double pl = fmin(1e-2 * fmax(1.0, fabs(sL[i])), 1e-2 * (sU[i] - sL[i]));
                const double pu = fmin(1e-2 * fmax(1.0, fabs(sU[i])), 1e-2 * (sU[i] - sL[i]));
                v = tw[i] ? fmin(fmax(c[i], sL[i] + pl), sU[i] - pu) : v;
            }
            s[i] = uon ? v : 0.0;
            yq[i] = 0.0;
            vl[i] = uon && tw[i] ? 1.0 : 0.0;
            vu[i] = uon ? 1.0 : 0.0;
        }
    }

    // objective gradient at a node (np_mpc...:129-140), z-space, unscaled
    auto cost_grad = [&](const double* xx, const double* uu, const double* pp, double* g) {
        g[0] = 2 * Qp * (xx[0] - r0); g[1] = 2 * Qv * (xx[1] - r1);
        g[2] = 2 * Qp * (xx[2] - r2); g[3] = 2 * Qv * (xx[3] - r3);
        const double d0 = uu[0] - pp[0], d1 = uu[1] - pp[1];
        g[4] = uon ? -2 * Rdu * d0 : 0.0; g[5] = uon ? -2 * Rdu * d1 : 0.0;
        g[6] = uon ? 2 * Ru * uu[0] + 2 * Rdu * d0 : 0.0; g[7] = uon ? 2 * Ru * uu[1] + 2 * Rdu * d1 : 0.0;
    };
    auto cost_val = [&](const double* xx, const double* uu, const double* pp) {
        double f = Qp * ((xx[0] - r0) * (xx[0] - r0) + (xx[2] - r2) * (xx[2] - r2)) +
                   Qv * ((xx[1] - r1) * (xx[1] - r1) + (xx[3] - r3) * (xx[3] - r3));
        const double d0 = uu[0] - pp[0], d1 = uu[1] - pp[1];
        return xon ? f + (uon ? Ru * (uu[0] * uu[0] + uu[1] * uu[1]) + Rdu * (d0 * d0 + d1 * d1) : 0.0) : 0.0;
    };
    // incoming defect g_k of node k (6 rows: physical 4 + up copy 2) for a trial point
    // sin / cos of both tilts of a node: the node lane takes alpha, its mirror lane beta, the pair
    // exchange both (the same bits as two evaluations per lane)
    auto rm_sincos2 = [&](const double* uu, double& sa, double& ca, double& sb, double& cb) {
        double s_, c_;
        tilt_sincos_econ(poly, mir ? uu[1] : uu[0], s_, c_);
        half_pair(s_, sa, sb);
        half_pair(c_, ca, cb);
    };
    auto defects = [&](const double* xx, const double* pp, const double* uu, double* g) {
        double sa, ca, sb, cb, xn[4];
        rm_sincos2(uu, sa, ca, sb, cb);
        rm_rk4(m, xx, sa, sb, xn, mir);
        double f[6];
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = from_prev(xn[i]);
        f[4] = from_prev(uu[0]); f[5] = from_prev(uu[1]);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = k == 0 ? xx[i] - x0[i] : xx[i] - f[i];
        g[4] = k == 0 ? pp[0] - upv[0] : pp[0] - f[4];
        g[5] = k == 0 ? pp[1] - upv[1] : pp[1] - f[5];
    };

    double gmax = 0.0;
    {
        double g[8];
        cost_grad(x, u, up, g);
#pragma unroll
        for (int i = 0; i < 8; ++i) gmax = fmax(gmax, xon ? fabs(g[i]) : 0.0);
    }
    gmax = wmax(gmax);
    const double sc = gmax > 100.0 ? 100.0 / gmax : 1.0;
    const double tol = a.tol, mu_min = tol / 10;
    const double nA = 6.0 * (N + 1), nI = 6.0 * N, nb = 12.0 * N;
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, eta_ph = 1e-8, gam_al = 0.05;

    double gdef[6];
    double theta;
    {
        defects(x, up, u, gdef);
        double zz[8] = {x[0], x[1], x[2], x[3], up[0], up[1], u[0], u[1]}, c[RM_NQ], th0 = 0.0;
        rm_iq3(zz, vmax, mir, c);
#pragma unroll
        for (int i = 0; i < 6; ++i) th0 += nod && xon ? fabs(gdef[i]) : 0.0;
#pragma unroll
        for (int i = 0; i < RM_NQ; ++i) th0 += uon ? fabs(c[i] - s[i]) : 0.0;
        theta = wsum_rl(th0);
    }
    const double th_max = 1e4 * fmax(1.0, theta), th_min = 1e-4 * fmax(1.0, theta);
    double fth = 0.0, fph = 0.0;
    int nfilt = 0;
    double mu = 0.1, delta_last = 0.0;
    int status = -1, it = 0;

    STAMP(0);
    // it = -1 (a.mult_init_max > 0): IPOPT's least-square estimate of the starting multipliers
    // (DefaultIterateInitializer::least_square_mults, constr_mult_init_max 1000) through the loop's own
    // stage QPs and Riccati sweep: unit weights on x and u (0 on the u_{k-1} copies, which are not
    // variables of the reference NLP), the slack columns eliminated with weight 1 (Hessian C^T C,
    // gradient C^T r_s, r_s = -v_L + v_U), r = scaled grad f - z_L + z_U, zero defects; the equality
    // multipliers are the step's new multipliers, y_d = C dz + r_s.  Mirrors oracle/rmpc_ipm.c.
    for (it = a.mult_init_max > 0.0 ? -1 : 0; it < a.max_iter; ++it) {
        const bool lsm = it < 0;
        // ---------------- derivatives, residuals, optimality error ---------------------------
        // stage data go to LDS as soon as they exist (Jacobian columns, dynamics Hessian, defect
        // column, dx~_0) to keep the register working set small
        double lamn[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) { const double t = from_next(lam[i]); lamn[i] = uon ? t : 0.0; }
        double jl[6];            // J^T lambda_{k+1} (x columns 0..3, tilt 4..5)
        {
            double sa, ca, sb, cb;
            rm_sincos2(u, sa, ca, sb, cb);
            // the RK4 stage data stay in registers through the adjoint and the three directions of
            // this lane (lanes k and k + 32 hold the same node: each has them without an LDS pass)
            double xn[4], huu[2], scr[4][4], sdr[4][2];
            rm_rk4_lin(m, x, sa, sb, xn, scr, sdr, mir);
            rm_adjoint_curv(m, scr, sdr, lamn, sa, sb, huu);
            STAMP(11);
            // lanes k and k + 32 own directions 0..2 and 3..5 of node k
            if (uon) rm_directions(m, scr, sdr, lamn, huu, m.gz * ca, m.gz * cb, mir ? 3 : 0, Mk, Hk, SH.JL[k]);
            __syncthreads();
            STAMP(12);
#pragma unroll
            for (int i = 0; i < 6; ++i) jl[i] = uon ? SH.JL[sr][i] : 0.0;
            double cdef[6];      // outgoing defect c_k = F(z_k) - x~_{k+1} -> defect column of M~
#pragma unroll
            for (int i = 0; i < 4; ++i) { const double t = from_next(x[i]); cdef[i] = xn[i] - t; }
            { const double t0 = from_next(up[0]), t1 = from_next(up[1]); cdef[4] = u[0] - t0; cdef[5] = u[1] - t1; }
            if (uon) {
#pragma unroll
                for (int r = 0; r < 6; ++r) Mk[8 * RmLds::NC + r] = lsm ? 0.0 : cdef[r];
            }
            double pl = 0.0;     // incoming defect g_k: primal residual, -g_0 = dx~_0
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double t = from_prev(cdef[i]);
                double gi = -t;
                if (k == 0) gi = i < 4 ? x[i] - x0[i] : up[i - 4] - upv[i - 4];
                pl = fmax(pl, xon ? fabs(gi) : 0.0);
                if (k == 0) S->dx0[i] = lsm ? 0.0 : -gi;
            }
            SH.JL[sr][6] = pl;
        }
        const double zz[8] = {x[0], x[1], x[2], x[3], up[0], up[1], u[0], u[1]};
        double cz[RM_NQ], rq[RM_NQ], sig[RM_NQ], psi[RM_NQ];
        rm_iq3(zz, vmax, mir, cz);
#pragma unroll
        for (int i = 0; i < RM_NQ; ++i) {
            rq[i] = uon ? cz[i] - s[i] : 0.0;
            const double dl = s[i] - sL[i], du_ = sU[i] - s[i];
            const double idl = tw[i] ? frcp(dl) : 0.0, idu = frcp(du_);
            sig[i] = uon ? (lsm ? 1.0 : fma(vl[i], idl, vu[i] * idu)) : 0.0;
            psi[i] = uon ? (lsm ? vu[i] - vl[i] : mu * (idu - idl)) : 0.0;     // (least squares: r_s)
            rq[i] = lsm ? 0.0 : rq[i];
        }
        double dinf = 0.0, pinf = SH.JL[sr][6], c0 = 0.0, cmin = 1e300, suml = 0.0, sumz = 0.0;
        {
            double gl[8];
            cost_grad(x, u, up, gl);
#pragma unroll
            for (int j = 0; j < 8; ++j) gl[j] *= sc;
#pragma unroll
            for (int i = 0; i < 6; ++i) gl[i] += lam[i];
            // - A~^T lam_{k+1} - B~^T lam_{k+1}
#pragma unroll
            for (int j = 0; j < 4; ++j) gl[j] -= jl[j];
            gl[6] -= jl[4] + lamn[4]; gl[7] -= jl[5] + lamn[5];
            // + C^T y, rows 3..5 from the mirror lane; the node's residual counts on the node lanes
            double yo[RM_NQ];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) yo[i] = __shfl_xor(yq[i], 32);
            gl[6] += yq[0]; gl[4] -= yq[0]; gl[7] += yq[1]; gl[5] -= yq[1];
            gl[1] += yq[2] - yo[0]; gl[3] += yo[1] - yo[2];
            gl[6] += -zl[0] + zu[0]; gl[7] += -zl[1] + zu[1];
#pragma unroll
            for (int j = 0; j < 8; ++j) dinf = fmax(dinf, nod && (j < 6 ? xon : uon) ? fabs(gl[j]) : 0.0);
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) dinf = fmax(dinf, uon ? fabs(-yq[i] - vl[i] + vu[i]) : 0.0);
#pragma unroll
            for (int i = 0; i < 6; ++i) suml += nod && xon ? fabs(lam[i]) : 0.0;
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                pinf = fmax(pinf, fabs(rq[i]));
                suml += fabs(yq[i]);
                if (uon) {
                    const double cu = vu[i] * (sU[i] - s[i]);
                    c0 = fmax(c0, cu); cmin = fmin(cmin, cu); sumz += vu[i];
                    if (tw[i]) { const double cl = vl[i] * (s[i] - sL[i]); c0 = fmax(c0, cl); cmin = fmin(cmin, cl); sumz += vl[i]; }
                }
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) if (uon && nod) {
                const double cl = zl[j] * (u[j] - lo), cu = zu[j] * (hi - u[j]);
                c0 = fmax(c0, fmax(cl, cu)); cmin = fmin(cmin, fmin(cl, cu)); sumz += zl[j] + zu[j];
            }
        }
        float r0 = (float)dinf, r1 = (float)pinf, r2 = (float)c0, r3 = (float)cmin, r4 = (float)suml, r5 = (float)sumz;
        wred_errors(r0, r1, r2, r3, r4, r5);
        dinf = r0; pinf = r1; c0 = r2;
        const double cminw = r3;
        suml = r4; sumz = r5;
        // IPOPT's scalings s_d, s_c (>= 1) as reciprocals
        const double is_d = 100.0 * frcp(fmax(100.0, (suml + sumz) * (1.0 / (nA + nI + nb))));
        const double is_c = 100.0 * frcp(fmax(100.0, sumz * (1.0 / nb)));
        if (!lsm && fmax(dinf * is_d, fmax(pinf, c0 * is_c)) <= tol) { status = 0; break; }
        for (; !lsm;) {
            const double cmu = fmax(c0 - mu, mu - cminw);
            if (fmax(dinf * is_d, fmax(pinf, cmu * is_c)) > 10.0 * mu || mu <= mu_min) break;
            mu = fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu)));
            nfilt = 0;
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                const double dl = s[i] - sL[i], du_ = sU[i] - s[i];
                const double idl = tw[i] ? frcp(dl) : 0.0, idu = frcp(du_);
                psi[i] = uon ? mu * (idu - idl) : 0.0;
            }
        }
        const double tau = fmax(0.99, 1.0 - mu);
        STAMP(1);

        // ---------------- stage QPs into LDS ---------------------------------------------------
        const double isl0 = uon ? frcp(u[0] - lo) : 0.0, isl1 = uon ? frcp(u[1] - lo) : 0.0;
        const double isu0 = uon ? frcp(hi - u[0]) : 0.0, isu1 = uon ? frcp(hi - u[1]) : 0.0;
        {
            // gradient column (index 8): scaled cost + box barrier + C^T (Sigma r + psi); the
            // cost / slack / barrier parts of the Hessian on top of the dynamics part
            double gq[8];
            cost_grad(x, u, up, gq);
#pragma unroll
            for (int j = 0; j < 8; ++j) gq[j] *= sc;
            // Sigma and Sigma r + psi of rows 3..5 from the mirror lane; the node lane writes the stage
            double tq[RM_NQ], so[RM_NQ], to[RM_NQ];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) tq[i] = sig[i] * rq[i] + psi[i];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) { so[i] = __shfl_xor(sig[i], 32); to[i] = __shfl_xor(tq[i], 32); }
            if (uon && nod) {
                if (lsm) {      // least squares: the box gradient -z_L + z_U, unit weights (0 on the copies)
                    gq[6] += zu[0] - zl[0]; gq[7] += zu[1] - zl[1];
                } else {
                    gq[6] += -mu * isl0 + mu * isu0; gq[7] += -mu * isl1 + mu * isu1;
                }
                gq[6] += tq[0]; gq[4] -= tq[0]; gq[7] += tq[1]; gq[5] -= tq[1];
                gq[1] += tq[2] - to[0];
                gq[3] += to[1] - to[2];
                const double wp = lsm ? 1.0 : sc * 2 * Qp, wv = lsm ? 1.0 : sc * 2 * Qv, wd = lsm ? 0.0 : sc * 2 * Rdu;
                const double wu0 = lsm ? 1.0 : sc * 2 * (Ru + Rdu) + zl[0] * isl0 + zu[0] * isu0;
                const double wu1 = lsm ? 1.0 : sc * 2 * (Ru + Rdu) + zl[1] * isl1 + zu[1] * isu1;
                Hk[hp(0, 0)] += wp; Hk[hp(2, 2)] += wp;
                Hk[hp(1, 1)] += wv + sig[2] + so[0];
                Hk[hp(3, 3)] += wv + so[1] + so[2];
                Hk[hp(6, 6)] += wu0 + sig[0];
                Hk[hp(7, 7)] += wu1 + sig[1];
                Hk[hp(4, 4)] = wd + sig[0]; Hk[hp(5, 5)] = wd + sig[1];
                Hk[hp(6, 4)] = -wd - sig[0]; Hk[hp(7, 5)] = -wd - sig[1];
#pragma unroll
                for (int j = 0; j < 8; ++j) Hk[hp(8, j)] = gq[j];
            }
            if (k == N && nod) {   // terminal surrogate G_N: value function [[Q_N, q_N], [q_N^T, 0]], Quu = I
                double* GN = S->G[N];
                for (int e = 0; e < tri(9); ++e) GN[e] = 0.0;
                GN[hp(0, 0)] = lsm ? 1.0 : sc * 2 * Qp; GN[hp(2, 2)] = lsm ? 1.0 : sc * 2 * Qp;
                GN[hp(1, 1)] = lsm ? 1.0 : sc * 2 * Qv; GN[hp(3, 3)] = lsm ? 1.0 : sc * 2 * Qv;
                GN[hp(6, 6)] = 1.0; GN[hp(7, 7)] = 1.0;
#pragma unroll
                for (int j = 0; j < 6; ++j) GN[hp(8, j)] = gq[j];
            }
        }
        __syncthreads();
        STAMP(2);
        if (lsm) {
            (void)riccati_sweep_aug(S, N);      // unit weights: positive definite
            closed_loop(S, N);
            double dxl[6], dUl[2], lmp[6];
            forward_sweep(S, N, k, dxl);
            const double* K0 = S->KK[uon ? k : 0][0];
            const double* K1 = S->KK[uon ? k : 0][1];
            double d0 = K0[6], d1 = K1[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) { d0 = fma(K0[j], dxl[j], d0); d1 = fma(K1[j], dxl[j], d1); }
            dUl[0] = uon ? d0 : 0.0; dUl[1] = uon ? d1 : 0.0;
            node_multiplier(S, xon ? k : 0, dxl, dUl, lmp);
            const double dzv[8] = {dxl[0], dxl[1], dxl[2], dxl[3], dxl[4], dxl[5], dUl[0], dUl[1]};
            double cdz[RM_NQ], yd[RM_NQ], ym = 0.0;
            rm_iq3(dzv, 0.0, mir, cdz);
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) { yd[i] = uon ? cdz[i] + psi[i] : 0.0; ym = fmax(ym, fabs(yd[i])); }
#pragma unroll
            for (int i = 0; i < 4; ++i) ym = fmax(ym, nod && xon ? fabs(lmp[i]) : 0.0);   // (copy rows are not IPOPT's)
            if (wmax(ym) <= a.mult_init_max) {
#pragma unroll
                for (int i = 0; i < 6; ++i) lam[i] = xon ? lmp[i] : 0.0;
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) yq[i] = yd[i];
            }
            continue;
        }

        // ---------------- Newton step: Riccati with inertia correction -----------------------
        double delta = 0.0, dapplied = 0.0;
        bool ok = riccati_sweep_aug(S, N);
        int attempt = 1;
        for (; attempt < 60 && !ok; ++attempt) {
            delta = (attempt == 1) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))   // IPOPT perturb_dec_fact 1/3
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            const double dd = delta - dapplied;
            if (uon && nod) {
#pragma unroll
                for (int j = 0; j < 8; ++j) Hk[hp(j, j)] += dd;
            }
            if (k == N && nod) {
                // the sweep never overwrites the terminal surrogate: add delta on its x~ block
#pragma unroll
                for (int j = 0; j < 6; ++j) S->G[N][hp(j, j)] += dd;
            }
            dapplied = delta;
            __syncthreads();
            ok = riccati_sweep_aug(S, N);
        }
        STAMP_ADD(9, attempt);
        STAMP(3);
        if (!ok) { status = -3; break; }
        if (delta > 0.0) delta_last = delta;
        closed_loop(S, N);
        STAMP(13);
        double dx[6], dU[2], lamp[6];
        forward_sweep(S, N, k, dx);
        STAMP(14);
        {
            const int kk = xon ? k : 0;
            const double* K0 = S->KK[uon ? k : 0][0];
            const double* K1 = S->KK[uon ? k : 0][1];
            double d0 = K0[6], d1 = K1[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) { d0 = fma(K0[j], dx[j], d0); d1 = fma(K1[j], dx[j], d1); }
            dU[0] = uon ? d0 : 0.0; dU[1] = uon ? d1 : 0.0;
            node_multiplier(S, kk, dx, dU, lamp);
        }
        STAMP(4);
        // slack and multiplier steps
        double dS[RM_NQ], dY[RM_NQ], dvl[RM_NQ], dvu[RM_NQ], dzl[2], dzu[2];
        {
            const double dzv[8] = {dx[0], dx[1], dx[2], dx[3], dx[4], dx[5], dU[0], dU[1]};
            double cdz[RM_NQ];
            rm_iq3(dzv, 0.0, mir, cdz);
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                dS[i] = uon ? cdz[i] + rq[i] : 0.0;
                dY[i] = uon ? sig[i] * dS[i] + psi[i] - yq[i] : 0.0;
                const double dl = s[i] - sL[i], du_ = sU[i] - s[i];
                const double idl = tw[i] ? frcp(dl) : 0.0, idu = frcp(du_);
                dvl[i] = uon && tw[i] ? fma(mu, idl, -vl[i]) - vl[i] * idl * dS[i] : 0.0;
                dvu[i] = uon ? fma(mu, idu, -vu[i]) + vu[i] * idu * dS[i] : 0.0;
            }
            dzl[0] = uon ? mu * isl0 - zl[0] - zl[0] * isl0 * dU[0] : 0.0;
            dzl[1] = uon ? mu * isl1 - zl[1] - zl[1] * isl1 * dU[1] : 0.0;
            dzu[0] = uon ? mu * isu0 - zu[0] + zu[0] * isu0 * dU[0] : 0.0;
            dzu[1] = uon ? mu * isu1 - zu[1] + zu[1] * isu1 * dU[1] : 0.0;
        }
        double amax = 1.0, az = 1.0;
        if (uon) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                // fractions to the boundary by frcp: reduced in f32 with a 2^-20 margin below
                if (dU[j] < 0) amax = fmin(amax, -tau * (u[j] - lo) * frcp(dU[j]));
                if (dU[j] > 0) amax = fmin(amax, tau * (hi - u[j]) * frcp(dU[j]));
                if (dzl[j] < 0) az = fmin(az, -tau * zl[j] * frcp(dzl[j]));
                if (dzu[j] < 0) az = fmin(az, -tau * zu[j] * frcp(dzu[j]));
            }
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                if (tw[i] && dS[i] < 0) amax = fmin(amax, -tau * (s[i] - sL[i]) * frcp(dS[i]));
                if (dS[i] > 0) amax = fmin(amax, tau * (sU[i] - s[i]) * frcp(dS[i]));
                if (tw[i] && dvl[i] < 0) az = fmin(az, -tau * vl[i] * frcp(dvl[i]));
                if (dvu[i] < 0) az = fmin(az, -tau * vu[i] * frcp(dvu[i]));
            }
        }
        float amax_f = (float)amax, az_f = (float)az;
        wmin2f(amax_f, az_f);
        amax = (double)amax_f * (1.0 - 1.0 / 1048576.0);
        az = (double)az_f * (1.0 - 1.0 / 1048576.0);

        STAMP(5);
        // ---------------- filter line search -------------------------------------------------
        auto barrier_args = [&](const double* uu, const double* ss) {
            double pa = 1.0;
            if (uon) {   // the tilt box and the du rows' lower bounds on the node lane, upper bounds of its rows on each
                const double pb = (uu[0] - lo) * (hi - uu[0]) * (uu[1] - lo) * (hi - uu[1]) * ((ss[0] - sL[0]) * (ss[1] - sL[1]));
                pa = nod ? pb : 1.0;
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) pa *= sU[i] - ss[i];
            }
            return pa;
        };
        double phil = nod ? sc * cost_val(x, u, up) : 0.0, gtdl = 0.0;
        {
            const double pa = barrier_args(u, s);
            phil -= uon ? mu * log_fast(pa) : 0.0;
            double gq[8];
            cost_grad(x, u, up, gq);
#pragma unroll
            for (int j = 0; j < 8; ++j) gq[j] *= sc;
#pragma unroll
            for (int i = 0; i < 6; ++i) gtdl += nod && xon ? gq[i] * dx[i] : 0.0;
            if (uon) {
                if (nod) gtdl += (gq[6] - mu * isl0 + mu * isu0) * dU[0] + (gq[7] - mu * isl1 + mu * isu1) * dU[1];
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) gtdl += psi[i] * dS[i];
            }
        }
        const double phi = wsum_rl(phil), gTd = wsum_rl(gtdl);
        const float lg_th = theta > 0.0 ? lg2(theta) : -3.0e38f;
        const float lg_gd = gTd < 0.0 ? lg2(-gTd) : 3.0e38f;
        const float lg_sw = (float)s_th * lg_th - (float)s_ph * lg_gd;
        double amin = gam_th;
        if (gTd < 0.0) amin = fmin(gam_th, fmin(gam_ph * theta * frcp(-gTd), (double)__builtin_amdgcn_exp2f(fmaxf(lg_sw, -126.0f))));
        amin *= gam_al;
        double alpha = amax, th_t = 0.0, ph_t = 0.0;
        bool accepted = false, ftype = false;
        // IPOPT's tiny-step test: max |d|/(1+|x|) < 10 eps_mach accepts the full step unfiltered
        float tnl = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            tnl = fmaxf(tnl, xon ? fabsf((float)dx[i]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)x[i])) : 0.0f);
        if (uon) {
#pragma unroll
            for (int j = 0; j < 2; ++j) tnl = fmaxf(tnl, fabsf((float)dU[j]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)u[j])));
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) tnl = fmaxf(tnl, fabsf((float)dS[i]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)s[i])));
        }
        const bool tiny = wmaxf(tnl) < 2.2e-15f;
        STAMP(6);
        int ls = 0;
        for (; ls < 80; ++ls) {
            double xt[4], pt[2], ut[2], st_[RM_NQ], gt[6];
#pragma unroll
            for (int i = 0; i < 4; ++i) xt[i] = fma(alpha, dx[i], x[i]);
            pt[0] = fma(alpha, dx[4], up[0]); pt[1] = fma(alpha, dx[5], up[1]);
            ut[0] = fma(alpha, dU[0], u[0]); ut[1] = fma(alpha, dU[1], u[1]);
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) st_[i] = fma(alpha, dS[i], s[i]);
            defects(xt, pt, ut, gt);
            double zt[8] = {xt[0], xt[1], xt[2], xt[3], pt[0], pt[1], ut[0], ut[1]}, ct[RM_NQ];
            rm_iq3(zt, vmax, mir, ct);
            double thl = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) thl += nod && xon ? fabs(gt[i]) : 0.0;
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) thl += uon ? fabs(ct[i] - st_[i]) : 0.0;
            double phl = nod ? sc * cost_val(xt, ut, pt) : 0.0;
            phl -= uon ? mu * log_fast(barrier_args(ut, st_)) : 0.0;
            th_t = wsum_rl(thl); ph_t = wsum_rl(phl);
            if (tiny) { accepted = true; ftype = true; break; }
            bool in_filter = !(th_t < th_max) || !isfinite(ph_t);
            in_filter = in_filter || wany(lane < nfilt && th_t >= fth && ph_t >= fph);
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
            if (lane == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
            ++nfilt;
        }
        // ---------------- accept ------------------------------------------------------------
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = xon ? fma(alpha, dx[i], x[i]) : x[i];
        up[0] = xon ? fma(alpha, dx[4], up[0]) : up[0];
        up[1] = xon ? fma(alpha, dx[5], up[1]) : up[1];
#pragma unroll
        for (int i = 0; i < 6; ++i) lam[i] = xon ? fma(alpha, lamp[i] - lam[i], lam[i]) : 0.0;
        if (uon) {
            u[0] = fma(alpha, dU[0], u[0]); u[1] = fma(alpha, dU[1], u[1]);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double il = frcp(u[j] - lo), iu = frcp(hi - u[j]);
                zl[j] = fmax(fmin(fma(az, dzl[j], zl[j]), 1e10 * mu * il), 1e-10 * mu * il);
                zu[j] = fmax(fmin(fma(az, dzu[j], zu[j]), 1e10 * mu * iu), 1e-10 * mu * iu);
            }
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                s[i] = fma(alpha, dS[i], s[i]);
                yq[i] = fma(alpha, dY[i], yq[i]);
                const double dl = s[i] - sL[i], du_ = sU[i] - s[i];
                const double idl = tw[i] ? frcp(dl) : 0.0, idu = frcp(du_);
                if (tw[i]) vl[i] = fmax(fmin(fma(az, dvl[i], vl[i]), 1e10 * mu * idl), 1e-10 * mu * idl);
                vu[i] = fmax(fmin(fma(az, dvu[i], vu[i]), 1e10 * mu * idu), 1e-10 * mu * idu);
            }
        }
        theta = th_t;
        STAMP(8);
    }

    // ---------------- outputs -------------------------------------------------------------
    const double fval = wsum_rl(nod ? cost_val(x, u, up) : 0.0);
    if (lane == 0) {
        a.u0[2 * b] = u[0]; a.u0[2 * b + 1] = u[1];
        a.f[b] = fval; a.status[b] = status; a.iters[b] = it;
    }
    if (a.w_out) {
        double* wo = a.w_out + (size_t)nw * b;
        if (nod && xon) {
#pragma unroll
            for (int i = 0; i < 4; ++i) wo[4 * k + i] = x[i];
        }
        if (nod && uon) { wo[4 * (N + 1) + 2 * k] = u[0]; wo[4 * (N + 1) + 2 * k + 1] = u[1]; }
    }
    STAMP_FLUSH_TO(g_stamp_rm, b);
}

// Standalone batched RLS.update (np_mpc...:17-27): one p = 7 filter per workgroup, lanes as entries.
__global__ __launch_bounds__(kWave) void rls_update_kernel(int B, double* theta, double* P, const double* phi,
                                                          const double* y, double lam) {
    __shared__ double Pphi[7], phiP[7], ph[7], th[7];
    const int b = blockIdx.x, l = threadIdx.x;
    double* Pb = P + 49 * b;
    if (l < 7) { ph[l] = phi[7 * b + l]; th[l] = theta[7 * b + l]; }
    __syncthreads();
    if (l < 7) {
        double s = 0.0;
        for (int j = 0; j < 7; ++j) s = fma(Pb[7 * l + j], ph[j], s);
        Pphi[l] = s;
    } else if (l < 14) {
        const int i = l - 7;
        double s = 0.0;
        for (int j = 0; j < 7; ++j) s = fma(ph[j], Pb[7 * j + i], s);
        phiP[i] = s;
    }
    __syncthreads();
    double den = lam, err = y[b];
    for (int i = 0; i < 7; ++i) { den = fma(ph[i], Pphi[i], den); err = fma(-ph[i], th[i], err); }
    double pn = 0.0;
    if (l < 49) pn = (Pb[l] - Pphi[l / 7] / den * phiP[l % 7]) / lam;
    __syncthreads();
    if (l < 49) Pb[l] = pn;
    if (l < 7) theta[7 * b + l] = th[l] + Pphi[l] / den * err;
}

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_rls(int B, double* theta, double* P, const double* phi, const double* y,
                                         double lam, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(dartmpc::rls_update_kernel, dim3(B), dim3(dartmpc::kWave), 0, stream, B, theta, P, phi, y, lam);
    return hipGetLastError();
}

extern "C" hipError_t dartmpc_launch_rmpc(const dartmpc::RmpcArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    if (args->N < 1 || args->N >= dartmpc::RM_NMAXS) return hipErrorInvalidValue;
    dartmpc::RmpcArgs a = *args;
    a.pack = (a.B <= 32) ? 8 : 1;            // blocks go round-robin over the 8 XCDs: one XCD, one L2 for the code
    hipLaunchKernelGGL(dartmpc::rmpc_ipm_kernel, dim3(a.B * a.pack), dim3(dartmpc::kWave), 0, stream, a);
    return hipGetLastError();
}

#ifdef DART_STAMPS
extern "C" hipError_t dartmpc_read_stamps_rmpc(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_rm), sizeof(unsigned long long) * 16, 0,
                               hipMemcpyDeviceToHost);
}
#endif
