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
//
// IPOPT's soft restoration and restoration phases (oracle/rmpc_ipm.c `soft_resto_step`, `restoration`):
// a measured |v| above vmax at the pinned node 0 (np_mpc...:123-127) makes the NLP locally infeasible and
// the filter line search fails.  rmpc_ipm_kernel<false> (every solve) carries no restoration code: an
// instance whose line search fails ends with the internal status kRmNeedResto and writes nothing else.  The
// launcher always follows it with rmpc_ipm_kernel<true> on the same stream; its blocks return at once unless
// their instance was handed over, the others solve the instance again from its start (the same iterates up
// to the failure) with both phases available, to the end of the solve.  No state crosses the hand-off but
// the status word in the caller's output array, so launches on different streams cannot interfere.
// Horizons N = 32..63: this file built a second time with -DDART_WG=2 (Makefile: rmpc_wg2.o) -- a workgroup of
// two waves per instance, wave w owning nodes 32 w .. 32 w + 31 with the lane roles above (wave.h: the wave
// reductions and node shifts combine the two waves, the Riccati and forward sweeps run in both on the shared
// LDS); its restoration-phase state lives in a per-instance global-memory area instead of LDS (RmpcArgs::
// resto_buf), which the 64-node arrays of the solve leave no room for.  The build's symbols sit in their own
// namespace.
#if DART_WG == 2
#define dartmpc dartmpc_wg2
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ocp_wave.h"
#include "rmpc_ipm.h"
#include "stamps.h"
#include "wave.h"

// this kernel runs at the register limit: its double sums use the readlane cross-row step (wsum_rl)

namespace dartmpc {

constexpr int RM_NMAXS = 32 * kWaves;      // max shooting nodes (N <= 31, two-wave build N <= 63)
constexpr int RM_NIQ = 6;         // inequality rows per node: du_x, du_y, vx-vmax, -vx-vmax, vy-vmax, -vy-vmax
constexpr int RM_NQ = 3;          // of them per lane: rows 0..2 on lane k, rows 3..5 on its mirror lane k + 32
static_assert(2 * RM_NQ == RM_NIQ, "the node and mirror lanes split the rows evenly");
using RmLds = OcpLds<6, RM_NMAXS>;
using RmSoft = AugSoftLds<RmLds, 4>;     // restoration: the four physical rows of every defect are soft
constexpr int kRmNeedResto = -100;      // hand-off of an instance to rmpc_ipm_kernel<true>

#ifdef DART_STAMPS
__device__ unsigned long long g_stamp_rm[32];
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

// Restoration-phase state in LDS (rmpc_ipm_kernel<true> only).  PN: node k's four physical incoming rows
// (written by the node lane): p, n, z_p, z_n, rp, rn, Sigma_p', Sigma_n'; x_R, D_R of the states, u_R, D_R of
// the tilts, and the original problem's u-bound multipliers at the start.  Q: each lane's three inequality
// rows: p, n, z_p, z_n, rp, rn, Sigma_s', Sigma_p', Sigma_n', sigma, off, psi, and the original slack and
// slack-bound multipliers at the start.  SV / SV2: a parked step (second-order correction, refinement).
enum { P_PC = 0, P_NC = 4, P_ZP = 8, P_ZN = 12, P_RP = 16, P_RN = 20, P_SP = 24, P_SN = 28, P_XR = 32, P_DRX = 36,
       P_UR = 40, P_DRU = 42, P_ZL0 = 44, P_ZU0 = 46, P_N = 48 };
enum { Q_QP = 0, Q_QN = 3, Q_ZQP = 6, Q_ZQN = 9, Q_RQP = 12, Q_RQN = 15, Q_SS = 18, Q_SP = 21, Q_SN = 24, Q_SIG = 27,
       Q_OFF = 30, Q_PSI = 33, Q_S0 = 36, Q_VL0 = 39, Q_VU0 = 42, Q_N = 45 };
enum { V_DX = 0, V_LP = 6, V_DU = 12, V_DY = 14, V_DS = 17, V_DQP = 20, V_DQN = 23, V_DPC = 26, V_DNC = 30, V_N = 34 };
struct RmResto {
    RmSoft soft;
    NodeArr<double[P_N], RM_NMAXS + 1> PN;
    NodeArr<double[Q_N], kWave * kWaves> Q;
    NodeArr<double[V_N], kWave * kWaves> SV, SV2;
};

// closed-loop rows of node k mapped through node k+1's soft rows: [Phi | f](r) <- Y(r, :) [[Phi | f]; 0 1]
struct RmSoftPost {
    RmLds* S;
    const RmSoft* R;
    __device__ void operator()(int k) const {
        const double* Y = R->T[k + 1];
        double F[6][7];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int j = 0; j < 7; ++j) F[r][j] = S->F[k][r][j];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                double t = j == 6 ? Y[7 * r + 6] : 0.0;
#pragma unroll
                for (int a = 0; a < 6; ++a) t = fma(Y[7 * r + a], F[a][j], t);
                S->F[k][r][j] = t;
            }
    }
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

// The LDS of the solve (one instance per workgroup), at namespace scope: a kernel is given the blocks its code
// reaches (70.6 KB without the restoration phases, 151.7 KB with them)
__shared__ RmShared g_rm_sh;
#if DART_WG == 1
__shared__ RmResto g_rm_resto;
#else
static_assert(sizeof(RmShared) + sizeof(g_wg_x) <= 160 * 1024, "the two-wave solve fits the LDS of a CU");
#endif

// The solve of instance b by the calling wave.  RESTO = false: the kernel of every launch, without IPOPT's
// restoration phases; an instance whose filter line search fails is handed over (status kRmNeedResto, no other
// output) and the function returns true.  RESTO = true: the solve of a handed-over instance again from its
// start, with both phases available (no state crosses the hand-off).
template <bool RESTO>
__device__ __forceinline__ bool rmpc_solve(const RmpcArgs& a, const int b) {
    RmShared& SH = g_rm_sh;
    RmLds* S = &SH.ocp;
    RmResto* RL = nullptr;
#if DART_WG == 1
    if constexpr (RESTO) RL = &g_rm_resto;
#else
    if constexpr (RESTO) RL = reinterpret_cast<RmResto*>(a.resto_buf) + b;
#endif
    STAMP_DECL
    // lane k and its mirror lane k + 32 both own node k: the node work runs on both, the slack rows are
    // split (rm_iq3), and sums over the wave count the node terms on the node lanes only
    const int lane = lane_id();
    const int k = node_base() + (lane & 31);
    const bool mir = lane >= 32, nod = !mir;
    const int ql = kWave * wave_idx() + lane;      // this lane's slot in the per-lane restoration arrays
    const int N = a.N;
    const bool xon = k <= N, uon = k < N;
    const double* pr = a.prm + 10 * b;
    const double Qp = pr[0], Qv = pr[1], Ru = pr[2], Rdu = pr[3];
    const double ulo = pr[4], uhi = pr[5], dulo = pr[6], duhi = pr[7], vmax = pr[8], veps = pr[9];

    // ---------------- fused RLS update (np_mpc...:17-27, rob_ctrl.py:340-343) -----------------
    if (!RESTO && a.rls_P) {      // (<true> re-solves with the theta <false> updated in place)
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
        if (wave_idx() == 0) {
#pragma unroll
            for (int r = 0; r < 2; ++r) if (idx[r] < 98) Pg[idx[r]] = pnew[r];
            if (lane < 14) a.theta[14 * b + lane] = thn;
        }
        if (lane < 14) SH.theta[lane] = thn;
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
        if constexpr (kWaves == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) f[i] = from_prev(xn[i]);
            f[4] = from_prev(uu[0]); f[5] = from_prev(uu[1]);
        } else {       // two waves: one exchange for the six shifts
            const double x6[6] = {xn[0], xn[1], xn[2], xn[3], uu[0], uu[1]};
            from_prev_n(x6, f);
        }
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
    int in_soft = 0, soft_count = 0;      // IPOPT's soft restoration phase (BacktrackingLineSearch; <true>)
    bool go_resto = false;
    double phi_rs = 0.0;
    int it_next = a.mult_init_max > 0.0 ? -1 : 0;
    // <true>: the iteration loop is left for each restoration phase, which runs after it (outside the loop,
    // so that its registers do not burden the iterations) and re-enters it at the next iteration
    for (;;) {
    for (it = it_next; it < a.max_iter; ++it) {
        const bool lsm = it < 0;
        // ---------------- derivatives, residuals, optimality error ---------------------------
        // stage data go to LDS as soon as they exist (Jacobian columns, dynamics Hessian, defect
        // column, dx~_0) to keep the register working set small
        double lamn[6];
        if constexpr (kWaves == 1) {
#pragma unroll
            for (int i = 0; i < 6; ++i) { const double t = from_next(lam[i]); lamn[i] = uon ? t : 0.0; }
        } else {
            double t6[6];
            from_next_n(lam, t6);
#pragma unroll
            for (int i = 0; i < 6; ++i) lamn[i] = uon ? t6[i] : 0.0;
        }
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
            double pcd[6];       // (two waves: the shifts in two exchanges, the incoming ones here)
            if constexpr (kWaves == 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i) { const double t = from_next(x[i]); cdef[i] = xn[i] - t; }
                { const double t0 = from_next(up[0]), t1 = from_next(up[1]); cdef[4] = u[0] - t0; cdef[5] = u[1] - t1; }
            } else {
                const double x6[6] = {x[0], x[1], x[2], x[3], up[0], up[1]};
                double t6[6];
                from_next_n(x6, t6);
#pragma unroll
                for (int i = 0; i < 4; ++i) cdef[i] = xn[i] - t6[i];
                cdef[4] = u[0] - t6[4]; cdef[5] = u[1] - t6[5];
                from_prev_n(cdef, pcd);
            }
            if (uon) {
#pragma unroll
                for (int r = 0; r < 6; ++r) Mk[8 * RmLds::NC + r] = lsm ? 0.0 : cdef[r];
            }
            double pl = 0.0;     // incoming defect g_k: primal residual, -g_0 = dx~_0
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double t = kWaves == 1 ? from_prev(cdef[i]) : pcd[i];
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
            nfilt = 0; in_soft = 0;       // BacktrackingLineSearch::Reset: the filter and the soft phase
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
        // (reduced here: riding with the line search's sums below measured 0.7 % slower, profiles/r06/c2_lockstep_ab.txt)
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
        // IPOPT's tiny-step test: max |d|/(1+|x|) < 10 eps_mach accepts the full step unfiltered; its maximum rides with
        // the two sums (one lock-step reduction)
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
        wsum2_rl_maxf(phil, gtdl, tnl);
        const double phi = phil, gTd = gtdl;
        const float lg_th = theta > 0.0 ? lg2(theta) : -3.0e38f;
        const float lg_gd = gTd < 0.0 ? lg2(-gTd) : 3.0e38f;
        const float lg_sw = (float)s_th * lg_th - (float)s_ph * lg_gd;
        double amin = gam_th;
        if (gTd < 0.0) amin = fmin(gam_th, fmin(gam_ph * theta * frcp(-gTd), (double)__builtin_amdgcn_exp2f(fmaxf(lg_sw, -126.0f))));
        amin *= gam_al;
        double alpha = amax, th_t = 0.0, ph_t = 0.0;
        bool accepted = false, ftype = false;
        const bool tiny = tnl < 2.2e-15f;
        STAMP(6);
        int ls = 0;
        for (; ls < 80 && !in_soft; ++ls) {
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
            wsum2_rl(thl, phl);
            th_t = thl; ph_t = phl;
            if (tiny) { accepted = true; ftype = true; break; }
            bool in_filter = !(th_t < th_max) || !isfinite(ph_t);
            in_filter = in_filter || wany_rep(lane < nfilt && th_t >= fth && ph_t >= fph);
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
#ifdef DART_RESTO_TRACE
        if (RESTO && blockIdx.x == 0 && lane == 0)      // diagnostic build: the oracle's ORACLE_DEBUG line
            printf("it %3d mu %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e az %.3e th %.2e\n", it, mu,
                   dinf * is_d, pinf, c0 * is_c, delta, amax, alpha, az, theta);
#endif
        if constexpr (!RESTO) {
            // a failed line search: IPOPT's restoration phases in rmpc_ipm_kernel<true> (or status -2 without)
            if (!accepted) { status = a.resto ? kRmNeedResto : -2; break; }
        }
        bool soft = false;
        if constexpr (RESTO) {
            // ---------------- IPOPT's soft restoration phase (BacktrackingLineSearch::TrySoftRestoStep) ----
            // the line search failed, or the soft phase is on: the primal-dual step damped only by the
            // fractions to the boundary (one length for x, s, lambda, y and the bound multipliers) is taken if
            // the original filter accepts it with alpha_primal_test = 0 (the phase ends) or if it cuts the
            // primal-dual system error at mu by the factor 0.9999; at most max_soft_resto_iters = 10 steps
            if (!accepted) {
                if (!in_soft) {         // PrepareRestoPhaseStart: the current point enters the filter
                    if (nfilt < kWave) {
                        if (lane == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
                        ++nfilt;
                    }
                    soft_count = 0;
                }
                if (!(in_soft && ++soft_count > 10)) {
                    const double as = fmin(amax, az);
                    double th_s, ph_s;
                    {
                        double xt[4], pt[2], ut[2], st_[RM_NQ], gt[6];
#pragma unroll
                        for (int i = 0; i < 4; ++i) xt[i] = fma(as, dx[i], x[i]);
                        pt[0] = fma(as, dx[4], up[0]); pt[1] = fma(as, dx[5], up[1]);
                        ut[0] = fma(as, dU[0], u[0]); ut[1] = fma(as, dU[1], u[1]);
#pragma unroll
                        for (int i = 0; i < RM_NQ; ++i) st_[i] = fma(as, dS[i], s[i]);
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
                        wsum2_rl(thl, phl);
                        th_s = thl; ph_s = phl;
                    }
                    bool orig = th_s < th_max && isfinite(ph_s) && !wany_rep(lane < nfilt && th_s >= fth && ph_s >= fph);
                    orig = orig && (cmp_le(th_s, (1 - gam_th) * theta, theta) || cmp_le(ph_s - phi, -gam_ph * theta, phi));
                    bool take = orig;
                    if (!take && isfinite(ph_s)) {
                        // IPOPT's primal-dual system error at mu (l1 norms of the primal infeasibility, the dual
                        // infeasibility and z s - mu, added) at the current point and at the trial point with
                        // every multiplier moved by the same step
                        double pd[2];
#pragma unroll 1
                        for (int pass = 0; pass < 2; ++pass) {
                            const double al = pass ? as : 0.0;
                            double xx[4], pp[2], uu[2], ss[RM_NQ], lm[6], yy[RM_NQ], wl[RM_NQ], wu[RM_NQ], zzl[2], zzu[2];
#pragma unroll
                            for (int i = 0; i < 4; ++i) xx[i] = fma(al, dx[i], x[i]);
                            pp[0] = fma(al, dx[4], up[0]); pp[1] = fma(al, dx[5], up[1]);
#pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                uu[j] = uon ? fma(al, dU[j], u[j]) : u[j];
                                zzl[j] = fma(al, dzl[j], zl[j]); zzu[j] = fma(al, dzu[j], zu[j]);
                            }
#pragma unroll
                            for (int i = 0; i < 6; ++i) lm[i] = xon ? fma(al, lamp[i] - lam[i], lam[i]) : 0.0;
#pragma unroll
                            for (int i = 0; i < RM_NQ; ++i) {
                                ss[i] = fma(al, dS[i], s[i]); yy[i] = fma(al, dY[i], yq[i]);
                                wl[i] = fma(al, dvl[i], vl[i]); wu[i] = fma(al, dvu[i], vu[i]);
                            }
                            double lmn[6], jl_[6], xn_[4];
#pragma unroll
                            for (int i = 0; i < 6; ++i) { const double t = from_next(lm[i]); lmn[i] = uon ? t : 0.0; }
                            {
                                double sa, ca, sb, cb, huu[2], scr[4][4], sdr[4][2];
                                rm_sincos2(uu, sa, ca, sb, cb);
                                rm_rk4_lin(m, xx, sa, sb, xn_, scr, sdr, mir);
                                rm_adjoint_curv(m, scr, sdr, lmn, sa, sb, huu);
                                if (uon) rm_directions(m, scr, sdr, lmn, huu, m.gz * ca, m.gz * cb, mir ? 3 : 0, Mk, Hk, SH.JL[k]);
                                __syncthreads();
#pragma unroll
                                for (int i = 0; i < 6; ++i) jl_[i] = uon ? SH.JL[sr][i] : 0.0;
                                __syncthreads();
                            }
                            double cdef[6], gg[6];
#pragma unroll
                            for (int i = 0; i < 4; ++i) { const double t = from_next(xx[i]); cdef[i] = xn_[i] - t; }
                            { const double t0 = from_next(pp[0]), t1 = from_next(pp[1]); cdef[4] = uu[0] - t0; cdef[5] = uu[1] - t1; }
#pragma unroll
                            for (int i = 0; i < 6; ++i) {
                                const double t = from_prev(cdef[i]);
                                gg[i] = k == 0 ? (i < 4 ? xx[i] - x0[i] : pp[i - 4] - upv[i - 4]) : -t;
                            }
                            double gl[8];
                            cost_grad(xx, uu, pp, gl);
#pragma unroll
                            for (int j = 0; j < 8; ++j) gl[j] *= sc;
#pragma unroll
                            for (int i = 0; i < 6; ++i) gl[i] += lm[i];
#pragma unroll
                            for (int j = 0; j < 4; ++j) gl[j] -= jl_[j];
                            gl[6] -= jl_[4] + lmn[4]; gl[7] -= jl_[5] + lmn[5];
                            double yo[RM_NQ];
#pragma unroll
                            for (int i = 0; i < RM_NQ; ++i) yo[i] = __shfl_xor(yy[i], 32);
                            gl[6] += yy[0]; gl[4] -= yy[0]; gl[7] += yy[1]; gl[5] -= yy[1];
                            gl[1] += yy[2] - yo[0]; gl[3] += yo[1] - yo[2];
                            gl[6] += -zzl[0] + zzu[0]; gl[7] += -zzl[1] + zzu[1];
                            double tot = 0.0;
#pragma unroll
                            for (int j = 0; j < 8; ++j) tot += nod && (j < 6 ? xon : uon) ? fabs(gl[j]) : 0.0;
#pragma unroll
                            for (int i = 0; i < 6; ++i) tot += nod && xon ? fabs(gg[i]) : 0.0;
                            if (uon && nod) tot += fabs(zzl[0] * (uu[0] - lo) - mu) + fabs(zzu[0] * (hi - uu[0]) - mu) +
                                                   fabs(zzl[1] * (uu[1] - lo) - mu) + fabs(zzu[1] * (hi - uu[1]) - mu);
                            if (uon) {
                                const double zz2[8] = {xx[0], xx[1], xx[2], xx[3], pp[0], pp[1], uu[0], uu[1]};
                                double cz2[RM_NQ];
                                rm_iq3(zz2, vmax, mir, cz2);
#pragma unroll
                                for (int i = 0; i < RM_NQ; ++i) {
                                    tot += fabs(-yy[i] - wl[i] + wu[i]) + fabs(cz2[i] - ss[i]);
                                    if (tw[i]) tot += fabs(wl[i] * (ss[i] - sL[i]) - mu);
                                    tot += fabs(wu[i] * (sU[i] - ss[i]) - mu);
                                }
                            }
                            pd[pass] = wsum_rl(tot);
                        }
                        take = pd[1] <= 0.9999 * pd[0];
                    }
                    if (take) {
                        accepted = true; soft = true; alpha = as; az = as; th_t = th_s;
                        in_soft = orig ? 0 : 1;
                        if (orig) soft_count = 0;
                    }
                }
            }
            if (!accepted) { phi_rs = phi; go_resto = true; break; }
        }
        if (!soft && !ftype && nfilt < kWave) {
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
    if (!RESTO || !go_resto) break;
    go_resto = false;
    // ---------------- IPOPT's restoration phase (MinC_1NrmRestorationPhase) -------------------------------
    // (oracle/rmpc_ipm.c `restoration`): min rho sum(p + n) + eta/2 |D_R (x - x_R)|^2 over the reference NLP's
    // variables, s.t. c(x) + n - p = 0 on the physical defect rows (x_0 pinning included; the u_{k-1} copy
    // rows stay hard), d(x) - s + n - p = 0 on the inequality rows with the slack bounds kept, p, n >= 0, the
    // U box; rho 1000, eta = sqrt(mu_R), D_R = 1 / max(1, |x_R|).  Start: mu_R = max(mu, |(c, d - s)|_inf),
    // closed-form p, n, z = mu_R / p, bound multipliers min(rho, z), least-square equality multipliers.  The
    // problem is solved by the same algorithm (its own filter and mu, inertia correction, second-order
    // correction, iterative refinement of every step); it returns when the original problem's theta falls to
    // 0.9 of its start value at a point the original filter accepts.  Defect rows: soft rows of the Riccati
    // recursion (riccati_sweep_aug_soft); inequality rows: slack, p and n in series, eliminated per stage,
    // y + dy = sigma (C dz + r) + off with 1 / sigma = 1 / Sigma_s' + 1 / Sigma_p' + 1 / Sigma_n'.
    {
        RmResto& RS = *RL;
        RmSoft* const SR = &RS.soft;
        double* const pn = RS.PN[xon ? k : RM_NMAXS];      // node k's physical rows (written by the node lane)
        double* const q = RS.Q[ql];                        // this lane's three inequality rows
        const double mu0 = mu, th0 = theta, phi0 = phi_rs, tau0 = fmax(0.99, 1.0 - mu0), rho = 1000.0;
        const double nbr = 24.0 * N + 8.0 * (N + 1);       // bound-multiplier count of the restoration problem
        aug_soft_init<RmLds, 4>(SR);
        if (nod) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { pn[P_XR + i] = x[i]; pn[P_DRX + i] = 1.0 / fmax(1.0, fabs(x[i])); }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                pn[P_UR + j] = u[j]; pn[P_DRU + j] = 1.0 / fmax(1.0, fabs(u[j]));
                pn[P_ZL0 + j] = zl[j]; pn[P_ZU0 + j] = zu[j];
            }
        }
#pragma unroll
        for (int i = 0; i < RM_NQ; ++i) { q[Q_S0 + i] = s[i]; q[Q_VL0 + i] = vl[i]; q[Q_VU0 + i] = vu[i]; }
        double rmu, eta;
        {   // RestoIterateInitializer
            double g0[6], cz[RM_NQ];
            defects(x, up, u, g0);
            const double zz[8] = {x[0], x[1], x[2], x[3], up[0], up[1], u[0], u[1]};
            rm_iq3(zz, vmax, mir, cz);
            double cmx = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) cmx = fmax(cmx, nod && xon ? fabs(g0[i]) : 0.0);
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) cmx = fmax(cmx, uon ? fabs(cz[i] - s[i]) : 0.0);
            rmu = fmax(mu0, wmax(cmx));
            eta = sqrt(rmu);
            auto pn_init = [&](double c, double& p, double& n) {
                const double aa = rmu / (2.0 * rho) - 0.5 * c, bb = c * rmu / (2.0 * rho);
                n = aa + sqrt(aa * aa + bb); p = c + n;
            };
            if (nod) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    double p = 1.0, n = 1.0;
                    if (xon) pn_init(g0[i], p, n);
                    pn[P_PC + i] = p; pn[P_NC + i] = n;
                    pn[P_ZP + i] = xon ? rmu / p : 0.0; pn[P_ZN + i] = xon ? rmu / n : 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                double p = 1.0, n = 1.0;
                if (uon) pn_init(cz[i] - s[i], p, n);
                q[Q_QP + i] = p; q[Q_QN + i] = n;
                q[Q_ZQP + i] = uon ? rmu / p : 0.0; q[Q_ZQN + i] = uon ? rmu / n : 0.0;
                vl[i] = fmin(rho, vl[i]); vu[i] = fmin(rho, vu[i]);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) { zl[j] = fmin(rho, zl[j]); zu[j] = fmin(rho, zu[j]); }
        }
        __syncthreads();
        // the derivative pass at the current point with the next node's multipliers lmn: Jacobian columns into
        // M~, the dynamics Hessian into H~, jl = J^T lmn (x columns 0..3, tilts 4..5), xn = x+ of node k
        double lmn[6], jl[6], xn[4], hd[6];
        auto rderiv = [&]() {
            if constexpr (kWaves == 1) {
#pragma unroll
                for (int i = 0; i < 6; ++i) { const double t = from_next(lam[i]); lmn[i] = uon ? t : 0.0; }
            } else {
                double t6[6];
                from_next_n(lam, t6);
#pragma unroll
                for (int i = 0; i < 6; ++i) lmn[i] = uon ? t6[i] : 0.0;
            }
            double sa, ca, sb, cb, huu[2], scr[4][4], sdr[4][2];
            rm_sincos2(u, sa, ca, sb, cb);
            rm_rk4_lin(m, x, sa, sb, xn, scr, sdr, mir);
            rm_adjoint_curv(m, scr, sdr, lmn, sa, sb, huu);
            if (uon) rm_directions(m, scr, sdr, lmn, huu, m.gz * ca, m.gz * cb, mir ? 3 : 0, Mk, Hk, SH.JL[k]);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 6; ++i) jl[i] = uon ? SH.JL[sr][i] : 0.0;
            const int dg[6] = {0, 1, 2, 3, 6, 7};
#pragma unroll
            for (int i = 0; i < 6; ++i) hd[i] = uon ? Hk[hp(dg[i], dg[i])] : 0.0;
            __syncthreads();
        };
        // incoming defects of node k (6 rows) from x+ of every node
        auto incoming = [&](double* g) {
            double cdef[6];
            if constexpr (kWaves == 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i) { const double t = from_next(x[i]); cdef[i] = xn[i] - t; }
                { const double t0 = from_next(up[0]), t1 = from_next(up[1]); cdef[4] = u[0] - t0; cdef[5] = u[1] - t1; }
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double t = from_prev(cdef[i]);
                    g[i] = k == 0 ? (i < 4 ? x[i] - x0[i] : up[i - 4] - upv[i - 4]) : -t;
                }
            } else {       // two waves: two exchanges
                double t6[6], pcd[6];
                { const double x6[6] = {x[0], x[1], x[2], x[3], up[0], up[1]}; from_next_n(x6, t6); }
#pragma unroll
                for (int i = 0; i < 4; ++i) cdef[i] = xn[i] - t6[i];
                cdef[4] = u[0] - t6[4]; cdef[5] = u[1] - t6[5];
                from_prev_n(cdef, pcd);
#pragma unroll
                for (int i = 0; i < 6; ++i) g[i] = k == 0 ? (i < 4 ? x[i] - x0[i] : up[i - 4] - upv[i - 4]) : -pcd[i];
            }
        };
        // the inequality rows (shift delta; lsq: the least-square multipliers' unit weights): Sigma's, sigma,
        // off, psi into Q
        auto iq_terms = [&](double delta, bool lsq) {
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                double Ss = 1.0, ps = 0.0, Sp = 1.0, Sn = 1.0, rp = 0.0, rn = 0.0, yv = 0.0;
                if (uon) {
                    if (lsq) {
                        ps = -vl[i] + vu[i]; rp = rho - q[Q_ZQP + i]; rn = rho - q[Q_ZQN + i];
                    } else {
                        const double dl = s[i] - sL[i], du_ = sU[i] - s[i];
                        Ss = (tw[i] ? vl[i] / dl : 0.0) + vu[i] / du_ + delta;
                        ps = (tw[i] ? -rmu / dl : 0.0) + rmu / du_;
                        Sp = q[Q_ZQP + i] / q[Q_QP + i] + delta; Sn = q[Q_ZQN + i] / q[Q_QN + i] + delta;
                        rp = q[Q_RQP + i]; rn = q[Q_RQN + i]; yv = yq[i];
                    }
                }
                const double sg = 1.0 / (1.0 / Ss + 1.0 / Sp + 1.0 / Sn);
                q[Q_SS + i] = Ss; q[Q_SP + i] = Sp; q[Q_SN + i] = Sn; q[Q_SIG + i] = sg; q[Q_PSI + i] = ps;
                q[Q_OFF + i] = uon ? sg * (ps / Ss + yv * (1.0 / Sp + 1.0 / Sn) - rn / Sn + rp / Sp) : 0.0;
            }
        };
        // stage Hessians (node lanes) and the terminal surrogate's Hessian; after iq_terms
        auto assemble_H = [&](double delta, bool lsq) {
            double sg[RM_NQ], so[RM_NQ];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) sg[i] = q[Q_SIG + i];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) so[i] = __shfl_xor(sg[i], 32);
            if (uon && nod) {
                if (lsq) {
                    for (int e = 0; e < RmLds::NT; ++e) Hk[e] = 0.0;
                    Hk[hp(0, 0)] = 1.0; Hk[hp(2, 2)] = 1.0;
                    Hk[hp(1, 1)] = 1.0 + sg[2] + so[0];
                    Hk[hp(3, 3)] = 1.0 + so[1] + so[2];
                    Hk[hp(6, 6)] = 1.0 + sg[0]; Hk[hp(7, 7)] = 1.0 + sg[1];
                    Hk[hp(4, 4)] = sg[0]; Hk[hp(5, 5)] = sg[1];
                } else {
                    double w[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) w[i] = eta * pn[P_DRX + i] * pn[P_DRX + i];
                    double wu[2];
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        wu[j] = eta * pn[P_DRU + j] * pn[P_DRU + j] + zl[j] / (u[j] - lo) + zu[j] / (hi - u[j]);
                    Hk[hp(0, 0)] = hd[0] + w[0] + delta;
                    Hk[hp(1, 1)] = hd[1] + w[1] + sg[2] + so[0] + delta;
                    Hk[hp(2, 2)] = hd[2] + w[2] + delta;
                    Hk[hp(3, 3)] = hd[3] + w[3] + so[1] + so[2] + delta;
                    Hk[hp(6, 6)] = hd[4] + wu[0] + sg[0] + delta;
                    Hk[hp(7, 7)] = hd[5] + wu[1] + sg[1] + delta;
                    Hk[hp(4, 4)] = sg[0] + delta; Hk[hp(5, 5)] = sg[1] + delta;
                }
                Hk[hp(6, 4)] = -sg[0]; Hk[hp(7, 5)] = -sg[1];
            }
            if (k == N && nod) {   // terminal surrogate: [[eta D_R^2 + delta, grad], [grad^T, 0]], Quu = I
                double* GN = S->G[N];
                for (int e = 0; e < RmLds::NT; ++e) GN[e] = 0.0;
#pragma unroll
                for (int i = 0; i < 6; ++i)
                    GN[hp(i, i)] = i < 4 ? (lsq ? 1.0 : eta * pn[P_DRX + i] * pn[P_DRX + i] + delta) : (lsq ? 0.0 : delta);
                GN[hp(6, 6)] = 1.0; GN[hp(7, 7)] = 1.0;
            }
        };
        // gradient rows: the proximity and barrier terms (or the override ov of a refinement solve), plus
        // C^T (sigma rin + offv) of the inequality rows; the terminal surrogate's gradient row
        auto assemble_g = [&](const double* rin, const double* offv, const double* ov, bool lsq) {
            double tq[RM_NQ], to[RM_NQ];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) tq[i] = uon ? q[Q_SIG + i] * rin[i] + offv[i] : 0.0;
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) to[i] = __shfl_xor(tq[i], 32);
            double gq[8];
            if (ov) {
#pragma unroll
                for (int j = 0; j < 8; ++j) gq[j] = ov[j];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) gq[i] = eta * pn[P_DRX + i] * pn[P_DRX + i] * (x[i] - pn[P_XR + i]);
                gq[4] = 0.0; gq[5] = 0.0;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    gq[6 + j] = eta * pn[P_DRU + j] * pn[P_DRU + j] * (u[j] - pn[P_UR + j]);
                    gq[6 + j] += lsq ? -zl[j] + zu[j] : -rmu / (u[j] - lo) + rmu / (hi - u[j]);
                }
            }
            if (uon && nod) {
                gq[6] += tq[0]; gq[4] -= tq[0]; gq[7] += tq[1]; gq[5] -= tq[1];
                gq[1] += tq[2] - to[0];
                gq[3] += to[1] - to[2];
#pragma unroll
                for (int j = 0; j < 8; ++j) Hk[hp(8, j)] = gq[j];
            }
            if (k == N && nod) {
#pragma unroll
                for (int j = 0; j < 6; ++j) S->G[N][hp(8, j)] = j < 4 ? gq[j] : (ov ? ov[j] : 0.0);
            }
        };
        // soft rows of node k's physical incoming rows (shift delta): Sigma_p', Sigma_n', 1 / D
        auto soft_set = [&](double delta, bool lsq) {
            if (nod) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const double sp_ = lsq ? 1.0 : pn[P_ZP + i] / pn[P_PC + i] + delta;
                    const double sn_ = lsq ? 1.0 : pn[P_ZN + i] / pn[P_NC + i] + delta;
                    pn[P_SP + i] = sp_; pn[P_SN + i] = sn_;
                    if (xon) SR->Dinv[k][i] = 1.0 / (1.0 / sp_ + 1.0 / sn_);
                }
            }
        };
        // right-hand side of the soft rows: rg = cgv - (rnv / Sigma_n' - rpv / Sigma_p') + D lamv (physical),
        // cgv (copy rows), into the defect column of M~ and dx~_0
        auto soft_rhs = [&](const double* cgv, const double* lamv, const double* rpv, const double* rnv) {
            double rg[6];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double sp_ = pn[P_SP + i], sn_ = pn[P_SN + i];
                rg[i] = cgv[i] - (rnv[i] / sn_ - rpv[i] / sp_) + (1.0 / sp_ + 1.0 / sn_) * lamv[i];
            }
            rg[4] = cgv[4]; rg[5] = cgv[5];
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                const double t = from_next(rg[r]);
                if (uon && nod) Mk[8 * RmLds::NC + r] = -t;
                if (k == 0 && nod) S->dx0[r] = -rg[r];
            }
        };
        // the step from the factorised soft system: dx~_0 and the closed-loop rows through the soft rows,
        // forward sweep, du = [K | k] [dx~; 1], lambda+ = -(P dx~ + p) with the unsoftened value function
        double dx[6], dU[2], lamp[6], dY[RM_NQ], dS[RM_NQ], dqp[RM_NQ], dqn[RM_NQ], dpc[4], dnc[4];
        auto rstep = [&]() {
            if (k == 0 && nod) {
                double d0[6];
#pragma unroll
                for (int r = 0; r < 6; ++r) d0[r] = S->dx0[r];
                const double* Y0 = SR->T[0];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double t = Y0[7 * r + 6];
#pragma unroll
                    for (int aa = 0; aa < 6; ++aa) t = fma(Y0[7 * r + aa], d0[aa], t);
                    S->dx0[r] = t;
                }
            }
            __syncthreads();
            closed_loop(S, N, RmSoftPost{S, SR});
            forward_sweep(S, N, k, dx);
            const double* K0 = S->KK[uon ? k : 0][0];
            const double* K1 = S->KK[uon ? k : 0][1];
            double d0 = K0[6], d1 = K1[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) { d0 = fma(K0[j], dx[j], d0); d1 = fma(K1[j], dx[j], d1); }
            dU[0] = uon ? d0 : 0.0; dU[1] = uon ? d1 : 0.0;
            node_multiplier(S, xon ? k : 0, dx, dU, lamp);
        };
        // the eliminated rows' steps: y + dy = sigma (C dz + rin) + offv, ds, dp, dn of the inequality rows,
        // dp, dn of the physical defect rows
        auto rdirs = [&](const double* rin, const double* offv, const double* psv, const double* rqpv,
                         const double* rqnv, const double* yv, const double* lamv, const double* rpv, const double* rnv) {
            const double dz[8] = {dx[0], dx[1], dx[2], dx[3], dx[4], dx[5], dU[0], dU[1]};
            double cdz[RM_NQ];
            rm_iq3(dz, 0.0, mir, cdz);
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                const double yn = q[Q_SIG + i] * (cdz[i] + rin[i]) + offv[i];
                dY[i] = uon ? yn - yv[i] : 0.0;
                dS[i] = uon ? (yn - psv[i]) / q[Q_SS + i] : 0.0;
                dqp[i] = uon ? (dY[i] - rqpv[i]) / q[Q_SP + i] : 0.0;
                dqn[i] = uon ? (-dY[i] - rqnv[i]) / q[Q_SN + i] : 0.0;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double dl = lamp[i] - lamv[i];
                dpc[i] = xon ? (dl - rpv[i]) / pn[P_SP + i] : 0.0;
                dnc[i] = xon ? (-dl - rnv[i]) / pn[P_SN + i] : 0.0;
            }
        };
        auto park = [&](double* v) {
#pragma unroll
            for (int i = 0; i < 6; ++i) { v[V_DX + i] = dx[i]; v[V_LP + i] = lamp[i]; }
#pragma unroll
            for (int j = 0; j < 2; ++j) v[V_DU + j] = dU[j];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) { v[V_DY + i] = dY[i]; v[V_DS + i] = dS[i]; v[V_DQP + i] = dqp[i]; v[V_DQN + i] = dqn[i]; }
#pragma unroll
            for (int i = 0; i < 4; ++i) { v[V_DPC + i] = dpc[i]; v[V_DNC + i] = dnc[i]; }
        };
        auto unpark = [&](const double* v, bool add) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                dx[i] = add ? dx[i] + v[V_DX + i] : v[V_DX + i];
                lamp[i] = add ? lamp[i] + v[V_LP + i] : v[V_LP + i];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) dU[j] = add ? dU[j] + v[V_DU + j] : v[V_DU + j];
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                dY[i] = add ? dY[i] + v[V_DY + i] : v[V_DY + i];
                dS[i] = add ? dS[i] + v[V_DS + i] : v[V_DS + i];
                dqp[i] = add ? dqp[i] + v[V_DQP + i] : v[V_DQP + i];
                dqn[i] = add ? dqn[i] + v[V_DQN + i] : v[V_DQN + i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dpc[i] = add ? dpc[i] + v[V_DPC + i] : v[V_DPC + i];
                dnc[i] = add ? dnc[i] + v[V_DNC + i] : v[V_DNC + i];
            }
        };
        const double zero6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};

        // ---- least-square equality multipliers of the restoration problem (unit weights on x, u, s, p, n) ----
        STAMP(7);               // (diagnostic stamps: 16.. the restoration phase proper)
        {
            if (nod) {
#pragma unroll
                for (int i = 0; i < 4; ++i) { pn[P_RP + i] = rho - pn[P_ZP + i]; pn[P_RN + i] = rho - pn[P_ZN + i]; }
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) lam[i] = 0.0;
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) yq[i] = 0.0;
            rderiv();
            iq_terms(0.0, true);
            assemble_H(0.0, true);
            assemble_g(zero6, q + Q_OFF, nullptr, true);
            soft_set(0.0, true);
            soft_rhs(zero6, zero6, pn + P_RP, pn + P_RN);
            __syncthreads();
            (void)riccati_sweep_aug_soft<RmLds, 4>(S, SR, N);      // unit weights: positive definite
            rstep();
            double ym = 0.0;
            bool fin = true;
            const double dz[8] = {dx[0], dx[1], dx[2], dx[3], dx[4], dx[5], dU[0], dU[1]};
            double cdz[RM_NQ], yd[RM_NQ];
            rm_iq3(dz, 0.0, mir, cdz);
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                yd[i] = uon ? q[Q_SIG + i] * cdz[i] + q[Q_OFF + i] : 0.0;
                ym = fmax(ym, fabs(yd[i]));
                fin = fin && isfinite(yd[i]);
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                if (i < 4) ym = fmax(ym, nod && xon ? fabs(lamp[i]) : 0.0);
                fin = fin && (!xon || isfinite(lamp[i]));
            }
            const bool use = !wany(!fin) && wmax(ym) <= 1e3;
#pragma unroll
            for (int i = 0; i < 6; ++i) lam[i] = (use && xon) ? lamp[i] : 0.0;
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) yq[i] = use ? yd[i] : 0.0;
        }
        int rit = it + 1, rnf = 0, rstat = -2;
        bool rfirst = true, rok = false;
        double rfth = 0.0, rfph = 0.0, rdelta_last = 0.0, thr = 0.0, rth_max = 0.0, rth_min = 0.0;
        double cg[6], cr[RM_NQ];
        STAMP(16);
        for (;; ++rit) {
            STAMP_ADD(27, 1);
            rderiv();
            {
                double g[6], cz[RM_NQ];
                incoming(g);
                const double zz[8] = {x[0], x[1], x[2], x[3], up[0], up[1], u[0], u[1]};
                rm_iq3(zz, vmax, mir, cz);
#pragma unroll
                for (int i = 0; i < 6; ++i) cg[i] = i < 4 ? g[i] + pn[P_NC + i] - pn[P_PC + i] : g[i];
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) cr[i] = uon ? cz[i] - s[i] + q[Q_QN + i] - q[Q_QP + i] : 0.0;
                if (rfirst) {
                    double t = 0.0;
#pragma unroll
                    for (int i = 0; i < 6; ++i) t += nod && xon ? fabs(cg[i]) : 0.0;
#pragma unroll
                    for (int i = 0; i < RM_NQ; ++i) t += uon ? fabs(cr[i]) : 0.0;
                    thr = wsum_rl(t);
                    rth_max = 1e4 * fmax(1.0, thr); rth_min = 1e-4 * fmax(1.0, thr);
                } else {
                    // RestoConvergenceCheck: the original problem's progress at the current point
                    double t = 0.0;
#pragma unroll
                    for (int i = 0; i < 6; ++i) t += nod && xon ? fabs(g[i]) : 0.0;
#pragma unroll
                    for (int i = 0; i < RM_NQ; ++i) t += uon ? fabs(cz[i] - s[i]) : 0.0;
                    const double tho = wsum_rl(t);
                    if (tho <= 0.9 * th0) {
                        double pl = nod ? sc * cost_val(x, u, up) : 0.0;
                        double pa = 1.0;
                        if (uon) {
                            const double pb = (u[0] - lo) * (hi - u[0]) * (u[1] - lo) * (hi - u[1]) * ((s[0] - sL[0]) * (s[1] - sL[1]));
                            pa = nod ? pb : 1.0;
#pragma unroll
                            for (int i = 0; i < RM_NQ; ++i) pa *= sU[i] - s[i];
                        }
                        pl -= uon ? mu0 * log_fast(pa) : 0.0;
                        const double pho = wsum_rl(pl);
                        bool accp = isfinite(pho) && !wany_rep(lane < nfilt && tho >= fth && pho >= fph);
                        accp = accp && (cmp_le(tho, (1 - gam_th) * th0, th0) || cmp_le(pho - phi0, -gam_ph * th0, phi0));
                        if (accp) { rok = true; theta = tho; break; }
                    }
                }
            }
            rfirst = false;
            // ---- optimality error of the restoration problem ----
            double dinf = 0.0, pinf = 0.0, c0r = 0.0, cminr = 1e300, suml = 0.0, sumz = 0.0;
            {
                double gl[8];
#pragma unroll
                for (int i = 0; i < 4; ++i) gl[i] = eta * pn[P_DRX + i] * pn[P_DRX + i] * (x[i] - pn[P_XR + i]);
                gl[4] = 0.0; gl[5] = 0.0;
#pragma unroll
                for (int j = 0; j < 2; ++j) gl[6 + j] = eta * pn[P_DRU + j] * pn[P_DRU + j] * (u[j] - pn[P_UR + j]);
#pragma unroll
                for (int i = 0; i < 6; ++i) gl[i] += lam[i];
#pragma unroll
                for (int j = 0; j < 4; ++j) gl[j] -= jl[j];
                gl[6] -= jl[4] + lmn[4]; gl[7] -= jl[5] + lmn[5];
                double yo[RM_NQ];
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) yo[i] = __shfl_xor(yq[i], 32);
                gl[6] += yq[0]; gl[4] -= yq[0]; gl[7] += yq[1]; gl[5] -= yq[1];
                gl[1] += yq[2] - yo[0]; gl[3] += yo[1] - yo[2];
                gl[6] += -zl[0] + zu[0]; gl[7] += -zl[1] + zu[1];
#pragma unroll
                for (int j = 0; j < 8; ++j) dinf = fmax(dinf, nod && (j < 6 ? xon : uon) ? fabs(gl[j]) : 0.0);
                if (uon) {
#pragma unroll
                    for (int i = 0; i < RM_NQ; ++i) {
                        const double y = yq[i];
                        dinf = fmax(dinf, fabs(-y - vl[i] + vu[i]));
                        dinf = fmax(dinf, fmax(fabs(rho - q[Q_ZQP + i] - y), fabs(rho - q[Q_ZQN + i] + y)));
                        pinf = fmax(pinf, fabs(cr[i]));
                        if (tw[i]) {
                            const double cl = vl[i] * (s[i] - sL[i]);
                            c0r = fmax(c0r, cl); cminr = fmin(cminr, cl); sumz += vl[i];
                        }
                        const double cu = vu[i] * (sU[i] - s[i]), cp = q[Q_ZQP + i] * q[Q_QP + i], cn = q[Q_ZQN + i] * q[Q_QN + i];
                        c0r = fmax(c0r, fmax(cu, fmax(cp, cn))); cminr = fmin(cminr, fmin(cu, fmin(cp, cn)));
                        sumz += vu[i] + q[Q_ZQP + i] + q[Q_ZQN + i];
                        suml += fabs(y);
                    }
                    if (nod) {
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const double cl = zl[j] * (u[j] - lo), cu = zu[j] * (hi - u[j]);
                            c0r = fmax(c0r, fmax(cl, cu)); cminr = fmin(cminr, fmin(cl, cu));
                            sumz += zl[j] + zu[j];
                        }
                    }
                }
                if (nod && xon) {
#pragma unroll
                    for (int i = 0; i < 6; ++i) { pinf = fmax(pinf, fabs(cg[i])); suml += fabs(lam[i]); }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        dinf = fmax(dinf, fmax(fabs(rho - pn[P_ZP + i] - lam[i]), fabs(rho - pn[P_ZN + i] + lam[i])));
                        const double cp = pn[P_ZP + i] * pn[P_PC + i], cn = pn[P_ZN + i] * pn[P_NC + i];
                        c0r = fmax(c0r, fmax(cp, cn)); cminr = fmin(cminr, fmin(cp, cn));
                        sumz += pn[P_ZP + i] + pn[P_ZN + i];
                    }
                }
                wred_errors_f64_rl(dinf, pinf, c0r, cminr, suml, sumz);
            }
            const double s_d = fmax(100.0, (suml + sumz) / (nA + nI + nbr)) / 100.0;
            const double s_c = fmax(100.0, sumz / nbr) / 100.0;
            const double errr = fmax(dinf / s_d, fmax(pinf, c0r / s_c));
            if (rit >= a.max_iter) { rstat = -1; break; }
            // the restoration problem converged: local infeasibility (IPOPT Infeasible_Problem_Detected, 2)
            if (errr <= tol && dinf <= 1.0 && pinf <= 1e-4 && c0r <= 1e-4) { rstat = 2; break; }
            for (;;) {
                const double cmu = fmax(c0r - rmu, rmu - cminr);
                if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * rmu || rmu <= mu_min) break;
                rmu = fmax(mu_min, fmin(0.2 * rmu, rmu * sqrt(rmu)));
                eta = sqrt(rmu);
                rnf = 0;
            }
            const double taur = fmax(0.99, 1.0 - rmu);
            if (nod) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    pn[P_RP + i] = rho - rmu / pn[P_PC + i] - lam[i];
                    pn[P_RN + i] = rho - rmu / pn[P_NC + i] + lam[i];
                }
            }
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                q[Q_RQP + i] = uon ? rho - rmu / q[Q_QP + i] - yq[i] : 0.0;
                q[Q_RQN + i] = uon ? rho - rmu / q[Q_QN + i] + yq[i] : 0.0;
            }
            STAMP(17);
            // ---- the step: plain (with inertia correction) or a second-order correction pass, one solve site;
            //      each solve refined iteratively (IPOPT's PDFullSpaceSolver) ----
            double delta = 0.0, amr = 1.0, azr = 1.0, phir = 0.0, gtdr = 0.0, aminr = 0.0, alr = 1.0;
            double pw_thr = 0.0, pw_gdr = 0.0;      // theta^s_th, (-gTd)^s_ph of the line search (gTd < 0)
            double csg[6], csr[RM_NQ], cgt[6], crt[RM_NQ], tht = 0.0, pht = 0.0, th_prev = 0.0;
            bool accr = false, ftr = false, okr = true;
            int soc = -1, ls = 0;
            // fractions to the boundary of the primal step (amr) and of every bound multiplier (azr)
            auto pn_steps = [&]() {
                double am = 1.0, a2 = 1.0;
                if (nod && xon) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const double p = pn[P_PC + i], n = pn[P_NC + i], zp = pn[P_ZP + i], zn = pn[P_ZN + i];
                        if (dpc[i] < 0) am = fmin(am, -taur * p / dpc[i]);
                        if (dnc[i] < 0) am = fmin(am, -taur * n / dnc[i]);
                        const double dzp = rmu / p - zp - zp / p * dpc[i], dzn = rmu / n - zn - zn / n * dnc[i];
                        if (dzp < 0) a2 = fmin(a2, -taur * zp / dzp);
                        if (dzn < 0) a2 = fmin(a2, -taur * zn / dzn);
                    }
                }
                if (uon) {
                    if (nod) {
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const double sl_ = u[j] - lo, su_ = hi - u[j];
                            if (dU[j] < 0) am = fmin(am, -taur * sl_ / dU[j]);
                            if (dU[j] > 0) am = fmin(am, taur * su_ / dU[j]);
                            const double dzl_ = rmu / sl_ - zl[j] - zl[j] / sl_ * dU[j];
                            const double dzu_ = rmu / su_ - zu[j] + zu[j] / su_ * dU[j];
                            if (dzl_ < 0) a2 = fmin(a2, -taur * zl[j] / dzl_);
                            if (dzu_ < 0) a2 = fmin(a2, -taur * zu[j] / dzu_);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < RM_NQ; ++i) {
                        const double dl = s[i] - sL[i], du_ = sU[i] - s[i];
                        if (tw[i] && dS[i] < 0) am = fmin(am, -taur * dl / dS[i]);
                        if (dS[i] > 0) am = fmin(am, taur * du_ / dS[i]);
                        const double p = q[Q_QP + i], n = q[Q_QN + i], zp = q[Q_ZQP + i], zn = q[Q_ZQN + i];
                        if (dqp[i] < 0) am = fmin(am, -taur * p / dqp[i]);
                        if (dqn[i] < 0) am = fmin(am, -taur * n / dqn[i]);
                        if (tw[i]) {
                            const double dv = rmu / dl - vl[i] - vl[i] / dl * dS[i];
                            if (dv < 0) a2 = fmin(a2, -taur * vl[i] / dv);
                        }
                        const double dv = rmu / du_ - vu[i] + vu[i] / du_ * dS[i];
                        if (dv < 0) a2 = fmin(a2, -taur * vu[i] / dv);
                        const double dzp = rmu / p - zp - zp / p * dqp[i], dzn = rmu / n - zn - zn / n * dqn[i];
                        if (dzp < 0) a2 = fmin(a2, -taur * zp / dzp);
                        if (dzn < 0) a2 = fmin(a2, -taur * zn / dzn);
                    }
                }
                wmin2d(am, a2);
                amr = am; azr = a2;
            };
            // one refinement pass: the residuals of the full Newton system at the step (stationarity of z, the
            // soft defect rows, the p / n rows of both kinds, the inequality and slack rows) solved for on the
            // same factorisation and added, while they exceed 1e-12 (1 + |step|); returns false when done
            auto refine = [&](const double* cgv, const double* crv) -> bool {
                double lpn_[6], pdx[6], pdu[2];
#pragma unroll
                for (int i = 0; i < 6; ++i) { const double t = from_next(lamp[i]); lpn_[i] = uon ? t : 0.0; }
#pragma unroll
                for (int i = 0; i < 6; ++i) pdx[i] = from_prev(dx[i]);
                pdu[0] = from_prev(dU[0]); pdu[1] = from_prev(dU[1]);
                double ex[8], ec[6], ep[4], en[4], eq[RM_NQ], eqp[RM_NQ], eqn[RM_NQ], es[RM_NQ];
                double emax = 0.0, smax = 0.0;
#pragma unroll
                for (int j = 0; j < 8; ++j) ex[j] = 0.0;
                if (uon && nod) {
                    const double dz[8] = {dx[0], dx[1], dx[2], dx[3], dx[4], dx[5], dU[0], dU[1]};
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        double t = Hk[hp(8, j)];
#pragma unroll
                        for (int i = 0; i < 8; ++i) t = fma(Hk[hp(j, i)], dz[i], t);
                        if (j < 6) t += lamp[j];
#pragma unroll
                        for (int mm = 0; mm < 6; ++mm) t -= Mk[j * RmLds::NC + mm] * lpn_[mm];
                        ex[j] = t;
                        emax = fmax(emax, fabs(t));
                    }
                } else if (k == N && nod) {
                    const double* GN = S->G[N];
#pragma unroll
                    for (int j = 0; j < 6; ++j) {
                        double t = GN[hp(8, j)];
#pragma unroll
                        for (int i = 0; i < 6; ++i) t = fma(GN[hp(j, i)], dx[i], t);
                        ex[j] = t + lamp[j];
                        emax = fmax(emax, fabs(ex[j]));
                    }
                }
#pragma unroll
                for (int i = 0; i < 6; ++i) ec[i] = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) { ep[i] = 0.0; en[i] = 0.0; }
                if (nod && xon) {
                    const double* Mp = &S->M[k > 0 ? k - 1 : 0][0][0];
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        double jd = dx[i];
                        if (k > 0) {
#pragma unroll
                            for (int mm = 0; mm < 6; ++mm) jd -= Mp[mm * RmLds::NC + i] * pdx[mm];
                            jd -= Mp[6 * RmLds::NC + i] * pdu[0];
                            jd -= Mp[7 * RmLds::NC + i] * pdu[1];
                        }
                        smax = fmax(smax, fabs(dx[i]));
                        if (i < 4) {
                            const double dl = lamp[i] - lam[i];
                            ec[i] = jd + dnc[i] - dpc[i] + cgv[i];
                            ep[i] = pn[P_SP + i] * dpc[i] - dl + pn[P_RP + i];
                            en[i] = pn[P_SN + i] * dnc[i] + dl + pn[P_RN + i];
                            emax = fmax(emax, fmax(fabs(ep[i]), fabs(en[i])));
                            smax = fmax(smax, fmax(fabs(dpc[i]), fabs(dnc[i])));
                        } else {
                            ec[i] = jd + cgv[i];
                        }
                        emax = fmax(emax, fabs(ec[i]));
                    }
                }
                {
                    const double dz[8] = {dx[0], dx[1], dx[2], dx[3], dx[4], dx[5], dU[0], dU[1]};
                    double cdz[RM_NQ];
                    rm_iq3(dz, 0.0, mir, cdz);
#pragma unroll
                    for (int i = 0; i < RM_NQ; ++i) {
                        eq[i] = uon ? cdz[i] - dS[i] + dqn[i] - dqp[i] + crv[i] : 0.0;
                        eqp[i] = uon ? q[Q_SP + i] * dqp[i] - dY[i] + q[Q_RQP + i] : 0.0;
                        eqn[i] = uon ? q[Q_SN + i] * dqn[i] + dY[i] + q[Q_RQN + i] : 0.0;
                        es[i] = uon ? q[Q_SS + i] * dS[i] - (yq[i] + dY[i]) + q[Q_PSI + i] : 0.0;
                        emax = fmax(emax, fmax(fmax(fabs(eq[i]), fabs(eqp[i])), fmax(fabs(eqn[i]), fabs(es[i]))));
                        smax = fmax(smax, fmax(fabs(dS[i]), fmax(fabs(dqp[i]), fabs(dqn[i]))));
                    }
                }
                if (uon && nod) smax = fmax(smax, fmax(fabs(dU[0]), fabs(dU[1])));
                emax = wmax(emax); smax = wmax(smax);
#ifdef DART_RESTO_TRACE
                {
                    double e1 = 0.0, e2 = 0.0, e3 = 0.0, e4 = 0.0;
                    for (int j = 0; j < 8; ++j) e1 = fmax(e1, fabs(ex[j]));
                    for (int i = 0; i < 6; ++i) e2 = fmax(e2, fabs(ec[i]));
                    for (int i = 0; i < 4; ++i) e3 = fmax(e3, fmax(fabs(ep[i]), fabs(en[i])));
                    for (int i = 0; i < RM_NQ; ++i) e4 = fmax(e4, fmax(fmax(fabs(eq[i]), fabs(eqp[i])), fmax(fabs(eqn[i]), fabs(es[i]))));
                    e1 = wmax(e1); e2 = wmax(e2); e3 = wmax(e3); e4 = wmax(e4);
                    double dmn = 1e300, dmx = 0.0, smx = 0.0;
                    if (nod && xon) for (int i = 0; i < 4; ++i) { dmn = fmin(dmn, SR->Dinv[k][i]); dmx = fmax(dmx, SR->Dinv[k][i]); }
                    if (uon) for (int i = 0; i < RM_NQ; ++i) smx = fmax(smx, q[Q_SIG + i]);
                    dmn = wmin(dmn); dmx = wmax(dmx); smx = wmax(smx);
                    if (blockIdx.x == 0 && lane == 0)
                        printf("     refine emax %.3e (stat %.2e defect %.2e pn %.2e iq %.2e) smax %.3e  Dinv [%.2e, %.2e] sigma max %.2e\n",
                               emax, e1, e2, e3, e4, smax, dmn, dmx, smx);
                }
#endif
                if (!(emax > 1e-12 * (1.0 + smax))) return false;
                // the correction solve: lambda = y = 0, the residuals as gradient and right-hand sides
                park(RS.SV2[ql]);
                double gsave[8], offc[RM_NQ];
#pragma unroll
                for (int j = 0; j < 8; ++j) gsave[j] = (uon && nod) ? Hk[hp(8, j)] : (k == N && nod && j < 6 ? S->G[N][hp(8, j)] : 0.0);
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i)
                    offc[i] = uon ? q[Q_SIG + i] * (es[i] / q[Q_SS + i] - eqn[i] / q[Q_SN + i] + eqp[i] / q[Q_SP + i]) : 0.0;
                assemble_g(eq, offc, ex, false);
                soft_rhs(ec, zero6, ep, en);
                __syncthreads();
                (void)riccati_sweep_aug_soft<RmLds, 4>(S, SR, N);
                rstep();
                rdirs(eq, offc, es, eqp, eqn, zero6, zero6, ep, en);
                unpark(RS.SV2[ql], true);
                if (uon && nod) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) Hk[hp(8, j)] = gsave[j];
                } else if (k == N && nod) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) S->G[N][hp(8, j)] = gsave[j];
                }
                __syncthreads();
                return true;
            };
            // trial point of the restoration problem at step al: constraint values cgt / crt, theta, barrier
            auto trial_r = [&](double al) {
                double xt[4], pt[2], ut[2], st_[RM_NQ], gt[6];
#pragma unroll
                for (int i = 0; i < 4; ++i) xt[i] = fma(al, dx[i], x[i]);
                pt[0] = fma(al, dx[4], up[0]); pt[1] = fma(al, dx[5], up[1]);
#pragma unroll
                for (int j = 0; j < 2; ++j) ut[j] = uon ? fma(al, dU[j], u[j]) : u[j];
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) st_[i] = fma(al, dS[i], s[i]);
                defects(xt, pt, ut, gt);
                const double zt[8] = {xt[0], xt[1], xt[2], xt[3], pt[0], pt[1], ut[0], ut[1]};
                double ct[RM_NQ];
                rm_iq3(zt, vmax, mir, ct);
                double thl = 0.0, phl = 0.0, lb = 0.0;
                bool inside = true;
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    if (i < 4) {
                        const double p = fma(al, dpc[i], pn[P_PC + i]), n = fma(al, dnc[i], pn[P_NC + i]);
                        cgt[i] = gt[i] + n - p;
                        if (nod && xon) {
                            const double e = pn[P_DRX + i] * (xt[i] - pn[P_XR + i]);
                            phl += rho * (p + n) + 0.5 * eta * e * e;
                            inside = inside && p > 0.0 && n > 0.0;
                            lb += log_fast(p) + log_fast(n);
                        }
                    } else {
                        cgt[i] = gt[i];
                    }
                    thl += nod && xon ? fabs(cgt[i]) : 0.0;
                }
                if (uon) {
#pragma unroll
                    for (int i = 0; i < RM_NQ; ++i) {
                        const double p = fma(al, dqp[i], q[Q_QP + i]), n = fma(al, dqn[i], q[Q_QN + i]);
                        crt[i] = ct[i] - st_[i] + n - p;
                        thl += fabs(crt[i]);
                        phl += rho * (p + n);
                        const double dl = st_[i] - sL[i], du_ = sU[i] - st_[i];
                        inside = inside && p > 0.0 && n > 0.0 && du_ > 0.0 && (!tw[i] || dl > 0.0);
                        lb += log_fast(p) + log_fast(n) + (tw[i] ? log_fast(dl) : 0.0) + log_fast(du_);
                    }
                    if (nod) {
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const double e = pn[P_DRU + j] * (ut[j] - pn[P_UR + j]);
                            phl += 0.5 * eta * e * e;
                            inside = inside && ut[j] > lo && ut[j] < hi;
                            lb += log_fast(ut[j] - lo) + log_fast(hi - ut[j]);
                        }
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < RM_NQ; ++i) crt[i] = 0.0;
                }
                phl = inside ? phl - rmu * lb : __builtin_inf();
                wsum2_rl(thl, phl);
                tht = thl; pht = phl;
            };
            auto racc = [&](double al_test, bool& ft) {
                const bool in_f = !(tht < rth_max) || !isfinite(pht) || wany_rep(lane < rnf && tht >= rfth && pht >= rfph);
                if (in_f) return false;
                const bool sw = gtdr < 0.0 && al_test * pw_gdr > pw_thr;
                if (thr <= rth_min && sw) {
                    if (cmp_le(pht, phir + eta_ph * al_test * gtdr, phir)) { ft = true; return true; }
                    return false;
                }
                return cmp_le(tht, (1 - gam_th) * thr, thr) || cmp_le(pht - phir, -gam_ph * thr, phir);
            };
            for (;;) {
                if (soc < 0) {
                    int attempt = 0;
                    for (;;) {
                        iq_terms(delta, false);
                        assemble_H(delta, false);
                        assemble_g(cr, q + Q_OFF, nullptr, false);
                        soft_set(delta, false);
                        soft_rhs(cg, lam, pn + P_RP, pn + P_RN);
                        __syncthreads();
                        okr = riccati_sweep_aug_soft<RmLds, 4>(S, SR, N);
                        STAMP_ADD(24, 1);
                        if (okr || ++attempt >= 60) break;
                        delta = (attempt == 1) ? (rdelta_last == 0.0 ? 1e-4 : fmax(1e-20, rdelta_last * (1.0 / 3.0)))
                                               : delta * (rdelta_last == 0.0 ? 100.0 : 8.0);
                    }
                    if (!okr) break;
                    if (delta > 0.0) rdelta_last = delta;
                } else {
                    assemble_g(csr, q + Q_OFF, nullptr, false);
                    soft_rhs(csg, lam, pn + P_RP, pn + P_RN);
                    __syncthreads();
                    (void)riccati_sweep_aug_soft<RmLds, 4>(S, SR, N);
                    STAMP_ADD(24, 1);
                }
                STAMP(18);
                rstep();
                rdirs(soc < 0 ? cr : csr, q + Q_OFF, q + Q_PSI, q + Q_RQP, q + Q_RQN, yq, lam, pn + P_RP, pn + P_RN);
                for (int rr = 0; rr < 3 && refine(soc < 0 ? cg : csg, soc < 0 ? cr : csr); ++rr) { STAMP_ADD(25, 1); }
                pn_steps();
                STAMP(19);
                double al_try;
                if (soc < 0) {
                    // barrier objective of the restoration problem and its directional derivative
                    double pl = 0.0, gd = 0.0, lb = 0.0;
                    if (nod && xon) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const double p = pn[P_PC + i], n = pn[P_NC + i];
                            const double w = eta * pn[P_DRX + i] * pn[P_DRX + i];
                            const double e = pn[P_DRX + i] * (x[i] - pn[P_XR + i]);
                            pl += rho * (p + n) + 0.5 * eta * e * e;
                            lb += log_fast(p) + log_fast(n);
                            gd += w * (x[i] - pn[P_XR + i]) * dx[i] + (rho - rmu / p) * dpc[i] + (rho - rmu / n) * dnc[i];
                        }
                    }
                    if (uon) {
#pragma unroll
                        for (int i = 0; i < RM_NQ; ++i) {
                            const double p = q[Q_QP + i], n = q[Q_QN + i];
                            pl += rho * (p + n);
                            lb += log_fast(p) + log_fast(n) + (tw[i] ? log_fast(s[i] - sL[i]) : 0.0) + log_fast(sU[i] - s[i]);
                            gd += (rho - rmu / p) * dqp[i] + (rho - rmu / n) * dqn[i] + q[Q_PSI + i] * dS[i];
                        }
                        if (nod) {
#pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                const double w = eta * pn[P_DRU + j] * pn[P_DRU + j];
                                const double e = pn[P_DRU + j] * (u[j] - pn[P_UR + j]);
                                pl += 0.5 * eta * e * e;
                                lb += log_fast(u[j] - lo) + log_fast(hi - u[j]);
                                gd += (w * (u[j] - pn[P_UR + j]) - rmu / (u[j] - lo) + rmu / (hi - u[j])) * dU[j];
                            }
                        }
                    }
                    double plb = pl - rmu * lb;
                    wsum2_rl(plb, gd);
                    phir = plb; gtdr = gd;
                    // theta^s_th and (-gTd)^s_ph, fixed through the line search: once here, one on each half of the wave
                    pw_thr = 0.0; pw_gdr = 0.0;
                    if (gtdr < 0) half_pair(lane < 32 ? pow(thr, s_th) : pow(-gtdr, s_ph), pw_thr, pw_gdr);
                    aminr = gam_th;
                    if (gtdr < 0) aminr = fmin(gam_th, fmin(gam_ph * thr / (-gtdr), pw_thr / pw_gdr));
                    aminr *= gam_al;
                    alr = amr;
                    al_try = alr;
                } else {
                    al_try = amr;
                }
                bool resolve = false;
                for (;;) {
                    trial_r(al_try);
                    STAMP_ADD(26, 1);
                    if (soc < 0) {
                        if (racc(alr, ftr)) { accr = true; break; }
                        if (ls == 0 && a.max_soc > 0 && !(tht < thr)) {
                            // second-order correction on the restoration problem's constraints; the plain step
                            // is parked in LDS
                            park(RS.SV[ql]);
#pragma unroll
                            for (int i = 0; i < 6; ++i) csg[i] = fma(alr, cg[i], cgt[i]);
#pragma unroll
                            for (int i = 0; i < RM_NQ; ++i) csr[i] = fma(alr, cr[i], crt[i]);
                            th_prev = tht; soc = 0; resolve = true;
                            break;
                        }
                    } else {
                        bool ft = false;
                        if (racc(alr, ft)) { accr = true; ftr = ft; alr = al_try; break; }
                        if (soc + 1 < a.max_soc && tht <= 0.99 * th_prev) {
#pragma unroll
                            for (int i = 0; i < 6; ++i) csg[i] = fma(al_try, csg[i], cgt[i]);
#pragma unroll
                            for (int i = 0; i < RM_NQ; ++i) csr[i] = fma(al_try, csr[i], crt[i]);
                            th_prev = tht; ++soc; resolve = true;
                            break;
                        }
                        // the corrections failed: back to the plain step and its multiplier steps
                        unpark(RS.SV[ql], false);
                        const double amr_keep = amr;
                        pn_steps();
                        amr = amr_keep;
                        soc = -1;
                    }
                    ++ls;
                    alr *= 0.5;
                    if (alr < aminr || ls >= 80) break;
                    al_try = alr;
                }
                if (!resolve) break;
            }
            STAMP(20);
#ifdef DART_RESTO_TRACE
            if (blockIdx.x == 0 && lane == 0)
                printf("  resto it %3d mu %.2e err %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e th %.3e "
                       "th_t %.3e acc %d\n", rit, rmu, errr, dinf / s_d, pinf, c0r / s_c, delta, amr, alr, thr, tht, (int)accr);
#endif
            if (!okr) { rstat = -3; break; }
            if (!accr) { rstat = -2; break; }      // a failed line search in the restoration phase
            if (!ftr && rnf < kWave) {
                if (lane == rnf) { rfth = (1 - gam_th) * thr; rfph = phir - gam_ph * thr; }
                ++rnf;
            }
            // ---- accept the trial point ----
            if (nod && xon) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const double p = fma(alr, dpc[i], pn[P_PC + i]), n = fma(alr, dnc[i], pn[P_NC + i]);
                    const double zp = pn[P_ZP + i], zn = pn[P_ZN + i];
                    const double dzp = rmu / pn[P_PC + i] - zp - zp / pn[P_PC + i] * dpc[i];
                    const double dzn = rmu / pn[P_NC + i] - zn - zn / pn[P_NC + i] * dnc[i];
                    pn[P_PC + i] = p; pn[P_NC + i] = n;
                    pn[P_ZP + i] = fmax(fmin(fma(azr, dzp, zp), 1e10 * rmu / p), rmu / (1e10 * p));
                    pn[P_ZN + i] = fmax(fmin(fma(azr, dzn, zn), 1e10 * rmu / n), rmu / (1e10 * n));
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = xon ? fma(alr, dx[i], x[i]) : x[i];
            up[0] = xon ? fma(alr, dx[4], up[0]) : up[0];
            up[1] = xon ? fma(alr, dx[5], up[1]) : up[1];
#pragma unroll
            for (int i = 0; i < 6; ++i) lam[i] = xon ? fma(alr, lamp[i] - lam[i], lam[i]) : 0.0;
            if (uon) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double sl_ = u[j] - lo, su_ = hi - u[j];
                    const double dzl_ = rmu / sl_ - zl[j] - zl[j] / sl_ * dU[j];
                    const double dzu_ = rmu / su_ - zu[j] + zu[j] / su_ * dU[j];
                    u[j] = fma(alr, dU[j], u[j]);
                    const double nl = u[j] - lo, nu = hi - u[j];
                    zl[j] = fmax(fmin(fma(azr, dzl_, zl[j]), 1e10 * rmu / nl), rmu / (1e10 * nl));
                    zu[j] = fmax(fmin(fma(azr, dzu_, zu[j]), 1e10 * rmu / nu), rmu / (1e10 * nu));
                }
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) {
                    const double dl = s[i] - sL[i], du_ = sU[i] - s[i];
                    const double dvl_ = tw[i] ? rmu / dl - vl[i] - vl[i] / dl * dS[i] : 0.0;
                    const double dvu_ = rmu / du_ - vu[i] + vu[i] / du_ * dS[i];
                    const double p0 = q[Q_QP + i], n0 = q[Q_QN + i], zp = q[Q_ZQP + i], zn = q[Q_ZQN + i];
                    const double dzp = rmu / p0 - zp - zp / p0 * dqp[i], dzn = rmu / n0 - zn - zn / n0 * dqn[i];
                    const double p = fma(alr, dqp[i], p0), n = fma(alr, dqn[i], n0);
                    s[i] = fma(alr, dS[i], s[i]);
                    yq[i] = fma(alr, dY[i], yq[i]);
                    q[Q_QP + i] = p; q[Q_QN + i] = n;
                    q[Q_ZQP + i] = fmax(fmin(fma(azr, dzp, zp), 1e10 * rmu / p), rmu / (1e10 * p));
                    q[Q_ZQN + i] = fmax(fmin(fma(azr, dzn, zn), 1e10 * rmu / n), rmu / (1e10 * n));
                    const double nl = s[i] - sL[i], nu = sU[i] - s[i];
                    if (tw[i]) vl[i] = fmax(fmin(fma(azr, dvl_, vl[i]), 1e10 * rmu / nl), rmu / (1e10 * nl));
                    vu[i] = fmax(fmin(fma(azr, dvu_, vu[i]), 1e10 * rmu / nu), rmu / (1e10 * nu));
                }
            }
            thr = tht;
            __syncthreads();
            STAMP(22);
        }
        if (!rok) { status = rstat; it = rit; break; }
        // back to the original problem: the bound multipliers take the step (mu - z s_trial) / s that pretends
        // the restoration's progress was one Newton step, cut by the fraction to the boundary (tau of the
        // original iteration) and all reset to 1 if one exceeds 1000; the equality multipliers restart at 0
        {
            double a2 = 1.0, dzlo[2] = {0.0, 0.0}, dzuo[2] = {0.0, 0.0}, dvlo[RM_NQ], dvuo[RM_NQ];
            double zl0[2], zu0[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) { zl0[j] = pn[P_ZL0 + j]; zu0[j] = pn[P_ZU0 + j]; }
            if (uon) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double ur = pn[P_UR + j];
                    dzlo[j] = (mu0 - zl0[j] * (u[j] - lo)) / (ur - lo);
                    dzuo[j] = (mu0 - zu0[j] * (hi - u[j])) / (hi - ur);
                    if (dzlo[j] < 0) a2 = fmin(a2, -tau0 * zl0[j] / dzlo[j]);
                    if (dzuo[j] < 0) a2 = fmin(a2, -tau0 * zu0[j] / dzuo[j]);
                }
            }
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) {
                const double s0 = q[Q_S0 + i], v0l = q[Q_VL0 + i], v0u = q[Q_VU0 + i];
                dvlo[i] = uon && tw[i] ? (mu0 - v0l * (s[i] - sL[i])) / (s0 - sL[i]) : 0.0;
                dvuo[i] = uon ? (mu0 - v0u * (sU[i] - s[i])) / (sU[i] - s0) : 0.0;
                if (dvlo[i] < 0) a2 = fmin(a2, -tau0 * v0l / dvlo[i]);
                if (dvuo[i] < 0) a2 = fmin(a2, -tau0 * v0u / dvuo[i]);
            }
            const double azo = wmin(a2);
            double zmx = 0.0;
            if (uon) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    zl[j] = fma(azo, dzlo[j], zl0[j]); zu[j] = fma(azo, dzuo[j], zu0[j]);
                    zmx = fmax(zmx, fmax(zl[j], zu[j]));
                }
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) {
                    vl[i] = tw[i] ? fma(azo, dvlo[i], q[Q_VL0 + i]) : 0.0;
                    vu[i] = fma(azo, dvuo[i], q[Q_VU0 + i]);
                    zmx = fmax(zmx, fmax(vl[i], vu[i]));
                }
            }
            const bool reset = wmax(zmx) > 1e3;
            if (uon) {
#pragma unroll
                for (int i = 0; i < RM_NQ; ++i) {
                    if (reset) { vl[i] = tw[i] ? 1.0 : 0.0; vu[i] = 1.0; }
                    const double nl = s[i] - sL[i], nu = sU[i] - s[i];
                    if (tw[i]) vl[i] = fmax(fmin(vl[i], 1e10 * mu0 / nl), mu0 / (1e10 * nl));
                    vu[i] = fmax(fmin(vu[i], 1e10 * mu0 / nu), mu0 / (1e10 * nu));
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (reset) { zl[j] = 1.0; zu[j] = 1.0; }
                    const double nl = u[j] - lo, nu = hi - u[j];
                    zl[j] = fmax(fmin(zl[j], 1e10 * mu0 / nl), mu0 / (1e10 * nl));
                    zu[j] = fmax(fmin(zu[j], 1e10 * mu0 / nu), mu0 / (1e10 * nu));
                }
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) lam[i] = 0.0;
#pragma unroll
            for (int i = 0; i < RM_NQ; ++i) yq[i] = 0.0;
        }
        in_soft = 0; soft_count = 0;
        it_next = rit;
        __syncthreads();
        STAMP(21);
    }
    }

    // ---------------- outputs -------------------------------------------------------------
    if (!RESTO && status == kRmNeedResto) {     // handed over: rmpc_solve<true> writes the outputs
        if (lane == 0 && wave_idx() == 0) a.status[b] = status;
        return true;
    }
    const double fval = wsum_rl(nod ? cost_val(x, u, up) : 0.0);
    if (lane == 0 && wave_idx() == 0) {
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
    STAMP_FLUSH32_TO(g_stamp_rm, b);
    return false;
}

// RESTO = false: every launch; RESTO = true: the handed-over instances, queued behind it on the same stream.
// (Unlike PMPC and LMPC, RMPC does not run the restoration in the solving wave for small batches: a
// non-inlined restoration call at the end of this kernel -- rmpc_resto_tail, round 5 -- costs it its last free
// registers (the call ABI's SGPRs spill into a VGPR), and the spilled main loop measured C3 -4.7 % against
// +1.7 % for the saved dispatch; profiles/r05/fuse_ab.txt)
template <bool RESTO>
__global__ __launch_bounds__(kWave * kWaves) void rmpc_ipm_kernel(RmpcArgs a) {
    if (blockIdx.x % a.pack) return;          // small batches packed onto one XCD (launcher)
    const int b = blockIdx.x / a.pack;
    if constexpr (RESTO) {
        if (a.status[b] != kRmNeedResto) return;     // wave-uniform: solved by rmpc_ipm_kernel<false>
    }
    (void)rmpc_solve<RESTO>(a, b);
}

#if DART_WG == 1
// Standalone batched RLS.update (np_mpc...:17-27): one p = 7 filter per workgroup, lanes as entries.
__global__ __launch_bounds__(kWave) void rls_update_kernel(int B, double* theta, double* P, const double* phi,
                                                          const double* y, double lam) {
    __shared__ double Pphi[7], phiP[7], ph[7], th[7];
    const int b = blockIdx.x, l = lane_id();
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
#endif

}  // namespace dartmpc

#if DART_WG == 2
// N = 32..63 (dartmpc_launch_rmpc forwards here): one instance per two-wave workgroup
extern "C" size_t dartmpc_rmpc_wg2_resto_bytes() { return sizeof(dartmpc::RmResto); }
extern "C" hipError_t dartmpc_launch_rmpc_wg2(const void* args, hipStream_t stream) {
    dartmpc::RmpcArgs a = *static_cast<const dartmpc::RmpcArgs*>(args);
    if (a.N < (dartmpc::force_wg2() ? 1 : 32) || a.N >= dartmpc::RM_NMAXS) return hipErrorInvalidValue;
    if (a.resto && !a.resto_buf) return hipErrorInvalidValue;
    a.pack = 1;
    const dim3 block(dartmpc::kWave * dartmpc::kWaves);
    hipLaunchKernelGGL(dartmpc::rmpc_ipm_kernel<false>, dim3(a.B), block, 0, stream, a);
    if (a.resto) {
        if (hipError_t e = hipGetLastError()) return e;
        hipLaunchKernelGGL(dartmpc::rmpc_ipm_kernel<true>, dim3(a.B), block, 0, stream, a);
    }
    return hipGetLastError();
}
#else

extern "C" hipError_t dartmpc_launch_rls(int B, double* theta, double* P, const double* phi, const double* y,
                                         double lam, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(dartmpc::rls_update_kernel, dim3(B), dim3(dartmpc::kWave), 0, stream, B, theta, P, phi, y, lam);
    return hipGetLastError();
}

// internal (bench.py's saturated lines): instances of rmpc_ipm_kernel<false> resident per CU, by the runtime's own
// occupancy calculation (registers, LDS, waves); -1 on error
extern "C" int dartmpc_rmpc_blocks_per_cu(void) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dartmpc::rmpc_ipm_kernel<false>, dartmpc::kWave, 0) != hipSuccess)
        return -1;
    return n;
}

extern "C" hipError_t dartmpc_launch_rmpc(const dartmpc::RmpcArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    if ((args->N >= dartmpc::RM_NMAXS || dartmpc::force_wg2()) && args->N < 2 * dartmpc::RM_NMAXS)
        return dartmpc_launch_rmpc_wg2(args, stream);
    if (args->N < 1 || args->N >= dartmpc::RM_NMAXS) return hipErrorInvalidValue;
    dartmpc::RmpcArgs a = *args;
    a.pack = (a.B <= 32) ? 8 : 1;            // blocks go round-robin over the 8 XCDs: one XCD, one L2 for the code
    hipLaunchKernelGGL(dartmpc::rmpc_ipm_kernel<false>, dim3(a.B * a.pack), dim3(dartmpc::kWave), 0, stream, a);
    if (a.resto) {      // the instances whose line search failed, with IPOPT's restoration phases
        if (hipError_t e = hipGetLastError()) return e;
        // one block per instance (not B x pack; the blocks of the instances that were not handed over return at
        // once): 4.39 -> 4.40 us per launch, the dispatch itself.  Inlining the restoration behind the solve instead
        // costs C3 10.5 % (profiles/r05/rmpc_inline_ab.txt), a non-inlined call 4.7 % (fuse_ab.txt).
        dartmpc::RmpcArgs r = a;
        r.pack = 1;
        hipLaunchKernelGGL(dartmpc::rmpc_ipm_kernel<true>, dim3(r.B), dim3(dartmpc::kWave), 0, stream, r);
    }
    return hipGetLastError();
}

#ifdef DART_STAMPS
extern "C" hipError_t dartmpc_read_stamps_rmpc(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_rm), sizeof(unsigned long long) * 32, 0,
                               hipMemcpyDeviceToHost);
}
#endif
#endif  // DART_WG
