// pmpc_resto.h -- IPOPT's soft restoration and restoration phases of the PMPC solve, gfx950.
//
// pmpc_ipm.hip's register kernel solves every instance; one whose filter line search fails (where IPOPT
// enters its restoration phases: at N = 31 a few of C4's instances, with max_soc = 0 about one in ten) is
// handed over to pmpc_resto_solve below, which solves it again from its start on the full 6-state NLP of
// mpc_3d.py:28-85, with IPOPT's soft restoration phase (BacktrackingLineSearch::TrySoftRestoStep) and
// restoration phase (MinC_1NrmRestorationPhase) available, to the end of the solve: oracle/pmpc_ipm.c
// `soft_resto_step`, `restoration`, whose commentary applies.  By default no state crosses the hand-off but the
// instance index (the restart repeats the oracle's arithmetic order from the first iteration).  Opt-in
// (DART_PMPC_RESUME=1): the register kernel also hands over the iterate of the iteration whose line search
// failed -- per node x, u, lambda, z_L, z_U, then its filter, mu, the last inertia shift, the iteration and filter
// counters (pmpc_model.h kPmHo layout, PmpcArgs::resto_buf) -- and the solve repeats that iteration at the same
// shift instead of starting over (faster, but not the oracle's path on every restored instance).
// Two callers:
//  * small batches (B <= 32, the latency regime): the register kernel's own wave calls it right after the
//    failed line search (pmpc_ipm.hip `pmpc_resto_tail`, a non-inlined call, so the register kernel's
//    allocation is untouched): no second dispatch on any launch;
//  * larger batches: pmpc_resto_kernel (pmpc_resto.hip), queued behind the register kernel on the same stream
//    (status kPmNeedResto marks the handed-over instances; the others return at once), or launched by the
//    host entries only when their completion words show a handed-over instance.
//
// Why a second kernel: in the restoration problem the z sub-state carries the proximity term and soft
// defect rows, so its multipliers no longer vanish and the two axes couple through the tilt columns of the z
// rows -- the register kernel's per-axis recursion does not hold there.  This kernel runs the one-wave LDS
// Riccati engine of ocp_wave.h on the whole stage instead (x~ = the six states, every M column non-zero:
// gen_node_step; every defect row soft in the restoration phase: aug_soften with NS = 6).  It runs only for
// the handed-over instances, so it is written for clarity: exact double reductions, library sin / cos / log.
//
// Mapping: one wave64 per instance; lane k and its mirror k + 32 own shooting node k (N <= 31) and run the
// node's arithmetic alike (the same bits); the node lane writes LDS, and sums over the wave count node lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "ocp_wave.h"
#include "pmpc_ipm.h"
#include "pmpc_model.h"
#include "stamps.h"
#include "wave.h"

namespace dartmpc {

constexpr int PR_NMAXS = 32;                 // max shooting nodes (N <= 31)
using PrLds = OcpLds<6, PR_NMAXS>;
using PrSoft = AugSoftLds<PrLds, 6>;         // restoration: every defect row soft

// restoration-phase state of node k's incoming rows (written by the node lane): p, n, z_p, z_n, rp, rn,
// Sigma_p', Sigma_n'; x_R, D_R of the states; u_R, D_R of the tilts; the original u-bound multipliers
enum { R_PC = 0, R_NC = 6, R_ZP = 12, R_ZN = 18, R_RP = 24, R_RN = 30, R_SP = 36, R_SN = 42, R_XR = 48, R_DRX = 54,
       R_UR = 60, R_DRU = 62, R_ZL0 = 64, R_ZU0 = 66, R_N = 68 };
// a parked step (second-order correction, iterative refinement), one row per lane
enum { V_DX = 0, V_LP = 6, V_DU = 12, V_DPC = 14, V_DNC = 20, V_N = 26 };

struct PrShared {
    PrLds ocp;
    PrSoft soft;
    NodeArr<double[R_N], PR_NMAXS + 1> PN;
    NodeArr<double[V_N], kWave> SV, SV2;
    alignas(16) double U[PrLds::ND * PrLds::NC];     // gen_node_step's products
};

// closed-loop rows of node k mapped through node k+1's soft rows: [Phi | f](r) <- Y(r, :) [[Phi | f]; 0 1]
struct PrSoftPost {
    PrLds* S;
    const PrSoft* R;
    __device__ void operator()(int k) const {
        const double* Y = R->T[k + 1];
        double F[6][7];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int j = 0; j < 7; ++j) F[r][j] = S->F[k][r][j];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                double t = j == 6 ? Y[7 * r + 6] : 0.0;
#pragma unroll
                for (int c = 0; c < 6; ++c) t = fma(Y[7 * r + c], F[c][j], t);
                S->F[k][r][j] = t;
            }
    }
};

// filter of (theta, phi) pairs, entry q in slot q >> 6 of lane q & 63 (IPOPT's filter; <= 256 entries)
struct PrFilter {
    double th[4], ph[4];
    int n;
    __device__ __forceinline__ void reset() {
        n = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) { th[r] = 0.0; ph[r] = 0.0; }
    }
    __device__ __forceinline__ bool hit(double t, double p) const {
        bool h = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) h = h || (lane_id() + 64 * r < n && t >= th[r] && p >= ph[r]);
        return wany(h);
    }
    __device__ __forceinline__ void add(double t, double p) {
        if (n >= 256) return;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (lane_id() + 64 * r == n) { th[r] = t; ph[r] = p; }
        ++n;
    }
};

// Transcendental pairs: a node's lanes k and k + 32 hold the same operands, so lanes 0-31 evaluate the first
// of a pair and lanes 32-63 the second, and v_permlane32_swap hands each half the other's result (half_pair):
// the same function on the same operand -- the same bits -- at half the evaluations per lane.  EXEC full.
__device__ __forceinline__ bool pr_low_half() { return lane_id() < 32; }

#ifdef DART_STAMPS
// diagnostic build: per-phase s_memtime cycles of the last handed-over instance (tools/stamps_pmpc_resto.py)
__device__ unsigned long long g_stamp_pr[32];
#endif

// the solve of handed-over instance b by the calling wave (its LDS: the caller's kernel gets PrShared)
__device__ __forceinline__ void pmpc_resto_solve(const PmpcArgs& a, const int b) {
    __shared__ PrShared SH;
    STAMP_DECL
    PrLds* S = &SH.ocp;
    PrSoft* SR = &SH.soft;
    constexpr int NC = PrLds::NC;
    const int lane = lane_id();
    const int k = lane & 31;
    const bool nod = lane < 32;
    const int N = a.N;
    const bool xon = k <= N, uon = k < N;
    const bool wx = nod && xon, wu = nod && uon;      // node lanes: they count in sums and write LDS
    const double h = a.Ts, gz = a.g;
    const double* st = a.x0 + 6 * b;
    const double* rf = a.ref + 6 * b;
    const double* pr = a.prm + 6 * b;
    const double mu_f = pr[0], Qp = pr[1], Qv = pr[2], R = pr[3], ulo = pr[4], uhi = pr[5];
    // the RK4 maps of the axis and z models (as pmpc_ipm.hip): px+ = px + a12 vx + b1 sin(theta_x),
    // vx+ = a22 vx + b2 sin(theta_x) (y alike); pz+ = zp1 pz + zcp w, vz+ = zav vz + zcv w, w = -g |theta|^2
    double a12, a22, b1, b2, zp1, zav, zcp, zcv;
    axis_rk4(h, gz, mu_f, 0.0, 0.0, 1.0, a12, a22);
    axis_rk4(h, gz, mu_f, 1.0, 0.0, 0.0, b1, b2);
    z_rk4(h, 0.0, 1.0, 1.0, zp1, zav);
    z_rk4(h, 1.0, 0.0, 0.0, zcp, zcv);
    const double lo = ulo - 1e-8 * fmax(1.0, fabs(ulo)), hi = uhi + 1e-8 * fmax(1.0, fabs(uhi));
    const int nw = 6 * (N + 1) + 2 * N;
    const double* ww = a.w_warm ? a.w_warm + (size_t)nw * b : nullptr;

    // ---------------- starting point (oracle_pmpc_solve; pmpc_ipm.hip) ------------------------------
    double x[6], u[2], lam[6], zl[2], zu[2];
#pragma unroll
    for (int i = 0; i < 6; ++i) { x[i] = xon ? (ww ? ww[6 * k + i] : st[i]) : 0.0; lam[i] = 0.0; }
    {
        const double pl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo)), pu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            double t = uon && ww ? ww[6 * (N + 1) + 2 * k + j] : 0.0;
            if (t < lo + pl) t = lo + pl;
            if (t > hi - pu) t = hi - pu;
            u[j] = uon ? t : 0.0;
            zl[j] = uon ? 1.0 : 0.0; zu[j] = uon ? 1.0 : 0.0;
        }
    }
    double gmax = 0.0;
    if (wx) {
        gmax = fmax(fmax(fabs(2 * Qp * (x[0] - rf[0])), fabs(2 * Qv * (x[1] - rf[1]))),
                    fmax(fabs(2 * Qp * (x[2] - rf[2])), fabs(2 * Qv * (x[3] - rf[3]))));
        if (uon) gmax = fmax(gmax, fmax(fabs(2 * R * u[0]), fabs(2 * R * u[1])));
    }
    gmax = wmax(gmax);
    const double sc = gmax > 100.0 ? 100.0 / gmax : 1.0;          // nlp_scaling_max_gradient = 100
    const double tol = a.tol, mu_min = tol / 10;
    const double ng = 6.0 * (N + 1), nU = 2.0 * N;
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, eta_ph = 1e-8, gam_al = 0.05, kap_soc = 0.99;

    // ---------------- model and NLP pieces of node k -------------------------------------------------
    auto fwd = [&](const double* xx, const double* uu, double* xn) {          // f(x_k, u_k), mpc_3d.py:87-104
        double sx, sy;
        half_pair(sin(pr_low_half() ? uu[0] : uu[1]), sx, sy);
        const double w = -gz * (uu[0] * uu[0] + uu[1] * uu[1]);
        xn[0] = fma(a12, xx[1], fma(b1, sx, xx[0])); xn[1] = fma(a22, xx[1], b2 * sx);
        xn[2] = fma(a12, xx[3], fma(b1, sy, xx[2])); xn[3] = fma(a22, xx[3], b2 * sy);
        xn[4] = fma(zp1, xx[4], zcp * w); xn[5] = fma(zav, xx[5], zcv * w);
    };
    // incoming defect rows g_k = x_k - f(x_{k-1}, u_{k-1}) (:48), g_0 = x_0 - state (:37)
    auto defects = [&](const double* xx, const double* uu, double* g) {
        double xn[6];
        fwd(xx, uu, xn);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double t = from_prev(xn[i]);
            g[i] = k == 0 ? xx[i] - st[i] : xx[i] - t;
        }
    };
    auto next_of = [&](const double* v, double* vn) {       // node k+1's values (0 past the horizon)
#pragma unroll
        for (int i = 0; i < 6; ++i) { const double t = from_next(v[i]); vn[i] = uon ? t : 0.0; }
    };
    // J^T ln of node k at controls uu: A^T ln (ja[0..5]) and B^T ln (ja[6..7]), and the curvature
    // ln^T d2 f / d theta_a^2 of the tilt diagonal (hu) -- d2 of -ln^T f, the lambda-weighted dynamics Hessian
    auto jac_t = [&](const double* uu, const double* ln, double* ja, double* hu) {
        double sx, cx, sy, cy, sh, ch;
        sincos(pr_low_half() ? uu[0] : uu[1], &sh, &ch);
        half_pair(sh, sx, sy);
        half_pair(ch, cx, cy);
        const double lz = fma(zcp, ln[4], zcv * ln[5]);
        const double lx = fma(b1, ln[0], b2 * ln[1]), ly = fma(b1, ln[2], b2 * ln[3]);
        ja[0] = ln[0]; ja[1] = fma(a12, ln[0], a22 * ln[1]);
        ja[2] = ln[2]; ja[3] = fma(a12, ln[2], a22 * ln[3]);
        ja[4] = zp1 * ln[4]; ja[5] = zav * ln[5];
        ja[6] = fma(cx, lx, -2.0 * gz * uu[0] * lz);
        ja[7] = fma(cy, ly, -2.0 * gz * uu[1] * lz);
        hu[0] = fma(sx, lx, 2.0 * gz * lz);
        hu[1] = fma(sy, ly, 2.0 * gz * lz);
    };
    auto cost_grad = [&](const double* xx, double* gx) {                  // scaled, mpc_3d.py:44-46, :63-66
        gx[0] = sc * (2 * Qp * (xx[0] - rf[0])); gx[1] = sc * (2 * Qv * (xx[1] - rf[1]));
        gx[2] = sc * (2 * Qp * (xx[2] - rf[2])); gx[3] = sc * (2 * Qv * (xx[3] - rf[3]));
        gx[4] = 0.0; gx[5] = 0.0;
    };
    auto node_cost = [&](const double* xx, const double* uu) {            // unscaled
        const double ep = (xx[0] - rf[0]) * (xx[0] - rf[0]) + (xx[2] - rf[2]) * (xx[2] - rf[2]);
        const double ev = (xx[1] - rf[1]) * (xx[1] - rf[1]) + (xx[3] - rf[3]) * (xx[3] - rf[3]);
        double f = Qp * ep + Qv * ev;
        if (uon) f += R * (uu[0] * uu[0] + uu[1] * uu[1]);
        return wx ? f : 0.0;
    };
    auto l1 = [&](const double* g) {
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) t += fabs(g[i]);
        return wx ? t : 0.0;
    };
    // barrier objective of the original problem at barrier parameter m (+inf outside the box)
    auto barrier = [&](const double* xx, const double* uu, double m) {
        double lb = 0.0;
        bool out = false;
        double lsl[2], lsu[2];
        {
            const double uh = pr_low_half() ? uu[0] : uu[1];
            half_pair(log(uh - lo), lsl[0], lsl[1]);
            half_pair(log(hi - uh), lsu[0], lsu[1]);
        }
        if (wu) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double sl = uu[j] - lo, su = hi - uu[j];
                out = out || !(sl > 0) || !(su > 0);
                lb += lsl[j] + lsu[j];
            }
        }
        if (wany(out)) return (double)INFINITY;
        double nc = node_cost(xx, uu);
        wsum2(nc, lb);            // (the same bits as two wsum: the same reduction tree, in lock step)
        return sc * nc - m * lb;
    };

    // constant structure of M_k: zeroed once, then only the tilt and defect columns are written
    double* const Mk = &S->M[uon ? k : 0][0][0];
    double* const Hk = S->H[uon ? k : 0];
    if (wu) {
        for (int e = 0; e < PrLds::ND * NC; ++e) Mk[e] = 0.0;
        for (int e = 0; e < PrLds::NTP; ++e) Hk[e] = 0.0;
        Mk[0 * NC + 0] = 1.0;
        Mk[1 * NC + 0] = a12; Mk[1 * NC + 1] = a22;
        Mk[2 * NC + 2] = 1.0;
        Mk[3 * NC + 2] = a12; Mk[3 * NC + 3] = a22;
        Mk[4 * NC + 4] = zp1; Mk[5 * NC + 5] = zav;
        Mk[8 * NC + 6] = 1.0;                                     // homogeneous coordinate
    }
    // the tilt columns of M_k at controls uu
    auto write_tilt_cols = [&](const double* uu) {
        double cx, cy;
        half_pair(cos(pr_low_half() ? uu[0] : uu[1]), cx, cy);
        if (wu) {
            Mk[6 * NC + 0] = b1 * cx; Mk[6 * NC + 1] = b2 * cx;
            Mk[6 * NC + 4] = zcp * (-2.0 * gz * uu[0]); Mk[6 * NC + 5] = zcv * (-2.0 * gz * uu[0]);
            Mk[7 * NC + 2] = b1 * cy; Mk[7 * NC + 3] = b2 * cy;
            Mk[7 * NC + 4] = zcp * (-2.0 * gz * uu[1]); Mk[7 * NC + 5] = zcv * (-2.0 * gz * uu[1]);
        }
    };
    // stage Hessian diagonals hx (states), hu (tilts) and gradient gq of node k into H_k; node N's into the
    // terminal surrogate G_N (value function [[diag hx, gq], [gq^T, 0]], Quu = I)
    auto write_stage = [&](const double* hx, const double* hu, const double* gq) {
        if (wu) {
#pragma unroll
            for (int i = 0; i < 6; ++i) Hk[hp(i, i)] = hx[i];
            Hk[hp(6, 6)] = hu[0]; Hk[hp(7, 7)] = hu[1];
#pragma unroll
            for (int j = 0; j < 8; ++j) Hk[hp(8, j)] = gq[j];
        }
        if (nod && k == N) {
            double* GN = S->G[N];
            for (int e = 0; e < PrLds::NTP; ++e) GN[e] = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) { GN[hp(i, i)] = hx[i]; GN[hp(8, i)] = gq[i]; }
            GN[hp(6, 6)] = 1.0; GN[hp(7, 7)] = 1.0;
        }
    };
    // right-hand side rg of node k's incoming rows (J d = -rg: dx~_{k+1} = A dx~ + B du - rg_{k+1}, dx~_0 = -rg_0)
    auto write_rhs = [&](const double* rg) {
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            const double t = from_next(rg[r]);
            if (wu) Mk[8 * NC + r] = -t;
            if (nod && k == 0) S->dx0[r] = -rg[r];
        }
    };
    // the step from a factorised system: forward sweep, du = [K | k] [dx~; 1], lambda+ = -(P dx~ + p)
    auto finish_step = [&](double* dx, double* dU, double* lp) {
        forward_sweep(S, N, k, dx);
        const double* K0 = S->KK[uon ? k : 0][0];
        const double* K1 = S->KK[uon ? k : 0][1];
        double d0 = K0[6], d1 = K1[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) { d0 = fma(K0[j], dx[j], d0); d1 = fma(K1[j], dx[j], d1); }
        dU[0] = uon ? d0 : 0.0; dU[1] = uon ? d1 : 0.0;
        node_multiplier(S, xon ? k : 0, dx, dU, lp);
#pragma unroll
        for (int i = 0; i < 6; ++i) { lp[i] = xon ? lp[i] : 0.0; dx[i] = xon ? dx[i] : 0.0; }
    };
    auto solve_plain = [&](double* dx, double* dU, double* lp) {
        closed_loop(S, N);
        finish_step(dx, dU, lp);
    };
    // with soft rows: dx~_0 and every closed-loop row seen through the next node's soft rows
    auto solve_soft = [&](double* dx, double* dU, double* lp) {
        if (nod && k == 0) {
            double d0[6];
#pragma unroll
            for (int r = 0; r < 6; ++r) d0[r] = S->dx0[r];
            const double* Y0 = SR->T[0];
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                double t = Y0[7 * r + 6];
#pragma unroll
                for (int c = 0; c < 6; ++c) t = fma(Y0[7 * r + c], d0[c], t);
                S->dx0[r] = t;
            }
        }
        __syncthreads();
        closed_loop(S, N, PrSoftPost{S, SR});
        finish_step(dx, dU, lp);
    };

    // ---------------- the original problem ------------------------------------------------------------
    double g[6];
    defects(x, u, g);
    double theta = wsum(l1(g));
    const double th_max = 1e4 * fmax(1.0, theta), th_min = 1e-4 * fmax(1.0, theta);
    PrFilter F0;
    F0.reset();
    double mu = 0.1, delta_last = 0.0;
    int status = -1, it = 0, in_soft = 0, soft_count = 0;
    bool go_resto = false;
    double phi_rs = 0.0, tau_rs = 0.99;
    int it_next = a.mult_init_max > 0.0 ? -1 : 0;
    const double zero6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    // Resume (a.resto_buf): the register kernel's iterate of the iteration whose line search failed
    // (pmpc_model.h kPmHo), its filter, mu, last inertia shift and iteration counter.  That iteration is repeated
    // here -- the same point, hence the same Newton system, factored at the shift the register kernel used (0, or
    // its updated last shift: resume_first) -- and the restoration phases follow; the scaling sc and the filter's
    // theta bounds above belong to the starting point, as in the register kernel.
    bool resume_first = false;
    if (a.resto_buf) {
        const double* ho = a.resto_buf + (size_t)kPmHo * b;
        const double* row = ho + kPmHoRow * k;
#pragma unroll
        for (int i = 0; i < 6; ++i) { x[i] = xon ? row[i] : 0.0; lam[i] = xon ? row[8 + i] : 0.0; }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            u[j] = uon ? row[6 + j] : 0.0;
            zl[j] = uon ? row[14 + j] : 0.0; zu[j] = uon ? row[16 + j] : 0.0;
        }
        mu = ho[kPmHoScal]; delta_last = ho[kPmHoScal + 1];
        it_next = (int)ho[kPmHoScal + 2];
        const int nf = (int)ho[kPmHoScal + 3];
        F0.th[0] = lane < nf ? ho[kPmHoFilt + 2 * lane] : 0.0;
        F0.ph[0] = lane < nf ? ho[kPmHoFilt + 2 * lane + 1] : 0.0;
        F0.n = nf;
        resume_first = true;
    }
    __syncthreads();
    STAMP(0);

    for (;;) {
    for (it = it_next; it < a.max_iter; ++it) {
        const bool lsm = it < 0;      // IPOPT's least-square starting multipliers (constr_mult_init_max)
        STAMP_ADD(16, 1);
        SPAN_BEGIN(sp_e0);
        defects(x, u, g);             // (the accepted trial's: the same bits)
        theta = wsum(l1(g));
        SPAN_END(28, sp_e0);
        SPAN_BEGIN(sp_e1);
        double ln[6], ja[8], hdu[2], gx[6];
        next_of(lam, ln);
        jac_t(u, ln, ja, hdu);
        cost_grad(x, gx);
        SPAN_END(29, sp_e1);
        SPAN_BEGIN(sp_e2);
        // ---- optimality error, IPOPT eq. (5) ----
        double dinf = 0.0, pinf = 0.0, c0 = 0.0, cmin = 1e300, suml = 0.0, sumz = 0.0;
        if (wx) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                dinf = fmax(dinf, fabs(gx[i] + lam[i] - ja[i]));
                pinf = fmax(pinf, fabs(g[i]));
                suml += fabs(lam[i]);
            }
        }
        if (wu) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double sl = u[j] - lo, su = hi - u[j];
                dinf = fmax(dinf, fabs(sc * 2 * R * u[j] - zl[j] + zu[j] - ja[6 + j]));
                const double cl = zl[j] * sl, cu = zu[j] * su;
                c0 = fmax(c0, fmax(cl, cu)); cmin = fmin(cmin, fmin(cl, cu));
                sumz += zl[j] + zu[j];
            }
        }
        wred_errors_f64(dinf, pinf, c0, cmin, suml, sumz);
        SPAN_END(30, sp_e2);
        SPAN_BEGIN(sp_e3);
        const double s_d = fmax(100.0, (suml + sumz) / (ng + 2 * nU)) / 100.0;
        const double s_c = fmax(100.0, sumz / (2 * nU)) / 100.0;
        if (!lsm && fmax(dinf / s_d, fmax(pinf, c0 / s_c)) <= tol) { status = 0; break; }
        for (; !lsm;) {
            const double cmu = fmax(c0 - mu, mu - cmin);
            if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * mu || mu <= mu_min) break;
            mu = fmax(mu_min, fmin(0.2 * mu, pow(mu, 1.5)));
            F0.reset(); in_soft = 0;      // BacktrackingLineSearch::Reset: the filter and the soft phase
        }
        const double tau = fmax(0.99, 1.0 - mu);
        SPAN_END(31, sp_e3);
        STAMP(1);
        write_tilt_cols(u);
        // stage QP at inertia shift d (least squares: unit weights, the box gradient -z_L + z_U, no defects)
        auto assemble = [&](double d) {
            double hx[6], hu[2], gq[8];
            const double wq[6] = {sc * 2 * Qp, sc * 2 * Qv, sc * 2 * Qp, sc * 2 * Qv, 0.0, 0.0};
#pragma unroll
            for (int i = 0; i < 6; ++i) { hx[i] = lsm ? 1.0 : wq[i] + d; gq[i] = gx[i]; }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double sl = u[j] - lo, su = hi - u[j];
                hu[j] = lsm ? 1.0 : hdu[j] + (sc * 2 * R + zl[j] / sl + zu[j] / su + d);
                gq[6 + j] = lsm ? sc * 2 * R * u[j] - zl[j] + zu[j] : sc * 2 * R * u[j] - mu / sl + mu / su;
            }
            write_stage(hx, hu, gq);
        };
        assemble(0.0);
        write_rhs(lsm ? zero6 : g);
        __syncthreads();
        double dx[6], dU[2], lp[6];
        if (lsm) {
            (void)riccati_sweep_gen(S, N, SH.U);       // unit weights: positive definite
            solve_plain(dx, dU, lp);
            double ym = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) ym = fmax(ym, wx ? fabs(lp[i]) : 0.0);
            ym = wmax(ym);
            if (ym <= a.mult_init_max) {
#pragma unroll
                for (int i = 0; i < 6; ++i) lam[i] = xon ? lp[i] : 0.0;
            }
            continue;
        }
        // ---- Newton step: Riccati with inertia correction ----
        double delta = 0.0;
        SPAN_BEGIN(sp_ric);
        bool ok = riccati_sweep_gen(S, N, SH.U);
        SPAN_END(21, sp_ric);
        STAMP_ADD(22, 1);
        for (int attempt = 0; !ok && attempt < 60; ++attempt) {
            // (the resumed iteration: the register kernel's shift, which its update left in delta_last)
            delta = (attempt == 0) ? (resume_first && delta_last > 0.0 ? delta_last
                                      : delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))
                                   : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            assemble(delta);
            __syncthreads();
            ok = riccati_sweep_gen(S, N, SH.U);
        }
        resume_first = false;
        if (!ok) { status = -3; break; }
        if (delta > 0.0) delta_last = delta;
        STAMP(2);
        solve_plain(dx, dU, lp);
        // bound-multiplier steps and the fractions to the boundary
        double dzl[2], dzu[2], amax = 1.0, az = 1.0;
        auto duals = [&]() {
            double am = 1.0, a2 = 1.0;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double sl = u[j] - lo, su = hi - u[j];
                dzl[j] = wu ? mu / sl - zl[j] - zl[j] / sl * dU[j] : 0.0;
                dzu[j] = wu ? mu / su - zu[j] + zu[j] / su * dU[j] : 0.0;
                if (wu) {
                    if (dU[j] < 0) am = fmin(am, -tau * sl / dU[j]);
                    if (dU[j] > 0) am = fmin(am, tau * su / dU[j]);
                    if (dzl[j] < 0) a2 = fmin(a2, -tau * zl[j] / dzl[j]);
                    if (dzu[j] < 0) a2 = fmin(a2, -tau * zu[j] / dzu[j]);
                }
            }
            wmin2d(am, a2);
            amax = am; az = a2;
        };
        duals();
        STAMP(3);
        const double amax0 = amax, az0 = az;
        SPAN_BEGIN(sp_lsp);
        // ---- filter line search with second-order correction (W&B 2006, Alg. A) ----
        const double phi = barrier(x, u, mu);
        double gtd = 0.0;
        if (wx) {
#pragma unroll
            for (int i = 0; i < 6; ++i) gtd += gx[i] * dx[i];
        }
        if (wu) {
#pragma unroll
            for (int j = 0; j < 2; ++j) gtd += (sc * 2 * R * u[j] - mu / (u[j] - lo) + mu / (hi - u[j])) * dU[j];
        }
        const double gTd = wsum(gtd);
        // theta^s_th and (-gTd)^s_ph are fixed through the line search: formed once here, not at every trial
        double pw_th = 0.0, pw_gd = 0.0;
        if (gTd < 0) half_pair(pr_low_half() ? pow(theta, s_th) : pow(-gTd, s_ph), pw_th, pw_gd);
        double amin = gam_th;
        if (gTd < 0) amin = fmin(gam_th, fmin(gam_ph * theta / (-gTd), pw_th / pw_gd));
        if (theta == 0.0 && gTd < 0) amin = 0.0;
        amin *= gam_al;
        double tn = 0.0;
        if (wx) {
#pragma unroll
            for (int i = 0; i < 6; ++i) tn = fmax(tn, fabs(dx[i]) / (1.0 + fabs(x[i])));
        }
        if (wu) tn = fmax(tn, fmax(fabs(dU[0]) / (1.0 + fabs(u[0])), fabs(dU[1]) / (1.0 + fabs(u[1]))));
        const bool tiny = wmax(tn) < 10.0 * 2.220446049250313e-16;
        double xt[6], ut[2], gt[6], th_t = 0.0, ph_t = 0.0;
        auto trial = [&](double al) {
            SPAN_BEGIN(sp_tr);
#pragma unroll
            for (int i = 0; i < 6; ++i) xt[i] = xon ? fma(al, dx[i], x[i]) : x[i];
#pragma unroll
            for (int j = 0; j < 2; ++j) ut[j] = uon ? fma(al, dU[j], u[j]) : u[j];
            defects(xt, ut, gt);
            SPAN_END(23, sp_tr);
            SPAN_BEGIN(sp_ph);
            // theta and the barrier objective's two sums in one lock-step reduction (barrier(): the same bits)
            double thl = l1(gt), lb = 0.0;
            bool out = false;
            double lsl[2], lsu[2];
            {
                const double uh = pr_low_half() ? ut[0] : ut[1];
                half_pair(log(uh - lo), lsl[0], lsl[1]);
                half_pair(log(hi - uh), lsu[0], lsu[1]);
            }
            if (wu) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double sl = ut[j] - lo, su = hi - ut[j];
                    out = out || !(sl > 0) || !(su > 0);
                    lb += lsl[j] + lsu[j];
                }
            }
            double nc = node_cost(xt, ut);
            wsum3(thl, nc, lb);
            th_t = thl;
            ph_t = wany(out) ? (double)INFINITY : sc * nc - mu * lb;
            SPAN_END(24, sp_ph);
        };
        bool ftype = false;
        // FilterLSAcceptor::CheckAcceptabilityOfTrialPoint with alpha_primal_test = al
        auto accept = [&](double al) -> bool {
            if (!(th_t < th_max) || !isfinite(ph_t)) return false;
            if (F0.hit(th_t, ph_t)) return false;
            const bool sw = gTd < 0 && al * pw_gd > pw_th;
            if (theta <= th_min && sw) {
                if (cmp_le(ph_t, phi + eta_ph * al * gTd, phi)) { ftype = true; return true; }
                return false;
            }
            return cmp_le(th_t, (1 - gam_th) * theta, theta) || cmp_le(ph_t - phi, -gam_ph * theta, phi);
        };
        SPAN_END(15, sp_lsp);
        double alpha = amax;
        bool accepted = false;
        for (int ls = 0; ls < 80 && !accepted && !in_soft; ++ls) {
            if (alpha < amin && ls > 0) break;
            trial(alpha);
            STAMP_ADD(17, 1);
            if (tiny) { accepted = true; ftype = true; break; }
            SPAN_BEGIN(sp_acc);
            accepted = accept(alpha);
            SPAN_END(27, sp_acc);
            if (!accepted && ls == 0 && !(th_t < theta) && a.max_soc > 0) {
                // FilterLSAcceptor::TrySecondOrderCorrection on the plain step's factorisation
                double sdx[6], sdU[2], slp[6], cs[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) { sdx[i] = dx[i]; slp[i] = lp[i]; cs[i] = g[i]; }
                sdU[0] = dU[0]; sdU[1] = dU[1];
                double asoc = alpha, th_old = 0.0;
                for (int c = 0; c < a.max_soc; ++c) {
                    if (c > 0 && !(th_t <= kap_soc * th_old)) break;
                    th_old = th_t;
#pragma unroll
                    for (int i = 0; i < 6; ++i) cs[i] = fma(asoc, cs[i], gt[i]);
                    SPAN_BEGIN(sp_soc);
                    write_rhs(cs);
                    __syncthreads();
                    (void)riccati_sweep_gen(S, N, SH.U);
                    solve_plain(dx, dU, lp);
                    SPAN_END(25, sp_soc);
                    STAMP_ADD(26, 1);
                    double am = 1.0;
                    if (wu) {
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if (dU[j] < 0) am = fmin(am, -tau * (u[j] - lo) / dU[j]);
                            if (dU[j] > 0) am = fmin(am, tau * (hi - u[j]) / dU[j]);
                        }
                    }
                    asoc = wmin(am);
                    trial(asoc);
                    if (accept(alpha)) {      // the corrected step is the whole step, multiplier steps included
                        accepted = true; alpha = asoc;
                        duals();
                        amax = asoc;
                        break;
                    }
                }
                if (!accepted) {
#pragma unroll
                    for (int i = 0; i < 6; ++i) { dx[i] = sdx[i]; lp[i] = slp[i]; }
                    dU[0] = sdU[0]; dU[1] = sdU[1];
                }
            }
            if (!accepted) alpha *= 0.5;
        }
#ifdef DART_RESTO_TRACE
        if (blockIdx.x == 0 && lane == 0)
            printf("it %3d mu %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e az %.3e th %.2e\n", it, mu,
                   dinf / s_d, pinf, c0 / s_c, delta, amax0, alpha, az, theta);
#endif
        STAMP(4);
        bool soft = false;
        if (!accepted) {
            // ---- IPOPT's soft restoration phase (at most 10 steps; the current point enters the filter) ----
            if (!in_soft) {
                F0.add((1 - gam_th) * theta, phi - gam_ph * theta);
                soft_count = 0;
            }
            if (!(in_soft && ++soft_count > 10)) {
                // the plain step's multiplier steps and fractions to the boundary
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double sl = u[j] - lo, su = hi - u[j];
                    dzl[j] = wu ? mu / sl - zl[j] - zl[j] / sl * dU[j] : 0.0;
                    dzu[j] = wu ? mu / su - zu[j] + zu[j] / su * dU[j] : 0.0;
                }
                const double as = fmin(amax0, az0);
                trial(as);
                bool orig = th_t < th_max && isfinite(ph_t) && !F0.hit(th_t, ph_t);
                orig = orig && (cmp_le(th_t, (1 - gam_th) * theta, theta) || cmp_le(ph_t - phi, -gam_ph * theta, phi));
                bool take = orig;
                if (!take && isfinite(ph_t)) {
                    // IPOPT's primal-dual system error at mu (l1 norms of the primal and dual infeasibilities and
                    // of z s - mu, added) at the current point and at the trial point, every multiplier moved by as
                    auto pd_error = [&](const double* xx, const double* uu, const double* lm, const double* l_,
                                        const double* u_, const double* gg) {
                        double lnn[6], jaa[8], hh[2], gxx[6];
                        next_of(lm, lnn);
                        jac_t(uu, lnn, jaa, hh);
                        cost_grad(xx, gxx);
                        double t = 0.0;
                        if (wx) {
#pragma unroll
                            for (int i = 0; i < 6; ++i) t += fabs(gxx[i] + lm[i] - jaa[i]) + fabs(gg[i]);
                        }
                        if (wu) {
#pragma unroll
                            for (int j = 0; j < 2; ++j)
                                t += fabs(sc * 2 * R * uu[j] - l_[j] + u_[j] - jaa[6 + j]) +
                                     fabs(l_[j] * (uu[j] - lo) - mu) + fabs(u_[j] * (hi - uu[j]) - mu);
                        }
                        return wsum(t);
                    };
                    const double pd0 = pd_error(x, u, lam, zl, zu, g);
                    double lmt[6], zlt[2], zut[2];
#pragma unroll
                    for (int i = 0; i < 6; ++i) lmt[i] = xon ? fma(as, lp[i] - lam[i], lam[i]) : 0.0;
#pragma unroll
                    for (int j = 0; j < 2; ++j) { zlt[j] = fma(as, dzl[j], zl[j]); zut[j] = fma(as, dzu[j], zu[j]); }
                    const double pd1 = pd_error(xt, ut, lmt, zlt, zut, gt);
                    take = pd1 <= 0.9999 * pd0;
                }
                if (take) {
                    accepted = true; soft = true; alpha = as; az = as;
                    in_soft = orig ? 0 : 1;
                    if (orig) soft_count = 0;
                }
            }
            if (!accepted) { phi_rs = phi; tau_rs = tau; go_resto = true; break; }
        }
        STAMP(5);
        if (!soft && !ftype) F0.add((1 - gam_th) * theta, phi - gam_ph * theta);
        // ---- accept the step ----
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            x[i] = xon ? fma(alpha, dx[i], x[i]) : x[i];
            lam[i] = xon ? fma(alpha, lp[i] - lam[i], lam[i]) : 0.0;
        }
        if (uon) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                u[j] = fma(alpha, dU[j], u[j]);
                const double sl = u[j] - lo, su = hi - u[j];
                zl[j] = fmax(fmin(fma(az, dzl[j], zl[j]), 1e10 * mu / sl), mu / (1e10 * sl));     // kappa_sigma
                zu[j] = fmax(fmin(fma(az, dzu[j], zu[j]), 1e10 * mu / su), mu / (1e10 * su));
            }
        }
        __syncthreads();
        STAMP(6);
    }
    if (!go_resto) break;
    go_resto = false;
    STAMP(5);

    // ---------------- IPOPT's restoration phase (MinC_1NrmRestorationPhase; oracle/pmpc_ipm.c) -----------
    // min rho sum(p + n) + eta/2 |D_R (x - x_R)|^2 s.t. c(x) + n - p = 0 on every defect row (x_0 pinning
    // included), p, n >= 0, the U box; rho 1000, eta = sqrt(mu_R), D_R = 1 / max(1, |x_R|).  Start: mu_R =
    // max(mu, |c|_inf), closed-form p, n, z = mu_R / p, u-bound multipliers min(rho, z), least-square equality
    // multipliers.  Solved by the same algorithm (own filter and mu, inertia correction, second-order
    // correction, iterative refinement of every step); it returns when the original problem's theta falls to
    // 0.9 of its start value at a point the original filter accepts.  The defect rows are soft rows of the
    // Riccati recursion (riccati_sweep_gen_soft).
    {
        double* const pn = SH.PN[xon ? k : PR_NMAXS];
        const double mu0 = mu, th0 = theta, phi0 = phi_rs, tau0 = tau_rs, rho = 1000.0;
        const double nb = 4.0 * N + 2.0 * ng;              // bound-multiplier count of the restoration problem
        aug_soft_init<PrLds, 6>(SR);
        defects(x, u, g);
        if (nod) {
#pragma unroll
            for (int i = 0; i < 6; ++i) { pn[R_XR + i] = x[i]; pn[R_DRX + i] = 1.0 / fmax(1.0, fabs(x[i])); }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                pn[R_UR + j] = u[j]; pn[R_DRU + j] = 1.0 / fmax(1.0, fabs(u[j]));
                pn[R_ZL0 + j] = zl[j]; pn[R_ZU0 + j] = zu[j];
            }
        }
        double cmx = 0.0;
        if (wx) {
#pragma unroll
            for (int i = 0; i < 6; ++i) cmx = fmax(cmx, fabs(g[i]));
        }
        double rmu = fmax(mu0, wmax(cmx));
        double eta = sqrt(rmu);
        if (nod) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double p = 1.0, n = 1.0;
                if (xon) {
                    const double aa = rmu / (2.0 * rho) - 0.5 * g[i], bb = g[i] * rmu / (2.0 * rho);
                    n = aa + sqrt(aa * aa + bb); p = g[i] + n;
                }
                pn[R_PC + i] = p; pn[R_NC + i] = n;
                pn[R_ZP + i] = xon ? rmu / p : 0.0; pn[R_ZN + i] = xon ? rmu / n : 0.0;
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) { zl[j] = fmin(rho, zl[j]); zu[j] = fmin(rho, zu[j]); }
        __syncthreads();

        double ln[6], ja[8], hdu[2];
        // stage QP of the restoration problem at shift d: lsq the least-square multipliers' unit weights; ov a
        // gradient override (refinement)
        auto assemble_r = [&](double d, bool lsq, const double* ov) {
            double hx[6], hu[2], gq[8];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double w = eta * pn[R_DRX + i] * pn[R_DRX + i];
                hx[i] = lsq ? 1.0 : w + d;
                gq[i] = ov ? ov[i] : w * (x[i] - pn[R_XR + i]);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double sl = u[j] - lo, su = hi - u[j];
                const double w = eta * pn[R_DRU + j] * pn[R_DRU + j];
                hu[j] = lsq ? 1.0 : hdu[j] + (w + zl[j] / sl + zu[j] / su + d);
                gq[6 + j] = ov ? ov[6 + j] : w * (u[j] - pn[R_UR + j]) + (lsq ? -zl[j] + zu[j] : -rmu / sl + rmu / su);
            }
            write_stage(hx, hu, gq);
        };
        // soft rows of node k (shift d): Sigma_p', Sigma_n', 1 / D
        // (node and mirror lanes write the same values: each reads its node's row back without a barrier)
        auto soft_set = [&](double d, bool lsq) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double sp = lsq ? 1.0 : pn[R_ZP + i] / pn[R_PC + i] + d;
                const double sn = lsq ? 1.0 : pn[R_ZN + i] / pn[R_NC + i] + d;
                pn[R_SP + i] = sp; pn[R_SN + i] = sn;
                if (xon) SR->Dinv[k][i] = 1.0 / (1.0 / sp + 1.0 / sn);
            }
        };
        // right-hand side of the soft rows: rg = cgv - (rnv / Sigma_n' - rpv / Sigma_p') + D lamv
        auto soft_rhs = [&](const double* cgv, const double* lamv, const double* rpv, const double* rnv) {
            double rg[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double sp = pn[R_SP + i], sn = pn[R_SN + i];
                rg[i] = cgv[i] - (rnv[i] / sn - rpv[i] / sp) + (1.0 / sp + 1.0 / sn) * lamv[i];
            }
            write_rhs(rg);
        };
        double dx[6], dU[2], lp[6], dpc[6], dnc[6];
        // p, n steps of the soft rows from the multiplier step
        auto pn_dirs = [&](const double* lamv, const double* rpv, const double* rnv) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double dl = lp[i] - lamv[i];
                dpc[i] = xon ? (dl - rpv[i]) / pn[R_SP + i] : 0.0;
                dnc[i] = xon ? (-dl - rnv[i]) / pn[R_SN + i] : 0.0;
            }
        };
        auto park = [&](double* v) {
#pragma unroll
            for (int i = 0; i < 6; ++i) { v[V_DX + i] = dx[i]; v[V_LP + i] = lp[i]; v[V_DPC + i] = dpc[i]; v[V_DNC + i] = dnc[i]; }
            v[V_DU] = dU[0]; v[V_DU + 1] = dU[1];
        };
        auto unpark = [&](const double* v, bool add) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                dx[i] = add ? dx[i] + v[V_DX + i] : v[V_DX + i];
                lp[i] = add ? lp[i] + v[V_LP + i] : v[V_LP + i];
                dpc[i] = add ? dpc[i] + v[V_DPC + i] : v[V_DPC + i];
                dnc[i] = add ? dnc[i] + v[V_DNC + i] : v[V_DNC + i];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) dU[j] = add ? dU[j] + v[V_DU + j] : v[V_DU + j];
        };

        // ---- least-square equality multipliers of the restoration problem (unit weights on x, u, p, n) ----
        {
#pragma unroll
            for (int i = 0; i < 6; ++i) { pn[R_RP + i] = rho - pn[R_ZP + i]; pn[R_RN + i] = rho - pn[R_ZN + i]; }
#pragma unroll
            for (int i = 0; i < 6; ++i) lam[i] = 0.0;
            write_tilt_cols(u);
            hdu[0] = 0.0; hdu[1] = 0.0;
            assemble_r(0.0, true, nullptr);
            soft_set(0.0, true);
            soft_rhs(zero6, zero6, pn + R_RP, pn + R_RN);
            __syncthreads();
            (void)riccati_sweep_gen_soft<PrLds, 6>(S, SR, N, SH.U);      // unit weights: positive definite
            solve_soft(dx, dU, lp);
            double ym = 0.0;
            bool fin = true;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                ym = fmax(ym, wx ? fabs(lp[i]) : 0.0);
                fin = fin && (!wx || isfinite(lp[i]));
            }
            const bool use = !wany(!fin) && wmax(ym) <= 1e3;
#pragma unroll
            for (int i = 0; i < 6; ++i) lam[i] = (use && xon) ? lp[i] : 0.0;
        }
        double cg[6], cgt[6];
        auto resto_cons = [&](const double* gg, const double* pp, const double* nn, double* cc) {
#pragma unroll
            for (int i = 0; i < 6; ++i) cc[i] = xon ? gg[i] + nn[i] - pp[i] : 0.0;
            return wsum(l1(cc));
        };
        double thr;
        {
            double pv[6], nv[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) { pv[i] = pn[R_PC + i]; nv[i] = pn[R_NC + i]; }
            thr = resto_cons(g, pv, nv, cg);
        }
        const double rth_max = 1e4 * fmax(1.0, thr), rth_min = 1e-4 * fmax(1.0, thr);
        PrFilter F1;
        F1.reset();
        int rit = it + 1, rstat = -2;
        bool rfirst = true, rok = false;
        double rdelta_last = 0.0;
        STAMP(7);
        for (;; ++rit) {
            STAMP_ADD(18, 1);
            defects(x, u, g);
            {
                double pv[6], nv[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) { pv[i] = pn[R_PC + i]; nv[i] = pn[R_NC + i]; }
                (void)resto_cons(g, pv, nv, cg);
            }
            if (!rfirst) {
                // RestoConvergenceCheck: the original problem's progress at the current point
                const double tho = wsum(l1(g));
                if (tho <= 0.9 * th0) {
                    const double pho = barrier(x, u, mu0);
                    bool acc = isfinite(pho) && !F0.hit(tho, pho);
                    acc = acc && (cmp_le(tho, (1 - gam_th) * th0, th0) || cmp_le(pho - phi0, -gam_ph * th0, phi0));
                    if (acc) { rok = true; break; }
                }
            }
            rfirst = false;
            next_of(lam, ln);
            jac_t(u, ln, ja, hdu);
            // ---- optimality error of the restoration problem ----
            double dinf = 0.0, pinf = 0.0, c0r = 0.0, cminr = 1e300, suml = 0.0, sumz = 0.0;
            if (wx) {
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double w = eta * pn[R_DRX + i] * pn[R_DRX + i];
                    dinf = fmax(dinf, fabs(w * (x[i] - pn[R_XR + i]) + lam[i] - ja[i]));
                    pinf = fmax(pinf, fabs(cg[i]));
                    suml += fabs(lam[i]);
                    dinf = fmax(dinf, fmax(fabs(rho - pn[R_ZP + i] - lam[i]), fabs(rho - pn[R_ZN + i] + lam[i])));
                    const double cp = pn[R_ZP + i] * pn[R_PC + i], cn = pn[R_ZN + i] * pn[R_NC + i];
                    c0r = fmax(c0r, fmax(cp, cn)); cminr = fmin(cminr, fmin(cp, cn));
                    sumz += pn[R_ZP + i] + pn[R_ZN + i];
                }
            }
            if (wu) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double w = eta * pn[R_DRU + j] * pn[R_DRU + j];
                    dinf = fmax(dinf, fabs(w * (u[j] - pn[R_UR + j]) - zl[j] + zu[j] - ja[6 + j]));
                    const double cl = zl[j] * (u[j] - lo), cu = zu[j] * (hi - u[j]);
                    c0r = fmax(c0r, fmax(cl, cu)); cminr = fmin(cminr, fmin(cl, cu));
                    sumz += zl[j] + zu[j];
                }
            }
            wred_errors_f64(dinf, pinf, c0r, cminr, suml, sumz);
            const double s_d = fmax(100.0, (suml + sumz) / (ng + nb)) / 100.0;
            const double s_c = fmax(100.0, sumz / nb) / 100.0;
            const double errr = fmax(dinf / s_d, fmax(pinf, c0r / s_c));
            if (rit >= a.max_iter) { rstat = -1; break; }
            // the restoration problem converged: local infeasibility (IPOPT Infeasible_Problem_Detected, 2)
            if (errr <= tol && dinf <= 1.0 && pinf <= 1e-4 && c0r <= 1e-4) { rstat = 2; break; }
            for (;;) {
                const double cmu = fmax(c0r - rmu, rmu - cminr);
                if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * rmu || rmu <= mu_min) break;
                rmu = fmax(mu_min, fmin(0.2 * rmu, pow(rmu, 1.5)));
                eta = sqrt(rmu);
                F1.reset();
            }
            const double taur = fmax(0.99, 1.0 - rmu);
            STAMP(8);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                pn[R_RP + i] = rho - rmu / pn[R_PC + i] - lam[i];
                pn[R_RN + i] = rho - rmu / pn[R_NC + i] + lam[i];
            }
            write_tilt_cols(u);
            // ---- Newton step with inertia correction ----
            double delta = 0.0;
            bool okr;
            {
                assemble_r(0.0, false, nullptr);
                soft_set(0.0, false);
                soft_rhs(cg, lam, pn + R_RP, pn + R_RN);
                __syncthreads();
                okr = riccati_sweep_gen_soft<PrLds, 6>(S, SR, N, SH.U);
                for (int attempt = 0; !okr && attempt < 60; ++attempt) {
                    delta = (attempt == 0) ? (rdelta_last == 0.0 ? 1e-4 : fmax(1e-20, rdelta_last * (1.0 / 3.0)))
                                           : delta * (rdelta_last == 0.0 ? 100.0 : 8.0);
                    assemble_r(delta, false, nullptr);
                    soft_set(delta, false);
                    soft_rhs(cg, lam, pn + R_RP, pn + R_RN);
                    __syncthreads();
                    okr = riccati_sweep_gen_soft<PrLds, 6>(S, SR, N, SH.U);
                }
            }
            if (!okr) { rstat = -3; break; }
            if (delta > 0.0) rdelta_last = delta;
            STAMP(9);
            // one refinement pass (PDFullSpaceSolver): the residuals of the full Newton system at the step --
            // stationarity of x and u, the soft defect rows, the p / n rows -- solved for on the same
            // factorisation and added, while they exceed 1e-12 (1 + |step|); returns false when done
            auto refine = [&](const double* cgv) -> bool {
                double lpn[6], pdx[6], pdu[2];
                next_of(lp, lpn);
#pragma unroll
                for (int i = 0; i < 6; ++i) pdx[i] = from_prev(dx[i]);
                pdu[0] = from_prev(dU[0]); pdu[1] = from_prev(dU[1]);
                double ex[8], ec[6], ep[6], en[6], emax = 0.0, smax = 0.0;
#pragma unroll
                for (int j = 0; j < 8; ++j) ex[j] = 0.0;
                if (wu) {
                    const double dz[8] = {dx[0], dx[1], dx[2], dx[3], dx[4], dx[5], dU[0], dU[1]};
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        double t = Hk[hp(8, j)];
#pragma unroll
                        for (int i = 0; i < 8; ++i) t = fma(Hk[hp(j, i)], dz[i], t);
                        if (j < 6) t += lp[j];
#pragma unroll
                        for (int m = 0; m < 6; ++m) t -= Mk[j * NC + m] * lpn[m];
                        ex[j] = t;
                        emax = fmax(emax, fabs(t));
                    }
                } else if (nod && k == N) {
                    const double* GN = S->G[N];
#pragma unroll
                    for (int j = 0; j < 6; ++j) {
                        double t = GN[hp(8, j)];
#pragma unroll
                        for (int i = 0; i < 6; ++i) t = fma(GN[hp(j, i)], dx[i], t);
                        ex[j] = t + lp[j];
                        emax = fmax(emax, fabs(ex[j]));
                    }
                }
#pragma unroll
                for (int i = 0; i < 6; ++i) { ec[i] = 0.0; ep[i] = 0.0; en[i] = 0.0; }
                if (wx) {
                    const double* Mp = &S->M[k > 0 ? k - 1 : 0][0][0];
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        double jd = dx[i];
                        if (k > 0) {
#pragma unroll
                            for (int m = 0; m < 6; ++m) jd -= Mp[m * NC + i] * pdx[m];
                            jd -= Mp[6 * NC + i] * pdu[0];
                            jd -= Mp[7 * NC + i] * pdu[1];
                        }
                        const double dl = lp[i] - lam[i];
                        ec[i] = jd + dnc[i] - dpc[i] + cgv[i];
                        ep[i] = pn[R_SP + i] * dpc[i] - dl + pn[R_RP + i];
                        en[i] = pn[R_SN + i] * dnc[i] + dl + pn[R_RN + i];
                        emax = fmax(emax, fmax(fabs(ec[i]), fmax(fabs(ep[i]), fabs(en[i]))));
                        smax = fmax(smax, fmax(fabs(dx[i]), fmax(fabs(dpc[i]), fabs(dnc[i]))));
                    }
                }
                if (wu) smax = fmax(smax, fmax(fabs(dU[0]), fabs(dU[1])));
                emax = wmax(emax); smax = wmax(smax);
                if (!(emax > 1e-12 * (1.0 + smax))) return false;
                STAMP_ADD(20, 1);
                // the correction solve: lambda = 0, the residuals as gradient and right-hand sides
                park(SH.SV2[lane]);
                double gsave[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) gsave[j] = wu ? Hk[hp(8, j)] : (nod && k == N && j < 6 ? S->G[N][hp(8, j)] : 0.0);
                if (wu) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) Hk[hp(8, j)] = ex[j];
                } else if (nod && k == N) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) S->G[N][hp(8, j)] = ex[j];
                }
                soft_rhs(ec, zero6, ep, en);
                __syncthreads();
                (void)riccati_sweep_gen_soft<PrLds, 6>(S, SR, N, SH.U);
                solve_soft(dx, dU, lp);
                pn_dirs(zero6, ep, en);
                unpark(SH.SV2[lane], true);
                if (wu) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) Hk[hp(8, j)] = gsave[j];
                } else if (nod && k == N) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) S->G[N][hp(8, j)] = gsave[j];
                }
                __syncthreads();
                return true;
            };
            double amr = 1.0, azr = 1.0;
            // fractions to the boundary of the primal step (amr) and of every bound multiplier (azr)
            auto pn_steps = [&]() {
                double am = 1.0, a2 = 1.0;
                if (wx) {
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        const double p = pn[R_PC + i], n = pn[R_NC + i], zp = pn[R_ZP + i], zn = pn[R_ZN + i];
                        if (dpc[i] < 0) am = fmin(am, -taur * p / dpc[i]);
                        if (dnc[i] < 0) am = fmin(am, -taur * n / dnc[i]);
                        const double dzp = rmu / p - zp - zp / p * dpc[i], dzn = rmu / n - zn - zn / n * dnc[i];
                        if (dzp < 0) a2 = fmin(a2, -taur * zp / dzp);
                        if (dzn < 0) a2 = fmin(a2, -taur * zn / dzn);
                    }
                }
                if (wu) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const double sl = u[j] - lo, su = hi - u[j];
                        if (dU[j] < 0) am = fmin(am, -taur * sl / dU[j]);
                        if (dU[j] > 0) am = fmin(am, taur * su / dU[j]);
                        const double dzl_ = rmu / sl - zl[j] - zl[j] / sl * dU[j];
                        const double dzu_ = rmu / su - zu[j] + zu[j] / su * dU[j];
                        if (dzl_ < 0) a2 = fmin(a2, -taur * zl[j] / dzl_);
                        if (dzu_ < 0) a2 = fmin(a2, -taur * zu[j] / dzu_);
                    }
                }
                wmin2d(am, a2);
                amr = am; azr = a2;
            };
            // the step of the right-hand side cgv: solve, p / n steps, refinement, fractions to the boundary
            auto rstep = [&](const double* cgv) {
                solve_soft(dx, dU, lp);
                pn_dirs(lam, pn + R_RP, pn + R_RN);
                for (int r = 0; r < 3 && refine(cgv); ++r) {}
                pn_steps();
            };
            rstep(cg);
            STAMP(10);
            // barrier objective of the restoration problem and its directional derivative
            double phir, gtdr;
            {
                double pl = 0.0, gd = 0.0, lb = 0.0;
                double lgp[6], lgn[6], lgl[2], lgu[2];
#pragma unroll
                for (int i = 0; i < 6; ++i)
                    half_pair(log(pr_low_half() ? pn[R_PC + i] : pn[R_NC + i]), lgp[i], lgn[i]);
                {
                    const double uh = pr_low_half() ? u[0] : u[1];
                    half_pair(log(uh - lo), lgl[0], lgl[1]);
                    half_pair(log(hi - uh), lgu[0], lgu[1]);
                }
                if (wx) {
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        const double p = pn[R_PC + i], n = pn[R_NC + i];
                        const double w = eta * pn[R_DRX + i] * pn[R_DRX + i];
                        const double e = pn[R_DRX + i] * (x[i] - pn[R_XR + i]);
                        pl += rho * (p + n) + 0.5 * eta * e * e;
                        lb += lgp[i] + lgn[i];
                        gd += w * (x[i] - pn[R_XR + i]) * dx[i] + (rho - rmu / p) * dpc[i] + (rho - rmu / n) * dnc[i];
                    }
                }
                if (wu) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const double w = eta * pn[R_DRU + j] * pn[R_DRU + j];
                        const double e = pn[R_DRU + j] * (u[j] - pn[R_UR + j]);
                        pl += 0.5 * eta * e * e;
                        lb += lgl[j] + lgu[j];
                        gd += (w * (u[j] - pn[R_UR + j]) - rmu / (u[j] - lo) + rmu / (hi - u[j])) * dU[j];
                    }
                }
                wsum3(pl, lb, gd);
                phir = pl - rmu * lb;
                gtdr = gd;
            }
            double pw_thr = 0.0, pw_gdr = 0.0;
            if (gtdr < 0) half_pair(pr_low_half() ? pow(thr, s_th) : pow(-gtdr, s_ph), pw_thr, pw_gdr);
            double aminr = gam_th;
            if (gtdr < 0) aminr = fmin(gam_th, fmin(gam_ph * thr / (-gtdr), pw_thr / pw_gdr));
            aminr *= gam_al;
            double xt[6], ut[2], gt[6], tht = 0.0, pht = 0.0;
            // trial point of the restoration problem at step al: constraint values cgt, theta, barrier
            auto trial_r = [&](double al) {
#pragma unroll
                for (int i = 0; i < 6; ++i) xt[i] = xon ? fma(al, dx[i], x[i]) : x[i];
#pragma unroll
                for (int j = 0; j < 2; ++j) ut[j] = uon ? fma(al, dU[j], u[j]) : u[j];
                defects(xt, ut, gt);
                double thl = 0.0, phl = 0.0, lb = 0.0;
                bool out = false;
                double lgp[6], lgn[6], lgl[2], lgu[2];
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double p = fma(al, dpc[i], pn[R_PC + i]), n = fma(al, dnc[i], pn[R_NC + i]);
                    half_pair(log(pr_low_half() ? p : n), lgp[i], lgn[i]);
                }
                {
                    const double uh = pr_low_half() ? ut[0] : ut[1];
                    half_pair(log(uh - lo), lgl[0], lgl[1]);
                    half_pair(log(hi - uh), lgu[0], lgu[1]);
                }
                if (wx) {
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        const double p = fma(al, dpc[i], pn[R_PC + i]), n = fma(al, dnc[i], pn[R_NC + i]);
                        cgt[i] = gt[i] + n - p;
                        thl += fabs(cgt[i]);
                        const double e = pn[R_DRX + i] * (xt[i] - pn[R_XR + i]);
                        phl += rho * (p + n) + 0.5 * eta * e * e;
                        out = out || !(p > 0.0) || !(n > 0.0);
                        lb += lgp[i] + lgn[i];
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 6; ++i) cgt[i] = 0.0;
                }
                if (wu) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const double e = pn[R_DRU + j] * (ut[j] - pn[R_UR + j]);
                        phl += 0.5 * eta * e * e;
                        out = out || !(ut[j] > lo) || !(ut[j] < hi);
                        lb += lgl[j] + lgu[j];
                    }
                }
                wsum3(thl, phl, lb);
                tht = thl;
                pht = wany(out) ? (double)INFINITY : phl - rmu * lb;
            };
            bool ftr = false;
            auto racc = [&](double al) -> bool {
                if (!(tht < rth_max) || !isfinite(pht) || F1.hit(tht, pht)) return false;
                const bool sw = gtdr < 0.0 && al * pw_gdr > pw_thr;
                if (thr <= rth_min && sw) {
                    if (cmp_le(pht, phir + eta_ph * al * gtdr, phir)) { ftr = true; return true; }
                    return false;
                }
                return cmp_le(tht, (1 - gam_th) * thr, thr) || cmp_le(pht - phir, -gam_ph * thr, phir);
            };
            double alr = amr;
            bool accr = false;
            for (int ls = 0; ls < 80 && !accr; ++ls) {
                if (alr < aminr && ls > 0) break;
                trial_r(alr);
                STAMP_ADD(19, 1);
                accr = racc(alr);
                if (!accr && ls == 0 && !(tht < thr) && a.max_soc > 0) {
                    // second-order correction on the restoration problem's constraints; the plain step parked
                    park(SH.SV[lane]);
                    const double amr_keep = amr, azr_keep = azr;
                    double asoc = alr, th_old = 0.0, cs[6];
#pragma unroll
                    for (int i = 0; i < 6; ++i) cs[i] = cg[i];
                    for (int c = 0; c < a.max_soc; ++c) {
                        if (c > 0 && !(tht <= kap_soc * th_old)) break;
                        th_old = tht;
#pragma unroll
                        for (int i = 0; i < 6; ++i) cs[i] = fma(asoc, cs[i], cgt[i]);
                        soft_rhs(cs, lam, pn + R_RP, pn + R_RN);
                        __syncthreads();
                        (void)riccati_sweep_gen_soft<PrLds, 6>(S, SR, N, SH.U);
                        rstep(cs);
                        asoc = amr;
                        trial_r(asoc);
                        if (racc(alr)) { accr = true; alr = asoc; break; }
                    }
                    if (!accr) {      // back to the plain direction and its multiplier steps
                        unpark(SH.SV[lane], false);
                        amr = amr_keep; azr = azr_keep;
                    }
                }
                if (!accr) alr *= 0.5;
            }
#ifdef DART_RESTO_TRACE
            if (blockIdx.x == 0 && lane == 0)
                printf("  resto it %3d mu %.2e err %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e th %.3e "
                       "th_t %.3e acc %d\n", rit, rmu, errr, dinf / s_d, pinf, c0r / s_c, delta, amr, alr, thr, tht, (int)accr);
#endif
            STAMP(11);
            if (!accr) { rstat = -2; break; }      // a failed line search in the restoration phase
            if (!ftr) F1.add((1 - gam_th) * thr, phir - gam_ph * thr);
            // ---- accept the trial point ----
            if (nod) {
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    if (!xon) continue;
                    const double p0 = pn[R_PC + i], n0 = pn[R_NC + i], zp = pn[R_ZP + i], zn = pn[R_ZN + i];
                    const double dzp = rmu / p0 - zp - zp / p0 * dpc[i], dzn = rmu / n0 - zn - zn / n0 * dnc[i];
                    const double p = fma(alr, dpc[i], p0), n = fma(alr, dnc[i], n0);
                    pn[R_PC + i] = p; pn[R_NC + i] = n;
                    pn[R_ZP + i] = fmax(fmin(fma(azr, dzp, zp), 1e10 * rmu / p), rmu / (1e10 * p));
                    pn[R_ZN + i] = fmax(fmin(fma(azr, dzn, zn), 1e10 * rmu / n), rmu / (1e10 * n));
                }
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                x[i] = xon ? fma(alr, dx[i], x[i]) : x[i];
                lam[i] = xon ? fma(alr, lp[i] - lam[i], lam[i]) : 0.0;
            }
            if (uon) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double sl = u[j] - lo, su = hi - u[j];
                    const double dzl_ = rmu / sl - zl[j] - zl[j] / sl * dU[j];
                    const double dzu_ = rmu / su - zu[j] + zu[j] / su * dU[j];
                    u[j] = fma(alr, dU[j], u[j]);
                    const double nl = u[j] - lo, nu = hi - u[j];
                    zl[j] = fmax(fmin(fma(azr, dzl_, zl[j]), 1e10 * rmu / nl), rmu / (1e10 * nl));
                    zu[j] = fmax(fmin(fma(azr, dzu_, zu[j]), 1e10 * rmu / nu), rmu / (1e10 * nu));
                }
            }
            thr = tht;
            __syncthreads();
            STAMP(12);
        }
        STAMP(13);
        if (!rok) { status = rstat; it = rit; break; }
        // back to the original problem: the u-bound multipliers take the step (mu - z s_trial) / s that
        // pretends the restoration's progress was one Newton step, cut by the fraction to the boundary (tau
        // of the original iteration) and all reset to 1 if one exceeds 1000; the equality multipliers restart at 0
        {
            double a2 = 1.0, dzlo[2] = {0.0, 0.0}, dzuo[2] = {0.0, 0.0};
            if (wu) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double ur = pn[R_UR + j], zl0 = pn[R_ZL0 + j], zu0 = pn[R_ZU0 + j];
                    dzlo[j] = (mu0 - zl0 * (u[j] - lo)) / (ur - lo);
                    dzuo[j] = (mu0 - zu0 * (hi - u[j])) / (hi - ur);
                    if (dzlo[j] < 0) a2 = fmin(a2, -tau0 * zl0 / dzlo[j]);
                    if (dzuo[j] < 0) a2 = fmin(a2, -tau0 * zu0 / dzuo[j]);
                }
            }
            const double azo = wmin(a2);
            double zmx = 0.0;
            if (uon) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    zl[j] = pn[R_ZL0 + j] + azo * dzlo[j]; zu[j] = pn[R_ZU0 + j] + azo * dzuo[j];
                    zmx = fmax(zmx, fmax(zl[j], zu[j]));
                }
            }
            const bool reset = wmax(wu ? zmx : 0.0) > 1e3;
            if (uon) {
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
        }
        in_soft = 0; soft_count = 0;
        it_next = rit;
        __syncthreads();
    }
    }

    // ---------------- outputs (as pmpc_ipm.hip) ------------------------------------------------------
    STAMP(14);
#ifdef DART_STAMPS
    if (lane == 0)
        for (int q = 0; q < 32; ++q) g_stamp_pr[q] = t_acc_[q];
#endif
    const double fval = wsum(node_cost(x, u));
    if (lane == 0) {
        a.u0[2 * b] = u[0]; a.u0[2 * b + 1] = u[1];
        a.f[b] = fval; a.status[b] = status; a.iters[b] = it;
    }
    if (a.w_out) {
        double* wo = a.w_out + (size_t)nw * b;
        if (wx) {
#pragma unroll
            for (int i = 0; i < 6; ++i) wo[6 * k + i] = x[i];
        }
        if (wu) { wo[6 * (N + 1) + 2 * k] = u[0]; wo[6 * (N + 1) + 2 * k + 1] = u[1]; }
    }
    if (a.done && a.resto != 2) {
        // release at system scope: the wave's output stores are visible before the completion word
        __threadfence_system();
        if (lane == 0) __hip_atomic_store(a.done + b, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace dartmpc
