// pmpc_ipm.hip -- batched PMPC interior-point solve for gfx950 (MI355X / CDNA4).
//
// Replaces the per-timestep `ca.nlpsol('solver','ipopt',...)` call of
// PMPC.solve (PMPC/src/controller/mpc_3d.py:115-138) for a whole batch of
// independent tray-tilt NMPC instances.
//
// Structure exploited: the Newton system of the reference NLP
// (mpc_3d.py:28-85) splits into two independent scalar-input optimal-control
// problems -- the x axis (px, vx; theta_x) and the y axis (py, vy; theta_y) --
// plus the cost-free z sub-state (pz, vz).  Each axis is linear in its state
// with input sin(theta):  x+ = Phi x + Gamma sin(theta), Phi/Gamma being exactly
// the RK4 map of mpc_3d.py:99-104 applied to :91-92.  z is affine in its state
// and in vz_new = -g (theta_x^2 + theta_y^2) (:93-97): it carries no cost, so
// its multipliers stay 0 and it never enters the (x, y) Riccati solve, but its
// defect rows (:37, :48) are part of IPOPT's constraint violation.  The kernel
// therefore runs IPOPT's primal-dual barrier method on the FULL 6-state NLP:
// one mu, one step length, one filter; theta, the primal infeasibility, the
// tiny-step test and the second-order correction see the z rows, and z moves
// with its own Newton step (an affine scan driven by the tilt steps).
//
// Mapping: one wave64 per instance, lane k <-> shooting node k (0..N, N <= 63).
// Everything per node lives in VGPRs.  Stage-coupled recursions (Riccati
// backward sweep, forward state sweep, z sweep) are DPP scans or hand 2x2
// blocks to the neighbouring lane with DPP wave shifts (no LDS); norms and
// inner products are DPP row reductions.  No LDS and no global traffic inside
// the iteration loop.
// Horizons N = 32..63: this file built a third time with -DDART_WG=2 (Makefile: pmpc_wg2.o) -- the scan build
// (NAX = 1) on a workgroup of two waves per instance, wave w owning nodes 32 w .. 32 w + 31 with the one-wave lane
// roles (wave.h: the wave reductions and node shifts combine the two waves).  Every scan runs in both waves and is
// continued across the wave boundary by one LDS hand-over (pm_pass): the suffix scans of wave 0 start from the
// values of node 32 (wave 1), the prefix scans of wave 1 from those of node 31 (wave 0).  IPOPT's soft restoration
// phase runs in the kernel as in the sequential N > 31 build.  The build's symbols sit in their own namespace.
#if DART_WG == 2
#define dartmpc dartmpc_wg2
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "pmpc_ipm.h"
#include "pmpc_model.h"
#include "pmpc_resto.h"
#include "stamps.h"
#include "wave.h"

namespace dartmpc {

// This file is compiled twice (Makefile): as is, it holds the scan instantiations for N > 15, the
// launcher and the self-test; with -DPMPC_SEQ, the one-row instantiation (N <= 15) and the
// sequential (throughput) ones behind dartmpc_launch_pmpc_seq, so that each set gets the
// optimisation level that is fastest for it.
#ifdef DART_STAMPS
#ifndef PMPC_SEQ
__device__ unsigned long long g_stamp[16];
#define STAMP_FLUSH(b) STAMP_FLUSH_TO(g_stamp, b)
#else
__device__ unsigned long long g_stamp_seq[16];
#define STAMP_FLUSH(b) STAMP_FLUSH_TO(g_stamp_seq, b)
#endif
#else
#define STAMP_FLUSH(b) STAMP_FLUSH_TO(g_stamp, b)
#endif

// values of node `src_node` of wave `src_wave` (lane src_node: axis x, lane src_node + 32: axis y) in every lane of
// the same axis half of both waves.  One barrier: every call site SITE has its own slots, and between two passes
// of one site both waves cross other barriers (the reductions and shifts of an iteration), each after its reads
// of the slot have completed (__syncthreads waits for the wave's LDS accesses), so no pass overwrites a slot that
// is still to be read.  Two-wave build only (the one-wave build names it in discarded branches).
#if DART_WG == 2
__shared__ double g_pm_x[4][2][4];
#endif
template <int SITE, int NV>
__device__ __forceinline__ void pm_pass(int src_wave, int src_node, const double (&v)[NV], double (&o)[NV]) {
    static_assert(NV <= 4 && SITE < 4, "four slots, four sites");
#if DART_WG == 1
    (void)src_wave; (void)src_node;
#pragma unroll
    for (int i = 0; i < NV; ++i) o[i] = v[i];
#else
    const int l = lane_id();
    if (wave_idx() == src_wave && (l & 31) == src_node) {
#pragma unroll
        for (int i = 0; i < NV; ++i) g_pm_x[SITE][l >> 5][i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) o[i] = g_pm_x[SITE][l >> 5][i];
#endif
}

// DPP move with an identity fill (FILL = 0.0 or 1.0) for lanes whose source is outside the row or
// masked out.  With every row enabled a zero half comes from bound_ctrl (the DPP writes 0 where the
// source is out of range): no initialising move; 1.0 only needs its high word 0x3ff00000 set first.
// Rows masked off keep the old value, so a partial ROWMASK initialises both words.
template <int CTRL, int ROWMASK, int FILL>
__device__ __forceinline__ double dpp_fill(double x) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const int blo = (int)(unsigned)(b & 0xffffffffu), bhi = (int)(unsigned)(b >> 32);
    constexpr int fhi = FILL ? 0x3ff00000 : 0;
    int rlo, rhi;
    if constexpr (ROWMASK == 0xf) {
        rlo = __builtin_amdgcn_mov_dpp(blo, CTRL, 0xf, 0xf, true);
        if constexpr (FILL) rhi = __builtin_amdgcn_update_dpp(fhi, bhi, CTRL, 0xf, 0xf, false);
        else rhi = __builtin_amdgcn_mov_dpp(bhi, CTRL, 0xf, 0xf, true);
    } else {
        rlo = __builtin_amdgcn_update_dpp(0, blo, CTRL, ROWMASK, 0xf, false);
        rhi = __builtin_amdgcn_update_dpp(fhi, bhi, CTRL, ROWMASK, 0xf, false);
    }
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)rhi << 32) | (unsigned)rlo);
}
// one Hillis-Steele level of an inclusive scan of 2-D affine maps x -> F x + c (later o earlier):
// (F, c) <- (F, c) o (P, q) = (F P, F q + c), (P, q) fetched by DPP, identity where out of range
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void affine_scan_level(double& f11, double& f12, double& f21, double& f22, double& c1,
                                                  double& c2) {
    const double p11 = dpp_fill<CTRL, ROWMASK, 1>(f11), p12 = dpp_fill<CTRL, ROWMASK, 0>(f12);
    const double p21 = dpp_fill<CTRL, ROWMASK, 0>(f21), p22 = dpp_fill<CTRL, ROWMASK, 1>(f22);
    const double q1 = dpp_fill<CTRL, ROWMASK, 0>(c1), q2 = dpp_fill<CTRL, ROWMASK, 0>(c2);
    const double n11 = fma(f11, p11, f12 * p21), n12 = fma(f11, p12, f12 * p22);
    const double n21 = fma(f21, p11, f22 * p21), n22 = fma(f21, p12, f22 * p22);
    c1 = fma(f11, q1, fma(f12, q2, c1));
    c2 = fma(f21, q1, fma(f22, q2, c2));
    f11 = n11; f12 = n12; f21 = n21; f22 = n22;
}

// A composition level whose source lanes already hold pure constants (their map is 0 because
// their window reaches node 0 of an inclusive prefix scan): only the constant is fetched, c <- F q + c
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void affine_scan_const(double f11, double f12, double f21, double f22, double& c1,
                                                  double& c2) {
    const double q1 = dpp_fill<CTRL, ROWMASK, 0>(c1), q2 = dpp_fill<CTRL, ROWMASK, 0>(c2);
    c1 = fma(f11, q1, fma(f12, q2, c1));
    c2 = fma(f21, q1, fma(f22, q2, c2));
}
// the same two levels for scalar affine maps z -> m z + c (the z sub-state's Newton sweep)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void affine1_scan_level(double& m, double& c) {
    const double pm = dpp_fill<CTRL, ROWMASK, 1>(m), pc = dpp_fill<CTRL, ROWMASK, 0>(c);
    c = fma(m, pc, c);
    m = m * pm;
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void affine1_scan_const(double m, double& c) {
    c = fma(m, dpp_fill<CTRL, ROWMASK, 0>(c), c);
}

// One level of a suffix scan of 4x4 matrices (T <- T * F, F fetched from lane k + d by DPP
// row_shl:d, identity where out of range)
template <int CTRL, bool FIRST = false>
__device__ __forceinline__ void mat4_scan_level(double* T) {
    // FIRST: T is a lane's own stage map, whose column 0 is (1, 0, X11, 0), and so is that of the
    // neighbour's map or of the identity fill: those entries are not fetched and their products
    // with 0 / 1 are dropped (the compiler keeps 0 * x for NaN semantics)
    constexpr bool fz[16] = {FIRST, false, false, false, FIRST, false, false, false,
                             false, false, false, false, FIRST, false, false, false};
    double F[16];
#pragma unroll
    for (int e = 0; e < 16; ++e)
        F[e] = fz[e] ? (e == 0 ? 1.0 : 0.0)
                     : (e % 5 == 0) ? dpp_fill<CTRL, 0xf, 1>(T[e]) : dpp_fill<CTRL, 0xf, 0>(T[e]);
    double N[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double acc = T[4 * i + 3] * F[12 + j];
            if (fz[12 + j]) acc = 0.0;
            acc = fma(T[4 * i + 2], F[8 + j], acc);
            if (!fz[4 + j]) acc = fma(T[4 * i + 1], F[4 + j], acc);
            if (FIRST && i == 0) acc += F[j];                                  // T[0] = 1
            else if (!(FIRST && (i == 1 || i == 3))) acc = fma(T[4 * i], F[j], acc);   // T[4] = T[12] = 0
            N[4 * i + j] = acc;
        }
#pragma unroll
    for (int e = 0; e < 16; ++e) T[e] = N[e];
}

// ---------------------------------------------------------------------------
// the kernel: one wave64 = one instance.
//   NAX = 1 (N <= 31): lane = axis*32 + k, one axis per lane (x in lanes 0-31, y in 32-63)
//   NAX = 2 (N <= 63): lane = k, both axes in every lane
// ---------------------------------------------------------------------------
//   QSCAN: compile the quadratic-Riccati scan (latency regime); without it the kernel fits 2 waves
//   per SIMD (throughput regime)
//   ONEROW: N <= 15, every axis fits one 16-lane DPP row and the scans need no cross-row step (the
//   DART driver's default horizon is 15, main_parallel_enhanced.py:171-196)
//   SHORT2: N <= 23, the suffix of node 16 spans at most 8 lanes, so the quadratic scan stops
//   after 3 in-row levels and finishes rows 0 / 2 with two 4 x 2 compositions (no 4th 4 x 4 level)
//   (16 <= N <= 23 at one wave per SIMD; its two-wave instantiation, OCC2, also serves large N <= 15 batches)
//   Occupancy: the sequential NAX == 1 build is the throughput variant and must fit two waves per
//   SIMD (<= 256 registers); the ILP-oriented scheduler of this file (Makefile) would otherwise spend
//   the whole register file on one wave
//   RED: the reduced (x, y) path (opt-in, dart_mpc_config.pmpc_path = 1): theta, the filter and the
//   error measures leave the z rows out and there is no second-order correction, z is rolled out from
//   the final controls.  Same KKT point, fewer iterations, but not IPOPT's iterates.
// the solve of instance b by the calling wave (the body of pmpc_ipm_kernel and of the resident
// server pmpc_serve_kernel); true when the instance was handed over to IPOPT's restoration phases
// (status kPmNeedResto, no other output)
// branch-layout hints for the cold paths of the loop (inertia retries, the sequential fallback of the
// scan, the least-square iteration, second-order corrections, failures): C2 +2.1 % (A/B); the one-row
// build (N <= 15) measured 1 % slower with them and goes without
#define PM_EXPECT(x, v) (ONEROW ? (bool)(x) : (bool)__builtin_expect((long)(bool)(x), (v)))
template <int NAX, bool QSCAN, bool ONEROW, bool SHORT2, bool RED>
__device__ __forceinline__ bool pmpc_solve(const PmpcArgs& a, const int b) {
    STAMP_DECL
    const int lane = kWaves == 1 ? (int)threadIdx.x : lane_id();
    const int k = NAX == 1 ? node_base() + (lane & 31) : lane;      // shooting node of this lane
    const int ax0 = NAX == 1 ? (lane >> 5) : 0;               // axis of slot 0 (NAX == 1)
    const int N = a.N;
    const bool xon = k <= N, uon = k < N;
    constexpr bool one_row = ONEROW;
    constexpr bool short2 = SHORT2 && !ONEROW;
    const double h = a.Ts;

    // every input is read here, at the start (the host entry hands them over in mapped host memory,
    // dart_mpc_abi.hip)
    const double* st = a.x0 + 6 * b;
    const double* rf = a.ref + 6 * b;
    const double* pr = a.prm + 6 * b;
    const double mu_f = pr[0], Qp = pr[1], Qv = pr[2], R = pr[3], ulo = pr[4], uhi = pr[5];

    // RK4 map of the linear axis model applied to the basis: exact Phi = [[1,a12],[0,a22]], Gamma = [b1,b2]
    double a12, a22, b1, b2;
    axis_rk4(h, a.g, mu_f, 0.0, 0.0, 1.0, a12, a22);
    axis_rk4(h, a.g, mu_f, 1.0, 0.0, 0.0, b1, b2);
    // the same for the z sub-state, z+ = zA z + zC w with w = vz_new (mpc_3d.py:93-97, RK4 :99-104):
    // pz+ = pz + cp w, vz+ = av vz + cv w
    double zp1, zav, zcp, zcv;
    z_rk4(h, 0.0, 1.0, 1.0, zp1, zav);
    z_rk4(h, 1.0, 0.0, 0.0, zcp, zcv);
    const double lo = ulo - 1e-8 * fmax(1.0, fabs(ulo));       // IPOPT bound_relax_factor = 1e-8
    const double hi = uhi + 1e-8 * fmax(1.0, fabs(uhi));
    const bool poly = fmax(fabs(lo), fabs(hi)) <= 1.0;
    // per-lane stage map: the real Phi on stages k < N, zero on the terminal/idle lanes, so that the
    // backward sweep reproduces the terminal value function there without a branch
    const double f11 = uon ? 1.0 : 0.0, a12k = uon ? a12 : 0.0, a22k = uon ? a22 : 0.0;
    const double ai22 = 1.0 / a22, ai12 = -a12 * ai22;        // A^-1 = [[1, ai12], [0, ai22]]
    // the same per lane for the quadratic scan: identity stage maps on the terminal / idle lanes
    const double uonf = uon ? 1.0 : 0.0, ai12k = uon ? ai12 : 0.0, ai22k = uon ? ai22 : 1.0, a22i = uon ? a22 : 1.0;
    const double A11k = a12k * a12k, A12k = 2.0 * a12k * a22k, A22k = a22k * a22k;

    // per-lane axis slots; z slots: NAX == 1 keeps pz on the x half and vz on the y half, NAX == 2
    // keeps pz in slot 0 and vz in slot 1 of every lane
    double sp[NAX], sv[NAX], rp[NAX], rv[NAX];
    double p[NAX], v[NAX], th[NAX], lp[NAX], lv[NAX], zl[NAX], zu[NAX];
    double zA[NAX], zC[NAX], zs[NAX], zz[NAX];
    const int nw = 6 * (N + 1) + 2 * N;
    const double* ww = a.w_warm ? a.w_warm + (size_t)nw * b : nullptr;
    const double pushl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo));   // IPOPT bound_push / frac
    const double pushu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
    double gmax = 0.0;
#pragma unroll
    for (int j = 0; j < NAX; ++j) {
        const int ax = NAX == 1 ? ax0 : j;
        sp[j] = st[2 * ax]; sv[j] = st[2 * ax + 1];
        rp[j] = rf[2 * ax]; rv[j] = rf[2 * ax + 1];
        p[j] = xon ? (ww ? ww[6 * k + 2 * ax] : sp[j]) : 0.0;       // cold start: tile(state) (mpc_3d.py:123)
        v[j] = xon ? (ww ? ww[6 * k + 2 * ax + 1] : sv[j]) : 0.0;
        double t = uon ? (ww ? ww[6 * (N + 1) + 2 * k + ax] : 0.0) : 0.0;
        if (uon) t = fmin(fmax(t, lo + pushl), hi - pushu);
        th[j] = t;
        lp[j] = 0.0; lv[j] = 0.0;
        zl[j] = uon ? 1.0 : 0.0; zu[j] = uon ? 1.0 : 0.0;      // bound_mult_init_val = 1
        if (xon) gmax = fmax(gmax, fmax(fabs(2 * Qp * (p[j] - rp[j])), fabs(2 * Qv * (v[j] - rv[j]))));
        if (uon) gmax = fmax(gmax, fabs(2 * R * th[j]));
        // z slot (ax here is 0 = pz, 1 = vz)
        zA[j] = ax ? zav : zp1; zC[j] = ax ? zcv : zcp;
        zs[j] = st[4 + ax];
        zz[j] = xon ? (ww ? ww[6 * k + 4 + ax] : zs[j]) : 0.0;
    }
    gmax = wmax(gmax);
    const double sc = gmax > 100.0 ? 100.0 / gmax : 1.0;     // nlp_scaling_max_gradient = 100
    const double qp2 = sc * 2 * Qp, qv2 = sc * 2 * Qv, r2 = sc * 2 * R;
    const double scQp = sc * Qp, scQv = sc * Qv, scR = sc * R;

    const double tol = a.tol, mu_min = tol / 10;
    const double n_eq = 6.0 * (N + 1), n_b = 4.0 * N;       // IPOPT counts on the full NLP
    const double inv_neb = 1.0 / (n_eq + n_b), inv_nb = 1.0 / n_b;
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, eta_ph = 1e-8, gam_al = 0.05;

    // defect g_k = x_k - f(x_{k-1}, u_{k-1}) (mpc_3d.py:48), g_0 = x_0 - state (:37)
    auto defects = [&](double pj, double vj, double sj, double spj, double svj, double& g1, double& g2) {
        const double fp = fma(a12, vj, fma(b1, sj, pj));
        const double fv = fma(a22, vj, b2 * sj);
        double ip, iv;
        if constexpr (kWaves == 1) {
            ip = from_prev(fp); iv = from_prev(fv);
        } else {       // two waves: one exchange for both shifts
            const double x2[2] = {fp, fv};
            double o2[2];
            from_prev_n(x2, o2);
            ip = o2[0]; iv = o2[1];
        }
        g1 = (k == 0) ? pj - spj : pj - ip;
        g2 = (k == 0) ? vj - svj : vj - iv;
    };
    // the sum over both axes of a per-axis quantity of this lane's node (NAX == 1: the other half's
    // lane k + 32 / k - 32 holds the other axis)
    auto axes_sum = [&](const double (&q)[NAX]) -> double {
        if constexpr (NAX == 1) return half_pair_sum(q[0]);
        else return q[0] + q[1];
    };
    // z defects of this lane's node from the z slots zj and this lane's w = vz_new: the node k - 1
    // prediction zA z + zC w comes from the previous lane
    auto zdefect = [&](double zj, double wj, int j) -> double {
        const double fz = fma(zA[j], zj, zC[j] * wj);
        const double ip = from_prev(fz);
        return (k == 0) ? zj - zs[j] : zj - ip;
    };
    // w = vz_new = -g (theta_x^2 + theta_y^2) at this lane's node (mpc_3d.py:93), 0 past the horizon
    auto vz_new = [&](const double (&t)[NAX]) -> double {
        double sq[NAX];
#pragma unroll
        for (int j = 0; j < NAX; ++j) sq[j] = uon ? t[j] * t[j] : 0.0;
        return -a.g * axes_sum(sq);
    };

    // sines and defects of the current point: computed here once, then carried over from the
    // accepted line-search trial (the update x + alpha d repeats the trial's arithmetic exactly)
    double g1[NAX], g2[NAX], gz[NAX], snc[NAX];
    double th0 = 0.0;
    {
        const double w0 = vz_new(th);
#pragma unroll
        for (int j = 0; j < NAX; ++j) {
            double s0, c0_;
            tilt_sincos(poly, th[j], s0, c0_);
            snc[j] = uon ? s0 : 0.0;
            defects(p[j], v[j], snc[j], sp[j], sv[j], g1[j], g2[j]);
            gz[j] = RED ? 0.0 : zdefect(zz[j], w0, j);
            if (xon) th0 += fabs(g1[j]) + fabs(g2[j]) + fabs(gz[j]);
        }
    }
    double theta = wsum(th0);                                  // filter's constraint violation
    const double th_max = 1e4 * fmax(1.0, theta), th_min = 1e-4 * fmax(1.0, theta);

    double fth = 0.0, fph = 0.0;      // filter entry held by lane (slot = lane id)
    int nfilt = 0;
    double mu = 0.1, delta_last = 0.0;
    int status = -1, it = 0;
    // IPOPT's soft restoration phase (round 5): in_soft while its steps are being taken, soft_count of them
    int in_soft = 0, soft_count = 0;
    STAMP(0);

#ifdef DART_STAMPS
    const unsigned long long t_loop0 = __builtin_amdgcn_s_memtime();
#endif
    // it = -1 (a.mult_init_max > 0): IPOPT's least-square estimate of the starting equality
    // multipliers (DefaultIterateInitializer::least_square_mults, constr_mult_init_max = 1000): the
    // step solve of the loop body with unit weights (X = I, R = 1), the gradient r = grad f - z_L + z_U
    // and a zero constraint right-hand side gives y = argmin ||r + J^T y|| as its new multipliers
    // (LeastSquareMultipliers: [I J^T; J 0] [d; y] = [-r; 0]).  Cold start: the z rows' input columns
    // vanish (theta = 0), so the estimate separates per axis and y_z = 0.
    for (it = a.mult_init_max > 0.0 ? -1 : 0; it < a.max_iter; ++it) {
        const bool lsm = it < 0;
#ifdef DART_STAMPS
        if (it == 1) t_acc_[12] = __builtin_amdgcn_s_memtime() - t_loop0;      // the first iteration (cold code)
#endif
        // -------- point quantities and optimality error (IPOPT eq. 5) ------------
        double sn[NAX], cs[NAX], isl[NAX], isu[NAX], lpn[NAX], lvn[NAX];
        double dinf = 0.0, pinf = 0.0, c0 = 0.0, cmin = 1e300, suml = 0.0, sumz = 0.0;
#pragma unroll
        for (int j = 0; j < NAX; ++j) {
            sn[j] = snc[j];
            const double c_ = tilt_cos_econ(poly, th[j]);
            cs[j] = uon ? c_ : 0.0;
            double ln, vn;       // unconditional: EXEC stays full
            if constexpr (kWaves == 1) {
                ln = from_next(lp[j]); vn = from_next(lv[j]);
            } else {
                const double x2[2] = {lp[j], lv[j]};
                double o2[2];
                from_next_n(x2, o2);
                ln = o2[0]; vn = o2[1];
            }
            lpn[j] = uon ? ln : 0.0; lvn[j] = uon ? vn : 0.0;
            const double sl = th[j] - lo, su = hi - th[j];
            isl[j] = uon ? frcp(sl) : 0.0; isu[j] = uon ? frcp(su) : 0.0;
            const double r1 = fma(qp2, p[j] - rp[j], lp[j] - lpn[j]);
            const double r2x = fma(qv2, v[j] - rv[j], lv[j] - fma(a12, lpn[j], a22 * lvn[j]));
            const double ru = fma(r2, th[j], -cs[j] * fma(b1, lpn[j], b2 * lvn[j])) - zl[j] + zu[j];
            dinf = fmax(dinf, xon ? fmax(fabs(r1), fabs(r2x)) : 0.0);
            dinf = fmax(dinf, uon ? fabs(ru) : 0.0);
            pinf = fmax(pinf, xon ? fmax(fmax(fabs(g1[j]), fabs(g2[j])), fabs(gz[j])) : 0.0);
            suml += xon ? fabs(lp[j]) + fabs(lv[j]) : 0.0;
            c0 = fmax(c0, uon ? fmax(zl[j] * sl, zu[j] * su) : 0.0);
            cmin = fmin(cmin, uon ? fmin(zl[j] * sl, zu[j] * su) : 1e300);
            sumz += zl[j] + zu[j];
        }
        float dinf_f = (float)dinf, pinf_f = (float)pinf, c0_f = (float)c0, cmin_f = (float)cmin;
        float suml_f = (float)suml, sumz_f = (float)sumz;
        wred_errors(dinf_f, pinf_f, c0_f, cmin_f, suml_f, sumz_f);
        const double dinf_w = dinf_f, pinf_w = pinf_f, c0_w = c0_f;
        const double cmin_w = cmin_f;
        // IPOPT's scalings s_d, s_c (>= 1) as reciprocals: one division each instead of one per test
        const float sz_w = sumz_f;
        const double is_d = 100.0 * frcp(fmax(100.0, (double)(suml_f + sz_w) * inv_neb));
        const double is_c = 100.0 * frcp(fmax(100.0, (double)sz_w * inv_nb));
        dinf = dinf_w; pinf = pinf_w; c0 = c0_w;
        STAMP(1);
        if (!lsm && fmax(dinf * is_d, fmax(pinf, c0 * is_c)) <= tol) { status = 0; break; }
        // -------- monotone barrier update (Fiacco-McCormick, may fire repeatedly) --
        // max_i |z_i s_i - mu| = max(max z s - mu, mu - min z s): one reduction pair, scalar loop
        for (; !lsm;) {
            const double cmu = fmax(c0 - mu, mu - cmin_w);
            if (fmax(dinf * is_d, fmax(pinf, cmu * is_c)) > 10.0 * mu || mu <= mu_min) break;
            mu = fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu)));
            nfilt = 0; in_soft = 0;       // BacktrackingLineSearch::Reset: the filter and the soft phase
        }
        const double tau = fmax(0.99, 1.0 - mu);
        STAMP(2);

        // -------- Newton step: Riccati recursion + inertia correction ---------------
        double be1[NAX], be2[NAX], E11[NAX], E12[NAX], E22[NAX], Rt0[NAX], rt[NAX], q1[NAX], q2[NAX];
#pragma unroll
        for (int j = 0; j < NAX; ++j) {
            be1[j] = b1 * cs[j]; be2[j] = b2 * cs[j];           // B_k = Gamma cos(theta_k); 0 on idle lanes
            E11[j] = be1[j] * be1[j]; E12[j] = 2.0 * be1[j] * be2[j]; E22[j] = be2[j] * be2[j];
            // Hessian of the Lagrangian in theta: 2R + lam_{k+1}^T Gamma sin(theta) + Sigma
            Rt0[j] = uon ? fma(sn[j], fma(b1, lpn[j], b2 * lvn[j]), r2 + zl[j] * isl[j] + zu[j] * isu[j]) : 1.0;
            // the barrier gradient in theta (least-square estimate: r_u = grad f - z_L + z_U)
            rt[j] = uon ? (lsm ? r2 * th[j] - zl[j] + zu[j] : fma(r2, th[j], mu * (isu[j] - isl[j]))) : 0.0;
            q1[j] = qp2 * (p[j] - rp[j]); q2[j] = qv2 * (v[j] - rv[j]);
        }
        double W1[NAX], W2[NAX], P11[NAX], P12[NAX], P22[NAX], iQs[NAX];
        double delta = 0.0;
        bool ok = false;
        int attempt = 0;
        for (; attempt < 60 && !ok; ++attempt) {
            if (PM_EXPECT(attempt > 0, 0))
                delta = (attempt == 1) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))   // IPOPT perturb_dec_fact 1/3
                                       : delta * (delta_last == 0.0 ? 100.0 : 8.0);
            const double X11d = lsm ? 1.0 : qp2 + delta, X22d = lsm ? 1.0 : qv2 + delta;
            double Quu[NAX], Rt[NAX];
#pragma unroll
            for (int j = 0; j < NAX; ++j) {      // terminal value function in every lane
                P11[j] = X11d; P12[j] = 0.0; P22[j] = X22d;
                Rt[j] = (lsm ? 1.0 : Rt0[j]) + delta;
            }
            // Quadratic part as a scan: with P = Y U^-1 the stage map P_k = X + A^T (P_{k+1}^-1 + G_k)^-1 A
            // (G_k = B_k B_k^T / R_k) is linear on [U; Y]: [U; Y]_k = S_k [U; Y]_{k+1},
            // S_k = [[A^-1, A^-1 G], [X A^-1, X A^-1 G + A^T]], so [U; Y]_k = S_k ... S_{N-1} [I; X]
            // is a suffix product (5 DPP levels).  Exact in the reals; in fp64 it matches the
            // sequential sweep to ~1e-15 while every stage is mildly stiff (B_k B_k^T X / R_k <= 2
            // per axis, checked here); otherwise, and for NAX == 2, the sequential sweep runs.
            bool use_scan = false;
            if constexpr (NAX == 1 && QSCAN) {
                const double ratio = fmax(E11[0] * X11d, E22[0] * X22d);
                use_scan = !wany(uon && !(Rt[0] > 0.0 && ratio <= 2.0 * Rt[0]));
            }
            STAMP_ADD(11, use_scan ? 1 : 0);
            if (PM_EXPECT(use_scan, 1)) {
                const double iR = uon ? frcp(Rt[0]) : 0.0;
                const double G11 = be1[0] * be1[0] * iR, G12 = be1[0] * be2[0] * iR, G22 = be2[0] * be2[0] * iR;
                const double g11 = G11 + ai12k * G12, g12 = G12 + ai12k * G22, g21 = ai22k * G12, g22 = ai22k * G22;
                // idle / terminal lanes: A^-1 = I, G = 0 (iR = 0), X = 0, A^T = I give T = I without a select
                const double X11k = X11d * uonf, X22k = X22d * uonf;
                double T[16] = {1.0, ai12k, g11, g12,
                                0.0, ai22k, g21, g22,
                                X11k, X11k * ai12k, fma(X11k, g11, 1.0), X11k * g12,
                                0.0, X22k * ai22k, fma(X22k, g21, a12k), fma(X22k, g22, a22i)};
                mat4_scan_level<0x101, true>(T);
                mat4_scan_level<0x102>(T);
                mat4_scan_level<0x104>(T);
                if constexpr (!short2 && !one_row) mat4_scan_level<0x108>(T);
                // [U; Y] = T [I; X] of the row-local suffix
                double W[8] = {fma(T[2], X11d, T[0]), fma(T[3], X22d, T[1]), fma(T[6], X11d, T[4]),
                               fma(T[7], X22d, T[5]), fma(T[10], X11d, T[8]), fma(T[11], X22d, T[9]),
                               fma(T[14], X11d, T[12]), fma(T[15], X22d, T[13])};
                if constexpr (short2 || one_row) {
                    // after 3 levels lane k holds S_k ... S_{min(k+7, row end)}: lanes 16-23 (48-55)
                    // already reach the terminal (N <= 23), lanes 8-15 the row end (and the terminal
                    // when N <= 15).  Lanes 8-15 compose with the 4 x 2 of lane 16 (ds_swizzle; not
                    // for N <= 15), then lanes 0-7 with that of lane k + 8 (DPP).  Lanes past the
                    // terminal hold [I; X], so a suffix that is already complete stays unchanged.
                    double F[8];
                    if constexpr (short2) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) F[e] = half_bcast_c<16>(W[e]);
                    if ((lane & 16) == 0) {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
#pragma unroll
                            for (int jj = 0; jj < 2; ++jj)
                                W[2 * i + jj] = fma(T[4 * i], F[jj], fma(T[4 * i + 1], F[2 + jj],
                                                    fma(T[4 * i + 2], F[4 + jj], T[4 * i + 3] * F[6 + jj])));
                    }
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) F[e] = dpp_fill<0x108, 0xf, 0>(W[e]);
                    if ((lane & 24) == 0) {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
#pragma unroll
                            for (int jj = 0; jj < 2; ++jj)
                                W[2 * i + jj] = fma(T[4 * i], F[jj], fma(T[4 * i + 1], F[2 + jj],
                                                    fma(T[4 * i + 2], F[4 + jj], T[4 * i + 3] * F[6 + jj])));
                    }
                } else if constexpr (!one_row && kWaves == 1) {
                    // rows 0 and 2 of each half: [U; Y]_k = T_k(row) [U; Y]_16, the 4 x 2 of lane 16 (48)
                    // fetched by ds_swizzle (bitmask mode, or_mask 16: no address, no LDS access)
                    double F[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) F[e] = half_bcast_c<16>(W[e]);
                    if ((lane & 16) == 0) {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
#pragma unroll
                            for (int jj = 0; jj < 2; ++jj)
                                W[2 * i + jj] = fma(T[4 * i], F[jj], fma(T[4 * i + 1], F[2 + jj],
                                                    fma(T[4 * i + 2], F[4 + jj], T[4 * i + 3] * F[6 + jj])));
                    }
                }
                double pnx[3] = {0.0, 0.0, 0.0};      // two waves: P_32 (wave 1's node 32) in wave 0
                if constexpr (kWaves == 2) {
                    // two waves (N >= 32, rows as above): wave 1's suffixes reach the terminal; wave 0's continue
                    // from the value function of node 32, [U; Y]_k = T_k(..31) [I; P_32] (exact in the reals, as the
                    // scan itself)
                    auto rows = [&]() {
                        double F[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) F[e] = half_bcast_c<16>(W[e]);
                        if ((lane & 16) == 0) {
#pragma unroll
                            for (int i = 0; i < 4; ++i)
#pragma unroll
                                for (int jj = 0; jj < 2; ++jj)
                                    W[2 * i + jj] = fma(T[4 * i], F[jj], fma(T[4 * i + 1], F[2 + jj],
                                                        fma(T[4 * i + 2], F[4 + jj], T[4 * i + 3] * F[6 + jj])));
                        }
                    };
                    double v[3] = {0.0, 0.0, 0.0}, pn[3];
                    if (wave_idx() == 1) {
                        rows();
                        const double idet = frcp(fma(W[0], W[3], -W[1] * W[2]));
                        v[0] = fma(W[4], W[3], -W[5] * W[2]) * idet;
                        v[1] = 0.5 * (fma(W[5], W[0], -W[4] * W[1]) * idet + fma(W[6], W[3], -W[7] * W[2]) * idet);
                        v[2] = fma(W[7], W[0], -W[6] * W[1]) * idet;
                    }
                    pm_pass<0>(1, 0, v, pn);
                    pnx[0] = pn[0]; pnx[1] = pn[1]; pnx[2] = pn[2];
                    if (wave_idx() == 0) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            W[2 * i] = fma(T[4 * i + 3], pn[1], fma(T[4 * i + 2], pn[0], T[4 * i]));
                            W[2 * i + 1] = fma(T[4 * i + 3], pn[2], fma(T[4 * i + 2], pn[1], T[4 * i + 1]));
                        }
                        rows();
                    }
                }
                // P = Y U^-1 (symmetrised)
                const double U11 = W[0], U12 = W[1], U21 = W[2], U22 = W[3];
                const double Y11 = W[4], Y12 = W[5], Y21 = W[6], Y22 = W[7];
                const double idet = frcp(fma(U11, U22, -U12 * U21));
                const double q11 = fma(Y11, U22, -Y12 * U21) * idet, q12 = fma(Y12, U11, -Y11 * U12) * idet;
                const double q21 = fma(Y21, U22, -Y22 * U21) * idet, q22 = fma(Y22, U11, -Y21 * U12) * idet;
                P11[0] = q11; P12[0] = 0.5 * (q12 + q21); P22[0] = q22;
                // the stage quantities of node k from P_{k+1}
                double n11, n12, n22;
                if constexpr (kWaves == 1) {
                    n11 = from_next(P11[0]); n12 = from_next(P12[0]); n22 = from_next(P22[0]);
                } else {
                    // two waves: node 32's value function is already in wave 0 (pnx), no exchange
                    n11 = dpp<kWaveShl1>(P11[0]); n12 = dpp<kWaveShl1>(P12[0]); n22 = dpp<kWaveShl1>(P22[0]);
                    if (wave_idx() == 0 && (lane & 31) == 31) { n11 = pnx[0]; n12 = pnx[1]; n22 = pnx[2]; }
                }
                const double e1 = be1[0], e2 = be2[0];
                const double Q = fma(E11[0], n11, fma(E12[0], n12, fma(E22[0], n22, Rt[0])));
                const double PB1 = fma(n11, e1, n12 * e2), PB2 = fma(n12, e1, n22 * e2);
                const double U1 = PB1, U2 = fma(PB1, a12k, PB2 * a22k);
                const double iQ = frcp(Q);
                W1[0] = iQ * U1; W2[0] = iQ * U2;
                Quu[0] = Q; iQs[0] = iQ;
            } else
            // backward sweep: every lane maps its neighbour's value function through its own
            // stage; after step j lane N-1-j is final.  Terminal/idle lanes have Phi = 0, B = 0.
            for (int step = 0; step < N; ++step) {
                double n11[NAX], n12[NAX], n22[NAX];
#pragma unroll
                for (int j = 0; j < NAX; ++j) {
                    n11[j] = from_next(P11[j]); n12[j] = from_next(P12[j]); n22[j] = from_next(P22[j]);
                }
#pragma unroll
                for (int j = 0; j < NAX; ++j) {
                    const double e1 = be1[j], e2 = be2[j];
                    const double Q = fma(E11[j], n11[j], fma(E12[j], n12[j], fma(E22[j], n22[j], Rt[j])));
                    const double PB1 = fma(n11[j], e1, n12[j] * e2), PB2 = fma(n12[j], e1, n22[j] * e2);
                    const double U1 = PB1, U2 = fma(PB1, a12k, PB2 * a22k);
                    const double X12 = fma(n11[j], a12k, n12[j] * a22k);
                    const double X22 = fma(A11k, n11[j], fma(A12k, n12[j], fma(A22k, n22[j], X22d)));
                    const double iQ = frcp(Q);
                    const double w1 = iQ * U1, w2 = iQ * U2;
                    P11[j] = fma(-w1, U1, fma(f11, n11[j], X11d));
                    P12[j] = fma(-w1, U2, X12);
                    P22[j] = fma(-w2, U2, X22);
                    W1[j] = w1; W2[j] = w2;
                    Quu[j] = Q; iQs[j] = iQ;
                }
            }
            bool bad = false;
#pragma unroll
            for (int j = 0; j < NAX; ++j) bad = bad || !(Quu[j] > 0.0) || !isfinite(Quu[j]);
            ok = !wany(bad);
        }
        STAMP_ADD(9, attempt);
        STAMP(3);
        if (PM_EXPECT(!ok, 0)) { status = -3; break; }
        if (delta > 0.0) delta_last = delta;

        // -------- the step for the constraint right-hand side (g1, g2, gz) ---------------
        // One call site serves the Newton step and IPOPT's second-order correction passes
        // (FilterLSAcceptor::TrySecondOrderCorrection, kappa_soc 0.99): a correction re-solves the
        // factorised system with c_soc <- alpha_soc c_soc + c(x_trial) (from c(x), alpha_soc = alpha)
        // in place of the defects, so while it runs g1 / g2 / gz hold c_soc.
        double dp[NAX], dv[NAX], dth[NAX], dlp[NAX], dlv[NAX], dzl[NAX], dzu[NAX], dz[NAX];
        double amax = 1.0, az = 1.0;
        float am_lf = 1.0f, az_lf = 1.0f;     // this lane's fractions to the boundary (the wave minima: amax, az)
        const double (&g1o)[NAX] = g1, (&g2o)[NAX] = g2, (&gzo)[NAX] = gz;
        auto direction = [&]() {
            double p1[NAX], p2[NAX], kff[NAX], gn1[NAX], gn2[NAX], g1[NAX], g2[NAX], gz[NAX];
#pragma unroll
            for (int j = 0; j < NAX; ++j) {      // right-hand side: the defects (0 for the multiplier estimate)
                g1[j] = lsm ? 0.0 : g1o[j]; g2[j] = lsm ? 0.0 : g2o[j]; gz[j] = lsm ? 0.0 : gzo[j];
            }
            double nPw[3];       // two waves: P_{k+1} fetched with g_{k+1} in one exchange
            if constexpr (kWaves == 1) {
#pragma unroll
                for (int j = 0; j < NAX; ++j) { gn1[j] = from_next(g1[j]); gn2[j] = from_next(g2[j]); }
            } else {
                const double x5[5] = {g1[0], g2[0], P11[0], P12[0], P22[0]};
                double o5[5];
                from_next_n(x5, o5);
                gn1[0] = o5[0]; gn2[0] = o5[1]; nPw[0] = o5[2]; nPw[1] = o5[3]; nPw[2] = o5[4];
            }
            if constexpr (NAX == 1) {
                // linear part of the value function, p_k = M_k p_{k+1} + m_k with M_k = A_k^T - w_k e_k^T
                // and m_k = q_k - w_k rt_k - M_k P_{k+1} g_{k+1}: a suffix scan of affine maps (row_shl
                // 1/2/4/8 inside the rows, then row 1 -> row 0 of each half by a lane shuffle); the
                // terminal/idle lanes carry M = 0, so each suffix stops at node N
                const double e1 = be1[0], e2 = be2[0], w1 = W1[0], w2 = W2[0];
                const double nP11 = kWaves == 1 ? from_next(P11[0]) : nPw[0];
                const double nP12 = kWaves == 1 ? from_next(P12[0]) : nPw[1];
                const double nP22 = kWaves == 1 ? from_next(P22[0]) : nPw[2];
                const double t1 = fma(nP11, gn1[0], nP12 * gn2[0]), t2 = fma(nP12, gn1[0], nP22 * gn2[0]);
                double m11 = fma(-w1, e1, f11), m12 = -w1 * e2, m21 = fma(-w2, e1, a12k), m22 = fma(-w2, e2, a22k);
                const double rtk = rt[0];
                double c1 = fma(-w1, rtk, q1[0]) - fma(m11, t1, m12 * t2);
                double c2 = fma(-w2, rtk, q2[0]) - fma(m21, t1, m22 * t2);
                double p32[2] = {0.0, 0.0};      // two waves: p of node 32 (wave 1) in wave 0
                (void)p32;
                affine_scan_level<0x101, 0xf>(m11, m12, m21, m22, c1, c2);   // row_shl:1
                affine_scan_level<0x102, 0xf>(m11, m12, m21, m22, c1, c2);   // row_shl:2
                affine_scan_level<0x104, 0xf>(m11, m12, m21, m22, c1, c2);   // row_shl:4
                if constexpr (short2 || one_row) {
                    // N <= 23: lanes 16-23 (48-55) are final after 3 levels; lanes 8-15 compose with the
                    // constant of lane 16 (N <= 15: already final), then lanes 0-7 with the (final)
                    // constant of lane k + 8
                    if constexpr (short2) {
                        const double r1 = half_bcast_c<16>(c1), r2 = half_bcast_c<16>(c2);
                        if ((lane & 24) == 8) {
                            c1 = fma(m11, r1, fma(m12, r2, c1));
                            c2 = fma(m21, r1, fma(m22, r2, c2));
                        }
                    }
                    const double s1 = dpp_fill<0x108, 0xf, 0>(c1), s2 = dpp_fill<0x108, 0xf, 0>(c2);
                    if ((lane & 24) == 0) {
                        c1 = fma(m11, s1, fma(m12, s2, c1));
                        c2 = fma(m21, s1, fma(m22, s2, c2));
                    }
                } else {
                    affine_scan_level<0x108, 0xf>(m11, m12, m21, m22, c1, c2);   // row_shl:8
                    // rows 0 and 2 compose with the suffix held by the first lane of rows 1 and 3
                    const bool lo_row = (lane & 16) == 0;
                    if constexpr (kWaves == 1) {
                        const double r1 = half_bcast_c<16>(c1), r2 = half_bcast_c<16>(c2);   // only the constant is needed now
                        if (lo_row) {
                            c1 = fma(m11, r1, fma(m12, r2, c1));
                            c2 = fma(m21, r1, fma(m22, r2, c2));
                        }
                    } else {
                        auto rows = [&]() {
                            const double r1 = half_bcast_c<16>(c1), r2 = half_bcast_c<16>(c2);
                            if (lo_row) {
                                c1 = fma(m11, r1, fma(m12, r2, c1));
                                c2 = fma(m21, r1, fma(m22, r2, c2));
                            }
                        };
                        // two waves: wave 0's rows 1 / 3 (their maps span nodes k..31) continue from p_32 of wave 1
                        if (wave_idx() == 1) rows();
                        double r[2];
                        { const double v[2] = {c1, c2}; pm_pass<1>(1, 0, v, r); }
                        p32[0] = r[0]; p32[1] = r[1];
                        if (wave_idx() == 0) {
                            if (!lo_row) {
                                c1 = fma(m11, r[0], fma(m12, r[1], c1));
                                c2 = fma(m21, r[0], fma(m22, r[1], c2));
                            }
                            rows();
                        }
                    }
                }
                p1[0] = c1; p2[0] = c2;
                // feed-forward k_k = -(e^T h + rt) / Q with h = p_{k+1} - P_{k+1} g_{k+1}
                double np1, np2;
                if constexpr (kWaves == 1) {
                    np1 = from_next(c1); np2 = from_next(c2);
                } else {
                    // two waves: node 32's p is already in wave 0 (p32), no exchange
                    np1 = dpp<kWaveShl1>(c1); np2 = dpp<kWaveShl1>(c2);
                    if (wave_idx() == 0 && (lane & 31) == 31) { np1 = p32[0]; np2 = p32[1]; }
                }
                const double h1 = np1 - t1, h2 = np2 - t2;
                kff[0] = -iQs[0] * fma(e1, h1, fma(e2, h2, rtk));

                // forward sweep of the state step: dx_k = F_{k-1} dx_{k-1} + f_{k-1} - g_k as an
                // inclusive scan of affine maps within each 32-lane axis half (DPP row_shr 1/2/4/8 inside
                // the 16-lane rows, then row_bcast:15 into the second row of each half)
                double pw1, pw2, pkf, pb1, pb2;
                if constexpr (kWaves == 1) {
                    pw1 = from_prev(W1[0]); pw2 = from_prev(W2[0]); pkf = from_prev(kff[0]);
                    pb1 = from_prev(be1[0]); pb2 = from_prev(be2[0]);
                } else {
                    const double x5[5] = {W1[0], W2[0], kff[0], be1[0], be2[0]};
                    double o5[5];
                    from_prev_n(x5, o5);
                    pw1 = o5[0]; pw2 = o5[1]; pkf = o5[2]; pb1 = o5[3]; pb2 = o5[4];
                }
                double f11_ = 1.0 - pb1 * pw1, f12_ = fma(-pb1, pw2, a12), f21_ = -pb2 * pw1, f22_ = fma(-pb2, pw2, a22);
                double d1 = fma(pb1, pkf, -g1[0]), d2 = fma(pb2, pkf, -g2[0]);
                if (k == 0) { f11_ = 0.0; f12_ = 0.0; f21_ = 0.0; f22_ = 0.0; d1 = -g1[0]; d2 = -g2[0]; }
                affine_scan_level<0x111, 0xf>(f11_, f12_, f21_, f22_, d1, d2);   // row_shr:1
                affine_scan_level<0x112, 0xf>(f11_, f12_, f21_, f22_, d1, d2);   // row_shr:2
                affine_scan_level<0x114, 0xf>(f11_, f12_, f21_, f22_, d1, d2);   // row_shr:4
                // after 3 levels the windows of lanes 0-7 reach node 0 (map 0, a constant): with N <= 23
                // the row_shr:8 level only moves constants (row 1's lanes 16-23 read nothing); lane 15 is
                // a constant once row 0 is done, so the row_bcast:15 level into rows 1 / 3 is one too
                if constexpr (one_row || short2) affine_scan_const<0x118, 0xf>(f11_, f12_, f21_, f22_, d1, d2);
                else affine_scan_level<0x118, 0xf>(f11_, f12_, f21_, f22_, d1, d2);   // row_shr:8
                if constexpr (kWaves == 1) {
                    if constexpr (!one_row) affine_scan_const<0x142, 0xa>(f11_, f12_, f21_, f22_, d1, d2);   // row_bcast:15 -> rows 1, 3
                } else {
                    // two waves: wave 1's rows 0 / 2 (their maps span nodes 32..k) continue from dx_31 of wave 0
                    if (wave_idx() == 0) affine_scan_const<0x142, 0xa>(f11_, f12_, f21_, f22_, d1, d2);
                    double r[2];
                    { const double v[2] = {d1, d2}; pm_pass<2>(0, 31, v, r); }
                    if (wave_idx() == 1) {
                        if ((lane & 16) == 0) {
                            d1 = fma(f11_, r[0], fma(f12_, r[1], d1));
                            d2 = fma(f21_, r[0], fma(f22_, r[1], d2));
                        }
                        affine_scan_const<0x142, 0xa>(f11_, f12_, f21_, f22_, d1, d2);
                    }
                }
                dp[0] = d1; dv[0] = d2;
            } else {
                // linear part of the value function (sequential): p_k = q_k + A_k^T h - w_k (e^T h + rt)
                double nP11[NAX], nP12[NAX], nP22[NAX];
#pragma unroll
                for (int j = 0; j < NAX; ++j) {
                    nP11[j] = from_next(P11[j]); nP12[j] = from_next(P12[j]); nP22[j] = from_next(P22[j]);
                    p1[j] = q1[j]; p2[j] = q2[j]; kff[j] = 0.0;
                }
                for (int step = 0; step < N; ++step) {
                    double n1[NAX], n2[NAX];
#pragma unroll
                    for (int j = 0; j < NAX; ++j) { n1[j] = from_next(p1[j]); n2[j] = from_next(p2[j]); }
#pragma unroll
                    for (int j = 0; j < NAX; ++j) {
                        const double h1 = n1[j] - fma(nP11[j], gn1[j], nP12[j] * gn2[j]);
                        const double h2 = n2[j] - fma(nP12[j], gn1[j], nP22[j] * gn2[j]);
                        const double qu = fma(be1[j], h1, fma(be2[j], h2, rt[j]));
                        kff[j] = -iQs[j] * qu;
                        p1[j] = fma(-W1[j], qu, fma(f11, h1, q1[j]));
                        p2[j] = fma(-W2[j], qu, q2[j] + fma(a12k, h1, a22k * h2));
                    }
                }
#pragma unroll
                for (int j = 0; j < NAX; ++j) { dp[j] = -g1[j]; dv[j] = -g2[j]; }
                for (int step = 0; step < N; ++step) {
                    double op[NAX], ov[NAX];
#pragma unroll
                    for (int j = 0; j < NAX; ++j) {
                        const double dt_ = fma(-W1[j], dp[j], fma(-W2[j], dv[j], kff[j]));
                        op[j] = fma(a12, dv[j], fma(be1[j], dt_, dp[j]));
                        ov[j] = fma(a22, dv[j], be2[j] * dt_);
                    }
#pragma unroll
                    for (int j = 0; j < NAX; ++j) {
                        const double ip = from_prev(op[j]), iv = from_prev(ov[j]);
                        dp[j] = k >= 1 ? ip - g1[j] : dp[j];
                        dv[j] = k >= 1 ? iv - g2[j] : dv[j];
                    }
                }
            }
            double am = 1.0, az_ = 1.0, twd[NAX];
#pragma unroll
            for (int j = 0; j < NAX; ++j) {
                dth[j] = uon ? fma(-W1[j], dp[j], fma(-W2[j], dv[j], kff[j])) : 0.0;
                // new multipliers lam+ = -(P dx + p), step = lam+ - lam
                dlp[j] = xon ? -fma(P11[j], dp[j], fma(P12[j], dv[j], p1[j])) - lp[j] : 0.0;
                dlv[j] = xon ? -fma(P12[j], dp[j], fma(P22[j], dv[j], p2[j])) - lv[j] : 0.0;
                const double sl = th[j] - lo, su = hi - th[j];
                const double zlx = zl[j] * isl[j], zux = zu[j] * isu[j];
                dzl[j] = uon ? fma(-zlx, dth[j], fma(mu, isl[j], -zl[j])) : 0.0;
                dzu[j] = uon ? fma(zux, dth[j], fma(mu, isu[j], -zu[j])) : 0.0;
                const double ith = frcp(dth[j]);
                const double cand = dth[j] < 0 ? -tau * sl * ith : (dth[j] > 0 ? tau * su * ith : 1.0);
                const double czl = dzl[j] < 0 ? -tau * zl[j] * frcp(dzl[j]) : 1.0;
                const double czu = dzu[j] < 0 ? -tau * zu[j] * frcp(dzu[j]) : 1.0;
                am = fmin(am, uon ? cand : 1.0);
                az_ = fmin(az_, uon ? fmin(czl, czu) : 1.0);
                twd[j] = 2.0 * th[j] * dth[j];
            }
            // f32 minima rounded down (tau <= 0.99 leaves far more slack than the f32 rounding); reduced by the
            // caller (frac_minima, or with the line search's sums)
            am_lf = (float)am; az_lf = (float)az_;
            // z step: dz_k = zA dz_{k-1} + zC dw_{k-1} - gz_k, dw = -g (2 theta_x dtheta_x + 2 theta_y dtheta_y)
            const double wd = RED ? 0.0 : -a.g * axes_sum(twd);
            if constexpr (RED) {
#pragma unroll
                for (int j = 0; j < NAX; ++j) dz[j] = 0.0;
            } else if constexpr (NAX == 1) {
                const double src = from_prev(zC[0] * wd);
                double m = k == 0 ? 0.0 : zA[0], c = k == 0 ? -gz[0] : src - gz[0];
                affine1_scan_level<0x111, 0xf>(m, c);   // row_shr:1
                affine1_scan_level<0x112, 0xf>(m, c);   // row_shr:2
                affine1_scan_level<0x114, 0xf>(m, c);   // row_shr:4
                if constexpr (one_row || short2) affine1_scan_const<0x118, 0xf>(m, c);
                else affine1_scan_level<0x118, 0xf>(m, c);   // row_shr:8
                if constexpr (kWaves == 1) {
                    if constexpr (!one_row) affine1_scan_const<0x142, 0xa>(m, c);   // row_bcast:15 -> rows 1, 3
                } else {       // two waves: as the state sweep
                    if (wave_idx() == 0) affine1_scan_const<0x142, 0xa>(m, c);
                    double r[1];
                    { const double v[1] = {c}; pm_pass<3>(0, 31, v, r); }
                    if (wave_idx() == 1) {
                        if ((lane & 16) == 0) c = fma(m, r[0], c);
                        affine1_scan_const<0x142, 0xa>(m, c);
                    }
                }
                dz[0] = c;
            } else {
#pragma unroll
                for (int j = 0; j < NAX; ++j) dz[j] = -gz[j];
                for (int step = 0; step < N; ++step) {
#pragma unroll
                    for (int j = 0; j < NAX; ++j) {
                        const double ip = from_prev(fma(zA[j], dz[j], zC[j] * wd));
                        dz[j] = k >= 1 ? ip - gz[j] : dz[j];
                    }
                }
            }
        };

        // amax, az from this lane's fractions (f32 minima rounded down)
        auto frac_set = [&]() {
            amax = (double)am_lf * (1.0 - 1.0 / 1048576.0);
            az = (double)az_lf * (1.0 - 1.0 / 1048576.0);
        };

        // -------- filter line search (Waechter & Biegler 2006, Alg. A) with second-order correction
        double alpha = 1.0, amain = 1.0, th_t = 0.0, ph_t = 0.0, th_old = 0.0, phi = 0.0, gTd = 0.0, amin = 0.0;
        float lg_sw = 0.0f;
        bool accepted = false, ftype = false, tiny = false;
        int ls = 0, soc = 0;        // soc: 0 Newton step, 1.. correction pass, -1 Newton step again after failed passes
        double snt[NAX], g1t[NAX], g2t[NAX], gzt[NAX];     // the trial's sines and defects (carried on acceptance)
        // trial point x + al d: defects, wave-summed theta and barrier objective
        auto trial = [&](double al) {
            double thl = 0.0, phl = 0.0, tt[NAX];
            if constexpr (kWaves == 2 && NAX == 1 && !RED) {
                // two waves: the three node shifts of the trial's defects (defects, zdefect) in one exchange
                const double pt = fma(al, dp[0], p[0]), vt = fma(al, dv[0], v[0]);
                tt[0] = fma(al, dth[0], th[0]);
                double s_, c_;
                tilt_sincos(poly, tt[0], s_, c_);
                snt[0] = uon ? s_ : 0.0;
                const double wt = vz_new(tt);
                const double zt = fma(al, dz[0], zz[0]);
                const double x3[3] = {fma(a12, vt, fma(b1, snt[0], pt)), fma(a22, vt, b2 * snt[0]),
                                      fma(zA[0], zt, zC[0] * wt)};
                double o3[3];
                from_prev_n(x3, o3);
                g1t[0] = (k == 0) ? pt - sp[0] : pt - o3[0];
                g2t[0] = (k == 0) ? vt - sv[0] : vt - o3[1];
                gzt[0] = (k == 0) ? zt - zs[0] : zt - o3[2];
                const double ep = pt - rp[0], ev = vt - rv[0];
                thl += xon ? fabs(g1t[0]) + fabs(g2t[0]) : 0.0;
                phl += xon ? fma(scQp * ep, ep, scQv * ev * ev) : 0.0;
                phl += uon ? fma(scR * tt[0], tt[0], -mu * log_fast((tt[0] - lo) * (hi - tt[0]))) : 0.0;
                thl += xon ? fabs(gzt[0]) : 0.0;
                wsum2(thl, phl);
                th_t = thl; ph_t = phl;
                return;
            }
#pragma unroll
            for (int j = 0; j < NAX; ++j) {
                const double pt = fma(al, dp[j], p[j]), vt = fma(al, dv[j], v[j]);
                tt[j] = fma(al, dth[j], th[j]);
                double s_, c_;
                tilt_sincos(poly, tt[j], s_, c_);
                snt[j] = uon ? s_ : 0.0;
                defects(pt, vt, snt[j], sp[j], sv[j], g1t[j], g2t[j]);
                const double ep = pt - rp[j], ev = vt - rv[j];
                thl += xon ? fabs(g1t[j]) + fabs(g2t[j]) : 0.0;
                phl += xon ? fma(scQp * ep, ep, scQv * ev * ev) : 0.0;
                phl += uon ? fma(scR * tt[j], tt[j], -mu * log_fast((tt[j] - lo) * (hi - tt[j]))) : 0.0;
            }
            if constexpr (RED) {
#pragma unroll
                for (int j = 0; j < NAX; ++j) gzt[j] = 0.0;
            } else {
                const double wt = vz_new(tt);
#pragma unroll
                for (int j = 0; j < NAX; ++j) {
                    gzt[j] = zdefect(fma(al, dz[j], zz[j]), wt, j);
                    thl += xon ? fabs(gzt[j]) : 0.0;
                }
            }
            wsum2(thl, phl);
            th_t = thl; ph_t = phl;
        };
        // filter acceptance of (th_t, ph_t) for the step size al_test (IPOPT alpha_primal_test)
        auto acceptable = [&](double al_test, bool& ft) {
            bool in_filter = !(th_t < th_max) || !isfinite(ph_t);
            in_filter = in_filter || wany_rep(lane < nfilt && th_t >= fth && ph_t >= fph);   // (replicated filter)
            if (in_filter) return false;
            const bool sw = gTd < 0.0 && lg2(al_test) > lg_sw;
            if (theta <= th_min && sw) {
                if (cmp_le(ph_t, phi + eta_ph * al_test * gTd, phi)) { ft = true; return true; }
                return false;
            }
            return cmp_le(th_t, (1 - gam_th) * theta, theta) || cmp_le(ph_t - phi, -gam_ph * theta, phi);
        };
        if (PM_EXPECT(lsm, 0)) {
            direction();
            // constr_mult_init_max: an estimate larger than it (max norm) is discarded (multipliers 0)
            double ym = 0.0;
#pragma unroll
            for (int j = 0; j < NAX; ++j) ym = fmax(ym, xon ? fmax(fabs(dlp[j]), fabs(dlv[j])) : 0.0);
            if (wmax(ym) <= a.mult_init_max) {
#pragma unroll
                for (int j = 0; j < NAX; ++j) { lp[j] += dlp[j]; lv[j] += dlv[j]; }
            }
            continue;
        }
        for (;;) {
            direction();
            if (PM_EXPECT(soc != 0, 0)) { wmin2f(am_lf, az_lf); frac_set(); }
            STAMP(4);
            if (PM_EXPECT(soc == 0, 1)) {
                double phil = 0.0, gtdl = 0.0;
#pragma unroll
                for (int j = 0; j < NAX; ++j) {
                    const double ep = p[j] - rp[j], ev = v[j] - rv[j];
                    const double sl = th[j] - lo, su = hi - th[j];
                    phil += xon ? fma(scQp * ep, ep, scQv * ev * ev) : 0.0;
                    gtdl += xon ? fma(qp2 * ep, dp[j], qv2 * ev * dv[j]) : 0.0;
                    phil += uon ? fma(scR * th[j], th[j], -mu * log_fast(sl * su)) : 0.0;
                    gtdl += uon ? rt[j] * dth[j] : 0.0;
                }
                // IPOPT's tiny-step test (max |d|/(1+|x|) < 10 eps_mach accepts the full step unfiltered): its maximum
                // rides with the two sums (one lock-step reduction; two waves: one exchange)
                float tn_w = 0.0f;
#pragma unroll
                for (int j = 0; j < NAX; ++j) {
                    tn_w = fmaxf(tn_w, xon ? fabsf((float)dp[j]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)p[j])) : 0.0f);
                    tn_w = fmaxf(tn_w, xon ? fabsf((float)dv[j]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)v[j])) : 0.0f);
                    tn_w = fmaxf(tn_w, xon ? fabsf((float)dz[j]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)zz[j])) : 0.0f);
                    tn_w = fmaxf(tn_w, uon ? fabsf((float)dth[j]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)th[j])) : 0.0f);
                }
                wsum2_maxf_min2f(phil, gtdl, tn_w, am_lf, az_lf);      // (the fraction minima ride along)
                frac_set();
                phi = phil; gTd = gtdl;
                // switching condition alpha (-gTd)^s_ph > delta theta^s_th, compared in log2 space
                const float lg_th = theta > 0.0 ? lg2(theta) : -3.0e38f;
                const float lg_gd = gTd < 0.0 ? lg2(-gTd) : 3.0e38f;
                lg_sw = (float)s_th * lg_th - (float)s_ph * lg_gd;    // log2(theta^s_th / (-gTd)^s_ph)
                amin = gam_th;
                if (gTd < 0.0) amin = fmin(gam_th, fmin(gam_ph * theta * frcp(-gTd), (double)__builtin_amdgcn_exp2f(fmaxf(lg_sw, -126.0f))));
                amin *= gam_al;
                tiny = tn_w < 2.2e-15f;
                alpha = amax; amain = amax;
            } else if (soc > 0) {
                alpha = amax;                 // alpha_soc: fraction to the boundary of the corrected step
            }
            STAMP(5);
            bool again = false;
            if constexpr ((NAX == 2 || kWaves == 2) && !RED) {
                if (PM_EXPECT(in_soft, 0)) break;      // in the soft restoration phase: its step only (below)
                if (PM_EXPECT(soc < 0 && alpha < amin, 0)) break;
            }
            for (;;) {
                trial(alpha);
                bool ft = false;
                if (PM_EXPECT(soc == 0 && tiny, 0)) { accepted = true; ftype = true; break; }
                if (acceptable(soc > 0 ? amain : alpha, ft)) { accepted = true; ftype = ft; break; }
                if (PM_EXPECT(!RED && soc == 0 && ls == 0 && a.max_soc > 0 && !(th_t < theta), 0)) {
                    // first correction: c_soc = alpha c(x) + c(x_trial)
#pragma unroll
                    for (int j = 0; j < NAX; ++j) {
                        g1[j] = fma(alpha, g1[j], g1t[j]); g2[j] = fma(alpha, g2[j], g2t[j]);
                        gz[j] = fma(alpha, gz[j], gzt[j]);
                    }
                    th_old = th_t; soc = 1; again = true;
                    break;
                }
                if (PM_EXPECT(soc > 0, 0)) {
                    if (soc < a.max_soc && th_t <= 0.99 * th_old) {      // next pass: c_soc <- alpha_soc c_soc + c(trial)
#pragma unroll
                        for (int j = 0; j < NAX; ++j) {
                            g1[j] = fma(alpha, g1[j], g1t[j]); g2[j] = fma(alpha, g2[j], g2t[j]);
                            gz[j] = fma(alpha, gz[j], gzt[j]);
                        }
                        th_old = th_t; ++soc; again = true;
                        break;
                    }
                    // the corrections failed: the defects of the current point back (the same
                    // arithmetic as their first evaluation), the Newton step again, backtrack from alpha/2
                    const double w0 = RED ? 0.0 : vz_new(th);
#pragma unroll
                    for (int j = 0; j < NAX; ++j) {
                        defects(p[j], v[j], snc[j], sp[j], sv[j], g1[j], g2[j]);
                        gz[j] = RED ? 0.0 : zdefect(zz[j], w0, j);
                    }
                    // (NAX == 2 or two waves, the soft phase below: always through the loop top, so that a line search that fails
                    // here leaves the plain step in the direction registers; alpha < amin stops it there)
                    soc = -1; ls = 1; alpha = 0.5 * amain;
                    again = ((NAX == 2 || kWaves == 2) && !RED) || !(alpha < amin);
                    break;
                }
                ++ls;
                alpha *= 0.5;
                if (alpha < amin || ls >= 80) break;
            }
            if (!again) break;
        }
        STAMP_ADD(10, ls + 1);
        STAMP_ADD(15, soc > 0 ? 1 : 0);
        STAMP(6);
        // A failed line search: IPOPT's soft restoration phase here (BacktrackingLineSearch::TrySoftRestoStep;
        // oracle/pmpc_ipm.c soft_resto_step), then, if it cannot proceed, the restoration phase proper in
        // pmpc_resto_solve (or status -2 without the phases).  The soft step is the plain primal-dual step damped
        // only by the fractions to the boundary (one length for x, lambda and z); it is taken if the original
        // filter accepts it with alpha_primal_test = 0 (the phase ends) or if it cuts IPOPT's primal-dual system
        // error at mu (the l1 norms of the primal and dual infeasibilities and of z s - mu, added) by 0.9999; at most
        // 10 such steps, and a mu decrease ends the phase.  Only for N > 31 (NAX == 2, two waves), where the restoration solve
        // on the LDS engine (pmpc_resto.h) does not fit: at the default options every PMPC line-search failure there
        // is settled in the soft phase (N = 40: 41 of C4's 1152 instances), which round 4 ended at -2.  For N <= 31
        // the handed-over instance is solved again on the LDS engine, whose sequential arithmetic takes the oracle's
        // iterations exactly; run here, the soft phase measured 87-93 % equal iteration counts on the restored
        // instances and cost C2 5 % (its register allocation; profiles/r05/pmpc_soft_in_register_kernel.txt).
        bool soft = false;
        if (PM_EXPECT(!accepted, 0)) {
            if constexpr (!RED && (NAX == 2 || kWaves == 2)) {
                if (a.soft) {
                    if (!in_soft) {       // PrepareRestoPhaseStart: the current point enters the filter
                        if (nfilt < kWave) {
                            if (lane == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
                            ++nfilt;
                        }
                        soft_count = 0;
                    }
                    if (!(in_soft && ++soft_count > 10)) {
                        // the fractions to the boundary of the plain step in f64 (the line search's f32 minima
                        // are rounded down by up to 2^-20; a soft step takes them whole, so they are formed exactly)
                        double am = 1.0, a2 = 1.0;
#pragma unroll
                        for (int j = 0; j < NAX; ++j) {
                            if (uon) {
                                const double sl = th[j] - lo, su = hi - th[j];
                                if (dth[j] < 0) am = fmin(am, -tau * sl / dth[j]);
                                if (dth[j] > 0) am = fmin(am, tau * su / dth[j]);
                                if (dzl[j] < 0) a2 = fmin(a2, -tau * zl[j] / dzl[j]);
                                if (dzu[j] < 0) a2 = fmin(a2, -tau * zu[j] / dzu[j]);
                            }
                        }
                        const double as = fmin(wmin(am), wmin(a2));
                        trial(as);
                        bool ft_ = false;
                        const bool orig = acceptable(0.0, ft_);
                        bool take = orig;
                        if (!take && isfinite(ph_t)) {
                            // the primal-dual system error at the point (pass 0) and at the trial with every
                            // multiplier moved by as (pass 1); one code site for both
                            double pd[2];
#pragma unroll 1
                            for (int pass = 0; pass < 2; ++pass) {
                                const double sa = pass ? as : 0.0;
                                double t = 0.0;
#pragma unroll
                                for (int j = 0; j < NAX; ++j) {
                                    const double pp = fma(sa, dp[j], p[j]), vv = fma(sa, dv[j], v[j]);
                                    const double tt = fma(sa, dth[j], th[j]);
                                    const double lpv = fma(sa, dlp[j], lp[j]), lvv = fma(sa, dlv[j], lv[j]);
                                    const double zlv = uon ? fma(sa, dzl[j], zl[j]) : 0.0;
                                    const double zuv = uon ? fma(sa, dzu[j], zu[j]) : 0.0;
                                    const double ga = pass ? g1t[j] : g1[j], gb = pass ? g2t[j] : g2[j];
                                    const double gc = pass ? gzt[j] : gz[j];
                                    const double ln = from_next(lpv), vn = from_next(lvv);
                                    const double lpn_ = uon ? ln : 0.0, lvn_ = uon ? vn : 0.0;
                                    const double r1 = fma(qp2, pp - rp[j], lpv - lpn_);
                                    const double r2x = fma(qv2, vv - rv[j], lvv - fma(a12, lpn_, a22 * lvn_));
                                    const double c_ = tilt_cos_econ(poly, tt);
                                    const double ru = fma(r2, tt, -c_ * fma(b1, lpn_, b2 * lvn_)) - zlv + zuv;
                                    const double sl = tt - lo, su = hi - tt;
                                    t += xon ? fabs(r1) + fabs(r2x) + fabs(ga) + fabs(gb) + fabs(gc) : 0.0;
                                    t += uon ? fabs(ru) + fabs(zlv * sl - mu) + fabs(zuv * su - mu) : 0.0;
                                }
                                pd[pass] = wsum(t);
                            }
                            take = pd[1] <= 0.9999 * pd[0];
                        }
                        if (take) {
                            accepted = true; soft = true; alpha = as; az = as;
                            in_soft = orig ? 0 : 1;
                            if (orig) soft_count = 0;
                        }
                    }
                }
            }
            if (!accepted) { status = a.resto ? kPmNeedResto : -2; break; }
        }
        if (!soft && !ftype && nfilt < kWave) {
            if (lane == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
            ++nfilt;
        }
        // -------- accept the step ----------------------------------------------------
#pragma unroll
        for (int j = 0; j < NAX; ++j) {
            snc[j] = snt[j]; g1[j] = g1t[j]; g2[j] = g2t[j]; gz[j] = gzt[j];
            p[j] = fma(alpha, dp[j], p[j]); v[j] = fma(alpha, dv[j], v[j]);
            zz[j] = fma(alpha, dz[j], zz[j]);
            lp[j] = fma(alpha, dlp[j], lp[j]); lv[j] = fma(alpha, dlv[j], lv[j]);
            th[j] = fma(alpha, dth[j], th[j]);
            const double il = frcp(th[j] - lo), iu = frcp(hi - th[j]);
            const double zln = fmax(fmin(fma(az, dzl[j], zl[j]), 1e10 * mu * il), 1e-10 * mu * il);   // kappa_sigma
            const double zun = fmax(fmin(fma(az, dzu[j], zu[j]), 1e10 * mu * iu), 1e-10 * mu * iu);
            zl[j] = uon ? zln : 0.0; zu[j] = uon ? zun : 0.0;
        }
        theta = th_t;
        STAMP(7);
    }

    // -------- outputs ---------------------------------------------------------------
    if (PM_EXPECT(status == kPmNeedResto, 0)) {     // handed over: pmpc_resto_solve writes the outputs
        if constexpr (NAX == 1 && kWaves == 1 && !RED) {
            if (a.resto_buf) {      // the iterate of the failed iteration (pmpc_model.h kPmHo layout)
                double* ho = a.resto_buf + (size_t)kPmHo * b;
                double* row = ho + kPmHoRow * k;
                if (xon) {
                    row[2 * ax0] = p[0]; row[2 * ax0 + 1] = v[0]; row[4 + ax0] = zz[0];
                    row[8 + 2 * ax0] = lp[0]; row[8 + 2 * ax0 + 1] = lv[0]; row[8 + 4 + ax0] = 0.0;
                }
                if (uon) { row[6 + ax0] = th[0]; row[14 + ax0] = zl[0]; row[16 + ax0] = zu[0]; }
                if (lane < nfilt) { ho[kPmHoFilt + 2 * lane] = fth; ho[kPmHoFilt + 2 * lane + 1] = fph; }
                if (lane == 0) {
                    ho[kPmHoScal] = mu; ho[kPmHoScal + 1] = delta_last;
                    ho[kPmHoScal + 2] = (double)it; ho[kPmHoScal + 3] = (double)nfilt;
                }
            }
        }
        if (lane == 0 && wave_idx() == 0) a.status[b] = status;
        if (a.done && a.resto == 2) {
            __threadfence_system();
            if (lane == 0) __hip_atomic_store(a.done + b, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return true;
    }
    // objective (mpc_3d.py:44-46, :63-66), unscaled
    double fl = 0.0;
#pragma unroll
    for (int j = 0; j < NAX; ++j) {
        const double ep = p[j] - rp[j], ev = v[j] - rv[j];
        fl += xon ? Qp * ep * ep + Qv * ev * ev : 0.0;
        fl += uon ? R * th[j] * th[j] : 0.0;
    }
    const double fval = wsum(fl);
    // theta_x and theta_y of this lane's node
    double tx, ty;
    if (NAX == 1) {
        const double other = __shfl_xor(th[0], 32);
        tx = ax0 == 0 ? th[0] : other;
        ty = ax0 == 0 ? other : th[0];
    } else {
        tx = th[0]; ty = th[NAX - 1];
    }
    if (lane == 0 && wave_idx() == 0) {
        a.u0[2 * b] = tx;
        a.u0[2 * b + 1] = ty;
        a.f[b] = fval;
        a.status[b] = status;
        a.iters[b] = it;
    }
    if (a.w_out) {
        double* wo = a.w_out + (size_t)nw * b;
        if constexpr (RED) {
            // the z sub-state follows the final controls through the reference RK4 (mpc_3d.py:93-97, :99-104)
            const double w = uon ? -a.g * (tx * tx + ty * ty) : 0.0;
            double pz = st[4], vz = st[5];
            for (int step = 0; step < N; ++step) {
                double pzn, vzn;
                z_rk4(h, w, pz, vz, pzn, vzn);
                const double ip = from_prev(pzn), iv = from_prev(vzn);
                pz = k >= 1 ? ip : pz; vz = k >= 1 ? iv : vz;
            }
#pragma unroll
            for (int j = 0; j < NAX; ++j) zz[j] = (NAX == 1 ? ax0 : j) ? vz : pz;
        }
#pragma unroll
        for (int j = 0; j < NAX; ++j) {
            const int ax = NAX == 1 ? ax0 : j;
            if (xon) { wo[6 * k + 2 * ax] = p[j]; wo[6 * k + 2 * ax + 1] = v[j]; wo[6 * k + 4 + ax] = zz[j]; }
            if (uon) wo[6 * (N + 1) + 2 * k + ax] = th[j];
        }
    }
    if (a.done) {
        // release at system scope: the wave's output stores (any lane) are visible before the word
        __threadfence_system();
        if constexpr (kWaves == 2) __syncthreads();       // and those of the other wave
        if (lane == 0 && wave_idx() == 0) __hip_atomic_store(a.done + b, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    STAMP(8);
    STAMP_FLUSH(b);
    return false;
}

// IPOPT's restoration phases for instance b in the wave that handed it over (resto mode 3, batches of at
// most 32): a call, not inlined, so that the register kernel keeps its own register allocation; the
// launch arguments are read from the kernel's argument segment (PmpcArgs is the kernel's first argument,
// kernarg_addr; the resident server passes its request's sequence and w_warm / w_out flags, which its waves
// change).  The kernel takes pmpc_resto_solve's LDS (PrShared), which costs nothing at one instance per CU.
__device__ __noinline__ void pmpc_resto_tail(const int b, const uint32_t seq, const uint32_t fl,
                                             const unsigned long long kargs) {
    PmpcArgs a = kernarg_load<PmpcArgs>(kargs);
    a.seq = seq;
    if (!(fl & 1u)) a.w_warm = nullptr;
    if (!(fl & 2u)) a.w_out = nullptr;
    __syncthreads();            // the hand-off's status store (lane 0) is the only prior write
    pmpc_resto_solve(a, b);
}

// FUSE: resto mode 3, the handed-over instance continues in pmpc_resto_tail (no second launch)
template <int NAX, bool QSCAN, bool ONEROW = false, bool SHORT2 = false, bool RED = false, bool OCC2 = false,
          bool FUSE = false>
__global__ __launch_bounds__(kWave * kWaves) __attribute__((amdgpu_waves_per_eu(OCC2 ? 2 : ((QSCAN || NAX == 2) ? 1 : 2))))
void pmpc_ipm_kernel(PmpcArgs a) {
    // small batches: the launcher deals 8 blocks per instance and only every 8th works, so all
    // instances land on one XCD (blocks go round-robin over the 8 XCDs) and share its L2 for the code
    if (blockIdx.x % a.pack) return;
    const int b = blockIdx.x / a.pack;
    const bool handed = pmpc_solve<NAX, QSCAN, ONEROW, SHORT2, RED>(a, b);
    if constexpr (FUSE) {
        if (PM_EXPECT(handed, 0)) pmpc_resto_tail(b, a.seq, 3u, kernarg_addr());
    }
}

// Resident solver (dart_mpc_serve_start): the waves of one launch stay on the GPU and take request
// after request from a mailbox in mapped host memory, so a host call costs no kernel launch, no
// dispatch and no cold instruction cache.  Mailbox: one 64-bit request word written by the host in
// one release store, sequence | batch B << 32 | flags << 48 (bit 0: w_warm given, bit 1: w_out
// wanted) | stop << 56.  Inputs and outputs live at fixed mapped addresses (the PmpcArgs pointers).  Every
// wave leaves the loop on stop or after sv.idle_ticks of s_memrealtime (100 MHz) without a request,
// so the grid always drains.
// FUSE (B_serve <= 32, resto mode 3): a handed-over instance continues in pmpc_resto_tail, so the grid stays
// resident through a restoration
template <int NAX, bool ONEROW, bool SHORT2, bool FUSE = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(1)))
void pmpc_serve_kernel(PmpcArgs a, PmpcServe sv) {
    if (blockIdx.x % a.pack) return;
    const int b = blockIdx.x / a.pack;
    uint32_t seen = a.seq;
    unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        // one uncached 8-byte read over the link: the request word (sequence | batch << 32 | flags << 48 |
        // stop << 56), written by the host in one store
        const unsigned long long w =
            __hip_atomic_load((const unsigned long long*)sv.mailbox, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(w & 0xffffffffu));
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(w >> 32));
        const uint32_t sq = lo;
        if (hi >> 24) break;                                            // stop
        if (sq == seen) {
            if (__builtin_amdgcn_s_memrealtime() - t_last > sv.idle_ticks) break;
            __builtin_amdgcn_s_sleep(4);
            continue;
        }
        seen = sq;
        const uint32_t B = hi & 0xffffu, fl = (hi >> 16) & 0xffu;
        if ((uint32_t)b < B) {
            PmpcArgs r = a;
            r.B = (int)B; r.seq = sq;
            r.w_warm = (fl & 1u) ? a.w_warm : nullptr;
            r.w_out = (fl & 2u) ? a.w_out : nullptr;
            const bool handed = pmpc_solve<NAX, true, ONEROW, SHORT2, false>(r, b);
            if constexpr (FUSE) {
                if (PM_EXPECT(handed, 0)) pmpc_resto_tail(b, sq, fl, kernarg_addr());
            }
        }
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

#if !defined(PMPC_SEQ) && DART_WG == 1
// self-test of the wave primitives: out[0..63] = from_next(lane), out[64..127] = from_prev(lane),
// out[128] = wsum(lane), out[129] = wmax(lane), out[130] = wmin(lane + 1),
// out[131..194] = relative error of the raw v_rcp_f64 on x_i = 1.37^(i-32)*pi (diagnostic),
// out[195] = wsumf(lane), out[196] = wmaxf(v), out[197] = wminf(v + 0.5) with v = (37 lane) mod 64,
// out[198] = wmaxf(0 except lane 40: inf), out[199] / out[200] = half_bcast<3>(lane) at lanes 0 / 40,
// out[201..264] = half_pair_sum(lane^2)
__global__ __launch_bounds__(kWave) void wave_selftest_kernel(double* out) {
    const double x = (double)threadIdx.x;
    const double n = from_next(x), p = from_prev(x);
    const double s = wsum(x), mx = wmax(x), mn = wmin(x + 1.0);
    out[threadIdx.x] = n;
    out[64 + threadIdx.x] = p;
    if (threadIdx.x == 0) { out[128] = s; out[129] = mx; out[130] = mn; }
    const double y = 3.141592653589793 * pow(1.37, (double)threadIdx.x - 32.0);
    out[131 + threadIdx.x] = fma(y, __builtin_amdgcn_rcp(y), -1.0);
    const float v = (float)((37 * threadIdx.x) % 64);
    const float sf = wsumf((float)threadIdx.x), mxf = wmaxf(v), mnf = wminf(v + 0.5f);
    const float inf1 = wmaxf(threadIdx.x == 40 ? __builtin_inff() : 0.0f);
    const double hb = half_bcast_c<3>(x);
    if (threadIdx.x == 0) { out[195] = sf; out[196] = mxf; out[197] = mnf; out[198] = inf1; out[199] = hb; }
    if (threadIdx.x == 40) out[200] = hb;
    out[201 + threadIdx.x] = half_pair_sum(x * x);
}

#endif  // PMPC_SEQ

}  // namespace dartmpc

#if DART_WG == 2
// N = 32..63 on IPOPT's path (dartmpc_launch_pmpc forwards here): the scan build, one instance per two-wave
// workgroup; grid = B x pack blocks as for the one-wave builds
extern "C" hipError_t dartmpc_launch_pmpc_wg2(const void* args, unsigned grid, hipStream_t stream) {
    const dartmpc::PmpcArgs& a = *static_cast<const dartmpc::PmpcArgs*>(args);
    if (a.N < 32 || a.N > 63 || a.reduced || a.resto) return hipErrorInvalidValue;
    hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true>), dim3(grid), dim3(dartmpc::kWave * dartmpc::kWaves), 0,
                       stream, a);
    return hipGetLastError();
}
#elif defined(PMPC_SEQ)
// one-row scan build (onerow != 0, N <= 15), else the sequential (throughput) builds: two waves per
// SIMD, used once B exceeds the scan limit or N > 31
template <bool RED>
static void launch_seq(const dartmpc::PmpcArgs* a, unsigned grid, hipStream_t stream, int onerow) {
    if (onerow && !RED && a->resto == 3)
        hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, true, false, false, false, true>), dim3(grid),
                           dim3(dartmpc::kWave), 0, stream, *a);
    else if (onerow)
        hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, true, false, RED>), dim3(grid), dim3(dartmpc::kWave), 0,
                           stream, *a);
    else if (a->N <= 31)
        hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, false, false, false, RED>), dim3(grid), dim3(dartmpc::kWave), 0,
                           stream, *a);
    else
        hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<2, false, false, false, RED>), dim3(grid), dim3(dartmpc::kWave), 0,
                           stream, *a);
}
extern "C" hipError_t dartmpc_launch_pmpc_seq(const dartmpc::PmpcArgs* a, unsigned grid, hipStream_t stream,
                                              int onerow) {
    if (a->reduced) launch_seq<true>(a, grid, stream, onerow);
    else launch_seq<false>(a, grid, stream, onerow);
    return hipGetLastError();
}
extern "C" hipError_t dartmpc_launch_pmpc_serve_onerow(const dartmpc::PmpcArgs* a, const dartmpc::PmpcServe* sv,
                                                      unsigned grid, hipStream_t stream) {
    if (a->resto == 3)
        hipLaunchKernelGGL((dartmpc::pmpc_serve_kernel<1, true, false, true>), dim3(grid), dim3(dartmpc::kWave), 0,
                           stream, *a, *sv);
    else
        hipLaunchKernelGGL((dartmpc::pmpc_serve_kernel<1, true, false>), dim3(grid), dim3(dartmpc::kWave), 0, stream,
                           *a, *sv);
    return hipGetLastError();
}
#ifdef DART_STAMPS
// diagnostic build only: the stamps of the one-row (N <= 15) and sequential builds of this object
extern "C" hipError_t dartmpc_read_stamps_seq(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_seq), sizeof(unsigned long long) * 16, 0,
                               hipMemcpyDeviceToHost);
}
#endif
#else
extern "C" hipError_t dartmpc_launch_pmpc_seq(const dartmpc::PmpcArgs* a, unsigned grid, hipStream_t stream,
                                              int onerow);
extern "C" hipError_t dartmpc_launch_pmpc_serve_onerow(const dartmpc::PmpcArgs* a, const dartmpc::PmpcServe* sv,
                                                      unsigned grid, hipStream_t stream);
extern "C" hipError_t dartmpc_launch_pmpc_wg2(const void* args, unsigned grid, hipStream_t stream);

// the resident server for B_serve slots (IPOPT's path, N <= 31): one wave per slot, one XCD when it fits
extern "C" hipError_t dartmpc_launch_pmpc_serve(const dartmpc::PmpcArgs* args, const dartmpc::PmpcServe* sv,
                                               hipStream_t stream) {
    if (args->B <= 0 || args->N > 31) return hipErrorInvalidValue;
    dartmpc::PmpcArgs a = *args;
    a.pack = (a.B <= 32) ? 8 : 1;
    // B_serve <= 32: the restoration phases run in the wave that handed the instance over (mode 3); larger
    // servers hand it to the host (mode 2: dart_mpc_abi.hip served_resto)
    if (a.resto && a.pack == 8 && dartmpc::resto_fuse_enabled()) a.resto = 3;
    else if (a.resto) a.resto = 2;
    const unsigned grid = (unsigned)(a.B * a.pack);
    if (a.N <= 15) return dartmpc_launch_pmpc_serve_onerow(&a, sv, grid, stream);
    if (a.N <= 23 && a.resto == 3)
        hipLaunchKernelGGL((dartmpc::pmpc_serve_kernel<1, false, true, true>), dim3(grid), dim3(dartmpc::kWave), 0,
                           stream, a, *sv);
    else if (a.N <= 23)
        hipLaunchKernelGGL((dartmpc::pmpc_serve_kernel<1, false, true>), dim3(grid), dim3(dartmpc::kWave), 0, stream, a,
                           *sv);
    else if (a.resto == 3)
        hipLaunchKernelGGL((dartmpc::pmpc_serve_kernel<1, false, false, true>), dim3(grid), dim3(dartmpc::kWave), 0,
                           stream, a, *sv);
    else
        hipLaunchKernelGGL((dartmpc::pmpc_serve_kernel<1, false, false>), dim3(grid), dim3(dartmpc::kWave), 0, stream, a,
                           *sv);
    return hipGetLastError();
}

extern "C" hipError_t dartmpc_launch_pmpc(const dartmpc::PmpcArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    dartmpc::PmpcArgs a = *args;
    a.pack = (a.B <= 32) ? 8 : 1;          // <= 32 waves fit one XCD's CUs
    // The quadratic scan shortens the dependent chain but needs more registers (one wave per SIMD
    // instead of two).  On IPOPT's path (z rows, second-order correction) the sequential build no
    // longer fits two waves per SIMD without scratch spills, and the scan build is faster at every
    // batch size measured (B = 4096: 15.9 against 14.7 M solves/s; 18432: 18.1 against 17.4 M), so
    // it serves every N <= 31 batch; the sequential builds remain for N > 31 and for the
    // DART_PMPC_QSCAN_MAX_B experiment knob (the round-2 crossover was ~1.7 k instances).
    const dim3 grid(a.B * a.pack);
    static const int qscan_max_b = [] {
        const char* e = getenv("DART_PMPC_QSCAN_MAX_B");
        return e ? atoi(e) : (1 << 30);
    }();
    // From two instances per SIMD of the device on (2048 on MI355X), batches of N <= 31 take the scan build
    // compiled for two waves per SIMD (40 VGPRs spilled, 164 B of scratch): the second wave fills the
    // first's dependency stalls (VALU busy ~63 % alone).  Below that, one wave per SIMD and no spills win
    // (N = 20, B = 1152: 10.8 against 9.4 M solves/s; even at 1536; B = 2048: 15.2 against 13.7 M; 18432:
    // 20.5-20.9 against 17.8 M; N = 31, 18432: 6.4 against 6.1 M).  N <= 15 takes the short-scan build there
    // (the one-row build loses at two waves, 19.4-19.7 against 19.9 M; the short-scan one wins, 2048: 15.4-15.5
    // against 15.0 M, 18432: 22.2-22.8 against 20.0 M).  profiles/r04/occ2_ab.txt; DART_PMPC_OCC2_MIN_B
    // overrides the threshold (experiments).
    static const int occ2_min_b = [] {
        if (const char* e = getenv("DART_PMPC_OCC2_MIN_B")) return atoi(e);
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return 1 << 30;
        return 2 * 4 * cus;
    }();
    const bool occ2 = !a.reduced && a.B >= occ2_min_b && a.B <= qscan_max_b;
    // N = 32..63 on IPOPT's path: the scan build on two waves per instance (DART_PMPC_SEQ_LONG=1: the one-wave
    // sequential build, NAX = 2, for A/B)
    static const bool long_wg2 = [] {
        const char* e = getenv("DART_PMPC_SEQ_LONG");
        return !(e && e[0] == '1');
    }();
    // batches of at most 32 (one XCD, one instance per CU): IPOPT's restoration phases run in the wave that
    // handed the instance over (resto mode 3, pmpc_resto_tail), so no restoration launch follows the solve.
    // Only the branches below that launch a FUSE instantiation take mode 3 (not the two-waves-per-SIMD build, not
    // the sequential builds past DART_PMPC_QSCAN_MAX_B): everywhere else the queued pmpc_resto_kernel (mode 1) stays
    if (a.resto == 1 && a.pack == 8 && !a.reduced && a.N <= 31 && !occ2 && a.B <= qscan_max_b &&
        dartmpc::resto_fuse_enabled())
        a.resto = 3;
    const bool fuse = a.resto == 3;
    if (a.N <= 23 && occ2) {        // (N <= 15 too: the short-scan build at two waves beats the one-row build at one)
        hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, false, true, false, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
    } else if (a.N <= 15 && a.B <= qscan_max_b) {
        if (hipError_t e = dartmpc_launch_pmpc_seq(&a, grid.x, stream, 1)) return e;
    } else if (a.N <= 23 && a.B <= qscan_max_b) {
        if (fuse)
            hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, false, true, false, false, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
        else if (a.reduced)
            hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, false, true, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
        else
            hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, false, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
    } else if (a.N <= 31 && a.B <= qscan_max_b) {
        if (occ2)
            hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, false, false, false, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
        else if (fuse)
            hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, false, false, false, false, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
        else if (a.reduced)
            hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true, false, false, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
        else
            hipLaunchKernelGGL((dartmpc::pmpc_ipm_kernel<1, true>), grid, dim3(dartmpc::kWave), 0, stream, a);
    } else if (a.N > 31 && !a.reduced && !a.resto && long_wg2) {
        if (hipError_t e = dartmpc_launch_pmpc_wg2(&a, grid.x, stream)) return e;
    } else {
        if (hipError_t e = dartmpc_launch_pmpc_seq(&a, grid.x, stream, 0)) return e;
    }
    if (a.resto == 1) {       // the instances whose line search failed, with IPOPT's restoration phases
        if (hipError_t e = hipGetLastError()) return e;
        return dartmpc_launch_pmpc_resto(&a, stream);
    }
    return hipGetLastError();
}

// internal (not part of include/dart_mpc.h): runs the wave-primitive self-test into device buffer d_out[131]
extern "C" hipError_t dartmpc_wave_selftest(double* d_out, hipStream_t stream) {
    hipLaunchKernelGGL(dartmpc::wave_selftest_kernel, dim3(1), dim3(dartmpc::kWave), 0, stream, d_out);
    return hipGetLastError();
}

#ifdef DART_STAMPS
// diagnostic build only: per-phase s_memtime cycles of block 0 from the last launch
extern "C" hipError_t dartmpc_read_stamps(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp), sizeof(unsigned long long) * 16, 0,
                               hipMemcpyDeviceToHost);
}
#endif
#endif  // PMPC_SEQ
