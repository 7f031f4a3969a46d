// lmpc_ipm.hip -- batched LMPC interior-point solve (8-state Stribeck / rolling model), gfx950.
//
// Replaces the solve of RLMPC._solver_worker (LMPC/src/controller/rlmpc2.py:229-533): the NLP
// :239-491 with the model safe_dynamics :260-429 (index map :301-344), RK4 :431-436, cost
// :444-464 (Q, Qt on the state error, R on [u; Delta u]), U box, and IPOPT's options
// (:480-489: max_iter, tol, acceptable_tol, acceptable_iter; the 0.05 s wall-clock cap is not
// reproduced: the solve is deterministic here).  The 34-vector pvec is an input, or, in the fused
// launch (dart_lmpc_policy_solve_batch), the output of the policy step run as the kernel's prologue.
//
// Separable structure: safe_dynamics never mixes the two horizontal directions -- [px, vx,
// theta_y, omega_y] are driven by tilt a alone (sliding friction, rolling slip vx - r_x omega_y,
// the omega_y torques, toppling sin theta_y; :352-427), [py, vy, theta_x, omega_x] by tilt b
// alone -- and Q, Qt, R and the U box are diagonal.  The NLP therefore splits into two
// independent scalar-input problems, coupled only through IPOPT's global quantities (mu, the
// step length, the filter, the scalings), all of which are wave-wide reductions here.  The two
// subsystems share one code path with per-half parameters: half h = lane >> 5 solves subsystem
// h, lane 32 h + k owns shooting node k (N <= 31).
//
// Method: IPOPT's primal-dual barrier method as in pmpc_ipm.hip / rmpc_ipm.hip (monotone mu,
// filter line search with second-order correction, inertia correction, bound_relax 1e-8,
// gradient-based scaling of the objective and of the constraint rows) with IPOPT's optimal /
// acceptable termination tests.  The Delta-u cost couples consecutive controls: each half runs
// the Riccati recursion on its augmented state x~_k = [x_k (4); u_{k-1}] (ocp_wave.h, OcpLdsS,
// one LDS round trip per node).  Exact derivatives as IPOPT gets them from CasADi: per
// direction of z = [x; u], the RK4 tangent (a column of the step Jacobian) and a second-order
// adjoint sweep back through the four stages (a column of the exact Hessian of lambda^T x+).
//
// Horizons N = 32..63: this file built a second time with -DDART_WG=2 (Makefile: lmpc_wg2.o) -- a workgroup of two
// waves per instance, wave w owning nodes 32 w .. 32 w + 31 of both halves (wave.h: the wave reductions and node
// shifts combine the two waves, the Riccati and forward sweeps run in both on the shared LDS).  The 64-node stage
// arrays fill the LDS, so that build keeps the second-order-correction scratch and the restoration-phase state in
// a per-instance device area after the hand-off states (LmpcArgs::resto_buf), runs the policy step of a fused call
// as its own launch, and queues the restoration kernel.  Its symbols sit in their own namespace.
#if DART_WG == 2
#define dartmpc dartmpc_wg2
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "lmpc_ipm.h"
#include "ocp_wave.h"
#include "stamps.h"
#include "wave.h"

namespace dartmpc {

constexpr int LM_NMAXS = 32 * kWaves;      // node slots per half (N <= 31; two-wave build N <= 63)
constexpr int LM_NSC = 5;         // stage-dependent tangent coefficients per RK stage
constexpr double LM_G = 9.81;     // rlmpc2.py:354
using LmLds = OcpLdsS<5, LM_NMAXS>;

#ifdef DART_STAMPS
__device__ unsigned long long g_stamp_lm[32];   // 16..23: the restoration phase (lmpc_ipm_kernel<true>)
#endif

struct Strb {           // stribeck_fric parameters (rlmpc2.py:372-376)
    double Fc, dF, B, ivs, ieps;    // dF = F_s - F_c, ivs = 1 / (v_s + 1e-12), ieps = 1 / eps
};

// One subsystem, local state [p, v, th, om], input a (x: [px, vx, theta_y, omega_y; a],
// y: [py, vy, theta_x, omega_x; b]):
//   pdot = v,  vdot = (m g sin a - c v - k p - Ff(v) - Fr(v + rs om)) / m,
//   thdot = om, omdot = (-r Fr(v + rs om) - Tn(om) - crot om - tq sin th) / I
// with rs = -r_x (x) / +r_y (y) the rolling-slip coupling (:391-395) and tq = m g h_com (:413-414).
struct LmSub {
    double im, m, c, k;
    Strb st;                // translational Stribeck: sliding (v) and rolling slip
    double rs, r, rr2;      // slip = v + rs om; torque -r Fr; rr2 = -r rs
    double iI, crot;
    Strb sr;                // rotational Stribeck
    double tq;
    double h;               // Ts
};

struct LmSoc {
    NodeArr<double[5], 2 * LM_NMAXS> CS;     // second-order correction: c_soc rows of node k (incoming defect)
    NodeArr<double[11], 2 * LM_NMAXS> SV;    // second-order correction: the plain step (dx~, lambda+, du)
};

struct LmShared {
    LmLds ocp;
#if DART_WG == 1
    LmSoc soc;                      // (two-wave build: in the device area, LmAux)
#endif
    LmSub sub[2];                   // uniform problem data of the two halves
    double W[2][2][4], tg[2][4], st0[2][4];   // [half][stage, terminal] weights, target, x_0 (local order)
    alignas(16) double Ps[2][LmLds::NTP];     // the explicit value function of riccati_s_sweep_p
};

// ---------------------------------------------------------------------------------------------
// IPOPT's restoration phase (MinC_1NrmRestorationPhase; oracle/lmpc_ipm.c `restoration`).  Every
// physical defect row of the feasibility problem carries a slack pair (p, n); eliminating it leaves
// the row soft, J dx - D dlam = rhs with D = (1/Sigma_p' + 1/Sigma_n') / d^2.  In the Riccati recursion
// the value function of node k+1 is then seen through its soft rows: eliminating the row slack w
// (Hessian D^-1 on the four physical rows) from V(x~ + w) is a second Schur complement over the value
// indices [x~ (5); 1],
//   Pt' = Pt - Pt(:, ph) S^-1 Pt(ph, :),   S = Pt(ph, ph) + D^-1,
// with Pt from G_{k+1} by the Schur complement on u, so the node step runs unchanged on the surrogate
// [[Pt', 0], [0, 1]]; the incoming rows of node k+1 map x~+ <- x~+ - E T [x~+; 1] with
// T = S^-1 Pt(ph, :) (4 x 6), and S positive definite is part of the inertia test.
// ---------------------------------------------------------------------------------------------
// iterative refinement of the restoration step: at most this many refinement solves per step, each
// only while the residual of the Newton system exceeds 1e-12 of the step (IPOPT's PDFullSpaceSolver
// refines every KKT solve).  Statuses equal to the oracle's on 99.958 % of 28,800 stress instances with
// it, 99.747 % without (tools/parity_sweep.py); the C5 stress line pays 6 %.  0 = off
#ifndef DART_RESTO_REFINE
#define DART_RESTO_REFINE 3
#endif
struct LmResto {
    NodeArr<double[24], 2 * LM_NMAXS> T;      // T of node k's soft rows (row-major 4 x 6, value indices)
    NodeArr<double[4], 2 * LM_NMAXS> Dinv;    // 1 / D of node k's four physical incoming rows
    NodeArr<double[20], 2 * LM_NMAXS> SV;     // a second-order correction: the plain step
    double Gs[2][LmLds::NTP];                 // the surrogate of G_{k+1} (one per half)
    // per-node state of the restoration problem (node k's four physical incoming rows), kept in LDS
    // rather than registers: p, n, z_p, z_n, rp, rn, Sigma_p', Sigma_n', x_R, D_R
    NodeArr<double[40], 2 * LM_NMAXS> PN;
};

// Backward sweep of both halves with soft physical rows (restoration phase): before the step of node
// k, each half forms the surrogate of G_{k+1} seen through node k+1's soft rows (RL->Gs) and keeps
// T_{k+1} for the forward map; T_0 of the soft initial rows comes last.  The transform of one node is
// one lane-parallel phase of the half-wave: every lane forms S = Pt(ph, ph) + D^-1 from G_{k+1}
// (Pt = Gzz - Gzu Gzu^T / Quu), factors it S = L diag(dd) L^T (each its own copy) and solves the column
// qv of T = S^-1 Pt(ph, :) its packed surrogate entry (pv, qv) needs, Pt(pv, qv) - Pt(pv, ph) T(:, qv);
// the lanes of row 6 of the packed triangle store T's six columns.  (Every product is formed as the
// earlier three-phase version formed it -- Pt(a, q) = fma(-Gzu(a) / Quu, Gzu(q), Gzz(a, q)) -- so the
// results are the same bits, with one barrier per node instead of three.)  G[slot N] must hold the
// terminal surrogate, RL->Dinv every node's 1 / D.  Returns false (wave-uniform) if some S or Quu is
// not positive definite.
__device__ bool riccati_s_sweep_soft(LmLds* S, LmResto* RL, int N, const RiccatiSRoles& R, bool early) {
    constexpr int NXA = LmLds::NXA, NP = LmLds::NP;
    static_assert(NXA == 5 && NP == 6, "packed row 6 = [x~ (5), u, 1] names T's six columns");
    const int h = lane_id() >> 5, base = h * LM_NMAXS;
    int zi = 0;
    while (tri(zi + 1) <= R.e) ++zi;
    const int zj = R.e - tri(zi);
    const bool uent = zi == NXA || zj == NXA;                              // z index 5 = u
    const int pv = zi == NXA + 1 ? NXA : (zi < NXA ? zi : 0), qv = zj == NXA + 1 ? NXA : (zj < NXA ? zj : 0);
    // the writer of T(:, qv): the lanes of packed row 6 (entries (6, zj), zj != u), each a different qv
    const bool twrite = R.on && zi == NXA + 1 && zj != NXA;
    bool ok = true;
    auto soften = [&](int j, bool surrogate) {
        const double* Gn = S->G[j];
        const double qj = Gn[hp(NXA, NXA)];
        ok = ok && qj > 0.0 && isfinite(qj);
        const double iq = frcp(qj);
        const double* dinv = RL->Dinv[j];
        double gu[4], di[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) { gu[a] = Gn[gszu<NXA>(a)]; di[a] = dinv[a]; }
        const double gq = Gn[gszu<NXA>(qv)], gp = Gn[gszu<NXA>(pv)];
        double P[4][4], rq[4], rp[4];          // Pt(i, c) for c <= i < 4; Pt(ph, qv); Pt(ph, pv)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int c = 0; c <= i; ++c) P[i][c] = fma(-gu[i] * iq, gu[c], Gn[gszz<NXA>(i, c)]);
            rq[i] = fma(-gu[i] * iq, gq, Gn[gszz<NXA>(i, qv)]);
            rp[i] = fma(-gu[i] * iq, gp, Gn[gszz<NXA>(i, pv)]);
        }
        const double pvq = fma(-gp * iq, gq, Gn[gszz<NXA>(pv, qv)]);
        double L[4][4], id[4], dd[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            double t = P[c][c] + di[c];
#pragma unroll
            for (int m = 0; m < c; ++m) t -= L[c][m] * L[c][m] * dd[m];
            dd[c] = t;
            ok = ok && t > 0.0 && isfinite(t);
            id[c] = frcp(t);
#pragma unroll
            for (int i = c + 1; i < 4; ++i) {
                double u = P[i][c];
#pragma unroll
                for (int m = 0; m < c; ++m) u -= L[i][m] * L[c][m] * dd[m];
                L[i][c] = u * id[c];
            }
        }
        double y[4], t4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double t = rq[i];
#pragma unroll
            for (int m = 0; m < i; ++m) t -= L[i][m] * y[m];
            y[i] = t;
        }
#pragma unroll
        for (int i = 3; i >= 0; --i) {
            double t = y[i] * id[i];
#pragma unroll
            for (int m = i + 1; m < 4; ++m) t -= L[m][i] * t4[m];
            t4[i] = t;
        }
        if (twrite) {
#pragma unroll
            for (int i = 0; i < 4; ++i) RL->T[j][6 * i + qv] = t4[i];
        }
        if (surrogate) {
            double v = pvq;
#pragma unroll
            for (int a = 0; a < 4; ++a) v -= rp[a] * t4[a];
            RL->Gs[h][R.e] = uent ? ((zi == NXA && zj == NXA) ? 1.0 : 0.0) : v;
        }
        chain_sync();
    };
    for (int k = N - 1; k >= 0; --k) {
        // node k's M and H entries do not depend on the chain: read before the soft-row transform of node k+1
        // (whose closing fence no LDS access crosses), so their latency is off the chain
        const double hk = S->H[base + k][R.e];
        const double* Mk = &S->M[base + k][0][0];
        double vi[NP], vj[NP];
#pragma unroll
        for (int m = 0; m < NP; ++m) { vi[m] = Mk[R.ci + m]; vj[m] = Mk[R.cj + m]; }
        soften(base + k + 1, true);
        const double* Gn = RL->Gs[h];
        double t[NP];
#pragma unroll
        for (int m = 0; m < NP; ++m) t[m] = 0.0;
#pragma unroll
        for (int n = 0; n < NP; ++n)
#pragma unroll
            for (int m = 0; m < NP; ++m) t[m] = fma(Gn[gszz<NXA>(m, n)], vj[n], t[m]);
        double ga = hk;
#pragma unroll
        for (int m = 0; m < NP; ++m) ga = fma(vi[m], t[m], ga);
        S->G[base + k][R.e] = ga;
        chain_sync();
        // early: a failed inertia test (Quu or a soft block's pivot of either half) ends the sweep -- only for the
        // perturbation loop, whose caller discards a failed sweep and factors again with a new perturbation.  Every
        // lane of a half tests the same LDS values, and the two waves of a two-wave build run the sweep alike, so
        // the wave's own ballot decides uniformly; the return value is the full sweep's (ok only accumulates).
        // (Restoration tails: ~2 soft sweeps per iteration on the C5 stress instances,
        // profiles/r05/stamps_lmpc_resto.txt.)  The callers that use the sweep whatever it returns (least-square
        // multipliers, refinement, second-order correction) run it whole, so no node keeps a stale factorisation.
        if (early && __ballot(!ok) != 0ull) break;
    }
    if (!early || __ballot(!ok) == 0ull) soften(base, false);
    return !wany(!ok);
}

// dynamic LDS: LmShared, then the policy step's PolicyLds (fused launches of lmpc_ipm_kernel<false>) or
// LmResto (lmpc_ipm_kernel<true>) at the same offset
constexpr size_t kLmPolicyLdsOff = (sizeof(LmShared) + 15) & ~size_t(15);
#if DART_WG == 1
constexpr size_t kLmRestoOff = kLmPolicyLdsOff;
constexpr size_t kLmLdsBytes = kLmPolicyLdsOff + (sizeof(PolicyLds) > sizeof(LmResto) ? sizeof(PolicyLds) : sizeof(LmResto));
static_assert(kLmLdsBytes <= 160 * 1024, "LDS of one CU");
#else
// two-wave build: LmShared alone (the policy step runs as its own launch; LmSoc and LmResto in the device area)
constexpr size_t kLmLdsBytes = kLmPolicyLdsOff;
static_assert(kLmLdsBytes + sizeof(g_wg_x) <= 160 * 1024, "LDS of one CU");
struct LmAux {
    LmSoc soc;
    LmResto resto;
};
#endif
// hand-off of an instance whose filter line search failed: its iteration-start state goes to HBM
// (LmpcArgs::resto_buf, kLmNst doubles per lane) and lmpc_ipm_kernel<true> resumes it
constexpr int kLmNeedResto = -100;
constexpr int kLmNst = 16;

__device__ __forceinline__ double sq(double p) { return fabs(p) + 1e-6; }   // squash_param :296-298

__device__ __forceinline__ Strb make_strb(double Fs, double Fc, double B, double vs, double eps) {
    Strb s;
    s.Fc = Fc; s.dF = Fs - Fc; s.B = B; s.ivs = 1.0 / (vs + 1e-12); s.ieps = 1.0 / eps;
    return s;
}

// value of the friction law: tanh(v/eps) (F_c + (F_s - F_c) exp(-|v|/(v_s + 1e-12))) + B v
__device__ __forceinline__ double strb(const Strb& p, double v) {
    const double e = exp_econ(-fabs(v) * p.ivs);
    const double T = tanh_econ(v * p.ieps);
    return fma(T, fma(p.dF, e, p.Fc), p.B * v);
}
// value, first and second derivative (d|v|/dv = sign(v), sign(0) = 0, as CasADi)
__device__ __forceinline__ void strb_d(const Strb& p, double v, double& S, double& S1, double& S2) {
    const double sg = (v > 0.0) ? 1.0 : ((v < 0.0) ? -1.0 : 0.0);
    const double e = exp_econ(-fabs(v) * p.ivs);
    const double T = tanh_econ(v * p.ieps);
    const double C = fma(p.dF, e, p.Fc);
    const double T1 = (1.0 - T * T) * p.ieps, C1 = -p.dF * e * sg * p.ivs;
    const double T2 = -2.0 * T * T1 * p.ieps, C2 = p.dF * e * (sg * sg) * p.ivs * p.ivs;
    S = fma(T, C, p.B * v);
    S1 = fma(T1, C, fma(T, C1, p.B));
    S2 = fma(T2, C, fma(2.0 * T1, C1, T * C2));
}

__device__ __forceinline__ double sin_any(double x) {
    double s, c;
    if (fabs(x) <= 1.0) sincos_econ(x, s, c);
    else s = sin(x);
    return s;
}
__device__ __forceinline__ void sincos_any(double x, double& s, double& c) {
    if (fabs(x) <= 1.0) sincos_econ(x, s, c);
    else sincos(x, &s, &c);
}

// safe_dynamics (:260-429) of one subsystem: ydot for state y and tilt sine sa
__device__ __forceinline__ void sub_f(const LmSub& m, const double* y, double sa, double* f) {
    const double Ff = strb(m.st, y[1]);
    const double Fr = strb(m.st, fma(m.rs, y[3], y[1]));
    const double Tn = strb(m.sr, y[3]);
    f[0] = y[1];
    f[1] = (m.m * (LM_G * sa) - m.c * y[1] - m.k * y[0] - Ff - Fr) * m.im;
    f[2] = y[3];
    f[3] = (-m.r * Fr - Tn - m.crot * y[3] - m.tq * sin_any(y[2])) * m.iI;
}

__device__ __forceinline__ void sub_rk4(const LmSub& ml, const double* x, double sa, double* xn) {
    const LmSub m = ml;         // model to registers once (LDS round trips off the stage chains)
    double k[4], y[4], acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { y[i] = x[i]; acc[i] = 0.0; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        sub_f(m, y, sa, k);
#pragma unroll
        for (int i = 0; i < 4; ++i) { acc[i] = fma(wts, k[i], acc[i]); y[i] = fma(cst * m.h, k[i], x[i]); }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) xn[i] = fma(m.h / 6.0, acc[i], x[i]);
}

// Value pass of RK4 that also stores, per stage s, the tangent coefficients
// sc[s] = [dvdot/dv, dvdot/dom, domdot/dv, domdot/dth, domdot/dom] at y_s and the second-derivative
// data sd[s] = [Ff''(v), Fr''(slip), Tn''(om), sin th].
__device__ __forceinline__ void sub_rk4_lin(const LmSub& ml, const double* x, double sa, double* xn,
                                            double (*sc)[LM_NSC], double (*sd)[4]) {
    const LmSub m = ml;
    double y[4], acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { y[i] = x[i]; acc[i] = 0.0; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        double k[4];
        k[0] = y[1]; k[2] = y[3];
        double Sf, Sf1, Sf2, Sr, Sr1, Sr2, Sn, Sn1, Sn2, sth, cth;
        strb_d(m.st, y[1], Sf, Sf1, Sf2);
        strb_d(m.st, fma(m.rs, y[3], y[1]), Sr, Sr1, Sr2);
        sd[s][0] = Sf2; sd[s][1] = Sr2;
        sc[s][0] = (-m.c - Sf1 - Sr1) * m.im;
        sc[s][1] = -m.rs * Sr1 * m.im;
        sc[s][2] = -m.r * Sr1 * m.iI;
        k[1] = (m.m * (LM_G * sa) - m.c * y[1] - m.k * y[0] - Sf - Sr) * m.im;
        k[3] = -m.r * Sr;                                          // completed below
        strb_d(m.sr, y[3], Sn, Sn1, Sn2);
        sincos_any(y[2], sth, cth);
        sd[s][2] = Sn2; sd[s][3] = sth;
        sc[s][3] = -m.tq * cth * m.iI;
        sc[s][4] = (m.rr2 * Sr1 - Sn1 - m.crot) * m.iI;
        k[3] = (k[3] - Sn - m.crot * y[3] - m.tq * sth) * m.iI;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = fma(wts, k[i], acc[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = fma(cst * m.h, k[i], x[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) xn[i] = fma(m.h / 6.0, acc[i], x[i]);
}

// q = (d f / d y at stage s)^T v from the stage's tangent coefficients
__device__ __forceinline__ void sub_jtv(double kx1, const double* c, const double* v, double* q) {
    q[0] = kx1 * v[1];
    q[1] = fma(c[0], v[1], fma(c[2], v[3], v[0]));
    q[2] = c[3] * v[3];
    q[3] = fma(c[1], v[1], fma(c[4], v[3], v[2]));
}

// First-order adjoint of L = nl^T x+ (nl = -lambda_{k+1}) through the four RK4 stages; converts the
// stage second-derivative data sd[s] in place into the curvature coefficients of kb_s^T f'' at y_s:
// [A1, A2, A3, C] with the (v, om) block [[A1, A2], [A2, A3]] and th: C; returns the tilt
// curvature huu = sum_s kb_s^T f_aa.
__device__ __forceinline__ double sub_adjoint_curv(const LmSub& m, const double (*sc)[LM_NSC], double (*sd)[4],
                                                   const double* lamn, double sa) {
    double kb[4], yb[4];
    const double h = m.h, kx1 = -m.k * m.im;
#pragma unroll
    for (int i = 0; i < 4; ++i) kb[i] = -(h / 6.0) * lamn[i];        // kb_4
    double huu = 0.0;
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        double* d = sd[s];
        const double c_v = kb[1] * (-d[0] * m.im);
        const double c_s = kb[1] * (-d[1] * m.im) + kb[3] * (-m.r * d[1] * m.iI);
        const double c_o = kb[3] * (-d[2] * m.iI);
        const double c_t = kb[3] * (m.tq * d[3] * m.iI);
        d[0] = c_v + c_s; d[1] = m.rs * c_s; d[2] = fma(m.rs * m.rs, c_s, c_o); d[3] = c_t;
        huu = fma(kb[1], -LM_G * sa, huu);
        if (s > 0) {      // kb_{s-1} = w_{s-1} h/6 nl + c_s h J_s^T kb_s  (c = 1, 1/2, 1/2 for s = 3, 2, 1)
            sub_jtv(kx1, sc[s], kb, yb);
            const double cs = s == 3 ? h : 0.5 * h, ws = (s == 1 ? 1.0 : 2.0) * h / 6.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) kb[i] = fma(cs, yb[i], -ws * lamn[i]);
        }
    }
    return huu;
}

// Direction d (0..3 state, 4 tilt): tangent of RK4 -> column d of the step Jacobian (written to
// column jc(d) of M~, returns col . lamn), then the second-order adjoint sweep back through the
// stages -> column d of the exact Hessian of -lambda^T x+ over z = [x; u], written to the packed
// stage Hessian (rows i >= d).
__device__ __forceinline__ double sub_direction(const LmSub& m, const double (*sc)[LM_NSC], const double (*cv)[4],
                                                double huu, double gca, int d, const double* lamn, double* Mk,
                                                double* Hk, double cadd) {
    double yd[4][4], acc[4], e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { e[i] = (i == d) ? 1.0 : 0.0; yd[0][i] = e[i]; acc[i] = 0.0; }
    const double fa = d == 4 ? gca : 0.0;
    const double kx1 = -m.k * m.im;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double wts = (s == 0 || s == 3) ? 1.0 : 2.0, cst = s < 2 ? 0.5 : (s == 2 ? 1.0 : 0.0);
        const double* c = sc[s];
        const double* y = yd[s];
        double k[4];
        k[0] = y[1]; k[2] = y[3];
        k[1] = fma(kx1, y[0], fma(c[0], y[1], fma(c[1], y[3], fa)));
        k[3] = fma(c[2], y[1], fma(c[4], y[3], c[3] * y[2]));
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = fma(wts, k[i], acc[i]);
        if (s < 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) yd[s + 1][i] = fma(cst * m.h, k[i], e[i]);
        }
    }
    const int jc = d < 4 ? d : 5;
    double dot = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double col = fma(m.h / 6.0, acc[i], e[i]);
        Mk[jc * LmLds::NC + i] = col;
        dot = fma(col, lamn[i], dot);
    }
    // second-order adjoint: kbd_s = d/dd kb_s, q_s = J_s^T kbd_s + (kb_s^T f'')_s yd_s
    double kbd[4], hx[4], hu = d == 4 ? huu : 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) { kbd[i] = 0.0; hx[i] = 0.0; }
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        const double* cc = cv[s];
        const double* y = yd[s];
        double q[4];
        sub_jtv(kx1, sc[s], kbd, q);
        q[1] = fma(cc[0], y[1], fma(cc[1], y[3], q[1]));
        q[3] = fma(cc[1], y[1], fma(cc[2], y[3], q[3]));
        q[2] = fma(cc[3], y[2], q[2]);
        hu = fma(gca, kbd[1], hu);
#pragma unroll
        for (int i = 0; i < 4; ++i) hx[i] += q[i];
        const double cs = s == 3 ? m.h : 0.5 * m.h;
#pragma unroll
        for (int i = 0; i < 4; ++i) kbd[i] = cs * q[i];
    }
    // rows i >= d of column d (z indices: x 0..3, up 4, tilt 5); cadd = the cost / barrier curvature
    // of the diagonal entry (d, d)
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i >= d) Hk[hp(i, jc)] = i == d ? hx[i] + cadd : hx[i];
    Hk[hp(5, jc)] = d == 4 ? hu + cadd : hu;
    return dot;
}

// The solve of instance b by the calling wave; returns true when <false> handed the instance over.
template <bool RESTO>
__device__ __forceinline__ bool lmpc_solve(const LmpcArgs& a, const int b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LmShared& SH = *reinterpret_cast<LmShared*>(smem);
    LmLds* S = &SH.ocp;
#if DART_WG == 1
    LmResto* RL = reinterpret_cast<LmResto*>(smem + kLmRestoOff);
    LmSoc& SO = SH.soc;
#else
    LmAux* const AX = reinterpret_cast<LmAux*>(a.resto_buf + (size_t)a.B * kWave * kWaves * kLmNst) + b;
    LmResto* RL = &AX->resto;
    LmSoc& SO = AX->soc;
#endif
    const RiccatiSRoles RR = riccati_s_roles<LmLds>();
    STAMP_DECL
    const int lane = lane_id();
    const int ql = kWave * wave_idx() + lane;      // this lane's slot in the per-lane hand-off state
    const int hf = lane >> 5;                  // subsystem: 0 = x [px, vx, th_y, om_y; a], 1 = y [py, vy, th_x, om_x; b]
    const int k = node_base() + (lane & 31);   // shooting node
    const int sl = hf * LM_NMAXS + k;          // node slot of this lane (every lane owns one)
    const int N = a.N;
    // fused policy step (C5: the learned parameter net in the same launch as the shooting defects it
    // parameterises): its LDS sits after LmShared, its output vector is this solve's pvec
    const double* pvec = a.fuse_policy ? (RESTO ? a.pol.model_params + LM_NPV * b : nullptr) : a.pvec + LM_NPV * b;
    if (!RESTO && a.fuse_policy) {
        PolicyLds& PL = *reinterpret_cast<PolicyLds*>(smem + kLmPolicyLdsOff);
        policy_step_wave(a.pol, b, PL);
        pvec = PL.pv;
    }
    // IPOPT max_cpu_time (rlmpc2.py:485): the solve's clock starts here; the resumed kernel continues it from
    // the time its instance had spent when it was handed over (the wait for the rest of the first launch is
    // not counted: the cap is per-instance GPU time); 100 MHz constant clock, a scalar read, so the test
    // below is wave-uniform
    unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    if constexpr (RESTO)
        t_start -= (unsigned long long)a.resto_buf[(size_t)b * kWave * kWaves * kLmNst + 6 * kLmNst + kLmNst - 1];
    auto out_of_time = [&]() {
#if DART_WG == 1
        return a.max_ticks > 0 && (long long)(__builtin_amdgcn_s_memrealtime() - t_start) > a.max_ticks;
#else
        // (each wave reads its own clock: the two decide together)
        return wany(a.max_ticks > 0 && (long long)(__builtin_amdgcn_s_memrealtime() - t_start) > a.max_ticks);
#endif
    };
    const bool xon = k <= N, uon = k < N;
    constexpr int NC = LmLds::NC;
    // full-state index of the subsystem's local state i
    auto gidx = [&](int i) { return hf == 0 ? (i == 0 ? 0 : i == 1 ? 1 : i == 2 ? 6 : 7) : (i == 0 ? 2 : i == 1 ? 3 : i == 2 ? 4 : 5); };

    // ---------------- model parameters (uniform per half, staged in LDS) -----------------------
    if (lane == 0 || lane == 32) {
        LmSub& m = SH.sub[hf];
        const double* p = pvec;
        const double m_x = sq(p[0]), m_y = sq(p[1]);
        if (hf == 0) {     // x: m_x, c_x, k_x, Stribeck x, I_y, r_x, c_rot_y, rotational Stribeck y, h_com_y
            m.m = m_x; m.c = sq(p[2]); m.k = sq(p[4]);
            m.st = make_strb(p[6], p[7], p[8], sq(p[9]), sq(p[10]));
            m.iI = 1.0 / (sq(p[17]) + 1e-12);
            m.r = sq(p[18]); m.rs = -m.r; m.crot = sq(p[21]);
            m.sr = make_strb(p[27], p[28], p[29], sq(p[30]), sq(p[31]));
            m.tq = m_x * LM_G * sq(p[33]);
        } else {           // y: m_y, c_y, k_y, Stribeck y, I_x, r_y, c_rot_x, rotational Stribeck x, h_com_x
            m.m = m_y; m.c = sq(p[3]); m.k = sq(p[5]);
            m.st = make_strb(p[11], p[12], p[13], sq(p[14]), sq(p[15]));
            m.iI = 1.0 / (sq(p[16]) + 1e-12);
            m.r = sq(p[19]); m.rs = m.r; m.crot = sq(p[20]);
            m.sr = make_strb(p[22], p[23], p[24], sq(p[25]), sq(p[26]));
            m.tq = m_y * LM_G * sq(p[32]);
        }
        m.im = 1.0 / m.m;
        m.rr2 = -m.r * m.rs;
        m.h = a.Ts;
    }
    const double* pr = a.prm + LM_NPRM * b;
    if (k < 4) {
        const int gi = gidx(k);
        SH.W[hf][0][k] = pr[gi]; SH.W[hf][1][k] = pr[8 + gi];
        SH.tg[hf][k] = a.target[8 * b + gi]; SH.st0[hf][k] = a.state[8 * b + gi];
    }
    __syncthreads();
    const LmSub& m = SH.sub[hf];
    const double* Wq = SH.W[hf][k < N ? 0 : 1];    // stage or terminal weights (lane N is the terminal node)
    const double* Qtv = SH.W[hf][1];
    const double* tg = SH.tg[hf];
    const double* st0 = SH.st0[hf];
    const double Ru = pr[16 + hf], Rdu = pr[18 + hf];
    const double ulo = pr[20], uhi = pr[21];

    const double lo = ulo - 1e-8 * fmax(1.0, fabs(ulo)), hi = uhi + 1e-8 * fmax(1.0, fabs(uhi));
    const bool poly = fmax(fabs(lo), fabs(hi)) <= 1.0;

    // ---------------- constant structure of the stage blocks ------------------------------------
    double* Mk = &S->M[sl][0][0];
    double* Hk = S->H[sl];
    if (uon) {
        for (int e = 0; e < LmLds::ND * NC; ++e) Mk[e] = 0.0;
        for (int e = 0; e < LmLds::NTP; ++e) Hk[e] = 0.0;
        Mk[5 * NC + 4] = 1.0;                 // up+ = u
        Mk[6 * NC + 5] = 1.0;                 // homogeneous coordinate
    }

    // ---------------- initial point (lane 32 h + k = node k of subsystem h) -----------------------
    const double upv = a.u_prev[2 * b + hf];
    const int nw = 8 * (N + 1) + 2 * N;
    const double* ww = a.w_warm ? a.w_warm + (size_t)nw * b : nullptr;
    double x[4], up, u, lam[5], zl, zu;
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = xon && ww ? ww[8 * k + gidx(i)] : 0.0;   // warm start w0 (zeros first, :492)
    const double pushl = fmin(1e-2 * fmax(1.0, fabs(lo)), 1e-2 * (hi - lo));
    const double pushu = fmin(1e-2 * fmax(1.0, fabs(hi)), 1e-2 * (hi - lo));
    {
        const double t = uon && ww ? ww[8 * (N + 1) + 2 * k + hf] : 0.0;
        u = uon ? fmin(fmax(t, lo + pushl), hi - pushu) : 0.0;
        zl = uon ? 1.0 : 0.0; zu = uon ? 1.0 : 0.0;
    }
    {
        const double p0 = from_prev(u);
        up = k == 0 ? upv : p0;
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) lam[i] = 0.0;

    auto cost_grad = [&](const double* xx, double uu, double pp, double* g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = 2.0 * Wq[i] * (xx[i] - tg[i]);
        const double d0 = uu - pp;
        g[4] = uon ? -2.0 * Rdu * d0 : 0.0;
        g[5] = uon ? fma(2.0 * Ru, uu, 2.0 * Rdu * d0) : 0.0;
    };
    auto cost_val = [&](const double* xx, double uu, double pp) {
        double f = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) f = fma(Wq[i] * (xx[i] - tg[i]), xx[i] - tg[i], f);
        const double d0 = uu - pp;
        const double fu = Ru * uu * uu + Rdu * d0 * d0;
        return xon ? f + (uon ? fu : 0.0) : 0.0;
    };
    // incoming augmented defect g_k of node k for a trial point (value-only RK4 of lane k-1)
    auto defects = [&](const double* xx, double pp, double uu, double* g) {
        double sa, ca, xn[4];
        tilt_sincos_econ(poly, uu, sa, ca);
        sub_rk4(m, xx, sa, xn);
        double f[5];
        if constexpr (kWaves == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) f[i] = from_prev(xn[i]);
            f[4] = from_prev(uu);
        } else {       // two waves: one exchange for the five shifts
            const double x5[5] = {xn[0], xn[1], xn[2], xn[3], uu};
            from_prev_n(x5, f);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = k == 0 ? xx[i] - st0[i] : xx[i] - f[i];
        g[4] = k == 0 ? pp - upv : pp - f[4];
    };

    // objective scaling (max |grad f| at the start point), constraint-row scaling (max |grad g_i|)
    double gmax = 0.0;
    {
        double g[6];
        cost_grad(x, u, up, g);
#pragma unroll
        for (int i = 0; i < 6; ++i) gmax = fmax(gmax, xon ? fabs(g[i]) : 0.0);
    }
    gmax = wmax(gmax);
    const double sc = gmax > 100.0 ? 100.0 / gmax : 1.0;

    // the derivative pass of iteration 0 runs here, once: its Jacobian columns give the constraint-row
    // scaling, and the loop's first iteration (same point, lambda = 0) takes M~, H~ and x+ as they stand
    double dsc[4];          // scaling of the incoming physical defect rows of node k (up row: 1)
    {
        double sa, ca, xn[4];
        const double lz[5] = {0, 0, 0, 0, 0};
        tilt_sincos_econ(poly, u, sa, ca);
        double scr[4][LM_NSC], cvr[4][4];
        sub_rk4_lin(m, x, sa, xn, scr, cvr);
        const double huu = sub_adjoint_curv(m, scr, cvr, lz, sa);
        if (uon) {
            const LmSub mr = m;
            const double isl = frcp(u - lo), isu = frcp(hi - u);
            const double cu = sc * 2.0 * (Ru + Rdu) + zl * isl + zu * isu;
#pragma unroll 1
            for (int d = 0; d < 5; ++d)
                sub_direction(mr, scr, cvr, huu, LM_G * ca, d, lz, Mk, Hk, d < 4 ? sc * 2.0 * Wq[d] : cu);
            Hk[hp(4, 4)] = sc * 2.0 * Rdu;
            Hk[hp(5, 4)] = -sc * 2.0 * Rdu;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) SO.CS[sl][i] = xn[i];       // x+ of iteration 0 (CS is free until then)
        double rs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double mx = 1.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) mx = fmax(mx, fabs(Mk[j * NC + i]));
            mx = fmax(mx, fabs(Mk[5 * NC + i]));
            rs[i] = uon ? (mx > 100.0 ? 100.0 / mx : 1.0) : 1.0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double t = kWaves == 1 ? from_prev(rs[i]) : 0.0;
            dsc[i] = k == 0 ? 1.0 : t;
        }
        if constexpr (kWaves == 2) {
            double t4[4];
            from_prev_n(rs, t4);
#pragma unroll
            for (int i = 0; i < 4; ++i) dsc[i] = k == 0 ? 1.0 : t4[i];
        }
    }

    const double tol = a.tol, mu_min = tol / 10;
    const double nA = 10.0 * (N + 1), nb = 4.0 * N;     // IPOPT's counts on the full NLP
    const double gam_th = 1e-5, gam_ph = 1e-8, s_th = 1.1, s_ph = 2.3, eta_ph = 1e-8, gam_al = 0.05;

    auto theta_of = [&](const double* g) {
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) t = fma(dsc[i], fabs(g[i]), t);
        return xon ? t + fabs(g[4]) : 0.0;
    };
    double theta;
    {
        double g0[5];
        defects(x, up, u, g0);
        theta = wsum(theta_of(g0));
    }
    const double th_max = 1e4 * fmax(1.0, theta), th_min = 1e-4 * fmax(1.0, theta);
    double fth = 0.0, fph = 0.0;      // filter entry held by lane (slot = lane id)
    int nfilt = 0, acc_count = 0;
    double mu = 0.1, delta_last = 0.0;
    int status = -1, it = 0;

    STAMP(0);
    // it = -1 (a.mult_init_max > 0): IPOPT's least-square estimate of the starting multipliers
    // (DefaultIterateInitializer::least_square_mults, constr_mult_init_max 1000) by the loop's own
    // Riccati machinery: [W J^T; J 0] [d; y] = [-r; 0] with unit weights on x and u, weight 0 on the
    // u_{k-1} copies (their columns then absorb the Delta-u gradient exactly and the defect multipliers
    // are those of the reference NLP, which has no copy rows), r = scaled grad f - z_L + z_U, and a zero
    // defect column; y = the step's new multipliers.  Mirrors ls_multipliers in oracle/lmpc_ipm.c.
    const bool lsinit = a.mult_init_max > 0.0;
    int in_soft = 0, soft_count = 0;       // IPOPT's soft restoration phase (BacktrackingLineSearch)
    bool pformed = false;                  // the inertia tests run on riccati_s_sweep_p (set once, see there)
    int it_start = lsinit ? -1 : 0;
    if constexpr (RESTO) {      // resume a handed-off instance at the start of its failed iteration
        const double* st = a.resto_buf + ((size_t)b * kWave * kWaves + ql) * kLmNst;
        const double* sc0 = a.resto_buf + (size_t)b * kWave * kWaves * kLmNst + kLmNst - 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = st[i];
        up = st[4]; u = st[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) lam[i] = st[6 + i];
        zl = st[11]; zu = st[12]; fth = st[13]; fph = st[14];
        mu = sc0[0]; theta = sc0[kLmNst]; delta_last = sc0[2 * kLmNst];
        it_start = (int)sc0[3 * kLmNst]; nfilt = (int)sc0[4 * kLmNst]; acc_count = (int)sc0[5 * kLmNst];
        pformed = sc0[7 * kLmNst] != 0.0;
#ifdef DART_RESTO_TRACE
        if (lane == 0)
            printf("resume wave %d: mu %.6e theta %.6e delta_last %.6e it %d nfilt %d acc %d\n", wave_idx(), mu, theta,
                   delta_last, it_start, nfilt, acc_count);
#endif
    }

    // ---- helpers of the restoration phases (cold path) -----------------------------------------
    // derivative pass at (xx, uu) with the next node's multipliers lmn: Jacobian columns into M~, the
    // exact dynamics Hessian into H~ (diagonal + cadd), jl = J^T lmn, xn = x+ of node k
    auto deriv_pass = [&](const double* xx, double uu, const double* lmn, const double* cadd4, double cadd_u,
                          double* jl_, double* xn_) {
        double sa, ca;
        tilt_sincos_econ(poly, uu, sa, ca);
        double scr[4][LM_NSC], cvr[4][4];
        sub_rk4_lin(m, xx, sa, xn_, scr, cvr);
        const double huu = sub_adjoint_curv(m, scr, cvr, lmn, sa);
#pragma unroll
        for (int i = 0; i < 5; ++i) jl_[i] = 0.0;
        if (uon) {
            const LmSub mr = m;
#pragma unroll 1
            for (int d = 0; d < 5; ++d)
                jl_[d] = sub_direction(mr, scr, cvr, huu, LM_G * ca, d, lmn, Mk, Hk, d < 4 ? cadd4[d] : cadd_u);
        }
    };
    // incoming augmented defects g_k of node k from x+ of every node (as at the top of the loop)
    auto incoming = [&](const double* xx, double ppv, double uu, const double* xn_, double* g) {
        double cdef[5];
        if constexpr (kWaves == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { const double t = from_next(xx[i]); cdef[i] = xn_[i] - t; }
            { const double t0 = from_next(ppv); cdef[4] = uu - t0; }
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const double t = from_prev(cdef[i]);
                g[i] = k == 0 ? (i < 4 ? xx[i] - st0[i] : ppv - upv) : -t;
            }
        } else {       // two waves: two exchanges
            double t5[5], pcd[5];
            { const double x5[5] = {xx[0], xx[1], xx[2], xx[3], ppv}; from_next_n(x5, t5); }
#pragma unroll
            for (int i = 0; i < 4; ++i) cdef[i] = xn_[i] - t5[i];
            cdef[4] = uu - t5[4];
            from_prev_n(cdef, pcd);
#pragma unroll
            for (int i = 0; i < 5; ++i) g[i] = k == 0 ? (i < 4 ? xx[i] - st0[i] : ppv - upv) : -pcd[i];
        }
    };
    // IPOPT's primal-dual system error at mu (l1 norms of the scaled primal infeasibility, the dual
    // infeasibility and z s - mu, added; IpoptCalculatedQuantities::curr_primal_dual_system_error) at
    // (xx, ppv, uu) with multipliers lm, zlv, zuv.  Overwrites M~ / H~.
    auto pd_l1 = [&](const double* xx, double ppv, double uu, const double* lm, double zlv, double zuv) {
        double lmn[5], jl_[5], xn_[4], g[5], gl[6];
        const double c0z[4] = {0.0, 0.0, 0.0, 0.0};
        if constexpr (kWaves == 1) {
#pragma unroll
            for (int i = 0; i < 5; ++i) { const double t = from_next(lm[i]); lmn[i] = uon ? t : 0.0; }
        } else {
            const double x5[5] = {lm[0], lm[1], lm[2], lm[3], lm[4]};
            double t5[5];
            from_next_n(x5, t5);
#pragma unroll
            for (int i = 0; i < 5; ++i) lmn[i] = uon ? t5[i] : 0.0;
        }
        deriv_pass(xx, uu, lmn, c0z, 0.0, jl_, xn_);
        incoming(xx, ppv, uu, xn_, g);
        double tot = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) tot += xon ? dsc[i] * fabs(g[i]) : 0.0;
        tot += xon ? fabs(g[4]) : 0.0;
        cost_grad(xx, uu, ppv, gl);
#pragma unroll
        for (int j = 0; j < 6; ++j) gl[j] *= sc;
#pragma unroll
        for (int i = 0; i < 5; ++i) gl[i] += lm[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) gl[j] -= jl_[j];
        gl[5] -= jl_[4] + lmn[4] + zlv - zuv;
#pragma unroll
        for (int j = 0; j < 6; ++j) tot += ((j < 5) ? xon : uon) ? fabs(gl[j]) : 0.0;
        tot += uon ? fabs(zlv * (uu - lo) - mu) + fabs(zuv * (hi - uu) - mu) : 0.0;
        return wsum(tot);
    };

    // RESTO: the iteration loop is left for each restoration phase, which runs after it (outside the loop,
    // so that its registers do not burden the iterations) and re-enters it at the next iteration
    bool go_resto = false;
    double phi_rs = 0.0;
    int it_next = it_start;
    for (;;) {
    for (it = it_next;; ++it) {
        const bool lsm = it < 0;
        // the iteration-start values a hand-off parks (the rest of the state changes only on acceptance)
        const double mu_it = mu, dl_it = delta_last;
        const int nfilt_it = nfilt, acc_it = acc_count;
        // hand-off to lmpc_ipm_kernel<true> (<false> only): the state of this iteration's start to HBM; pf = the
        // inertia tests of the resumed iteration run on the explicit value function (riccati_s_sweep_p)
        auto handoff = [&](bool pf) {
            double* st = a.resto_buf + ((size_t)b * kWave * kWaves + ql) * kLmNst;
#pragma unroll
            for (int i = 0; i < 4; ++i) st[i] = x[i];
            st[4] = up; st[5] = u;
#pragma unroll
            for (int i = 0; i < 5; ++i) st[6 + i] = lam[i];
            st[11] = zl; st[12] = zu; st[13] = fth; st[14] = fph;
#ifdef DART_RESTO_TRACE
            if (lane == 0)
                printf("hand-off wave %d: mu %.6e theta %.6e delta_last %.6e it %d nfilt %d acc %d pformed %d\n", wave_idx(),
                       mu_it, theta, dl_it, it, nfilt_it, acc_it, (int)pf);
#endif
            st[15] = lane == 0 ? mu_it : lane == 1 ? theta : lane == 2 ? dl_it : lane == 3 ? (double)it
                   : lane == 4 ? (double)nfilt_it : lane == 5 ? (double)acc_it
                   : lane == 7 ? (pf ? 1.0 : 0.0)
                   : (double)(__builtin_amdgcn_s_memrealtime() - t_start);     // elapsed ticks (lane 6)
            status = kLmNeedResto;
        };
        (void)handoff;
        // ---------------- derivatives, residuals, optimality error ---------------------------
        const double isl = uon ? frcp(u - lo) : 0.0, isu = uon ? frcp(hi - u) : 0.0;
        double lamn[5];
        if constexpr (kWaves == 1) {
#pragma unroll
            for (int i = 0; i < 5; ++i) { const double t = from_next(lam[i]); lamn[i] = uon ? t : 0.0; }
        } else {
            double t5[5];
            from_next_n(lam, t5);
#pragma unroll
            for (int i = 0; i < 5; ++i) lamn[i] = uon ? t5[i] : 0.0;
        }
        double jl[5];       // J^T lambda_{k+1} (x columns 0..3, tilt 4)
        double pinf, pinf_u;  // primal residual maxima
        {
            double xn[4];
            if (it <= 0 && (lsm || !lsinit)) {      // the setup's derivative pass (lambda = 0: J^T lambda = 0)
#pragma unroll
                for (int i = 0; i < 4; ++i) xn[i] = SO.CS[sl][i];
#pragma unroll
                for (int i = 0; i < 5; ++i) jl[i] = 0.0;
            } else {
                double sa, ca;
                tilt_sincos_econ(poly, u, sa, ca);
                // stage data of the RK4 pass stay in registers through the adjoint and the five directions
                double scr[4][LM_NSC], cvr[4][4];
                sub_rk4_lin(m, x, sa, xn, scr, cvr);
                {
                    const double huu = sub_adjoint_curv(m, scr, cvr, lamn, sa);
                    STAMP(13);
                    // exact dynamics Hessian (x, u blocks) and the Jacobian columns of node k
                    if (uon) {
                        const LmSub mr = m;     // model to registers once for the five directions
                        // with the cost / barrier terms of z = [x(4), up, u, 1] on the diagonal (gradient row later)
                        const double cu = sc * 2.0 * (Ru + Rdu) + zl * isl + zu * isu;
#pragma unroll
                        for (int d = 0; d < 5; ++d)
                            jl[d] = sub_direction(mr, scr, cvr, huu, LM_G * ca, d, lamn, Mk, Hk, d < 4 ? sc * 2.0 * Wq[d] : cu);
                        Hk[hp(4, 4)] = sc * 2.0 * Rdu;
                        Hk[hp(5, 4)] = -sc * 2.0 * Rdu;
                    } else {
#pragma unroll
                        for (int i = 0; i < 5; ++i) jl[i] = 0.0;
                    }
                    STAMP(14);
                }
            }
            // outgoing augmented defect c_k = [F(z_k); u_k] - x~_{k+1} -> defect column of M~
            double cdef[5];
            double pcd[5];       // (two waves: the shifts in two exchanges, the incoming ones here)
            if constexpr (kWaves == 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i) { const double t = from_next(x[i]); cdef[i] = xn[i] - t; }
                { const double t0 = from_next(up); cdef[4] = u - t0; }
            } else {
                const double x5[5] = {x[0], x[1], x[2], x[3], up};
                double t5[5];
                from_next_n(x5, t5);
#pragma unroll
                for (int i = 0; i < 4; ++i) cdef[i] = xn[i] - t5[i];
                cdef[4] = u - t5[4];
                from_prev_n(cdef, pcd);
            }
            if (uon) {
#pragma unroll
                for (int r = 0; r < 5; ++r) Mk[6 * NC + r] = cdef[r];
            }
            // incoming defect g_k: primal residuals now, -g_0 = dx~_0 for the forward sweep
            double pl = 0.0, plu = 0.0;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const double t = kWaves == 1 ? from_prev(cdef[i]) : pcd[i];
                double gi = -t;
                if (k == 0) gi = i < 4 ? x[i] - st0[i] : up - upv;
                const double d = i < 4 ? dsc[i] : 1.0;
                pl = fmax(pl, xon ? d * fabs(gi) : 0.0);
                plu = fmax(plu, xon ? fabs(gi) : 0.0);
                if (k == 0) S->dx0[hf][i] = -gi;
                SO.CS[sl][i] = gi;       // c(x) for a second-order correction
            }
            pinf = pl; pinf_u = plu;
        }
        double dinf = 0.0, c0 = 0.0, cmin = 1e300, suml = 0.0, sumz = 0.0;
        {
            double gl[6];
            cost_grad(x, u, up, gl);
#pragma unroll
            for (int j = 0; j < 6; ++j) gl[j] *= sc;
#pragma unroll
            for (int i = 0; i < 5; ++i) gl[i] += lam[i];
#pragma unroll
            for (int j = 0; j < 4; ++j) gl[j] -= jl[j];
            gl[5] -= jl[4] + lamn[4] + zl - zu;
#pragma unroll
            for (int j = 0; j < 6; ++j) dinf = fmax(dinf, (j < 5 ? xon : uon) ? fabs(gl[j]) : 0.0);
#pragma unroll
            for (int i = 0; i < 5; ++i) suml += xon ? fabs(lam[i]) * (i < 4 ? frcp(dsc[i]) : 1.0) : 0.0;
            if (uon) {
                const double cl = zl * (u - lo), cu = zu * (hi - u);
                c0 = fmax(cl, cu); cmin = fmin(cl, cu); sumz = zl + zu;
            }
        }
        float r0 = (float)dinf, r1 = (float)pinf, r2 = (float)pinf_u, r3 = (float)c0, r4 = (float)cmin;
        float r5 = (float)suml, r6 = (float)sumz;
        wred_errors4(r0, r1, r2, r3, r4, r5, r6);
        dinf = r0; pinf = r1; pinf_u = r2; c0 = r3;
        const double cminw = r4;
        suml = r5; sumz = r6;
        // IPOPT's scalings s_d, s_c (>= 1) as reciprocals
        const double is_d = 100.0 * frcp(fmax(100.0, (suml + sumz) * (1.0 / (nA + nb))));
        const double is_c = 100.0 * frcp(fmax(100.0, sumz * (1.0 / nb)));
        const double err = fmax(dinf * is_d, fmax(pinf, c0 * is_c));
        // IPOPT OptimalityErrorConvergenceCheck: optimal, then acceptable, then the iteration cap
        if (!lsm && err <= tol && dinf <= sc && pinf_u <= 1e-4 && c0 <= 1e-4 * sc) { status = 0; break; }
        if (lsm) {
        } else if (a.acc_iter > 0 && err <= a.acc_tol && pinf_u <= 1e-2 && c0 <= 1e-2 * sc) {
            if (++acc_count >= a.acc_iter) { status = 1; break; }
        } else {
            acc_count = 0;
        }
        if (it >= a.max_iter) { status = -1; break; }
        // IPOPT Maximum_CpuTime_Exceeded (not during the least-square estimate: IPOPT's initialisation)
        if (__builtin_expect(!lsm && out_of_time(), 0)) { status = -4; break; }
#ifdef DART_RESTO_TRACE
        if (lane == 0 && !lsm)
            printf("it %3d mu %.2e err %.2e dinf %.2e pinf %.2e c0 %.2e cmin %.2e suml %.3e sumz %.3e theta %.3e\n", it, mu, err,
                   dinf * is_d, pinf, c0 * is_c, cminw, suml, sumz, theta);
#endif
        for (; !lsm;) {
            const double cmu = fmax(c0 - mu, mu - cminw);
            if (fmax(dinf * is_d, fmax(pinf, cmu * is_c)) > 10.0 * mu || mu <= mu_min) break;
            mu = fmax(mu_min, fmin(0.2 * mu, mu * sqrt(mu)));
            nfilt = 0; in_soft = 0;       // BacktrackingLineSearch::Reset: the filter and the soft phase
        }
        const double tau = fmax(0.99, 1.0 - mu);
        STAMP(1);

        // ---------------- gradient rows (they depend on mu) ------------------------------------
        if (lsm) {      // the least-square system: unit weights on x and u, 0 on the copy, zero defects
            double gq[6];
            cost_grad(x, u, up, gq);
#pragma unroll
            for (int j = 0; j < 6; ++j) gq[j] *= sc;
            if (uon) {
                gq[5] += zu - zl;
                for (int e = 0; e < LmLds::NTP; ++e) Hk[e] = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) Hk[hp(i, i)] = 1.0;
                Hk[hp(5, 5)] = 1.0;
#pragma unroll
                for (int j = 0; j < 6; ++j) Hk[hp(6, j)] = gq[j];
#pragma unroll
                for (int r = 0; r < 5; ++r) Mk[6 * NC + r] = 0.0;
            }
            if (k == 0) {
#pragma unroll
                for (int r = 0; r < 5; ++r) S->dx0[hf][r] = 0.0;
            }
            if (k == N) {
                double* GN = S->G[sl];
                for (int e = 0; e < LmLds::NTP; ++e) GN[e] = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) GN[gszz<5>(i, i)] = 1.0;
#pragma unroll
                for (int j = 0; j < 5; ++j) GN[gszz<5>(5, j)] = gq[j];
                GN[hp(5, 5)] = 1.0;
            }
        } else {
            double gq[6];
            cost_grad(x, u, up, gq);
#pragma unroll
            for (int j = 0; j < 6; ++j) gq[j] *= sc;
            if (uon) {
                gq[5] += -mu * isl + mu * isu;
#pragma unroll
                for (int j = 0; j < 6; ++j) Hk[hp(6, j)] = gq[j];
            }
            if (k == N) {   // terminal surrogate G_N: value function [[2 Qt, q_N], [q_N^T, 0]] on x~, Quu = 1
                double* GN = S->G[sl];
                for (int e = 0; e < LmLds::NTP; ++e) GN[e] = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) GN[gszz<5>(i, i)] = sc * 2.0 * Qtv[i];
#pragma unroll
                for (int j = 0; j < 5; ++j) GN[gszz<5>(5, j)] = gq[j];
                GN[hp(5, 5)] = 1.0;
            }
        }
        __syncthreads();
        STAMP(2);
        if (lsm) {
            (void)riccati_s_sweep(S, N, RR);      // unit weights: every Quu >= 1
            closed_loop_s(S, N);
            double dxl[5], lmp[5];
            forward_sweep_s(S, N, k, dxl);
            const double* K = S->KK[uon ? sl : hf * LM_NMAXS];
            double d0 = K[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) d0 = fma(K[j], dxl[j], d0);
            node_multiplier_s(S, xon ? sl : hf * LM_NMAXS, dxl, uon ? d0 : 0.0, lmp);
            // constr_mult_init_max on IPOPT's (row-scaled) multipliers of the reference's rows
            double ym = 0.0;
            bool fin = true;        // an overflowed recursion (stiff, unstable dynamics) counts as too large
#pragma unroll
            for (int i = 0; i < 4; ++i) ym = fmax(ym, xon ? fabs(lmp[i]) * frcp(dsc[i]) : 0.0);
#pragma unroll
            for (int i = 0; i < 5; ++i) fin = fin && (!xon || isfinite(lmp[i]));
            if (!wany(!fin) && wmax(ym) <= a.mult_init_max) {
#pragma unroll
                for (int i = 0; i < 5; ++i) lam[i] = xon ? lmp[i] : 0.0;
            }
            continue;
        }

        // ---------------- Newton step and filter line search ----------------------------------
        // One copy of the Riccati solve serves the plain Newton step (with inertia correction) and
        // IPOPT's second-order correction passes (FilterLSAcceptor::TrySecondOrderCorrection; max_soc,
        // kappa_soc 0.99): a rejected full step with theta(trial) >= theta re-solves the system with
        // c_soc <- alpha_soc c_soc + c(x_trial) (from c(x), alpha_soc = alpha) in the defect column of
        // M~ and dx~_0 (H~, incl. the inertia shift, is unchanged) and tries x + alpha_soc d_soc.
        double dx[5], dU = 0.0, lamp[5], gt[5], dzl = 0.0, dzu = 0.0;
        double amax = 1.0, az = 1.0, phi = 0.0, gTd = 0.0, amin = 0.0, alpha = 1.0, th_t = 0.0, ph_t = 0.0;
        double th_prev = 0.0;
        float lg_sw = 0.0f;
        bool accepted = false, ftype = false, tiny = false, ok = true;
        int ls = 0, soc = -1;        // soc: -1 plain step, >= 0 second-order-correction pass
        // the Newton step from the factorised stage QPs: forward sweep, du = K [dx~; 1], lambda+
        auto recover_step = [&]() {
            forward_sweep_s(S, N, k, dx);
            STAMP(12);
            const double* K = S->KK[uon ? sl : hf * LM_NMAXS];
            double d0 = K[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) d0 = fma(K[j], dx[j], d0);
            dU = uon ? d0 : 0.0;
            node_multiplier_s(S, xon ? sl : hf * LM_NMAXS, dx, dU, lamp);
        };
        // primal fraction to the boundary of dU: this lane's, and the wave's (reduced in f32 with a 2^-20 margin)
        auto primal_ftb_l = [&]() {
            double am = 1.0;
            if (uon) {
                if (dU < 0) am = fmin(am, -tau * (u - lo) * frcp(dU));
                if (dU > 0) am = fmin(am, tau * (hi - u) * frcp(dU));
            }
            return (float)am;
        };
        auto primal_ftb = [&]() { return (double)wminf(primal_ftb_l()) * (1.0 - 1.0 / 1048576.0); };
        // bound-multiplier directions of dU and their fraction to the boundary: this lane's, and the wave's
        auto dual_step_l = [&]() {
            dzl = uon ? mu * isl - zl - zl * isl * dU : 0.0;
            dzu = uon ? mu * isu - zu + zu * isu * dU : 0.0;
            double az_ = 1.0;
            if (uon) {
                if (dzl < 0) az_ = fmin(az_, -tau * zl * frcp(dzl));
                if (dzu < 0) az_ = fmin(az_, -tau * zu * frcp(dzu));
            }
            return (float)az_;
        };
        auto dual_step = [&]() { return (double)wminf(dual_step_l()) * (1.0 - 1.0 / 1048576.0); };
        // trial point x + al d: incoming defects gt of node k, wave-summed theta and barrier objective
        auto trial = [&](double al) {
            double xt[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) xt[i] = fma(al, dx[i], x[i]);
            const double pt = fma(al, dx[4], up), ut = fma(al, dU, u);
            defects(xt, pt, ut, gt);
            double phl = sc * cost_val(xt, ut, pt);
            if (uon) phl -= mu * log_fast((ut - lo) * (hi - ut));
            double thl = theta_of(gt);
            wsum2(thl, phl);
            th_t = thl; ph_t = phl;
        };
        // filter acceptance of (th_t, ph_t) for the step size al_test (IPOPT alpha_primal_test)
        auto acceptable = [&](double al_test, bool& ft) {
            bool in_filter = !(th_t < th_max) || !isfinite(ph_t);
            in_filter = in_filter || wany_rep(lane < nfilt && th_t >= fth && ph_t >= fph);
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
                double cs[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) cs[i] = xon ? SO.CS[sl][i] : 0.0;
#pragma unroll
                for (int r = 0; r < 5; ++r) {
                    const double t = from_next(cs[r]);
                    if (uon) Mk[6 * NC + r] = -t;
                    if (k == 0) S->dx0[hf][r] = -cs[r];
                }
                __syncthreads();
                STAMP_ADD(15, 1);
            }
            {
                double delta = 0.0, dapplied = 0.0;
                int attempt = 0;
                for (;;) {
                    if constexpr (RESTO) ok = pformed ? riccati_s_sweep_p(S, SH.Ps, N, RR) : riccati_s_sweep(S, N, RR);
                    else ok = riccati_s_sweep(S, N, RR);
#ifdef DART_RESTO_TRACE
                    if (blockIdx.x == 0 && (it <= 0 || N > 31) && attempt < 3) {
                        bool fin = true;
                        if (uon) {
                            for (int e = 0; e < LmLds::NTP; ++e) fin = fin && isfinite(Hk[e]);
                            for (int e = 0; e < LmLds::ND * NC; ++e) fin = fin && isfinite(Mk[e]);
                        }
                        const double q = S->G[sl][hp(5, 5)];
                        const bool qbad = uon && !(q > 0.0 && isfinite(q));
                        const unsigned long long nf = __ballot(!fin), nq = __ballot(qbad);
                        if (lane == 0)
                            printf("  wave %d it %d attempt %d delta %.2e ok %d  lanes with non-finite H/M %llx  lanes with Quu<=0 %llx\n",
                                   wave_idx(), it, attempt, delta, (int)ok, nf, nq);
                        if (qbad && (nq & ((1ull << lane) - 1)) == 0)
                            printf("    wave %d first bad lane %d (node %d half %d) Quu %.3e  H diag %.3e %.3e %.3e %.3e %.3e %.3e\n", wave_idx(), lane, k,
                                   hf, q, Hk[hp(0, 0)], Hk[hp(1, 1)], Hk[hp(2, 2)], Hk[hp(3, 3)], Hk[hp(4, 4)], Hk[hp(5, 5)]);
                    }
#endif
                    if (ok || soc >= 0) break;
                    if (++attempt >= 60) {
                        // the folded recursion fails the inertia test at every perturbation: where the value function
                        // reaches ~1e18 its sign decisions part from the explicit form IPOPT-style recursions (and
                        // the oracle) take -- the whole perturbation sequence again with P formed, for the rest of
                        // the solve (profiles/r04/lmpc_riccati_probe_*.txt; 2 of 28,800 C5 stress instances).  That
                        // form lives in <true> only (the fast kernel keeps its registers): <false> hands over.
                        if (!RESTO || pformed) break;
                        pformed = true; attempt = 0; delta = 0.0;
                    } else {
                        delta = (attempt == 1) ? (delta_last == 0.0 ? 1e-4 : fmax(1e-20, delta_last * (1.0 / 3.0)))   // IPOPT perturb_dec_fact 1/3
                                               : delta * (delta_last == 0.0 ? 100.0 : 8.0);
                    }
                    const double dd = delta - dapplied;
                    if (uon) {
#pragma unroll
                        for (int j = 0; j < 6; ++j) Hk[hp(j, j)] += dd;
                    }
                    if (k == N) {
#pragma unroll
                        for (int j = 0; j < 5; ++j) S->G[sl][gszz<5>(j, j)] += dd;
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
            closed_loop_s(S, N);
            STAMP(11);
            recover_step();
            STAMP(4);
            double al_try;
            if (soc < 0) {
                // the two fraction minima, the line search's two sums and the tiny-step maximum: one lock-step
                // reduction (each value takes its own reduction's steps: the same bits)
                float amf = primal_ftb_l(), azf = dual_step_l();
                STAMP(5);
                double phil = sc * cost_val(x, u, up), gtdl = 0.0;
                if (uon) phil -= mu * log_fast((u - lo) * (hi - u));
                {
                    double gz_[6];
                    cost_grad(x, u, up, gz_);
#pragma unroll
                    for (int i = 0; i < 5; ++i) gtdl += xon ? sc * gz_[i] * dx[i] : 0.0;
                    if (uon) gtdl += (sc * gz_[5] - mu * isl + mu * isu) * dU;
                }
                float tnl = 0.0f;
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const double xi = i < 4 ? x[i] : up;
                    tnl = fmaxf(tnl, xon ? fabsf((float)dx[i]) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)xi)) : 0.0f);
                }
                if (uon) tnl = fmaxf(tnl, fabsf((float)dU) * __builtin_amdgcn_rcpf(1.0f + fabsf((float)u)));
                wsum2_maxf_min2f(phil, gtdl, tnl, amf, azf);
                amax = (double)amf * (1.0 - 1.0 / 1048576.0);
                az = (double)azf * (1.0 - 1.0 / 1048576.0);
                tiny = tnl < 2.2e-15f;
                phi = phil; gTd = gtdl;
                const float lg_th = theta > 0.0 ? lg2(theta) : -3.0e38f;
                const float lg_gd = gTd < 0.0 ? lg2(-gTd) : 3.0e38f;
                lg_sw = (float)s_th * lg_th - (float)s_ph * lg_gd;
                amin = gam_th;
                if (gTd < 0.0) amin = fmin(gam_th, fmin(gam_ph * theta * frcp(-gTd), (double)__builtin_amdgcn_exp2f(fmaxf(lg_sw, -126.0f))));
                amin *= gam_al;
                alpha = amax;
                al_try = alpha;
                STAMP(6);
            } else {
                al_try = primal_ftb();
            }
            bool resolve = false;
            for (; !in_soft;) {
                trial(al_try);
                if (soc < 0) {
                    if (tiny) { accepted = true; ftype = true; break; }
                    if (acceptable(alpha, ftype)) { accepted = true; break; }
                    if (ls == 0 && a.max_soc > 0 && !(th_t < theta)) {
                        if (xon) {      // c_soc = alpha c(x) + c(x_trial); keep the plain step
#pragma unroll
                            for (int i = 0; i < 5; ++i) {
                                SO.CS[sl][i] = fma(alpha, SO.CS[sl][i], gt[i]);
                                SO.SV[sl][i] = dx[i]; SO.SV[sl][5 + i] = lamp[i];
                            }
                            SO.SV[sl][10] = dU;
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
                            for (int i = 0; i < 5; ++i) SO.CS[sl][i] = fma(al_try, SO.CS[sl][i], gt[i]);
                        }
                        th_prev = th_t; ++soc; resolve = true;
                        break;
                    }
                    if (xon) {      // corrections failed: back to the plain step, backtrack
#pragma unroll
                        for (int i = 0; i < 5; ++i) { dx[i] = SO.SV[sl][i]; lamp[i] = SO.SV[sl][5 + i]; }
                        dU = SO.SV[sl][10];
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
        if (!ok) {
            if constexpr (!RESTO) {
                // (ok is false here only after 60 failed perturbations: a second-order-correction pass keeps its
                // sweep whatever the inertia test says, `if (soc >= 0) ok = true` above)
                if (a.resto) { handoff(true); break; }
            }
            status = -3;
            break;
        }
        STAMP_ADD(10, ls + 1);
        STAMP(7);
        // ---------------- IPOPT's soft restoration phase (BacktrackingLineSearch::TrySoftRestoStep) ------
        // the line search failed, or the soft phase is on: the primal-dual step damped only by the
        // fractions to the boundary (one length for x, lambda and z) is taken if the original filter
        // accepts it with alpha_primal_test = 0 (the phase ends) or if it cuts the primal-dual system
        // error at mu by the factor 0.9999; at most max_soft_resto_iters = 10 steps
        if constexpr (!RESTO) {
            if (!accepted && a.resto) {
                handoff(pformed);
                break;
            }
        }
        bool soft = false;
        if (RESTO && !accepted) {
            if (!in_soft) {         // PrepareRestoPhaseStart: the current point enters the filter
                if (nfilt < kWave) {
                    if (lane == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
                    ++nfilt;
                }
                soft_count = 0;
            }
            if (!(in_soft && ++soft_count > 10)) {
                const double as = fmin(amax, az);
                trial(as);
                bool ft = false;
                const bool orig = acceptable(0.0, ft);
                bool take = orig;
                if (!take && isfinite(ph_t)) {
                    double pd0 = 0.0, pd1 = 0.0;
#pragma unroll 1
                    for (int pass = 0; pass < 2; ++pass) {
                        const double al = pass ? as : 0.0;
                        double xx[4], lm[5];
#pragma unroll
                        for (int i = 0; i < 4; ++i) xx[i] = fma(al, dx[i], x[i]);
#pragma unroll
                        for (int i = 0; i < 5; ++i) lm[i] = fma(al, lamp[i] - lam[i], lam[i]);
                        const double e = pd_l1(xx, fma(al, dx[4], up), uon ? fma(al, dU, u) : u, lm, fma(al, dzl, zl),
                                               fma(al, dzu, zu));
                        if (pass) pd1 = e; else pd0 = e;
                    }
                    take = pd1 <= 0.9999 * pd0;
                }
                if (take) {
                    accepted = true; soft = true; alpha = as; az = as;
                    in_soft = orig ? 0 : 1;
                    if (orig) soft_count = 0;
                }
            }
        }
        // ---------------- IPOPT's restoration phase (MinC_1NrmRestorationPhase) -------------------------
        // (oracle/lmpc_ipm.c `restoration`; the soft-row Riccati sweep above).  rho 1000, eta = sqrt(mu_R),
        // D_R = 1 / max(1, |x_R|); start mu_R = max(mu, ||d c||_inf), closed-form p, n, z_p = mu_R / p,
        // z_n = mu_R / n, u-bound multipliers min(rho, z), least-square equality multipliers; its own
        // filter, mu, inertia correction and second-order correction; leaves when the original problem's
        // theta falls to 0.9 of its start value and the original filter accepts the point.
        if (RESTO && !accepted) { phi_rs = phi; go_resto = true; break; }
        if (!accepted) { status = -2; break; }
        if (!soft && !ftype && nfilt < kWave) {
            if (lane == nfilt) { fth = (1 - gam_th) * theta; fph = phi - gam_ph * theta; }
            ++nfilt;
        }
        // ---------------- accept ------------------------------------------------------------
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = xon ? fma(alpha, dx[i], x[i]) : x[i];
        up = xon ? fma(alpha, dx[4], up) : up;
#pragma unroll
        for (int i = 0; i < 5; ++i) lam[i] = xon ? fma(alpha, lamp[i] - lam[i], lam[i]) : 0.0;
        if (uon) {
            u = fma(alpha, dU, u);
            const double il = frcp(u - lo), iu = frcp(hi - u);
            zl = fmax(fmin(fma(az, dzl, zl), 1e10 * mu * il), 1e-10 * mu * il);
            zu = fmax(fmin(fma(az, dzu, zu), 1e10 * mu * iu), 1e-10 * mu * iu);
        }
        theta = th_t;
        STAMP(8);
    }
    if (!RESTO || !go_resto) break;
    go_resto = false;
    {
            const double tau = fmax(0.99, 1.0 - mu);
            const double mu0 = mu, th0 = theta, phi0 = phi_rs, tau0 = tau, rho = 1000.0;
            double* const pc = RL->PN[sl];
            double* const nc = pc + 4;
            double* const zp = pc + 8;
            double* const zn = pc + 12;
            double* const rp = pc + 16;
            double* const rn = pc + 20;
            double* const sp = pc + 24;
            double* const sn = pc + 28;
            double* const xr = pc + 32;
            double* const drx = pc + 36;
#pragma unroll
            for (int i = 0; i < 4; ++i) { xr[i] = x[i]; drx[i] = 1.0 / fmax(1.0, fabs(x[i])); }
            const double ur = u, dru = 1.0 / fmax(1.0, fabs(u));
            double g0[5];
            defects(x, up, u, g0);
            double cmx = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) cmx = fmax(cmx, xon ? dsc[i] * fabs(g0[i]) : 0.0);
            cmx = fmax(cmx, xon ? fabs(g0[4]) : 0.0);
            double rmu = fmax(mu0, wmax(cmx));
            double eta = sqrt(rmu);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double c = dsc[i] * g0[i];
                const double aa = rmu / (2.0 * rho) - 0.5 * c, bb = c * rmu / (2.0 * rho);
                nc[i] = xon ? aa + sqrt(aa * aa + bb) : 1.0;
                pc[i] = xon ? c + nc[i] : 1.0;
                zp[i] = xon ? rmu / pc[i] : 0.0;
                zn[i] = xon ? rmu / nc[i] : 0.0;
            }
            double rzl = uon ? fmin(rho, zl) : 0.0, rzu = uon ? fmin(rho, zu) : 0.0;
            double rl[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
            double jl[5], xn[4], lmn[5];
            // H~ of the restoration problem: the dynamics Hessian (derivative pass, cadd = 0), then eta D_R^2
            // and Sigma_u on the diagonal; no Delta-u cost
            auto stage = [&]() {
#pragma unroll
                for (int i = 0; i < 5; ++i) { const double t = from_next(rl[i]); lmn[i] = uon ? t : 0.0; }
                const double c0z[4] = {0.0, 0.0, 0.0, 0.0};
                deriv_pass(x, u, lmn, c0z, 0.0, jl, xn);
                if (uon) { Hk[hp(4, 4)] = 0.0; Hk[hp(5, 4)] = 0.0; }
            };
            // gradient rows of the stage QPs and the terminal surrogate (lsq: unit weights)
            auto grad_rows = [&](bool lsq) {
                if (uon) {
                    const double isl = frcp(u - lo), isu = frcp(hi - u);
#pragma unroll
                    for (int i = 0; i < 4; ++i) Hk[hp(6, i)] = eta * drx[i] * drx[i] * (x[i] - xr[i]);
                    Hk[hp(6, 4)] = 0.0;
                    Hk[hp(6, 5)] = lsq ? fma(eta * dru * dru, u - ur, rzu - rzl)
                                       : fma(eta * dru * dru, u - ur, rmu * isu - rmu * isl);
                }
                if (k == N) {
                    double* GN = S->G[sl];
                    for (int e = 0; e < LmLds::NTP; ++e) GN[e] = 0.0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        GN[gszz<5>(i, i)] = lsq ? 1.0 : eta * drx[i] * drx[i];
                        GN[gszz<5>(5, i)] = eta * drx[i] * drx[i] * (x[i] - xr[i]);
                    }
                    GN[hp(5, 5)] = 1.0;
                }
            };
            // soft rows of node k's incoming physical rows (Sigma + delta, 1 / D) and the right-hand
            // side from the constraint values cv: rg = cv / d - (rn / Sn - rp / Sp) / d + D lambda
            // (copy row: cv), into the defect column of M~ and dx~_0
            auto soft_rows = [&](double delta, bool lsq, const double* cv) {
                double rg[5];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const double d = dsc[i];
                    sp[i] = lsq ? 1.0 : zp[i] / pc[i] + delta;
                    sn[i] = lsq ? 1.0 : zn[i] / nc[i] + delta;
                    const double Dd = (1.0 / sp[i] + 1.0 / sn[i]) / (d * d);
                    RL->Dinv[sl][i] = 1.0 / Dd;
                    rg[i] = cv[i] / d - (rn[i] / sn[i] - rp[i] / sp[i]) / d + Dd * rl[i];
                }
                rg[4] = cv[4];
#pragma unroll
                for (int r = 0; r < 5; ++r) {
                    const double t = from_next(rg[r]);
                    if (uon) Mk[6 * NC + r] = -t;
                    if (k == 0) S->dx0[hf][r] = -rg[r];
                }
            };
            // the step from the factorised soft system: dx~_0 and the closed-loop rows through the soft
            // rows, forward sweep, du, lambda+
            auto post_soft = [&](int slt, int) {
                const double* T = RL->T[slt + 1];
                double F[5][6];
#pragma unroll
                for (int r = 0; r < 5; ++r)
#pragma unroll
                    for (int j = 0; j < 6; ++j) F[r][j] = S->F[slt][r][j];
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int j = 0; j < 6; ++j) {
                        double t = F[r][j] - (j == 5 ? T[6 * r + 5] : 0.0);
#pragma unroll
                        for (int aa = 0; aa < 5; ++aa) t -= T[6 * r + aa] * F[aa][j];
                        S->F[slt][r][j] = t;
                    }
            };
            double dxr[5], dUr = 0.0, lpr[5];
            auto resto_step = [&]() {
                if (k == 0) {
                    double d0[5];
#pragma unroll
                    for (int r = 0; r < 5; ++r) d0[r] = S->dx0[hf][r];
                    const double* T0 = RL->T[hf * LM_NMAXS];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        double t = d0[r] - T0[6 * r + 5];
#pragma unroll
                        for (int aa = 0; aa < 5; ++aa) t -= T0[6 * r + aa] * d0[aa];
                        S->dx0[hf][r] = t;
                    }
                }
                __syncthreads();
                closed_loop_s(S, N, post_soft);
                forward_sweep_s(S, N, k, dxr);
                const double* K = S->KK[uon ? sl : hf * LM_NMAXS];
                double d0 = K[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) d0 = fma(K[j], dxr[j], d0);
                dUr = uon ? d0 : 0.0;
                node_multiplier_s(S, xon ? sl : hf * LM_NMAXS, dxr, dUr, lpr);
            };
            // least-square equality multipliers of the restoration problem (unit weights on x, u, p, n:
            // D = 2 / d^2, right-hand side (rp - rn) / d with rp = rho - z_p, rn = rho - z_n)
#pragma unroll
            for (int i = 0; i < 4; ++i) { rp[i] = rho - zp[i]; rn[i] = rho - zn[i]; }
            {
                stage();
                if (uon) {
                    for (int e = 0; e < LmLds::NTP; ++e) Hk[e] = 0.0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) Hk[hp(i, i)] = 1.0;
                    Hk[hp(5, 5)] = 1.0;
                }
                grad_rows(true);
                const double cz[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
                soft_rows(0.0, true, cz);
                __syncthreads();
                (void)riccati_s_sweep_soft(S, RL, N, RR, false);
                resto_step();
                double ym = 0.0;
                bool fin = true;
#pragma unroll
                for (int i = 0; i < 4; ++i) ym = fmax(ym, xon ? fabs(lpr[i]) / dsc[i] : 0.0);
#pragma unroll
                for (int i = 0; i < 5; ++i) fin = fin && (!xon || isfinite(lpr[i]));
                const bool use = !wany(!fin) && wmax(ym) <= 1e3;
#pragma unroll
                for (int i = 0; i < 5; ++i) rl[i] = (use && xon) ? lpr[i] : 0.0;
            }
            STAMP(16);      // restoration start: reference point, p / n, least-square multipliers
            int rit = it + 1, rnf = 0, racc_count = 0, rstat = -2;
            bool rfirst = true, rok = false;
            double rfth = 0.0, rfph = 0.0, rdelta_last = 0.0, thr = 0.0, rth_max = 0.0, rth_min = 0.0;
            double cres[5];
            for (;; ++rit) {
                stage();
                STAMP(17);
                double g[5];
                incoming(x, up, u, xn, g);
#pragma unroll
                for (int i = 0; i < 4; ++i) cres[i] = xon ? dsc[i] * g[i] + nc[i] - pc[i] : 0.0;
                cres[4] = xon ? g[4] : 0.0;
                if (rfirst) {
                    double t = 0.0;
#pragma unroll
                    for (int i = 0; i < 5; ++i) t += fabs(cres[i]);
                    thr = wsum(t);
                    rth_max = 1e4 * fmax(1.0, thr); rth_min = 1e-4 * fmax(1.0, thr);
                } else {
                    // RestoConvergenceCheck: the original problem's progress at the current point
                    const double tho = wsum(theta_of(g));
                    if (tho <= 0.9 * th0) {
                        double pl = sc * cost_val(x, u, up);
                        if (uon) pl -= mu0 * log_fast((u - lo) * (hi - u));
                        const double pho = wsum(pl);
                        bool accp = isfinite(pho) && !wany_rep(lane < nfilt && tho >= fth && pho >= fph);
                        accp = accp && (cmp_le(tho, (1 - gam_th) * th0, th0) || cmp_le(pho - phi0, -gam_ph * th0, phi0));
                        if (accp) { rok = true; theta = tho; break; }
                    }
                }
                rfirst = false;
                // optimality error of the restoration problem
                double dinf = 0.0, pinf = 0.0, c0r = 0.0, cminr = 1e300, suml = 0.0, sumz = 0.0;
                {
                    double gl[6];
#pragma unroll
                    for (int i = 0; i < 4; ++i) gl[i] = eta * drx[i] * drx[i] * (x[i] - xr[i]) + rl[i] - jl[i];
                    gl[4] = rl[4];
                    gl[5] = eta * dru * dru * (u - ur) - jl[4] - lmn[4] - rzl + rzu;
#pragma unroll
                    for (int j = 0; j < 6; ++j) dinf = fmax(dinf, ((j < 5) ? xon : uon) ? fabs(gl[j]) : 0.0);
                    if (xon) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const double y = rl[i] / dsc[i];
                            dinf = fmax(dinf, fmax(fabs(rho - zp[i] - y), fabs(rho - zn[i] + y)));
                            pinf = fmax(pinf, fabs(cres[i]));
                            c0r = fmax(c0r, fmax(zp[i] * pc[i], zn[i] * nc[i]));
                            cminr = fmin(cminr, fmin(zp[i] * pc[i], zn[i] * nc[i]));
                            sumz += zp[i] + zn[i];
                            suml += fabs(y);
                        }
                        pinf = fmax(pinf, fabs(cres[4]));
                        suml += fabs(rl[4]);
                    }
                    if (uon) {
                        const double cl = rzl * (u - lo), cu = rzu * (hi - u);
                        c0r = fmax(c0r, fmax(cl, cu)); cminr = fmin(cminr, fmin(cl, cu));
                        sumz += rzl + rzu;
                    }
                    dinf = wmax(dinf); pinf = wmax(pinf); c0r = wmax(c0r); cminr = wmin(cminr);
                    suml = wsum(suml); sumz = wsum(sumz);
                }
                const double nbr = 4.0 * N + 16.0 * (N + 1);
                const double s_d = fmax(100.0, (suml + sumz) / (nA + nbr)) / 100.0;
                const double s_c = fmax(100.0, sumz / nbr) / 100.0;
                const double errr = fmax(dinf / s_d, fmax(pinf, c0r / s_c));
#ifdef DART_RESTO_TRACE
                const double errr_t = errr, dinf_t = dinf / s_d, pinf_t = pinf, c0_t = c0r / s_c;
#endif
                if (rit >= a.max_iter) { rstat = -1; break; }
                if (out_of_time()) { rstat = -4; break; }
                // the restoration problem converged: local infeasibility (IPOPT Infeasible_Problem_Detected, 2)
                if (errr <= tol && dinf <= 1.0 && pinf <= 1e-4 && c0r <= 1e-4) { rstat = 2; break; }
                if (a.acc_iter > 0 && errr <= a.acc_tol && pinf <= 1e-2 && c0r <= 1e-2) {
                    if (++racc_count >= a.acc_iter) { rstat = 2; break; }
                } else {
                    racc_count = 0;
                }
                for (;;) {
                    const double cmu = fmax(c0r - rmu, rmu - cminr);
                    if (fmax(dinf / s_d, fmax(pinf, cmu / s_c)) > 10.0 * rmu || rmu <= mu_min) break;
                    rmu = fmax(mu_min, fmin(0.2 * rmu, rmu * sqrt(rmu)));
                    eta = sqrt(rmu);
                    rnf = 0;
                }
                const double taur = fmax(0.99, 1.0 - rmu);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    rp[i] = rho - rmu / pc[i] - rl[i] / dsc[i];
                    rn[i] = rho - rmu / nc[i] + rl[i] / dsc[i];
                }
                const double isl = uon ? frcp(u - lo) : 0.0, isu = uon ? frcp(hi - u) : 0.0;
                if (uon) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) Hk[hp(i, i)] += eta * drx[i] * drx[i];
                    Hk[hp(5, 5)] += eta * dru * dru + rzl * isl + rzu * isu;
                }
                grad_rows(false);
                STAMP(18);
                double delta = 0.0, dapplied = 0.0;
                int attempt = 0;
                bool okr = false;
                for (;;) {
                    soft_rows(delta, false, cres);
                    __syncthreads();
                    okr = riccati_s_sweep_soft(S, RL, N, RR, true);
                    if (okr || ++attempt >= 60) break;
                    delta = (attempt == 1) ? (rdelta_last == 0.0 ? 1e-4 : fmax(1e-20, rdelta_last * (1.0 / 3.0)))
                                           : delta * (rdelta_last == 0.0 ? 100.0 : 8.0);
                    const double dd = delta - dapplied;
                    if (uon) {
#pragma unroll
                        for (int j = 0; j < 6; ++j) Hk[hp(j, j)] += dd;
                    }
                    if (k == N) {
#pragma unroll
                        for (int j = 0; j < 5; ++j) S->G[sl][gszz<5>(j, j)] += dd;
                    }
                    dapplied = delta;
                }
                STAMP(19);
                STAMP_ADD(24, attempt + 1);
                if (!okr) { rstat = -3; break; }
                if (delta > 0.0) rdelta_last = delta;
                // the step of p, n and every bound multiplier, and the fractions to the boundary
                double dpc[4], dnc[4], dzp[4], dzn[4], dzlr = 0.0, dzur = 0.0, amr = 1.0, azr = 1.0;
                auto pn_steps = [&]() {
                    double am = 1.0, a2 = 1.0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const double dy = (lpr[i] - rl[i]) / dsc[i];
                        dpc[i] = xon ? (dy - rp[i]) / sp[i] : 0.0;
                        dnc[i] = xon ? (-dy - rn[i]) / sn[i] : 0.0;
                        dzp[i] = xon ? rmu / pc[i] - zp[i] - zp[i] / pc[i] * dpc[i] : 0.0;
                        dzn[i] = xon ? rmu / nc[i] - zn[i] - zn[i] / nc[i] * dnc[i] : 0.0;
                        if (dpc[i] < 0) am = fmin(am, -taur * pc[i] / dpc[i]);
                        if (dnc[i] < 0) am = fmin(am, -taur * nc[i] / dnc[i]);
                        if (dzp[i] < 0) a2 = fmin(a2, -taur * zp[i] / dzp[i]);
                        if (dzn[i] < 0) a2 = fmin(a2, -taur * zn[i] / dzn[i]);
                    }
                    dzlr = uon ? rmu * isl - rzl - rzl * isl * dUr : 0.0;
                    dzur = uon ? rmu * isu - rzu + rzu * isu * dUr : 0.0;
                    if (uon) {
                        if (dUr < 0) am = fmin(am, -taur * (u - lo) / dUr);
                        if (dUr > 0) am = fmin(am, taur * (hi - u) / dUr);
                        if (dzlr < 0) a2 = fmin(a2, -taur * rzl / dzlr);
                        if (dzur < 0) a2 = fmin(a2, -taur * rzu / dzur);
                    }
                    amr = wmin(am); azr = wmin(a2);
                };
#if DART_RESTO_REFINE
                // one step of iterative refinement of the restoration step (IPOPT's PDFullSpaceSolver refines
                // every KKT solve): the residuals of the Newton system at (dx, du, lambda+) -- soft constraint
                // rows and stationarity rows -- as the right-hand side of the same factorised soft system
                // (D, Sigma and the quadratic parts unchanged), the correction added to the step
                auto refine = [&](const double* cv) -> bool {
                    double lpn_[5], pdx[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) { const double t = from_next(lpr[i]); lpn_[i] = uon ? t : 0.0; }
#pragma unroll
                    for (int i = 0; i < 5; ++i) pdx[i] = from_prev(dxr[i]);
                    const double pdu = from_prev(dUr);
                    double rc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
                    if (xon) {
                        const double* Mp = &S->M[k > 0 ? sl - 1 : sl][0][0];
#pragma unroll
                        for (int i = 0; i < 5; ++i) {
                            double jd = dxr[i];
                            if (k > 0) {
#pragma unroll
                                for (int m = 0; m < 5; ++m) jd -= Mp[m * NC + i] * pdx[m];
                                jd -= Mp[5 * NC + i] * pdu;
                            }
                            if (i < 4) {
                                const double dy = (lpr[i] - rl[i]) / dsc[i];
                                const double dpi = (dy - rp[i]) / sp[i], dni = (-dy - rn[i]) / sn[i];
                                rc[i] = dsc[i] * jd + dni - dpi + cv[i];
                            } else {
                                rc[i] = jd + cv[i];
                            }
                        }
                    }
                    double rs[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
                    double* GN = S->G[sl];
                    if (uon) {
                        const double zv[6] = {dxr[0], dxr[1], dxr[2], dxr[3], dxr[4], dUr};
#pragma unroll
                        for (int j = 0; j < 6; ++j) {
                            double t = Hk[hp(6, j)];
#pragma unroll
                            for (int i = 0; i < 6; ++i) t += Hk[hp(j, i)] * zv[i];
                            if (j < 5) t += lpr[j];
#pragma unroll
                            for (int m = 0; m < 5; ++m) t -= Mk[j * NC + m] * lpn_[m];
                            rs[j] = t;
                        }
                    } else if (k == N) {       // terminal node: G_N = [[Q_N, q_N], [q_N^T, .]] on x~
#pragma unroll
                        for (int j = 0; j < 5; ++j) {
                            double t = GN[gszz<5>(5, j)];
#pragma unroll
                            for (int i = 0; i < 5; ++i) t += GN[gszz<5>(j, i)] * dxr[i];
                            rs[j] = t + lpr[j];
                        }
                    }
                    // done once the residual is at rounding level relative to the step and the multipliers
                    double rmax = 0.0, smax = 0.0;
#pragma unroll
                    for (int i = 0; i < 5; ++i) rmax = fmax(rmax, fabs(rc[i]));
#pragma unroll
                    for (int j = 0; j < 6; ++j) rmax = fmax(rmax, fabs(rs[j]));
#pragma unroll
                    for (int i = 0; i < 5; ++i) smax = fmax(smax, xon ? fmax(fabs(dxr[i]), fabs(lpr[i])) : 0.0);
                    smax = fmax(smax, uon ? fabs(dUr) : 0.0);
                    rmax = wmax(rmax); smax = wmax(smax);
                    if (rmax <= 1e-12 * (1.0 + smax)) return false;
                    double gsave[6];
#pragma unroll
                    for (int j = 0; j < 6; ++j) gsave[j] = 0.0;
                    if (uon) {
#pragma unroll
                        for (int j = 0; j < 6; ++j) { gsave[j] = Hk[hp(6, j)]; Hk[hp(6, j)] = rs[j]; }
                    } else if (k == N) {
#pragma unroll
                        for (int j = 0; j < 5; ++j) { gsave[j] = GN[gszz<5>(5, j)]; GN[gszz<5>(5, j)] = rs[j]; }
                    }
                    double rg[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) rg[i] = xon ? (i < 4 ? rc[i] / dsc[i] : rc[i]) : 0.0;
#pragma unroll
                    for (int r = 0; r < 5; ++r) {
                        const double t = from_next(rg[r]);
                        if (uon) Mk[6 * NC + r] = -t;
                        if (k == 0) S->dx0[hf][r] = -rg[r];
                    }
                    __syncthreads();
                    (void)riccati_s_sweep_soft(S, RL, N, RR, false);
                    double dx0_[5], lp0_[5];
                    const double du0_ = dUr;
#pragma unroll
                    for (int i = 0; i < 5; ++i) { dx0_[i] = dxr[i]; lp0_[i] = lpr[i]; }
                    resto_step();
#pragma unroll
                    for (int i = 0; i < 5; ++i) { dxr[i] = dx0_[i] + dxr[i]; lpr[i] = lp0_[i] + lpr[i]; }
                    dUr = du0_ + dUr;
                    if (uon) {
#pragma unroll
                        for (int j = 0; j < 6; ++j) Hk[hp(6, j)] = gsave[j];
                    } else if (k == N) {
#pragma unroll
                        for (int j = 0; j < 5; ++j) GN[gszz<5>(5, j)] = gsave[j];
                    }
                    __syncthreads();
                    return true;
                };
#endif
                resto_step();
#if DART_RESTO_REFINE
                for (int rr = 0; rr < DART_RESTO_REFINE && refine(cres); ++rr) {}
#endif
                pn_steps();
                STAMP(20);
                // barrier objective of the restoration problem and its directional derivative
                double phir, gtdr;
                {
                    double pl = 0.0, gd = 0.0;
                    if (xon) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const double e = drx[i] * (x[i] - xr[i]);
                            pl += rho * (pc[i] + nc[i]) + 0.5 * eta * e * e - rmu * (log(pc[i]) + log(nc[i]));
                            gd += eta * drx[i] * e * dxr[i] + (rho - rmu / pc[i]) * dpc[i] + (rho - rmu / nc[i]) * dnc[i];
                        }
                    }
                    if (uon) {
                        const double e = dru * (u - ur);
                        pl += 0.5 * eta * e * e - rmu * (log(u - lo) + log(hi - u));
                        gd += (eta * dru * e - rmu * isl + rmu * isu) * dUr;
                    }
                    phir = wsum(pl); gtdr = wsum(gd);
                }
                double aminr = gam_th;
                if (gtdr < 0) aminr = fmin(gam_th, fmin(gam_ph * thr / (-gtdr), pow(thr, s_th) / pow(-gtdr, s_ph)));
                aminr *= gam_al;
                double ct[5], pct[4], nct[4];
                double tht = 0.0, pht = 0.0;
                auto trial_r = [&](double al) {
                    double xt[4], gt_[5];
#pragma unroll
                    for (int i = 0; i < 4; ++i) xt[i] = fma(al, dxr[i], x[i]);
                    const double pt = fma(al, dxr[4], up), ut = uon ? fma(al, dUr, u) : u;
                    defects(xt, pt, ut, gt_);
                    double thl = 0.0, phl = 0.0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        pct[i] = fma(al, dpc[i], pc[i]); nct[i] = fma(al, dnc[i], nc[i]);
                        ct[i] = xon ? dsc[i] * gt_[i] + nct[i] - pct[i] : 0.0;
                        const double e = drx[i] * (xt[i] - xr[i]);
                        if (xon) {
                            thl += fabs(ct[i]);
                            phl += (pct[i] > 0.0 && nct[i] > 0.0)
                                       ? rho * (pct[i] + nct[i]) + 0.5 * eta * e * e - rmu * (log(pct[i]) + log(nct[i]))
                                       : __builtin_inf();
                        }
                    }
                    ct[4] = xon ? gt_[4] : 0.0;
                    thl += fabs(ct[4]);
                    if (uon) {
                        const double e = dru * (ut - ur);
                        phl += (ut > lo && ut < hi) ? 0.5 * eta * e * e - rmu * (log(ut - lo) + log(hi - ut)) : __builtin_inf();
                    }
                    wsum2(thl, phl);
                    tht = thl; pht = phl;
                };
                auto racc = [&](double al_test, bool& ft) {
                    const bool in_f = !(tht < rth_max) || !isfinite(pht) || wany_rep(lane < rnf && tht >= rfth && pht >= rfph);
                    if (in_f) return false;
                    const bool sw = gtdr < 0.0 && al_test * pow(-gtdr, s_ph) > pow(thr, s_th);
                    if (thr <= rth_min && sw) {
                        if (cmp_le(pht, phir + eta_ph * al_test * gtdr, phir)) { ft = true; return true; }
                        return false;
                    }
                    return cmp_le(tht, (1 - gam_th) * thr, thr) || cmp_le(pht - phir, -gam_ph * thr, phir);
                };
                STAMP(21);
                double alr = amr;
                bool accr = false, ftr = false;
                for (int ls = 0; ls < 80 && !accr; ++ls) {
                    if (alr < aminr && ls > 0) break;
                    STAMP_ADD(26, 1);
                    trial_r(alr);
                    accr = racc(alr, ftr);
                    if (!accr && ls == 0 && !(tht < thr) && a.max_soc > 0) {
                        // second-order correction on the restoration problem's constraints; the plain step
                        // is parked in LDS
                        if (xon) {
                            double* sv = RL->SV[sl];
#pragma unroll
                            for (int i = 0; i < 5; ++i) { sv[i] = dxr[i]; sv[5 + i] = lpr[i]; }
                            sv[10] = dUr;
#pragma unroll
                            for (int i = 0; i < 4; ++i) { sv[11 + i] = dpc[i]; sv[15 + i] = dnc[i]; }
                        }
                        double csoc[5], asoc = alr, th_old = 0.0;
#pragma unroll
                        for (int i = 0; i < 5; ++i) csoc[i] = cres[i];
                        for (int c = 0; c < a.max_soc; ++c) {
                            if (c > 0 && !(tht <= 0.99 * th_old)) break;
                            th_old = tht;
#pragma unroll
                            for (int i = 0; i < 5; ++i) csoc[i] = fma(asoc, csoc[i], ct[i]);
                            soft_rows(delta, false, csoc);
                            __syncthreads();
                            (void)riccati_s_sweep_soft(S, RL, N, RR, false);
                            resto_step();
#if DART_RESTO_REFINE
                            for (int rr = 0; rr < DART_RESTO_REFINE && refine(csoc); ++rr) {}
#endif
                            pn_steps();
                            asoc = amr;
                            trial_r(asoc);
                            bool ft2 = false;
                            if (racc(alr, ft2)) { accr = true; ftr = ft2; alr = asoc; break; }
                        }
                        if (!accr) {        // back to the plain step
                            if (xon) {
                                const double* sv = RL->SV[sl];
#pragma unroll
                                for (int i = 0; i < 5; ++i) { dxr[i] = sv[i]; lpr[i] = sv[5 + i]; }
                                dUr = sv[10];
                            }
                            pn_steps();
                        }
                    }
                    if (!accr) alr *= 0.5;
                }
                STAMP(22);
#ifdef DART_RESTO_TRACE
                if (blockIdx.x == 0 && lane == 0)      // diagnostic build: the oracle's ORACLE_DEBUG line
                    printf("  resto it %3d mu %.2e err %.2e dinf %.2e pinf %.2e c0 %.2e delta %.1e amax %.3e alpha %.3e "
                           "th %.3e th_t %.3e phi %.6e ph_t %.6e gTd %.3e acc %d\n", rit, rmu, errr_t, dinf_t, pinf_t,
                           c0_t, delta, amr, alr, thr, tht, phir, pht, gtdr, (int)accr);
                {
                    double sx = 0.0, spn = 0.0, slp = 0.0, sla = 0.0, sz = 0.0, su = 0.0;
                    if (xon) {
                        for (int i = 0; i < 5; ++i) { sx += fabs(dxr[i]); slp += fabs(lpr[i]); sla += fabs(rl[i]); }
                        for (int i = 0; i < 4; ++i) { spn += fabs(dpc[i]) + fabs(dnc[i]); sz += zp[i] + zn[i]; }
                    }
                    if (uon) su = fabs(dUr);
                    sx = wsum(sx); spn = wsum(spn); slp = wsum(slp); sla = wsum(sla); sz = wsum(sz); su = wsum(su);
                    // the step against the linearised restoration rows of this lane's node (the oracle's
                    // "resto step check"): d J dx + dn - dp + c = 0 (physical), J dx + c = 0 (copy row)
                    double pdx[5];
                    for (int i = 0; i < 5; ++i) pdx[i] = from_prev(dxr[i]);
                    const double pdu = from_prev(dUr);
                    double e1 = 0.0;
                    if (xon) {
                        for (int i = 0; i < 5; ++i) {
                            double jd = dxr[i];
                            if (k > 0) {
                                const double* Mp = &S->M[sl - 1][0][0];
                                for (int m = 0; m < 5; ++m) jd -= Mp[m * NC + i] * pdx[m];
                                jd -= Mp[5 * NC + i] * pdu;
                            }
                            const double r = i < 4 ? dsc[i] * jd + dnc[i] - dpc[i] + cres[i] : jd + cres[i];
                            e1 = fmax(e1, fabs(r));
                        }
                    }
                    double rows[5] = {0, 0, 0, 0, 0};
                    if (xon) {
                        for (int i = 0; i < 5; ++i) {
                            double jd = dxr[i];
                            if (k > 0) {
                                const double* Mp = &S->M[sl - 1][0][0];
                                for (int m = 0; m < 5; ++m) jd -= Mp[m * NC + i] * pdx[m];
                                jd -= Mp[5 * NC + i] * pdu;
                            }
                            rows[i] = i < 4 ? dsc[i] * jd + dnc[i] - dpc[i] + cres[i] : jd + cres[i];
                        }
                    }
                    // the forward sweep against the closed-loop rows it composes: dx_k - F_{k-1} [dx_{k-1}; 1]
                    double e2 = 0.0;
                    if (xon && k > 0) {
                        for (int r = 0; r < 5; ++r) {
                            const double* Fr = S->F[sl - 1][r];
                            double t = Fr[5];
                            for (int j = 0; j < 5; ++j) t = fma(Fr[j], pdx[j], t);
                            e2 = fmax(e2, fabs(dxr[r] - t));
                        }
                    }
                    e2 = wmax(e2);
                    const double e1w = wmax(e1);
                    if (blockIdx.x == 0 && lane == 0) printf("   sweep check it %3d closed-loop %.2e\n", rit, e2);
                    if (blockIdx.x == 0 && lane == 0) printf("   step check it %3d constraint %.2e\n", rit, e1w);
                    if (blockIdx.x == 0 && xon && e1 > 0.05 * e1w && e1w > 1e-6)      // the rows that dominate it
                        printf("     lane %2d (half %d node %2d) rows %.2e %.2e %.2e %.2e %.2e  dx %.3e %.3e %.3e %.3e %.3e du %.3e\n",
                               lane, hf, k, rows[0], rows[1], rows[2], rows[3], rows[4], dxr[0], dxr[1], dxr[2], dxr[3],
                               dxr[4], dUr);
                    if (blockIdx.x == 0 && lane == 0)
                        printf("   chk it %3d th %.12e phi %.12e gTd %.12e dx %.12e dpn %.12e du %.12e lamp %.12e lam %.12e "
                               "zpn %.12e az %.12e\n", rit, thr, phir, gtdr, sx, spn, su, slp, sla, sz, azr);
                }
#endif
                if (!accr) { rstat = -2; break; }      // a failed line search in the restoration phase
                if (!ftr && rnf < kWave) {
                    if (lane == rnf) { rfth = (1 - gam_th) * thr; rfph = phir - gam_ph * thr; }
                    ++rnf;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = xon ? fma(alr, dxr[i], x[i]) : x[i];
                up = xon ? fma(alr, dxr[4], up) : up;
#pragma unroll
                for (int i = 0; i < 5; ++i) rl[i] = xon ? fma(alr, lpr[i] - rl[i], rl[i]) : 0.0;
                if (xon) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        pc[i] = pct[i]; nc[i] = nct[i];
                        zp[i] = fmax(fmin(fma(azr, dzp[i], zp[i]), 1e10 * rmu / pc[i]), rmu / (1e10 * pc[i]));
                        zn[i] = fmax(fmin(fma(azr, dzn[i], zn[i]), 1e10 * rmu / nc[i]), rmu / (1e10 * nc[i]));
                    }
                }
                if (uon) {
                    u = fma(alr, dUr, u);
                    const double sl_ = u - lo, su_ = hi - u;
                    rzl = fmax(fmin(fma(azr, dzlr, rzl), 1e10 * rmu / sl_), rmu / (1e10 * sl_));
                    rzu = fmax(fmin(fma(azr, dzur, rzu), 1e10 * rmu / su_), rmu / (1e10 * su_));
                }
                thr = tht;
                STAMP(23);
                STAMP_ADD(25, 1);
            }
            if (!rok) { status = rstat; it = rit; break; }
            // back to the original problem: the u-bound multipliers take the step (mu - z s_trial) / s that
            // pretends the restoration's progress was one Newton step, cut by the fraction to the boundary
            // (tau of the original iteration) and reset to 1 above 1000; the equality multipliers restart at 0
            {
                double dzlo = 0.0, dzuo = 0.0, a2 = 1.0;
                if (uon) {
                    const double slo = ur - lo, suo = hi - ur;
                    dzlo = (mu0 - zl * (u - lo)) / slo;
                    dzuo = (mu0 - zu * (hi - u)) / suo;
                    if (dzlo < 0) a2 = fmin(a2, -tau0 * zl / dzlo);
                    if (dzuo < 0) a2 = fmin(a2, -tau0 * zu / dzuo);
                }
                const double azo = wmin(a2);
                if (uon) { zl = fma(azo, dzlo, zl); zu = fma(azo, dzuo, zu); }
                const bool reset = wmax(uon ? fmax(zl, zu) : 0.0) > 1e3;
                if (uon) {
                    if (reset) { zl = 1.0; zu = 1.0; }
                    const double il = frcp(u - lo), iu = frcp(hi - u);
                    zl = fmax(fmin(zl, 1e10 * mu0 * il), 1e-10 * mu0 * il);
                    zu = fmax(fmin(zu, 1e10 * mu0 * iu), 1e-10 * mu0 * iu);
                }
#pragma unroll
                for (int i = 0; i < 5; ++i) lam[i] = 0.0;
            }
            in_soft = 0; soft_count = 0;
            it_next = rit;
            continue;
        }
    }

    // ---------------- outputs -------------------------------------------------------------
    const double fval = wsum(cost_val(x, u, up));
    if (lane == 0 && wave_idx() == 0) { a.f[b] = fval; a.status[b] = status; a.iters[b] = it; }
    if (k == 0) a.u0[2 * b + hf] = u;
    if (a.w_out) {
        double* wo = a.w_out + (size_t)nw * b;
        if (xon) {
#pragma unroll
            for (int i = 0; i < 4; ++i) wo[8 * k + gidx(i)] = x[i];
        }
        if (uon) wo[8 * (N + 1) + 2 * k + hf] = u;
    }
    STAMP_FLUSH32_TO(g_stamp_lm, b);
    return !RESTO && status == kLmNeedResto;
}

// IPOPT's restoration phases for instance b in the wave that handed it over (batches of at most 32, one
// instance per CU): lmpc_solve<true> resumes from the parked state as lmpc_ipm_kernel<true> would behind a
// second launch.  A call, not inlined, so that the fast kernel keeps its register allocation; the launch
// arguments are read from the kernel's argument segment (LmpcArgs is its first argument, kernarg_addr).  The policy
// prologue's LDS (fused C5 launches) is dead by then: the restoration state takes its place, and the policy's
// parameter vector is read back from model_params, as by the second launch.
__device__ __noinline__ void lmpc_resto_tail(const int b, const unsigned long long kargs) {
    const LmpcArgs a = kernarg_load<LmpcArgs>(kargs);
    __threadfence_block();
    __syncthreads();            // the parked state and the policy's parameter vector (global stores) first
    lmpc_solve<true>(a, b);
}

// RESTO = false: the fast kernel of every solve; an instance whose filter line search fails parks the state
// of that iteration's start in a.resto_buf and ends with status kLmNeedResto.  RESTO = true: the same solve
// with IPOPT's soft restoration and restoration phases inline (their registers would spill the fast kernel's
// loop); launched right after it for batches above 32, only flagged instances run: they redo the setup,
// reload the parked state and continue from the failed iteration.  FUSE (batches of at most 32): the flagged
// instances continue in lmpc_resto_tail in the same launch.
template <bool RESTO, bool FUSE = false>
__global__ __launch_bounds__(kWave * kWaves) void lmpc_ipm_kernel(LmpcArgs a) {
    // small batches packed onto one XCD (launcher; blocks go round robin over the 8 XCDs)
    if (blockIdx.x % a.pack != (unsigned)(a.xcd % a.pack)) return;
    const int b = blockIdx.x / a.pack;
    if constexpr (RESTO) {
        if (a.status[b] != kLmNeedResto) return;     // wave-uniform: the instance was solved by <false>
    }
    const bool handed = lmpc_solve<RESTO>(a, b);
    if constexpr (FUSE) {
        if (__builtin_expect(handed, 0)) lmpc_resto_tail(b, kernarg_addr());
    }
}

}  // namespace dartmpc

#if DART_WG == 2
// N = 32..63 (dartmpc_launch_lmpc forwards here): one instance per two-wave workgroup.  Device area per instance:
// the hand-off state of its 128 lanes, then LmAux (second-order-correction scratch, restoration state).
extern "C" size_t dartmpc_lmpc_wg2_area_doubles() {
    return (size_t)dartmpc::kWave * dartmpc::kWaves * dartmpc::kLmNst + (sizeof(dartmpc::LmAux) + 7) / 8;
}
extern "C" hipError_t dartmpc_launch_lmpc_wg2(const void* args, hipStream_t stream) {
    dartmpc::LmpcArgs a = *static_cast<const dartmpc::LmpcArgs*>(args);
    if (a.N < (dartmpc::force_wg2() ? 1 : 32) || a.N >= dartmpc::LM_NMAXS) return hipErrorInvalidValue;
    if (!a.resto_buf) return hipErrorInvalidValue;          // the device area is needed with or without resto
    static std::mutex mu;
    static bool attr_set[64] = {};
    const size_t lds = dartmpc::kLmLdsBytes;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> g(mu);
        if (!attr_set[dev]) {
            e = hipFuncSetAttribute((const void*)dartmpc::lmpc_ipm_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)dartmpc::lmpc_ipm_kernel<true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            attr_set[dev] = true;
        }
    }
    if (a.fuse_policy) {        // the policy step of every instance first (its own launch, same stream)
        e = dartmpc_launch_policy(&a.pol, stream);
        if (e != hipSuccess) return e;
        a.pvec = a.pol.model_params;
        a.fuse_policy = 0;
    }
    a.pack = 1; a.xcd = 0;
    const dim3 block(dartmpc::kWave * dartmpc::kWaves);
    hipLaunchKernelGGL(dartmpc::lmpc_ipm_kernel<false>, dim3(a.B), block, lds, stream, a);
    if (a.resto) {
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(dartmpc::lmpc_ipm_kernel<true>, dim3(a.B), block, lds, stream, a);
    }
    return hipGetLastError();
}
#else

extern "C" size_t dartmpc_lmpc_lds_bytes(void) { return dartmpc::kLmLdsBytes; }

// internal (bench.py's saturated lines): instances of lmpc_ipm_kernel<false> resident per CU in a batch of more than
// 32 (its LDS: LmShared alone), by the runtime's occupancy calculation; -1 on error (call after a launch, which
// sets the dynamic-LDS opt-in)
extern "C" int dartmpc_lmpc_blocks_per_cu(void) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dartmpc::lmpc_ipm_kernel<false>, dartmpc::kWave,
                                                     sizeof(dartmpc::LmShared)) != hipSuccess)
        return -1;
    return n;
}
extern "C" size_t dartmpc_lmpc_shared_bytes(void) { return sizeof(dartmpc::LmShared); }

extern "C" hipError_t dartmpc_launch_lmpc(const dartmpc::LmpcArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    if ((args->N >= dartmpc::LM_NMAXS || dartmpc::force_wg2()) && args->N < 2 * dartmpc::LM_NMAXS)
        return dartmpc_launch_lmpc_wg2(args, stream);
    if (args->N < 1 || args->N >= dartmpc::LM_NMAXS) return hipErrorInvalidValue;
    if (args->resto && !args->resto_buf) return hipErrorInvalidValue;
    // the dynamic-LDS opt-in is per device: set once for every device a launch goes to (thread-safe)
    static std::mutex mu;
    static bool attr_set[64] = {};
    const size_t lds = dartmpc::kLmLdsBytes;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> g(mu);
        if (!attr_set[dev]) {
            e = hipFuncSetAttribute((const void*)dartmpc::lmpc_ipm_kernel<false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)dartmpc::lmpc_ipm_kernel<true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)dartmpc::lmpc_ipm_kernel<false, true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            attr_set[dev] = true;
        }
    }
    dartmpc::LmpcArgs a = *args;
    a.pack = (a.B <= 32) ? 8 : 1;            // one XCD (and its L2) for the code of a small batch
    // the policy prologue's LDS only when the launch runs it (the opt-in above covers the maximum)
    const size_t lds_launch = a.fuse_policy ? dartmpc::kLmPolicyLdsOff + sizeof(dartmpc::PolicyLds) : sizeof(dartmpc::LmShared);
    if (a.resto && a.pack == 8 && dartmpc::resto_fuse_enabled()) {   // restoration in the solving wave: one launch
        const size_t lds_r = dartmpc::kLmRestoOff + sizeof(dartmpc::LmResto);
        hipLaunchKernelGGL((dartmpc::lmpc_ipm_kernel<false, true>), dim3(a.B * a.pack), dim3(dartmpc::kWave),
                           lds_launch > lds_r ? lds_launch : lds_r, stream, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(dartmpc::lmpc_ipm_kernel<false>, dim3(a.B * a.pack), dim3(dartmpc::kWave), lds_launch, stream, a);
    // IPOPT's restoration phases for the instances the first launch handed off (the others return at once)
    if (a.resto)
        hipLaunchKernelGGL(dartmpc::lmpc_ipm_kernel<true>, dim3(a.B * a.pack), dim3(dartmpc::kWave),
                           dartmpc::kLmRestoOff + sizeof(dartmpc::LmResto), stream, a);
    return hipGetLastError();
}

#ifdef DART_STAMPS
extern "C" hipError_t dartmpc_read_stamps_lmpc(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_lm), sizeof(unsigned long long) * 32, 0,
                               hipMemcpyDeviceToHost);
}
#endif
#endif  // DART_WG
