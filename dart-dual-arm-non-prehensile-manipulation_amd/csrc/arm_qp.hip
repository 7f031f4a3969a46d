// arm_qp.hip -- batched per-arm impedance QP (ARMCONTROL.solver_worker) for gfx950.
//
// Replaces the body of ARMCONTROL.solver_worker (PMPC/src/controller/arm.py:266-457; identical
// in RMPC/dev_dual/controller/parallel.py and LMPC/src/controller/parallel.py): per arm and
// simulation step, from the shared-memory snapshot that compute_dynamics (:111-199) publishes,
//   Minv = pinv(M, rcond 1e-6)                                  (:339-342)
//   Mx   = inv(Mx_inv) if |det Mx_inv| > 1e-8 else pinv(Mx_inv, rcond 1e-3)   (:344-350)
//   mu   = Mx (J Minv h + Jdot qd),  D = sqrtm|.|(Mx) sqrt(K) + sqrt(K) sqrtm|.|(Mx)   (:353-362)
//   cost = |J qdd + Jdot qd - Mx_inv F|^2_Wimp + |qdd - beta|^2_Wpos + |(qdd - qdd_prev)/dt|^2_Ws
//          with F = -D J qd + K twist + mu, beta = -2 sqrt(diag Kn) qd - Kn q     (:370-388)
//   s.t. Qmin <= q + qd dt + dt^2/2 qdd <= Qmax, Qdmin <= qd + dt qdd <= Qdmax,
//        taumin <= M qdd + h <= taumax                                            (:391-398)
// and the reference's outputs tau = M qdd + h, loss = cost(qdd), qdd (:428-437).  IPOPT's answer to
// this strictly convex QP is its unique KKT point (bounds relaxed by bound_relax_factor 1e-8); the
// kernel computes it with the Mehrotra predictor-corrector IPM of oracle/arm_qp.py:qp_ipm.
//
// Mapping: one wave64 per arm instance, everything in LDS.
//   * both symmetric eigenproblems (M: n x n, Mx_inv: 6 x 6, padded to 8 x 8) by parallel cyclic
//     Jacobi: 7 rounds of 4 disjoint rotations per sweep (round-robin pairing), lane = matrix entry
//     (i, j) of both matrices, each rotation round one LDS ping-pong step;
//   * the QP build as lane-per-entry small products;
//   * the IPM: lane i < 3n owns constraint row i (both sides: slacks, multipliers in registers),
//     lane (r, c) < n^2 owns an entry of the normal matrix K = H + A' W A, factored K = L D L' in
//     place (n LDS steps; a non-positive pivot = lost definiteness, as IPOPT / Cholesky see it);
//     lane r then keeps row r and column r of L in registers and both triangular solves of the
//     predictor and corrector run as readlane broadcasts (no LDS, no barriers).  An explicit
//     inverse would be cheaper to apply but loses the backward stability the IPM needs once
//     z / s of the active rows reaches 1e12+ (measured: Newton directions degrade, runs break down).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arm_qp.h"
#include "stamps.h"
#include "wave.h"

namespace dartmpc {

#ifdef DART_STAMPS
__device__ unsigned long long g_stamp_arm[16];
#endif

constexpr int AN = ARM_NMAX;

struct ArmShared {
    double snap[AN * AN + 16 * AN + 45];
    double prm[3 * AN * AN + 6 * AN + 73];
    double A[2][2][64];          // Jacobi ping-pong [buffer][matrix][8 x 8]
    double V[2][2][64];
    double rc[2][8], rt[2][8];   // rotation of index i this round: J(i, i) = c, J(partner, i) = t
    double y[8], mh[8], mxd[8];
    double Mx[36], S[36], D[36];
    double u1[6], vq[6], mu[6], F[6], e0[6], beta[AN];
    double WJ[6 * AN];
    double H[64], c[AN];
    double X[AN], DX[AN], RHS[AN];
    double ZD[3 * AN], W[3 * AN], VD[3 * AN];
    double K[2][64];             // LDL' ping-pong
    double eimp[6], epos[AN], qddd[AN];
};

// 1/sqrt(x) for x >= 1: v_rsq_f64 (~2^-26) + one Newton step -> ~1e-16 relative
__device__ __forceinline__ double frsq(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    return y * fma(-0.5 * x * y, y, 1.5);
}

// reduction over lanes 0..7 (quad reductions, then the two quad totals); lanes 8+ are ignored
template <class Op>
__device__ __forceinline__ double red8(double x, Op op) {
    x = op(x, dpp<0xB1>(x));     // quad_perm [1,0,3,2]
    x = op(x, dpp<0x4E>(x));     // quad_perm [2,3,0,1]
    return op(readlane(x, 0), readlane(x, 4));
}

// three maxima and one sum over lanes 0..7 in lock step (each takes red8's steps: the same bits)
__device__ __forceinline__ void red8_max3_sum(double& m0, double& m1, double& m2, double& s0) {
    m0 = fmax(m0, dpp<0xB1>(m0)); m1 = fmax(m1, dpp<0xB1>(m1)); m2 = fmax(m2, dpp<0xB1>(m2)); s0 = s0 + dpp<0xB1>(s0);
    m0 = fmax(m0, dpp<0x4E>(m0)); m1 = fmax(m1, dpp<0x4E>(m1)); m2 = fmax(m2, dpp<0x4E>(m2)); s0 = s0 + dpp<0x4E>(s0);
    m0 = fmax(readlane(m0, 0), readlane(m0, 4)); m1 = fmax(readlane(m1, 0), readlane(m1, 4));
    m2 = fmax(readlane(m2, 0), readlane(m2, 4)); s0 = readlane(s0, 0) + readlane(s0, 4);
}

// round-robin pairing of 8 indices, round r = 0..6 (index 7 fixed)
__device__ __forceinline__ int jpartner(int i, int r) {
    if (i == 7) return r;
    if (i == r) return 7;
    const int p = (2 * r - i) % 7;
    return p < 0 ? p + 7 : p;
}

template <int n>
__global__ __launch_bounds__(kWave) void arm_qp_kernel(ArmArgs a) {
    __shared__ ArmShared SH;
    STAMP_DECL
    const int b = blockIdx.x, l = threadIdx.x;
    const int SL = arm_snap_len(n), PL = arm_prm_len(n);
    {
        const double* gs = a.snap + (size_t)SL * b;
        const double* gp = a.prm + (size_t)a.prm_stride * b;
        for (int e = l; e < SL; e += kWave) SH.snap[e] = gs[e];
        for (int e = l; e < PL; e += kWave) SH.prm[e] = gp[e];
    }
    __syncthreads();
    const double* q = SH.snap;
    const double* qd = q + n;
    const double* qp = q + 2 * n;
    const double* mocap = q + 3 * n;
    const double* ee = mocap + 3;
    const double* rv = ee + 3;
    const double* J = q + 3 * n + 9;
    const double* Jd = J + 6 * n;
    const double* M = Jd + 6 * n;
    const double* hb = M + n * n;
    const double* Mxi = hb + n;
    const double* Wi = SH.prm;
    const double* Wp = Wi + 36;
    const double* Ws = Wp + n * n;
    const double* Qmin = Ws + n * n;
    const double* Qmax = Qmin + n;
    const double* Qdmin = Qmax + n;
    const double* Qdmax = Qdmin + n;
    const double* tmin = Qdmax + n;
    const double* tmax = tmin + n;
    const double* Kt = tmax + n;
    const double* Kn = Kt + 36;
    const double dt = Kn[n * n];
    STAMP(0);

    // ---------------- eigen-decompositions of M and Mx_inv (parallel cyclic Jacobi) -----------
    const int ei = l >> 3, ej = l & 7;
    {
        const double m0 = (ei < n && ej < n) ? 0.5 * (M[ei * n + ej] + M[ej * n + ei]) : 0.0;
        const double m1 = (ei < 6 && ej < 6) ? 0.5 * (Mxi[ei * 6 + ej] + Mxi[ej * 6 + ei]) : 0.0;
        SH.A[0][0][l] = m0;
        SH.A[0][1][l] = m1;
        SH.V[0][0][l] = ei == ej ? 1.0 : 0.0;
        SH.V[0][1][l] = ei == ej ? 1.0 : 0.0;
    }
    __syncthreads();
    int cur = 0;
    for (int sweep = 0; sweep < 16; ++sweep) {
        const double a0 = SH.A[cur][0][l], a1 = SH.A[cur][1][l];
        // the four sums in lock step (wsum2: each the same bits as its wsum)
        double off0 = ei != ej ? a0 * a0 : 0.0, dg0 = ei == ej ? a0 * a0 : 0.0;
        double off1 = ei != ej ? a1 * a1 : 0.0, dg1 = ei == ej ? a1 * a1 : 0.0;
        wsum2(off0, dg0);
        wsum2(off1, dg1);
        if (off0 <= 1e-32 * dg0 && off1 <= 1e-32 * dg1) break;
        STAMP_ADD(9, 1);
        for (int r = 0; r < 7; ++r) {
            if (l < 16) {   // rotation of index i of matrix mat this round
                const int mat = l >> 3, i = l & 7;
                const int pi = jpartner(i, r);
                const int p = i < pi ? i : pi, qq = i < pi ? pi : i;
                const double* Am = SH.A[cur][mat];
                const double apq = Am[p * 8 + qq], app = Am[p * 9], aqq = Am[qq * 9];
                double c = 1.0, s = 0.0;
                if (fabs(apq) > 1e-290) {
                    // classic Jacobi: tau = (a_qq - a_pp) / 2 a_pq, t = sign(tau) / (|tau| + sqrt(1 + tau^2));
                    // |tau| > 1e150 would overflow the square: t -> 1 / (2 |tau|) there
                    const double tau = (aqq - app) * (0.5 * frcp(apq));
                    const double at = fabs(tau);
                    const double den = at < 1e150 ? at + (1.0 + at * at) * frsq(1.0 + at * at) : 2.0 * at;
                    const double t = (tau >= 0.0 ? 1.0 : -1.0) * frcp(den);
                    c = frsq(1.0 + t * t);
                    s = t * c;
                }
                SH.rc[mat][i] = c;
                SH.rt[mat][i] = i == p ? -s : s;
            }
            __syncthreads();
            const int pi = jpartner(ei, r), pj = jpartner(ej, r);
#pragma unroll
            for (int mat = 0; mat < 2; ++mat) {
                const double* Am = SH.A[cur][mat];
                const double* Vm = SH.V[cur][mat];
                const double ci = SH.rc[mat][ei], ti = SH.rt[mat][ei], cj = SH.rc[mat][ej], tj = SH.rt[mat][ej];
                const double na = ci * (cj * Am[ei * 8 + ej] + tj * Am[ei * 8 + pj]) +
                                  ti * (cj * Am[pi * 8 + ej] + tj * Am[pi * 8 + pj]);
                const double nv = fma(Vm[ei * 8 + ej], cj, Vm[ei * 8 + pj] * tj);
                SH.A[cur ^ 1][mat][l] = na;
                SH.V[cur ^ 1][mat][l] = nv;
            }
            __syncthreads();
            cur ^= 1;
        }
    }
    STAMP(1);
    const double* A0 = SH.A[cur][0];
    const double* A1 = SH.A[cur][1];
    const double* V0 = SH.V[cur][0];
    const double* V1 = SH.V[cur][1];

    // ---------------- QP data (arm.py:335-388) -------------------------------------------------
    {   // pinv(M, rcond=1e-6) h: eigenvalues kept where |lambda| > 1e-6 max |lambda|
        const double lmax0 = wmax(l < n ? fabs(A0[(l < n ? l : 0) * 9]) : 0.0);
        if (l < n) {
            double y = 0.0;
            _Pragma("unroll") for (int k = 0; k < n; ++k) y = fma(V0[k * 8 + l], hb[k], y);
            const double lam = A0[l * 9];
            SH.y[l] = fabs(lam) > 1e-6 * lmax0 ? y / lam : 0.0;
        }
        // Mx: inv if |det| > 1e-8 else pinv(rcond=1e-3); eigen weights of Mx = 1/lambda or 0
        double det = 1.0, lmax1 = 0.0;
        _Pragma("unroll") for (int i = 0; i < 6; ++i) { det *= A1[i * 9]; lmax1 = fmax(lmax1, fabs(A1[i * 9])); }
        if (l < 6) {
            const double lam = A1[l * 9];
            const bool keep = fabs(det) > 1e-8 || fabs(lam) > 1e-3 * lmax1;
            SH.mxd[l] = keep ? 1.0 / lam : 0.0;
        }
    }
    __syncthreads();
    if (l < n) {
        double s = 0.0;
        _Pragma("unroll") for (int k = 0; k < n; ++k) s = fma(V0[l * 8 + k], SH.y[k], s);
        SH.mh[l] = s;
    }
    if (l < 36) {   // Mx and its safe square root (arm.py:355-358) from the same eigenvectors
        const int i = l / 6, j = l % 6;
        double mx = 0.0, sq = 0.0;
        _Pragma("unroll") for (int k = 0; k < 6; ++k) {
            const double vv = V1[i * 8 + k] * V1[j * 8 + k];
            mx = fma(vv, SH.mxd[k], mx);
            sq = fma(vv, sqrt(fabs(SH.mxd[k])), sq);
        }
        SH.Mx[l] = mx;
        SH.S[l] = sq;
    }
    __syncthreads();
    if (l < 6) {
        double u = 0.0, v = 0.0, w = 0.0;
        _Pragma("unroll") for (int k = 0; k < n; ++k) {
            u = fma(J[l * n + k], SH.mh[k], u);
            w = fma(Jd[l * n + k], qd[k], w);
            v = fma(J[l * n + k], qd[k], v);
        }
        SH.u1[l] = u + w;
        SH.vq[l] = v;
    }
    __syncthreads();
    if (l < 6) {
        double m_ = 0.0;
        _Pragma("unroll") for (int k = 0; k < 6; ++k) m_ = fma(SH.Mx[l * 6 + k], SH.u1[k], m_);
        SH.mu[l] = m_;
    }
    if (l < 36) {   // D = S sqrt(K) + sqrt(K) S, sqrt elementwise as np.sqrt(K)
        const int i = l / 6, j = l % 6;
        double d1 = 0.0, d2 = 0.0;
        _Pragma("unroll") for (int k = 0; k < 6; ++k) {
            d1 = fma(SH.S[i * 6 + k], sqrt(Kt[k * 6 + j]), d1);
            d2 = fma(sqrt(Kt[i * 6 + k]), SH.S[k * 6 + j], d2);
        }
        SH.D[l] = d1 + d2;
    }
    __syncthreads();
    if (l < 6) {    // F = -D (J qd) + K twist + mu
        double f1 = 0.0, f2 = 0.0;
        _Pragma("unroll") for (int k = 0; k < 6; ++k) {
            const double tw = k < 3 ? mocap[k] - ee[k] : rv[k - 3];
            f1 = fma(SH.D[l * 6 + k], SH.vq[k], f1);
            f2 = fma(Kt[l * 6 + k], tw, f2);
        }
        SH.F[l] = (-f1 + f2) + SH.mu[l];
    }
    if (l >= 8 && l < 8 + n) {   // beta = 2 sqrt(diag Kn) (-qd) + Kn (-q)
        const int r = l - 8;
        double s = 0.0;
        _Pragma("unroll") for (int k = 0; k < n; ++k) s = fma(Kn[r * n + k], -q[k], s);
        SH.beta[r] = 2.0 * sqrt(Kn[r * n + r]) * -qd[r] + s;
    }
    __syncthreads();
    if (l < 6) {    // Eimp = J qdd + e0, e0 = Jdot qd - Mx_inv F
        double e1 = 0.0, e2 = 0.0;
        _Pragma("unroll") for (int k = 0; k < n; ++k) e1 = fma(Jd[l * n + k], qd[k], e1);
        _Pragma("unroll") for (int k = 0; k < 6; ++k) e2 = fma(Mxi[l * 6 + k], SH.F[k], e2);
        SH.e0[l] = e1 - e2;
    }
    if (l < 6 * n) {   // sym(Wimp) J
        const int i = l / n, cc = l % n;
        double w = 0.0;
        _Pragma("unroll") for (int k = 0; k < 6; ++k) w = fma(0.5 * (Wi[i * 6 + k] + Wi[k * 6 + i]), J[k * n + cc], w);
        SH.WJ[l] = w;
    }
    __syncthreads();
    const double idt2 = 1.0 / (dt * dt);
    if (l < n * n) {   // H = 2 (J' sym(Wimp) J + sym(Wpos) + sym(Ws) / dt^2)
        const int r = l / n, cc = l % n;
        double hv = 0.0;
        _Pragma("unroll") for (int k = 0; k < 6; ++k) hv = fma(J[k * n + r], SH.WJ[k * n + cc], hv);
        hv += 0.5 * (Wp[r * n + cc] + Wp[cc * n + r]) + 0.5 * (Ws[r * n + cc] + Ws[cc * n + r]) * idt2;
        SH.H[r * 8 + cc] = 2.0 * hv;
    }
    if (l < n) {       // c = 2 (J' sym(Wimp) e0 - sym(Wpos) beta - sym(Ws) qdd_prev / dt^2)
        double c1 = 0.0, c2 = 0.0, c3 = 0.0;
        _Pragma("unroll") for (int k = 0; k < 6; ++k) c1 = fma(SH.WJ[k * n + l], SH.e0[k], c1);
        _Pragma("unroll") for (int k = 0; k < n; ++k) {
            c2 = fma(0.5 * (Wp[l * n + k] + Wp[k * n + l]), SH.beta[k], c2);
            c3 = fma(0.5 * (Ws[l * n + k] + Ws[k * n + l]) * idt2, qp[k], c3);
        }
        SH.c[l] = 2.0 * (c1 - c2 - c3);
    }

    __syncthreads();
    // ---------------- IPM: lane r < n owns joint r -- its position, velocity and torque rows ------
    // (arm.py:391-398; bounds relaxed as IPOPT's bound_relax_factor).  Everything iteration-local
    // lives in registers; cross-lane values move by readlane (uniform lane index), so the loop has
    // no LDS traffic and no barriers.
    const bool jl = l < n;
    const int r = jl ? l : 0;
    double Hrow[n], Mrow[n], Mcol[n];
#pragma unroll
    for (int k = 0; k < n; ++k) {
        Hrow[k] = SH.H[r * 8 + k];
        Mrow[k] = M[r * n + k];
        Mcol[k] = M[k * n + r];
    }
    const double cr = jl ? SH.c[r] : 0.0;
    const double a_pos = 0.5 * (dt * dt);
    bool onu[3], onl[3];
    double gu[3], gl[3];
    {
        const double bv[3] = {qd[r] * dt + q[r], qd[r], hb[r]};
        const double lov[3] = {Qmin[r], Qdmin[r], tmin[r]}, hiv[3] = {Qmax[r], Qdmax[r], tmax[r]};
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            onu[t] = jl && hiv[t] < 1e19;
            onl[t] = jl && lov[t] > -1e19;
            gu[t] = onu[t] ? (hiv[t] + 1e-8 * fmax(1.0, fabs(hiv[t]))) - bv[t] : 0.0;
            gl[t] = onl[t] ? bv[t] - (lov[t] - 1e-8 * fmax(1.0, fabs(lov[t]))) : 0.0;
        }
    }
    // a_t . v for the lane's three rows: dt^2/2 v_r, dt v_r, M(r, :) v
    auto rows_dot = [&](double vr, const double* vs, double* out) {
        out[0] = a_pos * vr;
        out[1] = dt * vr;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < n; ++k) s = fma(Mrow[k], vs[k], s);
        out[2] = s;
    };
    // (A' v)_r from the lane's own position / velocity entries and every lane's torque entry
    auto at_dot = [&](const double* v) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < n; ++k) s = fma(Mcol[k], readlane(v[2], k), s);
        return fma(a_pos, v[0], fma(dt, v[1], s));
    };
    auto bcast = [&](double v, double* vs) {
#pragma unroll
        for (int k = 0; k < n; ++k) vs[k] = readlane(v, k);
    };

    int cnt = 0;
#pragma unroll
    for (int t = 0; t < 3; ++t) cnt += __popcll(__ballot(onu[t])) + __popcll(__ballot(onl[t]));
    const double nact = fmax(1.0, (double)cnt);
    double gmx = 0.0;
#pragma unroll
    for (int t = 0; t < 3; ++t) gmx = fmax(gmx, fmax(onu[t] ? fabs(gu[t]) : 0.0, onl[t] ? fabs(gl[t]) : 0.0));
    const double sd = 1.0 + red8(jl ? fabs(cr) : 0.0, OpMax());
    const double sp = 1.0 + red8(gmx, OpMax());
    double x = jl ? qp[r] : 0.0;            // warm start x0 = qdd_prev (arm.py:401-408)
    double su[3], sl[3], zu[3], zl[3];
    {
        const double z0 = sd / nact;         // multipliers on the scale of the cost gradient
        double xs[n], ax[3];
        bcast(x, xs);
        rows_dot(x, xs, ax);
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            su[t] = onu[t] ? fmax(gu[t] - ax[t], 1.0) : 1.0;
            sl[t] = onl[t] ? fmax(gl[t] + ax[t], 1.0) : 1.0;
            zu[t] = onu[t] ? z0 : 0.0;
            zl[t] = onl[t] ? z0 : 0.0;
        }
    }
    const double tol = a.tol, acc_tol = a.acc_tol;
    const double isd = 1.0 / sd, isp = 1.0 / sp, inact = 1.0 / nact;
    STAMP(2);

    int status = -1, it = 0;
    for (it = 0; it < a.max_iter; ++it) {
        double xs[n], ax[3], isu[3], isl[3], rpu[3], rpl[3], zd[3];
        bcast(x, xs);
        rows_dot(x, xs, ax);
        double rpm = 0.0, szl = 0.0, zmx = 0.0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            isu[t] = frcp(su[t]);
            isl[t] = frcp(sl[t]);
            rpu[t] = onu[t] ? ax[t] + su[t] - gu[t] : 0.0;
            rpl[t] = onl[t] ? -ax[t] + sl[t] - gl[t] : 0.0;
            zd[t] = zu[t] - zl[t];
            rpm = fmax(rpm, fmax(fabs(rpu[t]), fabs(rpl[t])));
            szl += (onu[t] ? su[t] * zu[t] : 0.0) + (onl[t] ? sl[t] * zl[t] : 0.0);
            zmx = fmax(zmx, fmax(zu[t], zl[t]));
        }
        double rd = cr + at_dot(zd);
#pragma unroll
        for (int k = 0; k < n; ++k) rd = fma(Hrow[k], xs[k], rd);
        rd = jl ? rd : 0.0;
        double rdm = fabs(rd);
        red8_max3_sum(rdm, rpm, zmx, szl);          // (four red8 in lock step)
        const double mu = szl * inact;
        const double zmax = zmx;
        const double err = fmax(rdm * isd, fmax(rpm * isp, mu * isd));
        if (err <= tol) { status = 0; break; }
        if (zmax > 1e14 * sd) { status = -3; break; }
        STAMP(3);
        // row r of K = H + A' W A, then L D L' with row r of the factor in lane r
        double W[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) W[t] = (onu[t] ? zu[t] * isu[t] : 0.0) + (onl[t] ? zl[t] * isl[t] : 0.0);
        double Krow[n];
        {
            double mw[n];
#pragma unroll
            for (int k = 0; k < n; ++k) mw[k] = Mcol[k] * readlane(W[2], k);
            const double dg = fma(a_pos * a_pos, W[0], (dt * dt) * W[1]);
#pragma unroll
            for (int c = 0; c < n; ++c) {
                double kv = Hrow[c];
#pragma unroll
                for (int k = 0; k < n; ++k) kv = fma(mw[k], M[k * n + c], kv);
                Krow[c] = c == r ? kv + dg : kv;
            }
        }
        double iD[n];
        bool bad = false;
#pragma unroll
        for (int p = 0; p < n; ++p) {
            const double piv = readlane(Krow[p], p);
            bad = bad || !(piv > 0.0) || !isfinite(piv);
            const double ip = frcp(piv);
            iD[p] = ip;
            const double f = (r > p) ? Krow[p] * ip : 0.0;
#pragma unroll
            for (int c = p + 1; c < n; ++c) Krow[c] = fma(-f, readlane(Krow[c], p), Krow[c]);
        }
        if (bad) { status = err <= acc_tol ? 1 : -2; break; }
        STAMP(4);
        double Lrow[n], Lcol[n], iDr = 0.0;
#pragma unroll
        for (int k = 0; k < n; ++k) iDr = k == r ? iD[k] : iDr;
#pragma unroll
        for (int k = 0; k < n; ++k) {
            Lrow[k] = k < r ? Krow[k] * iD[k] : 0.0;
            Lcol[k] = k > r ? Krow[k] * iDr : 0.0;
        }
        STAMP(5);

        auto solve = [&](const double* rcu, const double* rcl, double* dsu, double* dsl, double* dzu, double* dzl,
                         double& dxr) {
            double vd[3];
#pragma unroll
            for (int t = 0; t < 3; ++t)
                vd[t] = (onu[t] ? (zu[t] * rpu[t] - rcu[t]) * isu[t] : 0.0) - (onl[t] ? (zl[t] * rpl[t] - rcl[t]) * isl[t] : 0.0);
            double y = -rd - at_dot(vd);
#pragma unroll
            for (int k = 0; k < n; ++k) y = fma(-Lrow[k], readlane(y, k), y);     // L y = rhs
            y *= iDr;                                                              // D z = y
#pragma unroll
            for (int k = n - 1; k >= 0; --k) y = fma(-Lcol[k], readlane(y, k), y); // L' dx = z
            dxr = jl ? y : 0.0;
            double dxs[n], adx[3];
            bcast(dxr, dxs);
            rows_dot(dxr, dxs, adx);
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                dsu[t] = onu[t] ? -rpu[t] - adx[t] : 0.0;
                dsl[t] = onl[t] ? -rpl[t] + adx[t] : 0.0;
                dzu[t] = onu[t] ? (-rcu[t] - zu[t] * dsu[t]) * isu[t] : 0.0;
                dzl[t] = onl[t] ? (-rcl[t] - zl[t] * dsl[t]) * isl[t] : 0.0;
            }
        };
        auto step_to_boundary = [&](const double* dsu, const double* dsl, const double* dzu, const double* dzl) {
            double tm = 1.0;
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                if (onu[t] && dsu[t] < 0.0) tm = fmin(tm, -su[t] * frcp(dsu[t]));
                if (onl[t] && dsl[t] < 0.0) tm = fmin(tm, -sl[t] * frcp(dsl[t]));
                if (onu[t] && dzu[t] < 0.0) tm = fmin(tm, -zu[t] * frcp(dzu[t]));
                if (onl[t] && dzl[t] < 0.0) tm = fmin(tm, -zl[t] * frcp(dzl[t]));
            }
            return red8(tm, OpMin());
        };
        double rcu[3], rcl[3], dsu[3], dsl[3], dzu[3], dzl[3], dxr;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            rcu[t] = onu[t] ? su[t] * zu[t] : 0.0;
            rcl[t] = onl[t] ? sl[t] * zl[t] : 0.0;
        }
        solve(rcu, rcl, dsu, dsl, dzu, dzl, dxr);
        const double aa = step_to_boundary(dsu, dsl, dzu, dzl);
        double mal = 0.0;
#pragma unroll
        for (int t = 0; t < 3; ++t)
            mal += (onu[t] ? (su[t] + aa * dsu[t]) * (zu[t] + aa * dzu[t]) : 0.0) +
                   (onl[t] ? (sl[t] + aa * dsl[t]) * (zl[t] + aa * dzl[t]) : 0.0);
        const double mu_aff = red8(mal, OpSum()) * inact;
        const double sr = mu > 0.0 ? mu_aff * frcp(mu) : 0.0, sigma = sr * sr * sr;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            rcu[t] = onu[t] ? su[t] * zu[t] + dsu[t] * dzu[t] - sigma * mu : 0.0;
            rcl[t] = onl[t] ? sl[t] * zl[t] + dsl[t] * dzl[t] - sigma * mu : 0.0;
        }
        solve(rcu, rcl, dsu, dsl, dzu, dzl, dxr);
        const double al = fmin(1.0, 0.99 * step_to_boundary(dsu, dsl, dzu, dzl));
        x = fma(al, dxr, x);
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            su[t] = onu[t] ? fma(al, dsu[t], su[t]) : 1.0;
            sl[t] = onl[t] ? fma(al, dsl[t], sl[t]) : 1.0;
            zu[t] = onu[t] ? fma(al, dzu[t], zu[t]) : 0.0;
            zl[t] = onl[t] ? fma(al, dzl[t], zl[t]) : 0.0;
        }
        STAMP(6);
    }
    STAMP(3);
    if (jl) SH.X[r] = x;
    __syncthreads();

    // ---------------- outputs (arm.py:428-437) -------------------------------------------------
    const size_t ob = (size_t)n * b;
    if (l < n) {
        double t = 0.0;
        _Pragma("unroll") for (int k = 0; k < n; ++k) t = fma(M[l * n + k], SH.X[k], t);
        a.tau[ob + l] = t + hb[l];
        a.qdd[ob + l] = SH.X[l];
        SH.epos[l] = SH.X[l] - SH.beta[l];
        SH.qddd[l] = (SH.X[l] - qp[l]) / dt;
    }
    if (l < 6) {
        double e = 0.0;
        _Pragma("unroll") for (int k = 0; k < n; ++k) e = fma(J[l * n + k], SH.X[k], e);
        SH.eimp[l] = e + SH.e0[l];
    }
    __syncthreads();
    double lt = 0.0;
    if (l < 36) lt += SH.eimp[l / 6] * Wi[l] * SH.eimp[l % 6];
    if (l < n * n) {
        const int r = l / n, cc = l % n;
        lt += SH.epos[r] * Wp[l] * SH.epos[cc] + SH.qddd[r] * Ws[l] * SH.qddd[cc];
    }
    lt = wsum(lt);
    if (l == 0) {
        a.loss[b] = lt;
        a.status[b] = status;
        a.iters[b] = it;
    }
    STAMP(7);
    STAMP_FLUSH_TO(g_stamp_arm, b);
}

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_arm(const dartmpc::ArmArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    const dim3 g(args->B), w(dartmpc::kWave);
    switch (args->n) {      // joint count as a compile-time constant: every inner loop unrolls
        case 1: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<1>, g, w, 0, stream, *args); break;
        case 2: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<2>, g, w, 0, stream, *args); break;
        case 3: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<3>, g, w, 0, stream, *args); break;
        case 4: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<4>, g, w, 0, stream, *args); break;
        case 5: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<5>, g, w, 0, stream, *args); break;
        case 6: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<6>, g, w, 0, stream, *args); break;
        case 7: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<7>, g, w, 0, stream, *args); break;
        case 8: hipLaunchKernelGGL(dartmpc::arm_qp_kernel<8>, g, w, 0, stream, *args); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

#ifdef DART_STAMPS
// diagnostic build only: per-phase s_memtime cycles of block 0 from the last launch
extern "C" hipError_t dartmpc_read_stamps_arm(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_arm), sizeof(unsigned long long) * 16, 0,
                               hipMemcpyDeviceToHost);
}
#endif
