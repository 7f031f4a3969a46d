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
#include "wave.h"

namespace dartmpc {

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

// round-robin pairing of 8 indices, round r = 0..6 (index 7 fixed)
__device__ __forceinline__ int jpartner(int i, int r) {
    if (i == 7) return r;
    if (i == r) return 7;
    const int p = (2 * r - i) % 7;
    return p < 0 ? p + 7 : p;
}

__global__ __launch_bounds__(kWave) void arm_qp_kernel(ArmArgs a) {
    __shared__ ArmShared SH;
    const int b = blockIdx.x, l = threadIdx.x, n = a.n;
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
        const double off0 = wsum(ei != ej ? a0 * a0 : 0.0), dg0 = wsum(ei == ej ? a0 * a0 : 0.0);
        const double off1 = wsum(ei != ej ? a1 * a1 : 0.0), dg1 = wsum(ei == ej ? a1 * a1 : 0.0);
        if (off0 <= 1e-32 * dg0 && off1 <= 1e-32 * dg1) break;
        for (int r = 0; r < 7; ++r) {
            if (l < 16) {
                const int mat = l >> 3, i = l & 7;
                const int pi = jpartner(i, r);
                const int p = i < pi ? i : pi, qq = i < pi ? pi : i;
                const double* Am = SH.A[cur][mat];
                const double apq = Am[p * 8 + qq], app = Am[p * 9], aqq = Am[qq * 9];
                double c = 1.0, s = 0.0;
                if (apq != 0.0) {
                    const double tau = (aqq - app) / (2.0 * apq);
                    const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                    c = 1.0 / sqrt(1.0 + t * t);
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
    const double* A0 = SH.A[cur][0];
    const double* A1 = SH.A[cur][1];
    const double* V0 = SH.V[cur][0];
    const double* V1 = SH.V[cur][1];

    // ---------------- QP data (arm.py:335-388) -------------------------------------------------
    {   // pinv(M, rcond=1e-6) h: eigenvalues kept where |lambda| > 1e-6 max |lambda|
        const double lmax0 = wmax(l < n ? fabs(A0[(l < n ? l : 0) * 9]) : 0.0);
        if (l < n) {
            double y = 0.0;
            for (int k = 0; k < n; ++k) y = fma(V0[k * 8 + l], hb[k], y);
            const double lam = A0[l * 9];
            SH.y[l] = fabs(lam) > 1e-6 * lmax0 ? y / lam : 0.0;
        }
        // Mx: inv if |det| > 1e-8 else pinv(rcond=1e-3); eigen weights of Mx = 1/lambda or 0
        double det = 1.0, lmax1 = 0.0;
        for (int i = 0; i < 6; ++i) { det *= A1[i * 9]; lmax1 = fmax(lmax1, fabs(A1[i * 9])); }
        if (l < 6) {
            const double lam = A1[l * 9];
            const bool keep = fabs(det) > 1e-8 || fabs(lam) > 1e-3 * lmax1;
            SH.mxd[l] = keep ? 1.0 / lam : 0.0;
        }
    }
    __syncthreads();
    if (l < n) {
        double s = 0.0;
        for (int k = 0; k < n; ++k) s = fma(V0[l * 8 + k], SH.y[k], s);
        SH.mh[l] = s;
    }
    if (l < 36) {   // Mx and its safe square root (arm.py:355-358) from the same eigenvectors
        const int i = l / 6, j = l % 6;
        double mx = 0.0, sq = 0.0;
        for (int k = 0; k < 6; ++k) {
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
        for (int k = 0; k < n; ++k) {
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
        for (int k = 0; k < 6; ++k) m_ = fma(SH.Mx[l * 6 + k], SH.u1[k], m_);
        SH.mu[l] = m_;
    }
    if (l < 36) {   // D = S sqrt(K) + sqrt(K) S, sqrt elementwise as np.sqrt(K)
        const int i = l / 6, j = l % 6;
        double d1 = 0.0, d2 = 0.0;
        for (int k = 0; k < 6; ++k) {
            d1 = fma(SH.S[i * 6 + k], sqrt(Kt[k * 6 + j]), d1);
            d2 = fma(sqrt(Kt[i * 6 + k]), SH.S[k * 6 + j], d2);
        }
        SH.D[l] = d1 + d2;
    }
    __syncthreads();
    if (l < 6) {    // F = -D (J qd) + K twist + mu
        double f1 = 0.0, f2 = 0.0;
        for (int k = 0; k < 6; ++k) {
            const double tw = k < 3 ? mocap[k] - ee[k] : rv[k - 3];
            f1 = fma(SH.D[l * 6 + k], SH.vq[k], f1);
            f2 = fma(Kt[l * 6 + k], tw, f2);
        }
        SH.F[l] = (-f1 + f2) + SH.mu[l];
    }
    if (l >= 8 && l < 8 + n) {   // beta = 2 sqrt(diag Kn) (-qd) + Kn (-q)
        const int r = l - 8;
        double s = 0.0;
        for (int k = 0; k < n; ++k) s = fma(Kn[r * n + k], -q[k], s);
        SH.beta[r] = 2.0 * sqrt(Kn[r * n + r]) * -qd[r] + s;
    }
    __syncthreads();
    if (l < 6) {    // Eimp = J qdd + e0, e0 = Jdot qd - Mx_inv F
        double e1 = 0.0, e2 = 0.0;
        for (int k = 0; k < n; ++k) e1 = fma(Jd[l * n + k], qd[k], e1);
        for (int k = 0; k < 6; ++k) e2 = fma(Mxi[l * 6 + k], SH.F[k], e2);
        SH.e0[l] = e1 - e2;
    }
    if (l < 6 * n) {   // sym(Wimp) J
        const int i = l / n, cc = l % n;
        double w = 0.0;
        for (int k = 0; k < 6; ++k) w = fma(0.5 * (Wi[i * 6 + k] + Wi[k * 6 + i]), J[k * n + cc], w);
        SH.WJ[l] = w;
    }
    __syncthreads();
    const double idt2 = 1.0 / (dt * dt);
    if (l < n * n) {   // H = 2 (J' sym(Wimp) J + sym(Wpos) + sym(Ws) / dt^2)
        const int r = l / n, cc = l % n;
        double hv = 0.0;
        for (int k = 0; k < 6; ++k) hv = fma(J[k * n + r], SH.WJ[k * n + cc], hv);
        hv += 0.5 * (Wp[r * n + cc] + Wp[cc * n + r]) + 0.5 * (Ws[r * n + cc] + Ws[cc * n + r]) * idt2;
        SH.H[r * 8 + cc] = 2.0 * hv;
    }
    if (l < n) {       // c = 2 (J' sym(Wimp) e0 - sym(Wpos) beta - sym(Ws) qdd_prev / dt^2)
        double c1 = 0.0, c2 = 0.0, c3 = 0.0;
        for (int k = 0; k < 6; ++k) c1 = fma(SH.WJ[k * n + l], SH.e0[k], c1);
        for (int k = 0; k < n; ++k) {
            c2 = fma(0.5 * (Wp[l * n + k] + Wp[k * n + l]), SH.beta[k], c2);
            c3 = fma(0.5 * (Ws[l * n + k] + Ws[k * n + l]) * idt2, qp[k], c3);
        }
        SH.c[l] = 2.0 * (c1 - c2 - c3);
    }

    // ---------------- constraint rows (arm.py:391-398), IPOPT bound relaxation ----------------
    const int m = 3 * n;
    const bool row = l < m;
    const int blk = row ? l / n : 0, ri = row ? l % n : 0;
    double bi = 0.0, lo = -1e20, hi = 1e20;
    if (row) {
        bi = blk == 0 ? qd[ri] * dt + q[ri] : (blk == 1 ? qd[ri] : hb[ri]);
        lo = blk == 0 ? Qmin[ri] : (blk == 1 ? Qdmin[ri] : tmin[ri]);
        hi = blk == 0 ? Qmax[ri] : (blk == 1 ? Qdmax[ri] : tmax[ri]);
    }
    const bool onu = row && hi < 1e19, onl = row && lo > -1e19;
    const double gu = onu ? (hi + 1e-8 * fmax(1.0, fabs(hi))) - bi : 0.0;
    const double gl = onl ? bi - (lo - 1e-8 * fmax(1.0, fabs(lo))) : 0.0;
    const double a_pos = 0.5 * (dt * dt);
    auto arow = [&](const double* v) {      // a_i . v
        if (blk == 0) return a_pos * v[ri];
        if (blk == 1) return dt * v[ri];
        double s = 0.0;
        for (int k = 0; k < n; ++k) s = fma(M[ri * n + k], v[k], s);
        return s;
    };
    auto atv = [&](const double* v) {       // (A' v)_l, lanes l < n
        double s = 0.0;
        for (int k = 0; k < n; ++k) s = fma(M[k * n + l], v[2 * n + k], s);
        return a_pos * v[l] + dt * v[n + l] + s;
    };
    if (l < n) SH.X[l] = qp[l];            // warm start x0 = qdd_prev (arm.py:401-408)
    __syncthreads();

    double su, sl, zu, zl;
    {
        const double ax = row ? arow(SH.X) : 0.0;
        su = onu ? fmax(gu - ax, 1.0) : 1.0;
        sl = onl ? fmax(gl + ax, 1.0) : 1.0;
        zu = onu ? 1.0 : 0.0;
        zl = onl ? 1.0 : 0.0;
    }
    const double nact = fmax(1.0, (double)(__popcll(__ballot(onu)) + __popcll(__ballot(onl))));
    const double sd = 1.0 + wmax(l < n ? fabs(SH.c[l < n ? l : 0]) : 0.0);
    const double sp = 1.0 + wmax(fmax(onu ? fabs(gu) : 0.0, onl ? fabs(gl) : 0.0));
    const double tol = a.tol, acc_tol = a.acc_tol;

    int status = -1, it = 0;
    for (it = 0; it < a.max_iter; ++it) {
        const double ax = row ? arow(SH.X) : 0.0;
        const double rpu = onu ? ax + su - gu : 0.0;
        const double rpl = onl ? -ax + sl - gl : 0.0;
        if (row) SH.ZD[l] = zu - zl;
        __syncthreads();
        double rd = 0.0;
        if (l < n) {
            double hx = 0.0;
            for (int k = 0; k < n; ++k) hx = fma(SH.H[l * 8 + k], SH.X[k], hx);
            rd = hx + SH.c[l] + atv(SH.ZD);
        }
        const double rdm = wmax(fabs(rd));
        const double rpm = wmax(fmax(fabs(rpu), fabs(rpl)));
        const double mu = wsum((onu ? su * zu : 0.0) + (onl ? sl * zl : 0.0)) / nact;
        const double zmax = wmax(fmax(zu, zl));
        const double err = fmax(rdm / sd, fmax(rpm / sp, mu / sd));
        if (err <= tol) { status = 0; break; }
        if (zmax > 1e14 * sd) { status = -3; break; }
        if (row) SH.W[l] = (onu ? zu / su : 0.0) + (onl ? zl / sl : 0.0);
        __syncthreads();
        if (l < n * n) {   // K = H + A' W A
            const int r = l / n, cc = l % n;
            double kv = SH.H[r * 8 + cc];
            if (r == cc) kv += (a_pos * a_pos) * SH.W[r] + (dt * dt) * SH.W[n + r];
            for (int k = 0; k < n; ++k) kv = fma(M[k * n + r] * SH.W[2 * n + k], M[k * n + cc], kv);
            SH.K[0][r * 8 + cc] = kv;
        }
        __syncthreads();
        // LDL' of K (right-looking, ping-pong): after step p the pivot D_p = F(p, p) and the
        // column F(r, p) = D_p L(r, p), r > p, are final
        int kb = 0;
        bool bad = false;
        for (int p = 0; p < n; ++p) {
            const double piv = SH.K[kb][p * 9];
            bad = bad || !(piv > 0.0) || !isfinite(piv);
            if (l < n * n) {
                const int r = l / n, cc = l % n;
                const double arc = SH.K[kb][r * 8 + cc];
                SH.K[kb ^ 1][r * 8 + cc] = (r > p && cc > p) ? arc - SH.K[kb][r * 8 + p] * SH.K[kb][p * 8 + cc] / piv : arc;
            }
            __syncthreads();
            kb ^= 1;
        }
        if (bad) { status = err <= acc_tol ? 1 : -2; break; }
        // lane r < n keeps row r (forward) and column r (backward) of the unit factor L and D_r
        double Lrow[AN], Lcol[AN], Dr = 1.0;
        {
            const double* F = SH.K[kb];
            const int r = l < n ? l : 0;
            Dr = F[r * 9];
#pragma unroll
            for (int k = 0; k < AN; ++k) {
                Lrow[k] = (k < r) ? F[r * 8 + k] / F[k * 9] : 0.0;
                Lcol[k] = (k > r && k < n) ? F[k * 8 + r] / Dr : 0.0;
            }
        }

        auto solve = [&](double rcu, double rcl, double& dsu, double& dsl, double& dzu, double& dzl) {
            if (row) SH.VD[l] = (onu ? (zu * rpu - rcu) / su : 0.0) - (onl ? (zl * rpl - rcl) / sl : 0.0);
            __syncthreads();
            double y = (l < n) ? -rd - atv(SH.VD) : 0.0;
#pragma unroll
            for (int k = 0; k < AN; ++k) {          // L y = rhs
                if (k < n) { const double yk = readlane(y, k); y = fma(-Lrow[k], yk, y); }
            }
            y /= Dr;                                 // D z = y
#pragma unroll
            for (int k = AN - 1; k >= 0; --k) {     // L' dx = z
                if (k < n) { const double xk = readlane(y, k); y = fma(-Lcol[k], xk, y); }
            }
            if (l < n) SH.DX[l] = y;
            __syncthreads();
            const double adx = row ? arow(SH.DX) : 0.0;
            dsu = onu ? -rpu - adx : 0.0;
            dsl = onl ? -rpl + adx : 0.0;
            dzu = onu ? (-rcu - zu * dsu) / su : 0.0;
            dzl = onl ? (-rcl - zl * dsl) / sl : 0.0;
        };
        auto step_to_boundary = [&](double dsu, double dsl, double dzu, double dzl) {
            double t = 1.0;
            if (onu && dsu < 0.0) t = fmin(t, -su / dsu);
            if (onl && dsl < 0.0) t = fmin(t, -sl / dsl);
            if (onu && dzu < 0.0) t = fmin(t, -zu / dzu);
            if (onl && dzl < 0.0) t = fmin(t, -zl / dzl);
            return wmin(t);
        };
        double dsu, dsl, dzu, dzl;
        solve(onu ? su * zu : 0.0, onl ? sl * zl : 0.0, dsu, dsl, dzu, dzl);
        const double aa = step_to_boundary(dsu, dsl, dzu, dzl);
        const double mu_aff = wsum((onu ? (su + aa * dsu) * (zu + aa * dzu) : 0.0) +
                                   (onl ? (sl + aa * dsl) * (zl + aa * dzl) : 0.0)) / nact;
        const double sr = mu > 0.0 ? mu_aff / mu : 0.0, sigma = sr * sr * sr;
        const double rcu = onu ? su * zu + dsu * dzu - sigma * mu : 0.0;
        const double rcl = onl ? sl * zl + dsl * dzl - sigma * mu : 0.0;
        solve(rcu, rcl, dsu, dsl, dzu, dzl);
        const double al = fmin(1.0, 0.99 * step_to_boundary(dsu, dsl, dzu, dzl));
        if (l < n) SH.X[l] = fma(al, SH.DX[l], SH.X[l]);
        su = onu ? fma(al, dsu, su) : 1.0;
        sl = onl ? fma(al, dsl, sl) : 1.0;
        zu = onu ? fma(al, dzu, zu) : 0.0;
        zl = onl ? fma(al, dzl, zl) : 0.0;
        __syncthreads();
    }
    __syncthreads();

    // ---------------- outputs (arm.py:428-437) -------------------------------------------------
    const size_t ob = (size_t)n * b;
    if (l < n) {
        double t = 0.0;
        for (int k = 0; k < n; ++k) t = fma(M[l * n + k], SH.X[k], t);
        a.tau[ob + l] = t + hb[l];
        a.qdd[ob + l] = SH.X[l];
        SH.epos[l] = SH.X[l] - SH.beta[l];
        SH.qddd[l] = (SH.X[l] - qp[l]) / dt;
    }
    if (l < 6) {
        double e = 0.0;
        for (int k = 0; k < n; ++k) e = fma(J[l * n + k], SH.X[k], e);
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
}

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_arm(const dartmpc::ArmArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    hipLaunchKernelGGL(dartmpc::arm_qp_kernel, dim3(args->B), dim3(dartmpc::kWave), 0, stream, *args);
    return hipGetLastError();
}
