// ocp_wave.h -- one-wave, LDS-staged Riccati engine for small dense optimal-control QPs (gfx950).
//
// Used by the coupled-model solvers (RMPC, later LMPC), whose stage blocks are too large for the
// lane-per-node register recursion of the PMPC kernel.  One wave64 owns one instance; the stage
// data of all nodes sit in LDS; the backward Riccati sweep runs over the nodes in sequence and
// the lanes share each node's dense algebra ("lanes as matrix entries"):
//
//   z = [x~ (NXA) ; u (2) ; 1]                      homogeneous stage vector, ND = NXA + 3
//   x~+ = M z,  M = [[A B c]; [0 0 1]]  (NP x ND)   linearised dynamics incl. the defect c
//   V(x~) = 1/2 [x~;1]^T Pt [x~;1]                  value function, NP = NXA + 1
//   G = M^T Pt M + Ht                               stage QP incl. gradient (last row/column)
//   Pt' = Schur complement of G on the u block      ->  gains K (2 x NXA), feed-forward k (2)
//
// One LDS round trip per node (riccati_sweep_aug): lanes 8 g + s form u_g = Pt_{k+1} a_g row by
// row from G_{k+1} (the Schur complement that defines Pt_{k+1} folded in), exchange it inside their
// 8-lane group by DPP and write the packed entries of G_k = M_k^T Pt_{k+1} M_k + Ht_k.  The gains
// [K | k] and the multipliers are recovered from the stored G_k afterwards, lane per node.
//
// The forward sweep dx~_{k+1} = Phi_k dx~_k + f_k (Phi = A + B K, f = c + B k, formed for all
// nodes in parallel, lane per node) runs redundantly in every lane: no exchange on the chain.
#pragma once
#include <hip/hip_runtime.h>

#include "wave.h"

namespace dartmpc {

// The end of a node step of a backward sweep (the next node reads what this one wrote).  One wave: the LDS
// instructions of a wave execute in the order they are issued, so the next node's reads of G_k follow this
// node's write without a wait for it -- only the compiler must keep program order (the empty asm with a
// memory clobber: no LDS access moves across it).  Two waves (DART_WG = 2): a workgroup barrier.
__device__ __forceinline__ void chain_sync() {
#if DART_WG == 1
    asm volatile("" ::: "memory");
#else
    __syncthreads();
#endif
}

__host__ __device__ constexpr int tri(int n) { return n * (n + 1) / 2; }
__host__ __device__ constexpr int hp(int i, int j) { return i >= j ? tri(i) + j : tri(j) + i; }
__host__ __device__ constexpr int even(int n) { return (n + 1) & ~1; }

// Per-node LDS array whose per-node stride is an odd number of 16-byte units: lane-per-node
// accesses (lane k reads or writes its own node's block) then spread over 16 bank groups (2-way at
// most for ds_*_b64) instead of the 2-4 that a power-of-two-ish stride gives, and every node block
// stays 16-byte aligned for ds_read_b128 (MI355X_MICROARCH.md §LDS: bank = (a/4) mod 64 / mod 32).
template <class T, int N>
struct NodeArr {
    static constexpr int W = (int)(sizeof(T) / sizeof(double));
    static constexpr int W2 = (W + 1) & ~1;
    static constexpr int SW = (W2 / 2) % 2 ? W2 : W2 + 2;
    alignas(16) double buf[N * SW];
    __device__ __forceinline__ T& operator[](int k) { return *reinterpret_cast<T*>(buf + k * SW); }
    __device__ __forceinline__ const T& operator[](int k) const { return *reinterpret_cast<const T*>(buf + k * SW); }
};

template <int NXA_, int NMAXS_>
struct OcpLds {
    static constexpr int NXA = NXA_;          // augmented state dimension
    static constexpr int NP = NXA + 1;        // value-function dimension (with homogeneous 1)
    static constexpr int ND = NXA + 3;        // stage vector dimension [x~; u; 1]
    static constexpr int NMAXS = NMAXS_;      // max shooting nodes (N + 1)
    static constexpr int NC = even(NP);       // padded column stride of M (16-byte aligned reads)
    static constexpr int NT = tri(ND);        // packed entries of G / Ht
    static constexpr int NTP = even(NT);
    static constexpr int NF = even(NXA + 1);  // closed-loop row stride [Phi row | f]
    NodeArr<double[ND][NC], NMAXS> M;         // M[k][j][m] = M_k(m, j): column j of M_k
    NodeArr<double[NTP], NMAXS> H;            // stage Hessian + gradient, packed symmetric
    NodeArr<double[NTP], NMAXS> G;            // G_k; G[N] = terminal surrogate (Pt_N, Quu = I)
    NodeArr<double[2][NC], NMAXS> KK;         // [K | k]_k rows
    NodeArr<double[NXA][NF], NMAXS> F;        // closed loop: F[k][r] = [Phi_k(r, :) | f_k(r)]
    NodeArr<double[NXA][NF], NMAXS / 2> F2;   // two-node maps of nodes 2q, 2q + 1 (compose_pairs)
    double dx0[NC];                           // forward sweep start dx~_0
    double dxs[NMAXS / 2 + 1][NF];            // forward sweep: dx~ of node 2q + 2 (slot q), odd node N (slot N / 2)
};

// Two-node closed-loop maps F2[q] = [Phi_{2q+1} Phi_{2q} | Phi_{2q+1} f_{2q} + f_{2q+1}] of every
// node pair of each of H independent chains (slot of node k of chain h: h * SLOTS + k; pair slot
// h * SLOTS / 2 + q), one row per task, tasks spread over the wave.  The forward sweep then runs
// N / 2 dependent steps instead of N.  Ends with a barrier.
template <int H, int SLOTS, int NXA, int RPT, class FA, class F2A>
__device__ __forceinline__ void compose_pairs(FA& F, F2A& F2, int N) {
    // task = RPT rows of one pair: RPT trades rounds over the wave against work per lane
    constexpr int NB = (NXA + RPT - 1) / RPT;
    const int np2 = N >> 1, per = np2 * NB;
    for (int t = lane_id(); t < H * per; t += 64) {
        const int h = H == 1 ? 0 : t / per, rem = t - h * per, q = rem / NB, r0 = (rem - q * NB) * RPT;
        const int s0 = h * SLOTS + 2 * q;
        double b[NXA][NXA + 1];
#pragma unroll
        for (int m = 0; m < NXA; ++m)
#pragma unroll
            for (int j = 0; j <= NXA; ++j) b[m][j] = F[s0][m][j];
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) {
            const int r = r0 + rr < NXA ? r0 + rr : NXA - 1;
            double a[NXA + 1];
#pragma unroll
            for (int j = 0; j <= NXA; ++j) a[j] = F[s0 + 1][r][j];
            double o[NXA + 1];
#pragma unroll
            for (int j = 0; j <= NXA; ++j) o[j] = j < NXA ? a[0] * b[0][j] : fma(a[0], b[0][j], a[NXA]);
#pragma unroll
            for (int m = 1; m < NXA; ++m)
#pragma unroll
                for (int j = 0; j <= NXA; ++j) o[j] = fma(a[m], b[m][j], o[j]);
            if (r0 + rr < NXA) {
#pragma unroll
                for (int j = 0; j <= NXA; ++j) F2[h * (SLOTS / 2) + q][r][j] = o[j];
            }
        }
    }
    __syncthreads();
}

// z index of value-function index p (the homogeneous coordinate sits last in both)
template <int NXA>
__host__ __device__ constexpr int zi_of_p(int p) { return p < NXA ? p : NXA + 2; }

// packed G offsets of the value-space block (p, q), the (p, u_a) block and Quu
template <int NXA>
__host__ __device__ constexpr int gzz(int p, int q) { return hp(zi_of_p<NXA>(p), zi_of_p<NXA>(q)); }
template <int NXA>
__host__ __device__ constexpr int gzu(int p, int a) { return hp(zi_of_p<NXA>(p), NXA + a); }

// Quu of a packed G, its positive-definiteness and its inverse (wave-uniform values)
template <int NXA>
__device__ __forceinline__ bool quu_inverse(const double* Gk, double& i00, double& i01, double& i11) {
    const double g00 = Gk[hp(NXA, NXA)], g01 = Gk[hp(NXA + 1, NXA)], g11 = Gk[hp(NXA + 1, NXA + 1)];
    const double det = g00 * g11 - g01 * g01;
    const double idet = frcp(det);
    i00 = g11 * idet; i01 = -g01 * idet; i11 = g00 * idet;
    return (g00 > 0.0) && (det > 0.0) && isfinite(det);
}

// Backward sweep for the Delta-u-augmented stage (x~ = [x (NXA - 2); u_prev (2)], z = [x~; u; 1]):
// the u_prev columns of M_k are zero (x~+ does not depend on u_{k-1}), so G_k = H_k on every entry
// with a u_prev index, and the products need only the NP non-zero columns c(g) = [x, u, 1] of M_k.
// The node step runs in two register phases with one DPP exchange between them, instead of every
// lane forming a whole NP x NP bilinear form:
//   phase 1, lane 8 g + s:  u_g[s] = (Pt_{k+1} a_g)[s] = (Gzz a_g)[s] - Gzu(s, :) Quu^-1 (Guz a_g)
//   phase 2, lane 8 g + s:  G_k(c(g), c(s)) = H_k + sum_m a_s[m] u_g[m]  for s <= g, with the eight
//                           u_g[m] of its group gathered by quad_perm / row_half_mirror DPP moves
// (m = s ^ x, x = 0..7; row 7 of every M column is the zero pad).  The 17 entries with a u_prev
// index are copied from H_k by lanes that write no product entry.  G[N] must hold the terminal
// surrogate.  Returns false (wave-uniform) if some Quu is not positive definite (inertia correction).
struct AugRoles {
    int cg, s, e;        // z column of the lane's group, lane in the group, packed entry written
    bool prod;           // a product entry (else a u_prev entry copied from H_k, or the pad slot)
    int goff[8];         // G_{k+1}(zs, z(n)) offsets of the value indices n
    int gsu0, gsu1;      // Gzu(s, 0), Gzu(s, 1)
    int cs;              // z column of the lane's value index s
};

template <class L>
__device__ __forceinline__ AugRoles aug_roles() {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND, NX = NXA - 2;
    static_assert(ND == NXA + 3 && NP <= 8 && L::NC == 8, "two inputs, value dimension <= 8, M columns padded to 8");
    AugRoles R;
    const int lane = lane_id();
    const int g = lane >> 3, s = lane & 7;
    const int ge = g < NP ? g : NP - 1, se = s < NP ? s : NP - 1;          // clamped (idle lanes stay finite)
    R.cg = ge < NX ? ge : ge + 2; R.cs = se < NX ? se : se + 2;           // z columns of the groups
    R.s = s;
    const int zs = se < NXA ? se : ND - 1;                                // z index of value index s
    // the packed entry this lane writes: a product entry (c(g), c(s)), s <= g < NP; or a u_prev entry
    // copied from H_k (q-th of the 17, enumerated row by row); or none
    R.prod = g < NP && s <= g;
    int q = -1;
    if (g >= NP) q = s;                                                   // lanes 56..63: q = 0..7
    else if (s > g) q = 8 + g * 7 - g * (g - 1) / 2 + (s - g - 1);        // upper-triangle lanes
    int ecopy = -1;
    if (q >= 0) {
        int n = 0;
        for (int i = 0; i < ND; ++i)
            for (int j = 0; j <= i; ++j)
                if (i == NX || i == NX + 1 || j == NX || j == NX + 1) {
                    if (n == q) ecopy = hp(i, j);
                    ++n;
                }
    }
    // lanes with no entry write the pad slot NT (straight-line stores, no exec masking)
    static_assert(L::NTP > L::NT, "a pad slot after the packed entries");
    R.e = R.prod ? hp(R.cg, R.cs) : (ecopy >= 0 ? ecopy : L::NT);
    // G_{k+1}(zs, z(n)) of the value indices n: packed row zs for z(n) <= zs, else column zs of row z(n)
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        const int zn = n < NXA ? n : ND - 1;
        R.goff[n] = zn <= zs ? tri(zs) + zn : tri(zn) + zs;
    }
    R.gsu0 = hp(NXA, zs); R.gsu1 = hp(NXA + 1, zs);
    return R;
}

// One node step: G_k from M_k, H_k and the value function held in Gn (G_{k+1}, or its soft-row
// surrogate); ok &= Quu of Gn positive definite.  Ends with chain_sync().
// Every LDS read of the step is issued before the first product, with no wait in between (the sched_barrier
// keeps the scheduler from sinking reads behind the arithmetic, where their latency would sit on the node
// chain): the M_k column of phase 1 first, then G_{k+1} -- the read that waits on the previous node's write --
// then the phase-2 column of M_k and the H entry, which are needed last.
// The step's operands that do not depend on the chain: the phase-1 and phase-2 columns of M_k and the H entry.
// The soft sweep reads them before the soft-row transform of node k+1 (aug_node_in), off the chain.
template <class L>
struct AugNodeIn {
    double a[L::NP], b[8], hk;
};
template <class L>
__device__ __forceinline__ void aug_node_in(const L* S, int k, const AugRoles& R, AugNodeIn<L>& in) {
    constexpr int NP = L::NP, NC = L::NC;
    const double* Mk = &S->M[k][0][0];
#pragma unroll
    for (int m = 0; m < NP; ++m) in.a[m] = Mk[R.cg * NC + m];
#pragma unroll
    for (int x = 0; x < 8; ++x) in.b[x] = Mk[R.cs * NC + (R.s ^ x)];
    in.hk = S->H[k][R.e];
}
template <class L, bool PRE = false>
__device__ __forceinline__ void aug_node_step(L* S, int k, const double* Gn, const AugRoles& R, bool& ok,
                                              const AugNodeIn<L>* pre = nullptr) {
    constexpr int NXA = L::NXA, NP = L::NP, NC = L::NC;
    const double* Mk = &S->M[k][0][0];
    double a[NP], b[8];
    if constexpr (PRE) {
#pragma unroll
        for (int m = 0; m < NP; ++m) a[m] = pre->a[m];
    } else {
#pragma unroll
        for (int m = 0; m < NP; ++m) a[m] = Mk[R.cg * NC + m];
    }
    __builtin_amdgcn_sched_barrier(0);
    double gz[NP], gu0[NP], gu1[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) { gu0[n] = Gn[gzu<NXA>(n, 0)]; gu1[n] = Gn[gzu<NXA>(n, 1)]; }
    const double q00 = Gn[hp(NXA, NXA)], q01 = Gn[hp(NXA + 1, NXA)], q11 = Gn[hp(NXA + 1, NXA + 1)];
#pragma unroll
    for (int n = 0; n < NP; ++n) gz[n] = Gn[R.goff[n]];
    const double gs0 = Gn[R.gsu0], gs1 = Gn[R.gsu1];
    __builtin_amdgcn_sched_barrier(0);
    double hk;
    if constexpr (PRE) {
#pragma unroll
        for (int x = 0; x < 8; ++x) b[x] = pre->b[x];
        hk = pre->hk;
    } else {
#pragma unroll
        for (int x = 0; x < 8; ++x) b[x] = Mk[R.cs * NC + (R.s ^ x)];
        hk = S->H[k][R.e];
    }
    __builtin_amdgcn_sched_barrier(0);
    double t0 = 0.0, t1 = 0.0, w0 = 0.0, w1 = 0.0;
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        w0 = fma(gu0[n], a[n], w0);
        w1 = fma(gu1[n], a[n], w1);
    }
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        if (n & 1) t1 = fma(gz[n], a[n], t1);
        else t0 = fma(gz[n], a[n], t0);
    }
    // r = Quu^-1 Guz(:, s) depends on G_{k+1} alone: it runs beside the products with a_g
    const double det = fma(q00, q11, -q01 * q01);
    ok = ok && (q00 > 0.0) && (det > 0.0) && isfinite(det);
    const double idet = frcp(det);
    const double r0 = fma(q11, gs0, -q01 * gs1) * idet, r1 = fma(q00, gs1, -q01 * gs0) * idet;
    const double u = (t0 + t1) - fma(r0, w0, r1 * w1);
    // phase 2: u_g[s ^ x] of the 8-lane group
    const double m7 = dpp<0x141>(u);                                 // row_half_mirror: lane s <- 7 - s
    const double ux[8] = {u, dpp<0xB1>(u), dpp<0x4E>(u), dpp<0x1B>(u), dpp<0x1B>(m7), dpp<0x4E>(m7),
                          dpp<0xB1>(m7), m7};
    double p0 = hk, p1 = 0.0;
#pragma unroll
    for (int x = 0; x < 8; x += 2) { p0 = fma(b[x], ux[x], p0); p1 = fma(b[x + 1], ux[x + 1], p1); }
    // all reads of G_{k+1} and M_k precede the write of G_k (distinct rows: no hazard)
    S->G[k][R.e] = R.prod ? p0 + p1 : hk;
    chain_sync();
}

template <class L>
__device__ bool riccati_sweep_aug(L* S, int N) {
    constexpr int NXA = L::NXA;
    const AugRoles R = aug_roles<L>();
    bool ok = true;
    // (unrolled by two like riccati_s_sweep, this kernel spills: C3 -20 %, profiles/r04/node_unroll_ab.txt)
    for (int k = N - 1; k >= 0; --k) aug_node_step<L>(S, k, S->G[k + 1], R, ok);
    double i00, i01, i11;
    return quu_inverse<NXA>(S->G[0], i00, i01, i11) && ok;
}

// ------------------------------------------------------------------------------------------
// Soft rows (IPOPT's restoration phase, rmpc_ipm.hip): the first NS rows of node j's incoming defect are
// soft, J dx - D dlam = rhs.  In the recursion the value function of node j is then seen through them:
// eliminating the row slack w (Hessian D^-1 on value indices ph = 0..NS-1) from V(x~ + w) gives
//   Pt' = P (I + D P)^-1 (over the value indices [x~; 1], P the Schur complement of G_j on u),
// and the node step runs unchanged on the surrogate [[Pt', 0], [0, I_u]] (Gs).  With S = P(ph, ph) + D^-1
// (positive definite: part of the inertia test) and W = S^-1 D^-1 every block is formed without
// cancellation, whatever the mix of nearly hard (D^-1 huge) and nearly free (D^-1 tiny) rows -- the
// Woodbury form P - P(:, ph) S^-1 P(ph, :) loses all accuracy on a free row's block at mu ~ 1e-9
// (D^-1 spans 1e-7 ... 1e15 there):
//   Pt'(ph, ph) = P(ph, ph) W,   Pt'(r, ph) = P(r, ph) W,   Pt'(r, r') = P(r, r') - P(r, ph) S^-1 P(ph, r')
// (r, r' the other value indices).  The incoming rows of node j map x~+ <- y with
//   y(ph) = W x~+(ph) - S^-1 P(ph, r) [x~+(r); 1] = Y [x~+; 1],  Y (NS x NP) kept per node.
template <class L, int NS>
struct AugSoftLds {
    NodeArr<double[NS * L::NP], L::NMAXS> T;  // Y_j row-major NS x NP (value indices)
    NodeArr<double[NS], L::NMAXS> Dinv;       // 1 / D of node j's soft rows
    alignas(16) double Gs[L::NTP];            // the surrogate of G_{k+1}
};

// the constant u rows of the surrogate (Gzu = 0, Quu = I); call once before the soft sweeps
template <class L, int NS>
__device__ __forceinline__ void aug_soft_init(AugSoftLds<L, NS>* RS) {
    constexpr int NXA = L::NXA;
    for (int e = lane_id(); e < L::NTP; e += 64) {
        int i = 0;
        while (tri(i + 1) <= e) ++i;
        const int j = e - tri(i);
        const bool ui = i == NXA || i == NXA + 1, uj = j == NXA || j == NXA + 1;
        if (ui || uj || e >= L::NT) RS->Gs[e] = (ui && i == j) ? 1.0 : 0.0;
    }
    __syncthreads();
}

// Node j's soft rows seen from G_j: lane e < tri(NP) owns the packed value entry (pv, qv), qv <= pv; every
// such lane forms S from G_j, factors it S = L diag(dd) L^T (its own copy) and solves one system S t = b for
// its entry -- b = e_qv (both indices soft: Pt'(pv, qv) = D^-1_qv P(pv, ph) t), b = P(ph, pv) (pv not soft,
// qv soft: Pt'(pv, qv) = D^-1_qv t_qv), b = P(ph, qv) (neither: Pt'(pv, qv) = P(pv, qv) - P(pv, ph) t); the
// diagonal soft lanes store Y's column qv (D^-1_qv t), the lanes of the homogeneous row with qv not soft store
// -t.  With `surrogate` every lane stores Pt'(pv, qv) into Gs.  ok &= (Quu of G_j and S positive definite).
// Ends with a barrier.
// The lane's packed value entry (pv, qv) of aug_soften, the same at every node: formed once per sweep.
struct SoftenRoles {
    int pv, qv;
};
template <class L>
__device__ __forceinline__ SoftenRoles soften_roles() {
    constexpr int NV = tri(L::NP);
    const int e0 = lane_id() < NV ? lane_id() : NV - 1;
    SoftenRoles R;
    R.pv = 0;
    while (tri(R.pv + 1) <= e0) ++R.pv;
    R.qv = e0 - tri(R.pv);
    return R;
}
template <class L, int NS>
__device__ __forceinline__ void aug_soften(L* S, AugSoftLds<L, NS>* RS, int j, bool surrogate, const SoftenRoles& SR,
                                           bool& ok) {
    constexpr int NXA = L::NXA, NP = L::NP, NV = tri(NP);
    const int pv = SR.pv, qv = SR.qv;
    const bool act = lane_id() < NV;
    const bool ps = pv < NS, qs = qv < NS;          // (qv <= pv: qs whenever ps)
    const double* Gn = S->G[j];
    const double q00 = Gn[hp(NXA, NXA)], q01 = Gn[hp(NXA + 1, NXA)], q11 = Gn[hp(NXA + 1, NXA + 1)];
    const double det = fma(q00, q11, -q01 * q01);
    ok = ok && (q00 > 0.0) && (det > 0.0) && isfinite(det);
    const double idet = frcp(det);
    const double i00 = q11 * idet, i01 = -q01 * idet, i11 = q00 * idet;
    // w(a) = Quu^-1 Gzu(a, :); P(a, b) = Gzz(a, b) - Gzu(b, :) w(a)
    double ga0[NS], ga1[NS], wa0[NS], wa1[NS];
#pragma unroll
    for (int a = 0; a < NS; ++a) {
        ga0[a] = Gn[gzu<NXA>(a, 0)]; ga1[a] = Gn[gzu<NXA>(a, 1)];
        wa0[a] = fma(i00, ga0[a], i01 * ga1[a]); wa1[a] = fma(i01, ga0[a], i11 * ga1[a]);
    }
    const int bc = (!ps && qs) ? pv : qv;           // the column of P(ph, :) on the right-hand side
    const double gq0 = Gn[gzu<NXA>(qv, 0)], gq1 = Gn[gzu<NXA>(qv, 1)];
    const double gp0 = Gn[gzu<NXA>(pv, 0)], gp1 = Gn[gzu<NXA>(pv, 1)];
    const double gb0 = Gn[gzu<NXA>(bc, 0)], gb1 = Gn[gzu<NXA>(bc, 1)];
    const double wq0 = fma(i00, gq0, i01 * gq1), wq1 = fma(i01, gq0, i11 * gq1);
    double P[NS][NS], rb[NS], rp[NS], di[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
#pragma unroll
        for (int c = 0; c <= i; ++c) P[i][c] = Gn[gzz<NXA>(i, c)] - fma(ga0[i], wa0[c], ga1[i] * wa1[c]);
        rb[i] = Gn[gzz<NXA>(i, bc)] - fma(gb0, wa0[i], gb1 * wa1[i]);     // P(i, bc)
        rp[i] = Gn[gzz<NXA>(i, pv)] - fma(gp0, wa0[i], gp1 * wa1[i]);     // P(i, pv)
        di[i] = RS->Dinv[j][i];
    }
    const double pvq = Gn[gzz<NXA>(pv, qv)] - fma(gp0, wq0, gp1 * wq1);
    double Lm[NS][NS], id[NS], dd[NS];
#pragma unroll
    for (int c = 0; c < NS; ++c) {
        double t = P[c][c] + di[c];
#pragma unroll
        for (int m = 0; m < c; ++m) t -= Lm[c][m] * Lm[c][m] * dd[m];
        dd[c] = t;
        ok = ok && t > 0.0 && isfinite(t);
        id[c] = 1.0 / t;
#pragma unroll
        for (int i = c + 1; i < NS; ++i) {
            double u = P[i][c];
#pragma unroll
            for (int m = 0; m < c; ++m) u -= Lm[i][m] * Lm[c][m] * dd[m];
            Lm[i][c] = u * id[c];
        }
    }
    double y[NS], t4[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        double t = qs && ps ? (i == qv ? 1.0 : 0.0) : rb[i];
#pragma unroll
        for (int m = 0; m < i; ++m) t -= Lm[i][m] * y[m];
        y[i] = t;
    }
#pragma unroll
    for (int i = NS - 1; i >= 0; --i) {
        double t = y[i] * id[i];
#pragma unroll
        for (int m = i + 1; m < NS; ++m) t -= Lm[m][i] * t4[m];
        t4[i] = t;
    }
    double dq = 0.0, tq = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        if (i == qv) { dq = di[i]; tq = t4[i]; }
    }
    if (act && ps && pv == qv) {
#pragma unroll
        for (int i = 0; i < NS; ++i) RS->T[j][NP * i + qv] = dq * t4[i];
    }
    if (act && !qs && pv == NP - 1) {
#pragma unroll
        for (int i = 0; i < NS; ++i) RS->T[j][NP * i + qv] = -t4[i];
    }
    if (surrogate && act) {
        double v;
        if (ps) {             // both soft: D^-1_qv P(pv, ph) S^-1 e_qv  (P(pv, i) = P[max][min])
            v = 0.0;
#pragma unroll
            for (int a = 0; a < NS; ++a) v = fma(rp[a], t4[a], v);
            v *= dq;
        } else if (qs) {      // pv not soft, qv soft: D^-1_qv (S^-1 P(ph, pv))_qv
            v = dq * tq;
        } else {
            v = pvq;
#pragma unroll
            for (int a = 0; a < NS; ++a) v -= rp[a] * t4[a];
        }
        RS->Gs[gzz<NXA>(pv, qv)] = v;
    }
    chain_sync();
}

// Backward sweep with the soft rows of every node (restoration phase): before the step of node k the
// surrogate of G_{k+1} seen through node k+1's soft rows, Y_{k+1} kept for the forward map; Y_0 of the soft
// initial rows last.  G[N] must hold the terminal surrogate, RS->Dinv every node's 1 / D, the u rows of
// RS->Gs their constants (aug_soft_init).  Returns false (wave-uniform) if some S or Quu is not positive
// definite.
template <class L, int NS>
__device__ bool riccati_sweep_aug_soft(L* S, AugSoftLds<L, NS>* RS, int N) {
    const AugRoles R = aug_roles<L>();
    const SoftenRoles SR = soften_roles<L>();
    bool ok = true;
    for (int k = N - 1; k >= 0; --k) {
        AugNodeIn<L> in;
        aug_node_in<L>(S, k, R, in);          // off the chain: issued before the transform's closing fence
        aug_soften<L, NS>(S, RS, k + 1, true, SR, ok);
        aug_node_step<L, true>(S, k, RS->Gs, R, ok, &in);
    }
    aug_soften<L, NS>(S, RS, 0, false, SR, ok);
    return !wany(!ok);
}

// ------------------------------------------------------------------------------------------
// Node step for stages whose M columns may all be non-zero (the PMPC restoration kernel, pmpc_resto.hip:
// x~ = the six states, no u_prev block).  Two LDS phases: lane NP i + s (i < ND, s < NP) forms
// u_i[s] = (Pt_{k+1} a_i)[s] = (Gzz a_i)[s] - Gzu(s, :) Quu^-1 (Guz a_i), a_i column i of M_k, parked in U
// (ND rows of stride NC); then lane e < NT forms the packed entry G_k(i, j) = H_k(i, j) + a_j^T u_i.
// ok &= Quu of Gn positive definite.  Two barriers.  R: the lane roles (gen_roles), the same at every node.
struct GenRoles {
    int i1, s1;          // phase 1: stage column i, value index s of lane NP i + s (clamped)
    int i2, j2;          // phase 2: the packed entry (i, j) of lane e < NT
};
template <class L>
__device__ __forceinline__ GenRoles gen_roles() {
    constexpr int NP = L::NP, ND = L::ND;
    GenRoles R;
    const int lane = lane_id();
    const int l = lane < ND * NP ? lane : ND * NP - 1;
    R.i1 = l / NP; R.s1 = l - R.i1 * NP;
    const int e = lane < L::NT ? lane : 0;
    int i = 0;
    while (tri(i + 1) <= e) ++i;
    R.i2 = i; R.j2 = e - tri(i);
    return R;
}
template <class L>
__device__ __forceinline__ void gen_node_step(L* S, int k, const double* Gn, double* U, const GenRoles& R, bool& ok) {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND, NC = L::NC;
    static_assert(ND * NP <= 64 && NP <= NC, "one lane per (stage column, value index)");
    const int lane = lane_id();
    const double* Mk = &S->M[k][0][0];
    const int i = R.i1, s = R.s1;
    // every read that does not depend on this step's own products is issued up front, in three groups (as
    // aug_node_step): column i of M_k, then G_{k+1} (the read that follows the previous node's write), then
    // the phase-2 column j of M_k and the H entry; the three accumulations below keep their order
    double an[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) an[n] = Mk[i * NC + n];
    __builtin_amdgcn_sched_barrier(0);
    const double q00 = Gn[hp(NXA, NXA)], q01 = Gn[hp(NXA + 1, NXA)], q11 = Gn[hp(NXA + 1, NXA + 1)];
    double gsn[NP], g0n[NP], g1n[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) { gsn[n] = Gn[gzz<NXA>(s, n)]; g0n[n] = Gn[gzu<NXA>(n, 0)]; g1n[n] = Gn[gzu<NXA>(n, 1)]; }
    const double gs0 = Gn[gzu<NXA>(s, 0)], gs1 = Gn[gzu<NXA>(s, 1)];
    __builtin_amdgcn_sched_barrier(0);
    const int i2 = R.i2, j2 = R.j2;
    double mj[NP];
#pragma unroll
    for (int m = 0; m < NP; ++m) mj[m] = Mk[j2 * NC + m];
    const double hk = S->H[k][lane < L::NT ? lane : 0];
    __builtin_amdgcn_sched_barrier(0);
    const double det = fma(q00, q11, -q01 * q01);
    ok = ok && (q00 > 0.0) && (det > 0.0) && isfinite(det);
    double t = 0.0, w0 = 0.0, w1 = 0.0;
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        t = fma(gsn[n], an[n], t);
        w0 = fma(g0n[n], an[n], w0);
        w1 = fma(g1n[n], an[n], w1);
    }
    const double r0 = fma(q11, gs0, -q01 * gs1) / det, r1 = fma(q00, gs1, -q01 * gs0) / det;
    if (lane < ND * NP) U[i * NC + s] = t - fma(r0, w0, r1 * w1);
    chain_sync();
    if (lane < L::NT) {
        double gv = hk;
#pragma unroll
        for (int m = 0; m < NP; ++m) gv = fma(mj[m], U[i2 * NC + m], gv);
        S->G[k][lane] = gv;
    }
    chain_sync();
}

// backward sweeps with gen_node_step: plain, and with the soft rows of every node (as riccati_sweep_aug[_soft])
template <class L>
__device__ bool riccati_sweep_gen(L* S, int N, double* U) {
    const GenRoles R = gen_roles<L>();
    bool ok = true;
    for (int k = N - 1; k >= 0; --k) gen_node_step<L>(S, k, S->G[k + 1], U, R, ok);
    double i00, i01, i11;
    return quu_inverse<L::NXA>(S->G[0], i00, i01, i11) && ok;
}
template <class L, int NS>
__device__ bool riccati_sweep_gen_soft(L* S, AugSoftLds<L, NS>* RS, int N, double* U) {
    const GenRoles R = gen_roles<L>();
    const SoftenRoles SR = soften_roles<L>();
    bool ok = true;
    // (the operands off the chain stay in the node step here: read ahead of the NS = 6 transform they spill)
    for (int k = N - 1; k >= 0; --k) {
        aug_soften<L, NS>(S, RS, k + 1, true, SR, ok);
        gen_node_step<L>(S, k, RS->Gs, U, R, ok);
    }
    aug_soften<L, NS>(S, RS, 0, false, SR, ok);
    return !wany(!ok);
}

struct NoPost {
    __device__ void operator()(int, int) const {}
};
template <class P> struct IsNoPost { static constexpr bool value = false; };
template <> struct IsNoPost<NoPost> { static constexpr bool value = true; };

// Gains and closed-loop matrices for the forward sweep, lanes k and k + 32 per node (of the calling wave): both
// form [K | k] = -Quu^-1 Guz, lane k writes it, and the rows of Phi_k = A_k + B_k K_k, f_k = c_k + B_k k_k
// split between them.  Ends with a barrier.
// post(k) (restoration phase: the rows mapped through node k+1's soft rows) runs on the node lanes k < N
// after every row of F_k is written, before the pair maps are composed.
template <class L, class Post = NoPost>
__device__ void closed_loop(L* S, int N, Post post = Post()) {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND, RH = (NXA + 1) / 2;
    const int k = node_base() + (lane_id() & 31), rb = lane_id() >= 32 ? RH : 0;
    if (k < N) {
        // LDS reads grouped ahead of the writes (the compiler cannot prove F, KK and M disjoint and
        // would otherwise wait out each read before the next write)
        const double* Gk = S->G[k];
        double gu0[NP], gu1[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) { gu0[p] = Gk[gzu<NXA>(p, 0)]; gu1[p] = Gk[gzu<NXA>(p, 1)]; }
        double i00, i01, i11;
        quu_inverse<NXA>(Gk, i00, i01, i11);
        double K0[NP], K1[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            K0[p] = -fma(i00, gu0[p], i01 * gu1[p]);
            K1[p] = -fma(i01, gu0[p], i11 * gu1[p]);
        }
        if (rb == 0) {
#pragma unroll
            for (int p = 0; p < NP; ++p) { S->KK[k][0][p] = K0[p]; S->KK[k][1][p] = K1[p]; }
        }
#pragma unroll
        for (int rr = 0; rr < RH; ++rr) {    // row r of M_k read whole before row r of F is written
            const int r = rb + rr < NXA ? rb + rr : NXA - 1;
            double mr[NXA + 3];
#pragma unroll
            for (int j = 0; j < NXA + 3; ++j) mr[j] = S->M[k][j < NXA + 2 ? j : ND - 1][r];
            const double b0 = mr[NXA], b1 = mr[NXA + 1];
#pragma unroll
            for (int j = 0; j < NXA; ++j) S->F[k][r][j] = fma(b0, K0[j], fma(b1, K1[j], mr[j]));
            S->F[k][r][NXA] = fma(b0, K0[NXA], fma(b1, K1[NXA], mr[NXA + 2]));
        }
    }
    __syncthreads();
    if constexpr (!IsNoPost<Post>::value) {
        if (k < N && lane_id() < 32) post(k);
        __syncthreads();
    }
    compose_pairs<1, L::NMAXS, NXA, 1>(S->F, S->F2, N);   // NXA floor(N / 2) tasks: one round over the wave for N <= 21 (RMPC), two beyond
}

// Multiplier of the dynamics row into node k: lam~_k = -Pt_k [dx~; 1] (first NXA rows), with
// Pt_k [dx~; 1] = Gzz [dx~; 1] + Gzu du (du = [K | k][dx~; 1]), read from G_k (lane per node).
template <class L>
__device__ __forceinline__ void node_multiplier(const L* S, int k, const double* dx, const double* du, double* lam) {
    constexpr int NXA = L::NXA, NP = L::NP;
    const double* Gk = S->G[k];
#pragma unroll
    for (int p = 0; p < NXA; ++p) {
        double t = Gk[gzz<NXA>(p, NP - 1)];
#pragma unroll
        for (int q = 0; q < NXA; ++q) t = fma(Gk[gzz<NXA>(p, q)], dx[q], t);
        t = fma(Gk[gzu<NXA>(p, 0)], du[0], t);
        t = fma(Gk[gzu<NXA>(p, 1)], du[1], t);
        lam[p] = -t;
    }
}

// One step of a paired forward chain: s = row r of F [d; 1], parked (every lane of a row holds the
// same s; all lanes store, no EXEC masking), then broadcast within the row into d.
template <int NXA>
__device__ __forceinline__ void pair_step(const double* F, double* d, double* park) {
    double s0 = F[NXA], s1 = 0.0;       // two accumulators: half the dependent FMA depth
#pragma unroll
    for (int j = 0; j < NXA; j += 2) {
        s0 = fma(F[j], d[j], s0);
        if (j + 1 < NXA) s1 = fma(F[j + 1], d[j + 1], s1);
    }
    const double s = s0 + s1;
    *park = s;
#pragma unroll
    for (int i = 0; i < NXA; ++i) d[i] = row_bcast_over(s, i, d[i]);
}

// The chain over the np2 pair maps of one half (pair slots p0 .. p0 + np2 - 1, row r), two pairs per
// trip with ping-pong rows: the rows of the next pair are loaded before the current step and held
// in registers across it (PREFETCH; the empty asm keeps the compiler from sinking the loads into the
// next step, where every step would wait out an LDS latency), else loaded when needed.
template <int NXA, bool PREFETCH, class F2A, class PA>
__device__ __forceinline__ void pair_chain(const F2A& F2, int p0, int np2, int r, double* d, PA park) {
    double Fa[NXA + 1], Fb[NXA + 1];
#pragma unroll
    for (int j = 0; j <= NXA; ++j) Fa[j] = F2[p0][r][j];
    for (int q = 0; q < np2; q += 2) {
        const bool two = q + 1 < np2;
        if constexpr (PREFETCH) {
#pragma unroll
            for (int j = 0; j <= NXA; ++j) Fb[j] = F2[p0 + (two ? q + 1 : q)][r][j];
        }
        pair_step<NXA>(Fa, d, park(q));
        if (!two) break;
        if constexpr (PREFETCH) {
#pragma unroll
            for (int j = 0; j <= NXA; ++j) asm volatile("" : "+v"(Fb[j]));
            const int qn = q + 2 < np2 ? q + 2 : q + 1;
#pragma unroll
            for (int j = 0; j <= NXA; ++j) Fa[j] = F2[p0 + qn][r][j];
        } else {
#pragma unroll
            for (int j = 0; j <= NXA; ++j) Fb[j] = F2[p0 + q + 1][r][j];
        }
        pair_step<NXA>(Fb, d, park(q + 1));
        if constexpr (PREFETCH) {
#pragma unroll
            for (int j = 0; j <= NXA; ++j) asm volatile("" : "+v"(Fa[j]));
        } else if (q + 2 < np2) {
#pragma unroll
            for (int j = 0; j <= NXA; ++j) Fa[j] = F2[p0 + q + 2][r][j];
        }
    }
}

// Forward sweep over node pairs: lane 16 w + r (r < NXA) of every row w owns row r of the two-node
// chain dx~_{2q+2} = F2[q] [dx~_{2q}; 1] -- the four rows run the same chain, so each row
// broadcasts the new state to itself by 64-bit DPP row_newbcast (no scalar round trip).  The rows of
// pair q + 1 are loaded while pair q is processed (held in registers across the step by an empty asm,
// or the compiler sinks the loads into the next step and every step waits out an LDS latency), and
// row 0 parks each new state in S->dxs instead of every lane selecting it into its own slot.  An odd
// N ends with one single-node step; the odd nodes in between follow afterwards, lane per node, from
// their even predecessor (off the chain).  Lane-per-node use: every lane returns in dxo the state step
// of node `node` = its lane (node > N keeps dx~_0).  S->dx0 must hold dx~_0; compose_pairs must have
// run.  Ends with a barrier.
template <class L, bool PREFETCH = true>
__device__ void forward_sweep(L* S, int N, int node, double* dxo) {
    constexpr int NXA = L::NXA;
    const int lr = lane_id() & 15;
    const int r = lr < NXA ? lr : 0;
    double d[NXA];
#pragma unroll
    for (int i = 0; i < NXA; ++i) d[i] = S->dx0[i];
    const int np2 = N >> 1;
    pair_chain<NXA, PREFETCH>(S->F2, 0, np2, r, d, [&](int q) { return &S->dxs[q][r]; });
    if (N & 1) {
        const double* row = S->F[N - 1][r];
        double s = row[NXA];
#pragma unroll
        for (int j = 0; j < NXA; ++j) s = fma(row[j], d[j], s);
        S->dxs[np2][r] = s;
    }
    __syncthreads();
    // even nodes 2 .. 2 np2 and an odd terminal node from the parked states, node 0 from dx~_0
    const bool even_n = !(node & 1) && node >= 2 && node <= 2 * np2;
    const bool odd_end = (N & 1) && node == N;
    const int slot = even_n ? (node >> 1) - 1 : np2;
#pragma unroll
    for (int i = 0; i < NXA; ++i) dxo[i] = (even_n || odd_end) ? S->dxs[slot][i] : S->dx0[i];
    double pv[NXA];
    if constexpr (kWaves == 1) {
#pragma unroll
        for (int i = 0; i < NXA; ++i) pv[i] = from_prev(dxo[i]);
    } else {       // two waves: one exchange
        double xo[NXA];
#pragma unroll
        for (int i = 0; i < NXA; ++i) xo[i] = dxo[i];
        from_prev_n(xo, pv);
    }
    if ((node & 1) && node < 2 * np2) {
#pragma unroll
        for (int rr = 0; rr < NXA; ++rr) {
            const double* row = S->F[node - 1][rr];
            double s = row[NXA];
#pragma unroll
            for (int j = 0; j < NXA; ++j) s = fma(row[j], pv[j], s);
            dxo[rr] = s;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Scalar-input variant for two independent subsystems per wave (LMPC: the x and y halves of the
// separable 8-state model, lmpc_ipm.hip).  Half h = lane >> 5 owns node slots 32 h + k; z =
// [x~ (NXA); u; 1], ND = NXA + 2, so the packed G_k of one subsystem (NT = 28 at NXA = 5) fits a
// half-wave: lane 32 h + e owns entry e of its half.  Quu is a scalar; the Schur complement is
// G_k(i, j) = Ht_ij + a_i^T Gzz a_j - (a_i^T Gzu)(Guz a_j) / Quu, one LDS round trip per node.
template <int NXA_, int NMAXS_>
struct OcpLdsS {
    static constexpr int NXA = NXA_;          // augmented state dimension of one subsystem
    static constexpr int NP = NXA + 1;        // value-function dimension (with homogeneous 1)
    static constexpr int ND = NXA + 2;        // stage vector [x~; u; 1]
    static constexpr int NMAXS = NMAXS_;      // node slots per half (N + 1 <= NMAXS)
    static constexpr int NC = even(NP);       // padded column stride of M
    static constexpr int NT = tri(ND), NTP = even(NT);
    static constexpr int NF = even(NXA + 1);
    static_assert(NT <= 32, "one packed entry per half-wave lane");
    NodeArr<double[ND][NC], 2 * NMAXS> M;     // M[s][j][m] = M_k(m, j), slot s = NMAXS h + k
    NodeArr<double[NTP], 2 * NMAXS> H;        // stage Hessian + gradient row, packed
    NodeArr<double[NTP], 2 * NMAXS> G;        // G_k; G[N] = terminal surrogate (Pt_N, Quu = 1)
    NodeArr<double[NC], 2 * NMAXS> KK;        // [K | k]_k
    NodeArr<double[NXA][NF], 2 * NMAXS> F;    // closed loop rows [Phi_k(r, :) | f_k(r)]
    NodeArr<double[NXA][NF], NMAXS> F2;       // two-node maps, pair slot (NMAXS / 2) h + q (compose_pairs)
    double dx0[2][NC];                        // forward sweep start of each half
    double dxs[2][NMAXS / 2 + 1][NF];         // forward sweep of each half: dx~ of node 2q + 2 (slot q), odd node N
};

template <int NXA>
__host__ __device__ constexpr int zsi_of_p(int p) { return p < NXA ? p : NXA + 1; }
template <int NXA>
__host__ __device__ constexpr int gszz(int p, int q) { return hp(zsi_of_p<NXA>(p), zsi_of_p<NXA>(q)); }
template <int NXA>
__host__ __device__ constexpr int gszu(int p) { return hp(zsi_of_p<NXA>(p), NXA); }

struct RiccatiSRoles {
    int ci, cj;     // column offsets (j * NC) of a_i, a_j in M_k
    int e;          // packed entry of this lane in its half
    bool on;
};

template <class L>
__device__ RiccatiSRoles riccati_s_roles() {
    RiccatiSRoles r{};
    const int e0 = lane_id() & 31;
    r.on = e0 < L::NT;
    r.e = r.on ? e0 : 0;
    int i = 0;
    while (tri(i + 1) <= r.e) ++i;
    r.ci = i * L::NC; r.cj = (r.e - tri(i)) * L::NC;
    return r;
}

// Backward sweep of both halves over nodes N-1 .. 0; G[slot N] must hold each half's terminal
// surrogate.  Returns false (wave-uniform) if some Quu of either half is not positive.
// One node step of both halves (riccati_s_sweep): straight-line body, every lane active (lanes past NT
// recompute entry 0 and store the same value): the loads of H_k and M_k do not wait on G_{k+1}, and Quu's
// reciprocal is taken after the products, so one LDS latency per node stays on the chain.  Ends with a
// barrier.
template <class L>
__device__ __forceinline__ void s_node_step(L* S, int sk, const RiccatiSRoles& R, bool& ok) {
    constexpr int NXA = L::NXA, NP = L::NP;
    // every LDS read of the step issued before the first product (sched_barrier), the column of M_k that the
    // first products need first, then G_{k+1} -- whose reads follow the previous node's write in the wave's LDS
    // order (chain_sync) -- then the other column and the H entry: one LDS latency on the chain, where the
    // compiler's own schedule re-used registers across the G_{k+1} reads and waited out several
    const double* Mk = &S->M[sk][0][0];
    double vi[NP], vj[NP];
#pragma unroll
    for (int m = 0; m < NP; ++m) vj[m] = Mk[R.cj + m];
    __builtin_amdgcn_sched_barrier(0);
    const double* Gn = S->G[sk + 1];
    double gzz_[NP][NP], gzu_[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
#pragma unroll
        for (int m = 0; m <= n; ++m) gzz_[m][n] = Gn[gszz<NXA>(m, n)];
        gzu_[n] = Gn[gszu<NXA>(n)];
    }
    const double q = Gn[hp(NXA, NXA)];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < NP; ++m) vi[m] = Mk[R.ci + m];
    const double hk = S->H[sk][R.e];
    __builtin_amdgcn_sched_barrier(0);
    double t[NP], b = 0.0, c = 0.0;
#pragma unroll
    for (int m = 0; m < NP; ++m) t[m] = 0.0;
#pragma unroll
    for (int n = 0; n < NP; ++n) {
#pragma unroll
        for (int m = 0; m < NP; ++m) t[m] = fma(m <= n ? gzz_[m][n] : gzz_[n][m], vj[n], t[m]);
        b = fma(vi[n], gzu_[n], b);
        c = fma(vj[n], gzu_[n], c);
    }
    double ga = hk, gb = 0.0;
#pragma unroll
    for (int m = 0; m < NP; m += 2) {
        ga = fma(vi[m], t[m], ga);
        if (m + 1 < NP) gb = fma(vi[m + 1], t[m + 1], gb);
    }
    ok = ok && q > 0.0 && isfinite(q);
    const double g = (ga + gb) - b * c * frcp(q);
    // all reads of G_{k+1} and M_k precede the write of G_k (distinct slots: no hazard)
    S->G[sk][R.e] = g;
    chain_sync();
}

// Backward sweep of both halves over nodes N-1 .. 0; G[slot N] must hold each half's terminal
// surrogate.  Returns false (wave-uniform) if some Quu of either half is not positive.  Two nodes per
// loop trip: the second node's LDS addresses are immediate offsets of the first's (C5 +0.3 %,
// profiles/r04/node_unroll_ab.txt).
template <class L>
__device__ bool riccati_s_sweep(L* S, int N, const RiccatiSRoles& R) {
    constexpr int NXA = L::NXA;
    const int base = (lane_id() >> 5) * L::NMAXS;
    bool ok = true;
    int k = N - 1;
    for (; k >= 1; k -= 2) {
        s_node_step<L>(S, base + k, R, ok);
        s_node_step<L>(S, base + k - 1, R, ok);
    }
    if (k == 0) s_node_step<L>(S, base, R, ok);
    const double q0 = S->G[base][hp(NXA, NXA)];
    ok = ok && q0 > 0.0 && isfinite(q0);
    return !wany(!ok);
}

// The same backward sweep with the value function formed explicitly at every node (the order of IPOPT-style
// dense recursions and of the C oracle, oracle/lmpc_ipm.c riccati_factor): phase 1, lane e of each half forms the
// packed entry e of P_{k+1} = Gzz - Gzu Guz / Quu from G_{k+1} into Ps[h] (u entries: 0, Quu: 1), one barrier;
// phase 2, the node step on that surrogate.  Where the value function reaches ~1e18 (LMPC stress instances with
// an unstable open loop) the two orders can decide Quu's sign differently (profiles/r04/lmpc_riccati_probe_*.txt);
// the LMPC kernel takes this form when the folded one fails the inertia test at every perturbation.  Returns
// false (wave-uniform) if some Quu is not positive.
template <class L>
__device__ bool riccati_s_sweep_p(L* S, double (*Ps)[L::NTP], int N, const RiccatiSRoles& R) {
    constexpr int NXA = L::NXA;
    const int h = lane_id() >> 5, base = h * L::NMAXS;
    int zi = 0;
    while (tri(zi + 1) <= R.e) ++zi;
    const int zj = R.e - tri(zi);
    const bool uent = zi == NXA || zj == NXA;
    bool ok = true;
    for (int k = N - 1; k >= 0; --k) {
        const double* Gn = S->G[base + k + 1];
        const double q = Gn[hp(NXA, NXA)];
        ok = ok && q > 0.0 && isfinite(q);
        const double gi = Gn[hp(zi, NXA)], gj = Gn[hp(zj, NXA)];
        const double pv = Gn[R.e] - gi * gj / q;
        Ps[h][R.e] = uent ? ((zi == NXA && zj == NXA) ? 1.0 : 0.0) : pv;
        chain_sync();
        // node step on the surrogate (s_node_step with Gn = Ps[h]: Gzu = 0, Quu = 1)
        const double hk = S->H[base + k][R.e];
        const double* Mk = &S->M[base + k][0][0];
        constexpr int NP = L::NP;
        double vi[NP], vj[NP];
#pragma unroll
        for (int m = 0; m < NP; ++m) { vi[m] = Mk[R.ci + m]; vj[m] = Mk[R.cj + m]; }
        const double* P = Ps[h];
        double t[NP];
#pragma unroll
        for (int m = 0; m < NP; ++m) t[m] = 0.0;
#pragma unroll
        for (int n = 0; n < NP; ++n)
#pragma unroll
            for (int m = 0; m < NP; ++m) t[m] = fma(P[gszz<NXA>(m, n)], vj[n], t[m]);
        double g = hk;
#pragma unroll
        for (int m = 0; m < NP; ++m) g = fma(vi[m], t[m], g);
        S->G[base + k][R.e] = g;
        chain_sync();
    }
    const double q0 = S->G[base][hp(NXA, NXA)];
    ok = ok && q0 > 0.0 && isfinite(q0);
    return !wany(!ok);
}

// [K | k] = -Guz / Quu and [Phi | f] of every node, lane 32 h + k per node (k < N); post(slot, k) then
// runs on each node's lane before the pair maps are composed (the LMPC restoration phase maps the rows
// through its soft defect rows there).  Ends with a barrier.
template <class L, class Post = NoPost>
__device__ void closed_loop_s(L* S, int N, Post post = Post()) {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND;
    const int k = node_base() + (lane_id() & 31), sl = (lane_id() >> 5) * L::NMAXS + k;
    if (k < N) {
        // every LDS read before the first write (the compiler cannot prove F, KK and M disjoint and
        // would otherwise wait out each read before the next write)
        const double* Gk = S->G[sl];
        const double* Mk = &S->M[sl][0][0];
        double gu[NP], mk[NXA + 2][NXA];
#pragma unroll
        for (int p = 0; p < NP; ++p) gu[p] = Gk[gszu<NXA>(p)];
#pragma unroll
        for (int j = 0; j < NXA + 2; ++j)
#pragma unroll
            for (int r = 0; r < NXA; ++r) mk[j][r] = Mk[(j < NXA ? j : j == NXA ? NXA : ND - 1) * L::NC + r];
        const double iq = frcp(Gk[hp(NXA, NXA)]);
        double K[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) K[p] = -gu[p] * iq;
#pragma unroll
        for (int p = 0; p < NP; ++p) S->KK[sl][p] = K[p];
#pragma unroll
        for (int r = 0; r < NXA; ++r) {
            const double bq = mk[NXA][r];
#pragma unroll
            for (int j = 0; j < NXA; ++j) S->F[sl][r][j] = fma(bq, K[j], mk[j][r]);
            S->F[sl][r][NXA] = fma(bq, K[NXA], mk[NXA + 1][r]);
        }
        post(sl, k);
    }
    __syncthreads();
    compose_pairs<2, L::NMAXS, NXA, 3>(S->F, S->F2, N);   // 2 x 2 x N / 2 tasks: one round
}

// lam~ = -Pt_k [dx~; 1] (first NXA rows) with Pt_k [dx~; 1] = Gzz [dx~; 1] + Gzu du, read from G of slot sl
template <class L>
__device__ __forceinline__ void node_multiplier_s(const L* S, int sl, const double* dx, double du, double* lam) {
    constexpr int NXA = L::NXA, NP = L::NP;
    const double* Gk = S->G[sl];
#pragma unroll
    for (int p = 0; p < NXA; ++p) {
        double t = Gk[gszz<NXA>(p, NP - 1)];
#pragma unroll
        for (int q = 0; q < NXA; ++q) t = fma(Gk[gszz<NXA>(p, q)], dx[q], t);
        lam[p] = -fma(Gk[gszu<NXA>(p)], du, t);
    }
}

// Forward sweep of both halves over node pairs: lane 16 w + r (r < NXA) owns row r of the two-node
// chain dx~_{2q+2} = F2 [dx~_{2q}; 1] of half h = w / 2 (both rows of a half run it, so each row
// broadcasts the new state to itself by 64-bit DPP row_newbcast); the next pair's rows are loaded
// during the step and rows 0 / 2 park each new state in S->dxs (as forward_sweep).  An odd N ends with
// one single-node step; the odd nodes in between follow afterwards, lane per node, from their even
// predecessor.  Every lane returns in dxo the step of node `node` (= lane & 31) of its half.  Ends
// with a barrier.
template <class L, bool PREFETCH = true>
__device__ void forward_sweep_s(L* S, int N, int node, double* dxo) {
    constexpr int NXA = L::NXA;
    const int h = lane_id() >> 5, base = h * L::NMAXS, pbase = h * (L::NMAXS / 2);
    const int lr = lane_id() & 15;
    const int r = lr < NXA ? lr : 0;
    double d[NXA];
#pragma unroll
    for (int i = 0; i < NXA; ++i) d[i] = S->dx0[h][i];
    const int np2 = N >> 1;
    pair_chain<NXA, PREFETCH>(S->F2, pbase, np2, r, d, [&](int q) { return &S->dxs[h][q][r]; });
    if (N & 1) {
        const double* row = S->F[base + N - 1][r];
        double s = row[NXA];
#pragma unroll
        for (int j = 0; j < NXA; ++j) s = fma(row[j], d[j], s);
        S->dxs[h][np2][r] = s;
    }
    __syncthreads();
    const bool even_n = !(node & 1) && node >= 2 && node <= 2 * np2;
    const bool odd_end = (N & 1) && node == N;
    const int slot = even_n ? (node >> 1) - 1 : np2;
#pragma unroll
    for (int i = 0; i < NXA; ++i) dxo[i] = (even_n || odd_end) ? S->dxs[h][slot][i] : S->dx0[h][i];
    double pv[NXA];
    if constexpr (kWaves == 1) {
#pragma unroll
        for (int i = 0; i < NXA; ++i) pv[i] = from_prev(dxo[i]);
    } else {       // two waves: one exchange
        double xo[NXA];
#pragma unroll
        for (int i = 0; i < NXA; ++i) xo[i] = dxo[i];
        from_prev_n(xo, pv);
    }
    if ((node & 1) && node < 2 * np2) {
#pragma unroll
        for (int rr = 0; rr < NXA; ++rr) {
            const double* row = S->F[base + node - 1][rr];
            double s = row[NXA];
#pragma unroll
            for (int j = 0; j < NXA; ++j) s = fma(row[j], pv[j], s);
            dxo[rr] = s;
        }
    }
}

}  // namespace dartmpc
