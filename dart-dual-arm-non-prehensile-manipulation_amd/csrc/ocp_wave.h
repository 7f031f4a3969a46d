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
// One LDS round trip per node: lane e owns packed entry (i, j) of G_k and forms it from the
// columns a_i, a_j of M_k (lane-private reads) and all of G_{k+1} (broadcast reads), with the
// Schur complement that defines Pt_{k+1} folded into the bilinear form.  The gains [K | k] and
// the multipliers are recovered from the stored G_k afterwards, lane per node, in parallel.
//
// The forward sweep dx~_{k+1} = Phi_k dx~_k + f_k (Phi = A + B K, f = c + B k, formed for all
// nodes in parallel, lane per node) runs redundantly in every lane: no exchange on the chain.
#pragma once
#include <hip/hip_runtime.h>

#include "wave.h"

namespace dartmpc {

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
    static constexpr int EPL = (NT + 63) / 64;     // packed entries of G per lane
    NodeArr<double[ND][NC], NMAXS> M;         // M[k][j][m] = M_k(m, j): column j of M_k
    NodeArr<double[NTP], NMAXS> H;            // stage Hessian + gradient, packed symmetric
    NodeArr<double[NTP], NMAXS> G;            // G_k; G[N] = terminal surrogate (Pt_N, Quu = I)
    NodeArr<double[2][NC], NMAXS> KK;         // [K | k]_k rows
    NodeArr<double[NXA][NF], NMAXS> F;        // closed loop: F[k][r] = [Phi_k(r, :) | f_k(r)]
    double dx0[NC];                           // forward sweep start dx~_0
};

// z index of value-function index p (the homogeneous coordinate sits last in both)
template <int NXA>
__host__ __device__ constexpr int zi_of_p(int p) { return p < NXA ? p : NXA + 2; }

// packed G offsets of the value-space block (p, q), the (p, u_a) block and Quu
template <int NXA>
__host__ __device__ constexpr int gzz(int p, int q) { return hp(zi_of_p<NXA>(p), zi_of_p<NXA>(q)); }
template <int NXA>
__host__ __device__ constexpr int gzu(int p, int a) { return hp(zi_of_p<NXA>(p), NXA + a); }

// Per-lane roles of the backward sweep (packed entries e = lane + 64 r of G), decoded once.
template <int EPL>
struct RiccatiRoles {
    int ci[EPL], cj[EPL];   // column offsets (j * NC) of a_i, a_j in M_k
    bool on[EPL];           // lane owns entry r
};

template <class L>
__device__ RiccatiRoles<L::EPL> riccati_roles() {
    constexpr int NT = L::NT, NC = L::NC;
    const int lane = threadIdx.x;
    RiccatiRoles<L::EPL> r{};
#pragma unroll
    for (int q = 0; q < L::EPL; ++q) {
        const int e0 = lane + 64 * q;
        const int e = e0 < NT ? e0 : 0;
        int i = 0;
        while (tri(i + 1) <= e) ++i;
        const int j = e - tri(i);
        r.ci[q] = i * NC; r.cj[q] = j * NC;
        r.on[q] = e0 < NT;
    }
    return r;
}

// Quu of a packed G, its positive-definiteness and its inverse (wave-uniform values)
template <int NXA>
__device__ __forceinline__ bool quu_inverse(const double* Gk, double& i00, double& i01, double& i11) {
    const double g00 = Gk[hp(NXA, NXA)], g01 = Gk[hp(NXA + 1, NXA)], g11 = Gk[hp(NXA + 1, NXA + 1)];
    const double det = g00 * g11 - g01 * g01;
    const double idet = frcp(det);
    i00 = g11 * idet; i01 = -g01 * idet; i11 = g00 * idet;
    return (g00 > 0.0) && (det > 0.0) && isfinite(det);
}

// Backward Riccati sweep over nodes N-1 .. 0, one LDS round trip per node.  With
// Pt_{k+1} = Gzz - Gzu Quu^-1 Guz (the Schur complement of G_{k+1}) folded in,
//   G_k(i, j) = Ht_ij + a_i^T Gzz a_j - (a_i^T Gzu) Quu^-1 (Guz a_j),
// lane e owning packed entry (i, j).  G[N] must hold the terminal surrogate.  Returns false
// (wave-uniform) if some Quu is not positive definite (inertia correction needed).
template <class L>
__device__ bool riccati_sweep(L* S, int N, const RiccatiRoles<L::EPL>& R) {
    constexpr int NXA = L::NXA, NP = L::NP;
    const int lane = threadIdx.x;
    bool ok = true;
    for (int k = N - 1; k >= 0; --k) {
        const double* Gn = S->G[k + 1];
        double i00, i01, i11;
        ok = quu_inverse<NXA>(Gn, i00, i01, i11) && ok;
        double gout[L::EPL];
#pragma unroll
        for (int q = 0; q < L::EPL; ++q) {
            if (!R.on[q]) continue;
            const double* ai = &S->M[k][0][0] + R.ci[q];
            const double* aj = &S->M[k][0][0] + R.cj[q];
            double vi[NP], vj[NP];
#pragma unroll
            for (int m = 0; m < NP; ++m) { vi[m] = ai[m]; vj[m] = aj[m]; }
            // NP + 4 independent accumulators updated round-robin: dependency distance NP + 4
            double t[NP];
            double b0 = 0.0, b1 = 0.0, c0 = 0.0, c1 = 0.0;
#pragma unroll
            for (int m = 0; m < NP; ++m) t[m] = 0.0;
#pragma unroll
            for (int n = 0; n < NP; ++n) {
#pragma unroll
                for (int m = 0; m < NP; ++m) t[m] = fma(Gn[gzz<NXA>(m, n)], vj[n], t[m]);
                b0 = fma(vi[n], Gn[gzu<NXA>(n, 0)], b0);
                b1 = fma(vi[n], Gn[gzu<NXA>(n, 1)], b1);
                c0 = fma(vj[n], Gn[gzu<NXA>(n, 0)], c0);
                c1 = fma(vj[n], Gn[gzu<NXA>(n, 1)], c1);
            }
            double ga = S->H[k][lane + 64 * q], gb = 0.0;
#pragma unroll
            for (int m = 0; m < NP; m += 2) {
                ga = fma(vi[m], t[m], ga);
                if (m + 1 < NP) gb = fma(vi[m + 1], t[m + 1], gb);
            }
            const double w0 = fma(i00, c0, i01 * c1), w1 = fma(i01, c0, i11 * c1);
            gout[q] = (ga + gb) - fma(b0, w0, b1 * w1);
        }
        // all reads of G_{k+1} and M_k precede the writes of G_k (distinct rows: no hazard)
#pragma unroll
        for (int q = 0; q < L::EPL; ++q)
            if (R.on[q]) S->G[k][lane + 64 * q] = gout[q];
        __syncthreads();
    }
    double i00, i01, i11;
    return quu_inverse<NXA>(S->G[0], i00, i01, i11) && ok;
}

// Gains and closed-loop matrices for the forward sweep, lane per node (lanes 0..N-1):
// [K | k] = -Quu^-1 Guz, Phi_k = A_k + B_k K_k, f_k = c_k + B_k k_k.  Ends with a barrier.
template <class L>
__device__ void closed_loop(L* S, int N) {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND;
    const int k = threadIdx.x;
    if (k < N) {
        const double* Gk = S->G[k];
        double i00, i01, i11;
        quu_inverse<NXA>(Gk, i00, i01, i11);
        double K0[NP], K1[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const double c0 = Gk[gzu<NXA>(p, 0)], c1 = Gk[gzu<NXA>(p, 1)];
            K0[p] = -fma(i00, c0, i01 * c1);
            K1[p] = -fma(i01, c0, i11 * c1);
            S->KK[k][0][p] = K0[p];
            S->KK[k][1][p] = K1[p];
        }
#pragma unroll
        for (int r = 0; r < NXA; ++r) {
            const double b0 = S->M[k][NXA][r], b1 = S->M[k][NXA + 1][r];
#pragma unroll
            for (int j = 0; j < NXA; ++j) S->F[k][r][j] = fma(b0, K0[j], fma(b1, K1[j], S->M[k][j][r]));
            S->F[k][r][NXA] = fma(b0, K0[NXA], fma(b1, K1[NXA], S->M[k][ND - 1][r]));
        }
    }
    __syncthreads();
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

// Forward sweep: lane r < NXA owns row r of the chain dx~_{k+1} = Phi_k dx~_k + f_k; the new
// state is broadcast to every lane by readlane (scalar registers), and row r's closed-loop data
// for node k+1 is prefetched while node k is processed.  Every lane returns in dxo the state step
// of node `node` (lane-per-node use; node > N keeps dx~_0).  S->dx0 must hold dx~_0.
template <class L>
__device__ void forward_sweep(L* S, int N, int node, double* dxo) {
    constexpr int NXA = L::NXA;
    const int lane = threadIdx.x;
    const int r = lane < NXA ? lane : 0;
    double d[NXA];
#pragma unroll
    for (int i = 0; i < NXA; ++i) { d[i] = S->dx0[i]; dxo[i] = d[i]; }
    double Fc[NXA + 1];
#pragma unroll
    for (int j = 0; j <= NXA; ++j) Fc[j] = S->F[0][r][j];
    for (int k = 0; k < N; ++k) {
        double Fn[NXA + 1];
        const int kn = k + 1 < N ? k + 1 : k;
#pragma unroll
        for (int j = 0; j <= NXA; ++j) Fn[j] = S->F[kn][r][j];
        double s = Fc[NXA];
#pragma unroll
        for (int j = 0; j < NXA; ++j) s = fma(Fc[j], d[j], s);
        const bool mine = node == k + 1;
#pragma unroll
        for (int i = 0; i < NXA; ++i) { d[i] = readlane(s, i); dxo[i] = mine ? d[i] : dxo[i]; }
#pragma unroll
        for (int j = 0; j <= NXA; ++j) Fc[j] = Fn[j];
    }
}

// ------------------------------------------------------------------------------------------
// Three-phase variant with an explicit value function, for wide augmented states (LMPC,
// NXA = 10): per node (A) T = Pt_{k+1} M_k (NP x ND entries, 11 FMA each), (B) G = Ht + M^T T
// (packed, 11 FMA each), (C) the 2 x 2 Schur complement -> Pt_k (packed) and [K | k].  Each
// lane holds only the operands of its own few entries (no uniform block in registers).
template <int NXA_, int NMAXS_>
struct OcpLds3 {
    static constexpr int NXA = NXA_, NP = NXA + 1, ND = NXA + 3, NMAXS = NMAXS_;
    static constexpr int NC = even(NP);
    static constexpr int NT = tri(ND), NTP = even(NT);
    static constexpr int NPT = tri(NP);
    static constexpr int NPK = even(NPT + 2 * NP);   // [Pt packed | K row 0 | K row 1] per node
    static constexpr int NF = even(NXA + 1);
    static constexpr int NTT = NP * ND;               // entries of T
    static constexpr int EA = (NTT + 63) / 64, EB = (NT + 63) / 64, EC = (NPT + 2 * NP + 63) / 64;
    double M[NMAXS][ND][NC];
    double H[NMAXS][NTP];
    double PK[NMAXS][NPK];
    static constexpr int NPF = even(NP);              // row stride of the full copy of Pt_{k+1}
    double T[ND][NP + 1];                             // scratch Pt_{k+1} M_k, transposed: T[j][m]
    double PF[NP][NPF];                               // scratch Pt_{k+1}, full rows (16-byte aligned)
    double G[NTP];                                    // scratch G_k
    double F[NMAXS][NXA][NF];
    double dx0[NC];
};

template <class L>
struct Riccati3Roles {
    int am[L::EA], aj[L::EA];            // (A) row m of Pt, column offset of a_j
    bool aon[L::EA];
    int bi[L::EB], bj[L::EB];            // (B) column offsets of a_i, T column j
    bool bon[L::EB];
    int ga0[L::EC], ga1[L::EC], gb0[L::EC], gb1[L::EC], gzz[L::EC];   // (C) packed G offsets
    bool isK[L::EC], con[L::EC];
    int ka[L::EC];
    int fpq[L::EC], fqp[L::EC];          // (C) offsets (p, q) and (q, p) of a value entry in the full copy
};

template <class L>
__device__ Riccati3Roles<L> riccati3_roles() {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND, NC = L::NC, NT = L::NT, NPT = L::NPT, NTT = L::NTT;
    const int lane = threadIdx.x;
    Riccati3Roles<L> r{};
#pragma unroll
    for (int q = 0; q < L::EA; ++q) {
        const int e0 = lane + 64 * q, e = e0 < NTT ? e0 : 0;
        r.am[q] = e / ND; r.aj[q] = (e % ND) * NC; r.aon[q] = e0 < NTT;
    }
#pragma unroll
    for (int q = 0; q < L::EB; ++q) {
        const int e0 = lane + 64 * q, e = e0 < NT ? e0 : 0;
        int i = 0;
        while (tri(i + 1) <= e) ++i;
        const int j = e - tri(i);
        r.bi[q] = i * NC; r.bj[q] = j; r.bon[q] = e0 < NT;
    }
#pragma unroll
    for (int q = 0; q < L::EC; ++q) {
        const int e = lane + 64 * q;
        int zi = 0, zj = 0;
        r.isK[q] = e >= NPT;
        r.ka[q] = 0;
        r.fpq[q] = 0; r.fqp[q] = 0;
        if (e < NPT) {
            int p = 0;
            while (tri(p + 1) <= e) ++p;
            const int qq = e - tri(p);
            zi = zi_of_p<NXA>(p); zj = zi_of_p<NXA>(qq);
            r.fpq[q] = p * L::NPF + qq; r.fqp[q] = qq * L::NPF + p;
        } else {
            const int rr = (e - NPT) < 2 * NP ? e - NPT : 0;
            r.ka[q] = rr / NP;
            zi = zi_of_p<NXA>(rr % NP); zj = zi;
        }
        r.ga0[q] = hp(zi, NXA); r.ga1[q] = hp(zi, NXA + 1);
        r.gb0[q] = hp(NXA, zj); r.gb1[q] = hp(NXA + 1, zj);
        r.gzz[q] = hp(zi, zj);
        r.con[q] = e < NPT + 2 * NP;
    }
    return r;
}

// Backward sweep; PK[N] (value part) must hold the terminal value function.
template <class L>
__device__ bool riccati3_sweep(L* S, int N, const Riccati3Roles<L>& R) {
    constexpr int NXA = L::NXA, NP = L::NP, NPT = L::NPT;
    const int lane = threadIdx.x;
    bool ok = true;
    {   // full copy of the terminal value function
        const int i = lane / NP, j = lane % NP;
        for (int e = lane; e < NP * NP; e += 64) {
            const int ii = e / NP, jj = e % NP;
            S->PF[ii][jj] = S->PK[N][ii >= jj ? tri(ii) + jj : tri(jj) + ii];
        }
        (void)i; (void)j;
    }
    __syncthreads();
    for (int k = N - 1; k >= 0; --k) {
        // (A) T(m, j) = sum_n Pt_{k+1}(m, n) M_k(n, j): row m of the full copy and column j of M_k are
        // both contiguous (16-byte aligned), stored transposed for (B)
        {
            double tv[L::EA];
#pragma unroll
            for (int q = 0; q < L::EA; ++q) {
                const double* aj = &S->M[k][0][0] + R.aj[q];
                const double* pm = S->PF[R.am[q]];
                double t = 0.0;
#pragma unroll
                for (int n = 0; n < NP; ++n) t = fma(pm[n], aj[n], t);
                tv[q] = t;
            }
#pragma unroll
            for (int q = 0; q < L::EA; ++q)
                if (R.aon[q]) S->T[(lane + 64 * q) % L::ND][(lane + 64 * q) / L::ND] = tv[q];
        }
        __syncthreads();
        // (B) G(i, j) = Ht(i, j) + sum_m M_k(m, i) T(m, j)
        {
            double gv[L::EB];
#pragma unroll
            for (int q = 0; q < L::EB; ++q) {
                const double* ai = &S->M[k][0][0] + R.bi[q];
                const double* tj = S->T[R.bj[q]];
                double g = S->H[k][(lane + 64 * q) < L::NT ? lane + 64 * q : 0];
#pragma unroll
                for (int mm = 0; mm < NP; ++mm) g = fma(ai[mm], tj[mm], g);
                gv[q] = g;
            }
#pragma unroll
            for (int q = 0; q < L::EB; ++q)
                if (R.bon[q]) S->G[lane + 64 * q] = gv[q];
        }
        __syncthreads();
        // (C) Schur complement on the u block -> packed Pt_k, gains, and the full copy for node k-1
        double i00, i01, i11;
        ok = quu_inverse<NXA>(S->G, i00, i01, i11) && ok;
        {
            double cv[L::EC];
#pragma unroll
            for (int q = 0; q < L::EC; ++q) {
                const double b0 = S->G[R.gb0[q]], b1 = S->G[R.gb1[q]];
                const double w0 = fma(i00, b0, i01 * b1), w1 = fma(i01, b0, i11 * b1);
                const double a0 = S->G[R.ga0[q]], a1 = S->G[R.ga1[q]], gz = S->G[R.gzz[q]];
                const double pv = gz - fma(a0, w0, a1 * w1);
                const double kv = R.ka[q] == 0 ? -w0 : -w1;
                cv[q] = R.isK[q] ? kv : pv;
            }
#pragma unroll
            for (int q = 0; q < L::EC; ++q) {
                if (R.con[q]) S->PK[k][lane + 64 * q] = cv[q];
                if (R.con[q] && !R.isK[q]) {
                    (&S->PF[0][0])[R.fpq[q]] = cv[q];
                    (&S->PF[0][0])[R.fqp[q]] = cv[q];
                }
            }
        }
        __syncthreads();
    }
    (void)NPT;
    return ok;
}

// [Phi | f] of every node from the stored gains, lane per node.  Ends with a barrier.
template <class L>
__device__ void closed_loop3(L* S, int N) {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND, NPT = L::NPT;
    const int k = threadIdx.x;
    if (k < N) {
        const double* K0 = S->PK[k] + NPT;
        const double* K1 = K0 + NP;
#pragma unroll
        for (int r = 0; r < NXA; ++r) {
            const double b0 = S->M[k][NXA][r], b1 = S->M[k][NXA + 1][r];
#pragma unroll
            for (int j = 0; j < NXA; ++j) S->F[k][r][j] = fma(b0, K0[j], fma(b1, K1[j], S->M[k][j][r]));
            S->F[k][r][NXA] = fma(b0, K0[NXA], fma(b1, K1[NXA], S->M[k][ND - 1][r]));
        }
    }
    __syncthreads();
}

// lam~_k = -Pt_k [dx~; 1] (first NXA rows), lane per node
template <class L>
__device__ __forceinline__ void node_multiplier3(const L* S, int k, const double* dx, double* lam) {
    constexpr int NXA = L::NXA;
    const double* Pk = S->PK[k];
#pragma unroll
    for (int p = 0; p < NXA; ++p) {
        double t = Pk[hp(NXA, p)];
#pragma unroll
        for (int q = 0; q < NXA; ++q) t = fma(Pk[hp(p, q)], dx[q], t);
        lam[p] = -t;
    }
}

}  // namespace dartmpc
