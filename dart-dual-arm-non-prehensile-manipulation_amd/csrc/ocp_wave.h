// ocp_wave.h -- one-wave, LDS-staged Riccati engine for small dense optimal-control QPs (gfx950).
//
// Used by the coupled-model solvers (RMPC, later LMPC), whose stage blocks are too large for the
// lane-per-node register recursion of the PMPC kernel.  One wave64 owns one instance; the stage
// data of all nodes sit in LDS; the backward Riccati sweep runs over the nodes in sequence and
// the 64 lanes share each node's dense linear algebra ("lanes as matrix entries"):
//
//   z = [x~ (NXA) ; u (2) ; 1]                      homogeneous stage vector, ND = NXA + 3
//   x~+ = M z,  M = [[A B c]; [0 0 1]]  (NP x ND)   linearised dynamics incl. the defect c
//   V(x~) = 1/2 [x~;1]^T Pt [x~;1]                  value function, NP = NXA + 1
//   G = M^T Pt M + Ht                               stage QP incl. gradient (last row/column)
//   Pt' = Schur complement of G on the u block      ->  gains K (2 x NXA), feed-forward k (2)
//
// Three lane-parallel products per node (Y = Pt M, G = M^T Y + Ht, Schur), each one LDS round trip.
#pragma once
#include <hip/hip_runtime.h>

namespace dartmpc {

__host__ __device__ constexpr int tri(int n) { return n * (n + 1) / 2; }
__device__ __forceinline__ int hp(int i, int j) { return i >= j ? tri(i) + j : tri(j) + i; }

template <int NXA_, int NMAXS_>
struct OcpLds {
    static constexpr int NXA = NXA_;          // augmented state dimension
    static constexpr int NP = NXA + 1;        // value-function dimension (with homogeneous 1)
    static constexpr int ND = NXA + 3;        // stage vector dimension [x~; u; 1]
    static constexpr int NMAXS = NMAXS_;      // max shooting nodes (N + 1)
    double M[NMAXS][ND][NP];                  // M columns: M[k][j][m] = M_k(m, j)
    double H[NMAXS][tri(ND)];                 // stage Hessian + gradient, packed symmetric
    double P[NMAXS][tri(NP)];                 // value functions Pt_k, packed symmetric
    double K[NMAXS][2][NP];                   // [K | k] per node (row a, column p; p = NXA is k)
    double Y[NP][ND];                         // scratch: Pt_{k+1} M_k
    double G[tri(ND)];                        // scratch: G_k
    double dz[NMAXS][ND];                     // forward sweep: [dx~_k ; du_k ; 1]
};

// z index of value-function index p (the homogeneous coordinate sits last in both)
template <int NXA>
__device__ __forceinline__ int zi_of_p(int p) { return p < NXA ? p : NXA + 2; }

// Backward Riccati sweep over nodes N-1 .. 0.  L->P[N] must hold the terminal value function.
// Returns false (wave-uniform) if some Quu is not positive definite (inertia correction needed).
template <class L>
__device__ bool riccati_sweep(L* S, int N) {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND;
    const int lane = threadIdx.x;
    bool ok = true;
    for (int k = N - 1; k >= 0; --k) {
        // (A) Y = Pt_{k+1} M_k : NP x ND entries
        for (int e = lane; e < NP * ND; e += 64) {
            const int m = e / ND, j = e % ND;
            double s = 0.0;
#pragma unroll
            for (int l = 0; l < NP; ++l) s = fma(S->P[k + 1][hp(m, l)], S->M[k][j][l], s);
            S->Y[m][j] = s;
        }
        __syncthreads();
        // (B) G = M^T Y + Ht (packed lower triangle)
        for (int e = lane; e < tri(ND); e += 64) {
            int i = 0;
            while (tri(i + 1) <= e) ++i;
            const int j = e - tri(i);
            double s = S->H[k][e];
#pragma unroll
            for (int m = 0; m < NP; ++m) s = fma(S->M[k][i][m], S->Y[m][j], s);
            S->G[e] = s;
        }
        __syncthreads();
        // (C) Schur complement on the u block (z indices NXA, NXA+1)
        const double g00 = S->G[hp(NXA, NXA)], g01 = S->G[hp(NXA, NXA + 1)], g11 = S->G[hp(NXA + 1, NXA + 1)];
        const double det = g00 * g11 - g01 * g01;
        ok = ok && (g00 > 0.0) && (det > 0.0) && isfinite(det);
        const double idet = 1.0 / det;
        const double i00 = g11 * idet, i01 = -g01 * idet, i11 = g00 * idet;
        for (int e = lane; e < tri(NP) + 2 * NP; e += 64) {
            if (e < tri(NP)) {
                int p = 0;
                while (tri(p + 1) <= e) ++p;
                const int q = e - tri(p);
                const int zi = zi_of_p<NXA>(p), zj = zi_of_p<NXA>(q);
                const double a0 = S->G[hp(zi, NXA)], a1 = S->G[hp(zi, NXA + 1)];
                const double b0 = S->G[hp(NXA, zj)], b1 = S->G[hp(NXA + 1, zj)];
                const double w0 = fma(i00, b0, i01 * b1), w1 = fma(i01, b0, i11 * b1);
                S->P[k][e] = S->G[hp(zi, zj)] - fma(a0, w0, a1 * w1);
            } else {
                const int r = e - tri(NP), a = r / NP, p = r % NP;
                const int zj = zi_of_p<NXA>(p);
                const double b0 = S->G[hp(NXA, zj)], b1 = S->G[hp(NXA + 1, zj)];
                S->K[k][a][p] = a == 0 ? -fma(i00, b0, i01 * b1) : -fma(i01, b0, i11 * b1);
            }
        }
        __syncthreads();
    }
    return ok;
}

// Forward sweep dx~_{k+1} = M_k [dx~_k; du_k; 1], du_k = K_k dx~_k + k_k.  L->dz[0][0..NXA) must hold
// dx~_0 on entry; fills dz[k] = [dx~_k; du_k; 1] for k = 0..N (du_N = 0).
template <class L>
__device__ void forward_sweep(L* S, int N) {
    constexpr int NXA = L::NXA, NP = L::NP, ND = L::ND;
    const int lane = threadIdx.x;
    for (int k = 0; k < N; ++k) {
        double du0 = S->K[k][0][NXA], du1 = S->K[k][1][NXA];
#pragma unroll
        for (int j = 0; j < NXA; ++j) {
            const double d = S->dz[k][j];
            du0 = fma(S->K[k][0][j], d, du0);
            du1 = fma(S->K[k][1][j], d, du1);
        }
        if (lane < NXA) {
            double s = S->M[k][ND - 1][lane];                 // c_k
#pragma unroll
            for (int j = 0; j < NXA; ++j) s = fma(S->M[k][j][lane], S->dz[k][j], s);
            s = fma(S->M[k][NXA][lane], du0, s);
            s = fma(S->M[k][NXA + 1][lane], du1, s);
            S->dz[k + 1][lane] = s;
        } else if (lane == NXA) {
            S->dz[k][NXA] = du0;
            S->dz[k][NXA + 1] = du1;
            S->dz[k][NXA + 2] = 1.0;
        }
        __syncthreads();
    }
    if (lane == 0) { S->dz[N][NXA] = 0.0; S->dz[N][NXA + 1] = 0.0; S->dz[N][NXA + 2] = 1.0; }
    __syncthreads();
    (void)NP;
}

}  // namespace dartmpc
