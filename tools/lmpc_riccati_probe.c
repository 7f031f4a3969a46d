/* Diagnostic (CPU): at iteration 0 of an LMPC oracle solve, the Riccati recursion three ways for a list of
 * inertia shifts delta -- the oracle's full-matrix form (P_{k+1} formed, then Quu = R + B^T P B), the kernel's
 * lanes-as-entries form (ocp_wave.h riccati_s_sweep: G_k(i, j) = H + a_i^T Gzz a_j - (a_i^T g)(g^T a_j) / q
 * from the pre-Schur G_{k+1}), and the kernel form with the Schur complement of G_{k+1} taken entrywise first
 * -- printing the nodes where Quu loses its sign.  Build: make -C oracle probe; input: tools/lmpc_riccati_probe.py. */
#include <stdio.h>
#define ORACLE_RICCATI_PROBE 1
#include "../oracle/lmpc_ipm.c"

enum { PV = NA + 1, PZ = NA + 3 };     /* value indices [x~; 1], stage indices [x~; u; 1] */
static int zi(int p) { return p < NA ? p : NA + 2; }

static void riccati_probe(const ctx_t *C, work_t *W) {
    const int N = C->P->N;
    const double deltas[] = {0.0, 1e-4, 1e-2, 1.0, 1e2, 1e4, 1e8, 1e16, 1e24};
    static double G[NMAX + 1][PZ][PZ];
    for (unsigned di = 0; di < sizeof deltas / sizeof deltas[0]; ++di) {
        const double delta = deltas[di];
        for (int form = 0; form < 4; ++form) {
            int first_bad = -1;
            double qbad = 0.0, maxg = 0.0;
            if (form == 3) {
                /* the exact recursion (quad precision) on the same stage data */
                typedef __float128 Q;
                static Q Pq[NMAX + 1][NA][NA];
                double pn[NA], Pn[NA][NA];
                terminal_qp(C, W, delta, Pn, pn);
                for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) Pq[N][i][j] = Pn[i][j];
                for (int k = N - 1; k >= 0; --k) {
                    double Hq[NZ][NZ], gq[NZ];
                    stage_qp(C, W, k, delta, Hq, gq);
                    Q PA[NA][NA], PB[NA][NU], Quu[NU][NU], Qxx[NA][NA], Qux[NU][NA];
                    for (int i = 0; i < NA; ++i) {
                        for (int j = 0; j < NA; ++j) { Q t = 0; for (int m = 0; m < NA; ++m) t += Pq[k + 1][i][m] * (Q)W->A[k][m][j]; PA[i][j] = t; }
                        for (int j = 0; j < NU; ++j) { Q t = 0; for (int m = 0; m < NA; ++m) t += Pq[k + 1][i][m] * (Q)W->Bm[k][m][j]; PB[i][j] = t; }
                    }
                    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) {
                        Q t = Hq[i][j]; for (int m = 0; m < NA; ++m) t += (Q)W->A[k][m][i] * PA[m][j]; Qxx[i][j] = t;
                    }
                    for (int a = 0; a < NU; ++a) {
                        for (int i = 0; i < NA; ++i) { Q t = Hq[NA + a][i]; for (int m = 0; m < NA; ++m) t += (Q)W->Bm[k][m][a] * PA[m][i]; Qux[a][i] = t; }
                        for (int b = 0; b < NU; ++b) { Q t = Hq[NA + a][NA + b]; for (int m = 0; m < NA; ++m) t += (Q)W->Bm[k][m][a] * PB[m][b]; Quu[a][b] = t; }
                    }
                    const Q det = Quu[0][0] * Quu[1][1] - Quu[0][1] * Quu[1][0];
                    if (di == 0 && k >= N - 8) printf("    node %2d Quu %.6e %.6e %.6e (quad)\n", k, (double)Quu[0][0], (double)Quu[0][1], (double)Quu[1][1]);
                    if (!(Quu[0][0] > 0 && det > 0)) { first_bad = k; qbad = (double)Quu[0][0]; break; }
                    const Q i00 = Quu[1][1] / det, i01 = -Quu[0][1] / det, i11 = Quu[0][0] / det;
                    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) {
                        const Q k0 = -(i00 * Qux[0][j] + i01 * Qux[1][j]), k1 = -(i01 * Qux[0][j] + i11 * Qux[1][j]);
                        Pq[k][i][j] = Qxx[i][j] + Qux[0][i] * k0 + Qux[1][i] * k1;
                        maxg = fmax(maxg, fabs((double)Pq[k][i][j]));
                    }
                }
            } else if (form == 0) {
                /* the oracle's recursion, Quu per node */
                double pn[NA];
                terminal_qp(C, W, delta, W->Pm[N], pn);
                for (int k = N - 1; k >= 0; --k) {
                    double Hq[NZ][NZ], gq[NZ];
                    stage_qp(C, W, k, delta, Hq, gq);
                    double (*A)[NA] = W->A[k], (*Bm)[NU] = W->Bm[k], (*Pp)[NA] = W->Pm[k + 1];
                    double PA[NA][NA], PB[NA][NU], Quu[NU][NU], Qxx[NA][NA], Lq[3];
                    for (int i = 0; i < NA; ++i) {
                        for (int j = 0; j < NA; ++j) { double s = 0; for (int m = 0; m < NA; ++m) s += Pp[i][m] * A[m][j]; PA[i][j] = s; }
                        for (int j = 0; j < NU; ++j) { double s = 0; for (int m = 0; m < NA; ++m) s += Pp[i][m] * Bm[m][j]; PB[i][j] = s; }
                    }
                    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j) {
                        double s = Hq[i][j]; for (int m = 0; m < NA; ++m) s += A[m][i] * PA[m][j]; Qxx[i][j] = s;
                        maxg = fmax(maxg, fabs(s));
                    }
                    double Qux[NU][NA], K[NU][NA];
                    for (int a = 0; a < NU; ++a) {
                        for (int i = 0; i < NA; ++i) { double s = Hq[NA + a][i]; for (int m = 0; m < NA; ++m) s += Bm[m][a] * PA[m][i]; Qux[a][i] = s; }
                        for (int b = 0; b < NU; ++b) { double s = Hq[NA + a][NA + b]; for (int m = 0; m < NA; ++m) s += Bm[m][a] * PB[m][b]; Quu[a][b] = s; }
                    }
                    if (di == 0 && k >= N - 8) printf("    node %2d Quu %.6e %.6e %.6e\n", k, Quu[0][0], Quu[0][1], Quu[1][1]);
                    if (!chol2(Quu[0][0], 0.5 * (Quu[0][1] + Quu[1][0]), Quu[1][1], Lq)) {
                        if (first_bad < 0) { first_bad = k; qbad = fmin(Quu[0][0], Quu[1][1]); }
                        break;
                    }
                    for (int i = 0; i < NA; ++i) {
                        double b2[2] = {Qux[0][i], Qux[1][i]}, x2[2];
                        chol2_solve(Lq, b2, x2); K[0][i] = -x2[0]; K[1][i] = -x2[1];
                    }
                    for (int i = 0; i < NA; ++i) for (int j = 0; j < NA; ++j)
                        W->Pm[k][i][j] = Qxx[i][j] + Qux[0][i] * K[0][j] + Qux[1][i] * K[1][j];
                    for (int i = 0; i < NA; ++i) for (int j = 0; j < i; ++j) { double s = 0.5 * (W->Pm[k][i][j] + W->Pm[k][j][i]); W->Pm[k][i][j] = W->Pm[k][j][i] = s; }
                }
            } else {
                /* the kernel's forms over the pre-Schur G */
                double pn[NA], Pn[NA][NA];
                terminal_qp(C, W, delta, Pn, pn);
                memset(G[N], 0, sizeof G[N]);
                for (int i = 0; i < NA; ++i) {
                    for (int j = 0; j < NA; ++j) G[N][i][j] = Pn[i][j];
                    G[N][i][NA + 2] = G[N][NA + 2][i] = pn[i];
                }
                G[N][NA][NA] = G[N][NA + 1][NA + 1] = 1.0;
                for (int k = N - 1; k >= 0; --k) {
                    double Hq[NZ][NZ], gq[NZ], H[PZ][PZ], M[PV][PZ];
                    stage_qp(C, W, k, delta, Hq, gq);
                    memset(H, 0, sizeof H); memset(M, 0, sizeof M);
                    for (int a = 0; a < NZ; ++a) { for (int b = 0; b < NZ; ++b) H[a][b] = Hq[a][b]; H[a][NA + 2] = H[NA + 2][a] = gq[a]; }
                    for (int r = 0; r < NA; ++r) {
                        for (int j = 0; j < NA; ++j) M[r][j] = W->A[k][r][j];
                        M[r][NA] = W->Bm[k][r][0]; M[r][NA + 1] = W->Bm[k][r][1];
                    }
                    M[NA][NA + 2] = 1.0;
                    const double (*Gn)[PZ] = G[k + 1];
                    const double q00 = Gn[NA][NA], q01 = Gn[NA][NA + 1], q11 = Gn[NA + 1][NA + 1];
                    const double det = q00 * q11 - q01 * q01;
                    const double i00 = q11 / det, i01 = -q01 / det, i11 = q00 / det;
                    double Pt[PV][PV];
                    for (int p = 0; p < PV; ++p) for (int q = 0; q < PV; ++q) {
                        const double g0p = Gn[zi(p)][NA], g1p = Gn[zi(p)][NA + 1], g0q = Gn[zi(q)][NA], g1q = Gn[zi(q)][NA + 1];
                        Pt[p][q] = Gn[zi(p)][zi(q)] - (g0p * (i00 * g0q + i01 * g1q) + g1p * (i01 * g0q + i11 * g1q));
                    }
                    if (di == 0 && form == 2) {
                        double dm = 0, pm = 0;
                        for (int p = 0; p < NA; ++p) for (int q = 0; q < NA; ++q) { dm = fmax(dm, fabs(Pt[p][q] - W->Pm[k + 1][p][q])); pm = fmax(pm, fabs(W->Pm[k + 1][p][q])); }
                        printf("    node %2d  max|P_oracle| %.3e  max|Pt - P_oracle| %.3e  Quu_{k+1} %.3e %.3e\n", k + 1, pm, dm, q00, q11);
                    }
                    for (int i = 0; i < PZ; ++i) for (int j = 0; j <= i; ++j) {
                        double v;
                        if (form == 1) {
                            double ga = H[i][j], b0 = 0, b1 = 0, c0 = 0, c1 = 0;
                            for (int m = 0; m < PV; ++m) {
                                double t = 0;
                                for (int n = 0; n < PV; ++n) t += Gn[zi(m)][zi(n)] * M[n][j];
                                ga += M[m][i] * t;
                                b0 += M[m][i] * Gn[zi(m)][NA]; b1 += M[m][i] * Gn[zi(m)][NA + 1];
                                c0 += M[m][j] * Gn[zi(m)][NA]; c1 += M[m][j] * Gn[zi(m)][NA + 1];
                            }
                            v = ga - (b0 * (i00 * c0 + i01 * c1) + b1 * (i01 * c0 + i11 * c1));
                        } else {
                            v = H[i][j];
                            for (int m = 0; m < PV; ++m) { double t = 0; for (int n = 0; n < PV; ++n) t += Pt[m][n] * M[n][j]; v += M[m][i] * t; }
                        }
                        G[k][i][j] = G[k][j][i] = v;
                        maxg = fmax(maxg, fabs(v));
                    }
                    const double u00 = G[k][NA][NA], u01 = G[k][NA][NA + 1], u11 = G[k][NA + 1][NA + 1];
                    if (di == 0 && form == 1 && k >= N - 8) printf("    node %2d Quu %.6e %.6e %.6e\n", k, u00, u01, u11);
                    if (!(u00 > 0 && u00 * u11 - u01 * u01 > 0)) { first_bad = k; qbad = fmin(u00, u11); break; }
                }
            }
            printf("delta %8.1e  %-22s %s", delta, form == 0 ? "oracle (P formed)" : form == 1 ? "kernel (pre-Schur G)" : form == 2 ? "kernel, Schur first" : "exact (quad)",
                   first_bad < 0 ? "PD at every node" : "");
            if (first_bad >= 0) printf("Quu not PD at node %d (min diag %.3e)", first_bad, qbad);
            printf("   max |entry| %.3e\n", maxg);
        }
    }
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s inputs.bin\n", argv[0]); return 1; }
    FILE *f = fopen(argv[1], "rb");
    double in[8 + 2 + 34 + 8 + 22];
    if (!f || fread(in, sizeof(double), sizeof in / sizeof in[0], f) != sizeof in / sizeof in[0]) { fprintf(stderr, "bad input\n"); return 1; }
    fclose(f);
    double u0[2], fv;
    int32_t it;
    const int st = oracle_lmpc_solve(30, 0.002, in, in + 8, in + 10, in + 44, in + 52, NULL, 50, 1e-4, 1e-3, 5, u0, &fv, NULL, &it);
    printf("oracle: status %d after %d iterations, u0 %.6e %.6e\n", st, it, u0[0], u0[1]);
    return 0;
}
