// rmpc_ipm.h -- launch arguments of the batched RMPC interior-point kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dartmpc {

struct RmpcArgs {
    int B, N;
    double Ts, tol, g;
    int max_iter;
    double mult_init_max;   // IPOPT constr_mult_init_max: > 0 least-square starting multipliers (default 1000)
    int pack;                // blocks per instance slot (set by the launcher; 8 = one XCD for small B)
    int resto;               // IPOPT's soft restoration and restoration phases (1 default; 0: a failed line search ends at -2)
    int max_soc;             // IPOPT max_soc of the restoration phase's line search (default 4)
    const double* x0;        // [B][4]
    const double* u_prev;    // [B][2]
    double* theta;           // [B][14] theta_hat (in), or RLS theta (in/out) when rls_P != nullptr
    double* rls_P;           // [B][2][7][7] in/out, nullable
    const double* rls_phi;   // [B][7]   phi_prev
    const double* rls_y;     // [B][2]   measured accelerations
    double rls_lambda;
    const double* Rref;      // [B][4(N+1)]
    const double* prm;       // [B][10]  Qp Qv Ru Rdu u_lo u_hi du_lo du_hi vmax v_eps
    const double* w_warm;    // [B][4(N+1)+2N] nullable
    double* u0;              // [B][2]
    double* f;               // [B]
    double* w_out;           // [B][4(N+1)+2N] nullable
    int32_t* status;         // [B]
    int32_t* iters;          // [B]
    double* resto_buf;       // N > 31 with resto: B x dartmpc_rmpc_wg2_resto_bytes() of device memory (the
                             // two-wave build's restoration state), else unused
};

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_rmpc(const dartmpc::RmpcArgs* args, hipStream_t stream);
extern "C" hipError_t dartmpc_launch_rmpc_wg2(const void* args, hipStream_t stream);
extern "C" size_t dartmpc_rmpc_wg2_resto_bytes();
extern "C" hipError_t dartmpc_launch_rls(int B, double* theta, double* P, const double* phi, const double* y,
                                         double lam, hipStream_t stream);
