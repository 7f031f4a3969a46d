// lmpc_ipm.h -- launch arguments of the batched LMPC interior-point kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lmpc_policy.h"

namespace dartmpc {

constexpr int LM_NPRM = 22;   // [Q(8), Qt(8), R(4), u_lo, u_hi]
constexpr int LM_NPV = 34;    // model parameter vector (LMPC/src/controller/rlmpc2.py:301-344)

struct LmpcArgs {
    int B, N;
    double Ts, tol, acc_tol;
    int max_iter, acc_iter;
    int max_soc;             // IPOPT max_soc: second-order corrections after a rejected first trial
    double mult_init_max;    // IPOPT constr_mult_init_max: > 0 least-square starting multipliers (default 1000)
    int resto;               // IPOPT's soft restoration and restoration phases after a failed line search (1)
    long long max_ticks;     // IPOPT max_cpu_time in ticks of the 100 MHz constant clock (s_memrealtime), 0 = off
    double* resto_buf;       // [B][64][16] hand-off of instances entering them (device workspace of the handle);
                             // N > 31: [B][128][16], then B x LmAux (dartmpc_lmpc_wg2_area_doubles per instance)
    int pack;                // blocks per instance slot (set by the launcher; 8 = one XCD for small B)
    int xcd;                 // that XCD (0-7): the working blocks are those with blockIdx % pack == xcd % pack
    const double* state;     // [B][8]  [px, vx, py, vy, theta_x, omega_x, theta_y, omega_y]
    const double* u_prev;    // [B][2]
    const double* pvec;      // [B][34]
    const double* target;    // [B][8]
    const double* prm;       // [B][22]
    const double* w_warm;    // [B][8(N+1)+2N] nullable
    double* u0;              // [B][2]
    double* f;               // [B]
    double* w_out;           // [B][8(N+1)+2N] nullable
    int32_t* status;         // [B]
    int32_t* iters;          // [B]
    // fused policy + solve (dart_lmpc_policy_solve_batch): every instance first runs its policy step
    // (policy_step_wave) and solves with the parameters it leaves in pol.model_params; pvec unused
    int fuse_policy;
    PolicyArgs pol;
};

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_lmpc(const dartmpc::LmpcArgs* args, hipStream_t stream);
extern "C" size_t dartmpc_lmpc_lds_bytes(void);
extern "C" hipError_t dartmpc_launch_lmpc_wg2(const void* args, hipStream_t stream);
extern "C" size_t dartmpc_lmpc_wg2_area_doubles();
