// arm_qp.h -- launch arguments of the batched per-arm impedance QP kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dartmpc {

constexpr int ARM_NMAX = 8;     // joints per arm (the reference's xArm has 7)
constexpr int ARM_NT = 6;       // task-space dimension (arm.py:129: [jacp; jacr])

// per-instance snapshot row (fp64): the shared-memory fields of arm.py:185-199 the solver reads
//   q[n] qd[n] qdd_prev[n] mocap_pos[3] ee_pos[3] rotvec[3] jac[6][n] jacDot[6][n] M[n][n] h[n]
//   Mx_inv[6][6]
__host__ __device__ constexpr int arm_snap_len(int n) { return n * n + 16 * n + 45; }
// parameter row (fp64): Wimp[6][6] Wpos[n][n] Wsmooth[n][n] Qmin[n] Qmax[n] Qdotmin[n] Qdotmax[n]
//   taumin[n] taumax[n] K[6][6] K_null[n][n] dt
__host__ __device__ constexpr int arm_prm_len(int n) { return 3 * n * n + 6 * n + 73; }

struct ArmArgs {
    int B, n;
    int prm_stride;          // 0: one parameter row for every instance, else arm_prm_len(n)
    int max_iter;
    double tol, acc_tol;
    const double* snap;      // [B][arm_snap_len(n)]
    const double* prm;       // [B or 1][arm_prm_len(n)]
    double* qdd;             // [B][n]   solution (the next qdd_prev)
    double* tau;             // [B][n]   M qdd + h
    double* loss;            // [B]
    int32_t* status;         // [B]
    int32_t* iters;          // [B]
};

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_arm(const dartmpc::ArmArgs* args, hipStream_t stream);
