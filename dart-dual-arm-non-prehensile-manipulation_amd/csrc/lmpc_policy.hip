// lmpc_policy.hip -- batched LMPC parameter policy step (inference + logit-space update), gfx950.
//
// Replaces the inference half of RLMPC._rl_worker (LMPC/src/controller/rlmpc2.py:537-769) for a
// batch of independent controllers, one wave64 per instance; the step itself is
// policy_step_wave (lmpc_policy.h), which the fused policy + solve launch of lmpc_ipm.hip runs as
// its prologue.  The weights are an input (the reference checkpoints are not loaded).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lmpc_policy.h"
#include "wave.h"

namespace dartmpc {

__global__ __launch_bounds__(kWave) void lmpc_policy_kernel(PolicyArgs a) {
    __shared__ PolicyLds L;
    policy_step_wave(a, blockIdx.x, L);
}

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_policy(const dartmpc::PolicyArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    hipLaunchKernelGGL(dartmpc::lmpc_policy_kernel, dim3(args->B), dim3(dartmpc::kWave), 0, stream, *args);
    return hipGetLastError();
}
