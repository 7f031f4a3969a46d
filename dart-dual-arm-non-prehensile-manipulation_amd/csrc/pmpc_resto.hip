// pmpc_resto.hip -- pmpc_resto_kernel: IPOPT's restoration phases (pmpc_resto.h) for the handed-over
// instances of a PMPC launch of more than 32 instances (smaller ones run them in the register kernel's own
// wave, pmpc_ipm.hip).  One wave64 per instance slot; every slot whose status word is not kPmNeedResto
// returns at once.
#include "pmpc_resto.h"

namespace dartmpc {

__global__ __launch_bounds__(kWave) void pmpc_resto_kernel(PmpcArgs a) {
    if (blockIdx.x % a.pack) return;
    const int b = blockIdx.x / a.pack;
    if (a.status[b] != kPmNeedResto) return;          // wave-uniform: solved by the register kernel
    pmpc_resto_solve(a, b);
}

}  // namespace dartmpc

// the handed-over instances of a PMPC launch (status kPmNeedResto), on the same stream behind it
extern "C" hipError_t dartmpc_launch_pmpc_resto(const dartmpc::PmpcArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    if (args->N < 1 || args->N >= dartmpc::PR_NMAXS) return hipErrorInvalidValue;
    dartmpc::PmpcArgs a = *args;
    a.pack = (a.B <= 32) ? 8 : 1;
    a.resto = 1;
    hipLaunchKernelGGL(dartmpc::pmpc_resto_kernel, dim3(a.B * a.pack), dim3(dartmpc::kWave), 0, stream, a);
    return hipGetLastError();
}

#ifdef DART_STAMPS
// diagnostic build only: per-phase cycles of the last instance pmpc_resto_kernel solved (32 counters)
extern "C" hipError_t dartmpc_read_stamps_pmpc_resto(unsigned long long* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(dartmpc::g_stamp_pr), sizeof(unsigned long long) * 32, 0,
                               hipMemcpyDeviceToHost);
}
#endif
