// pmpc_ipm.h -- launch arguments of the batched PMPC interior-point kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dartmpc {

struct PmpcArgs {
    int B, N;
    double Ts, tol, g;      // g = model.opt.gravity[2]
    int max_iter;
    int max_soc;            // IPOPT max_soc: second-order corrections after a rejected first trial (default 4)
    int reduced;            // 1: the reduced (x, y) path (dart_mpc_config.pmpc_path), 0: IPOPT's path
    double mult_init_max;   // IPOPT constr_mult_init_max: > 0 least-square starting multipliers (default 1000)
    int pack;               // blocks per instance slot: 8 packs a small batch onto one XCD (launcher)
    // IPOPT's restoration phases (N <= 31, IPOPT's path): 0 off (a failed line search ends at -2); 1 an
    // instance whose line search fails is handed to pmpc_resto_kernel (status kPmNeedResto, no other output,
    // no completion word), which dartmpc_launch_pmpc queues behind the solve on the same stream; 2 the same
    // hand-off with the completion word written (the resident server: the host runs the restoration kernel)
    int resto;
    // IPOPT's soft restoration phase in the register kernel (1 with the restoration phases on, at every N; the
    // restoration phase proper follows only where resto allows the hand-off, N <= 31)
    int soft;
    double* resto_buf;      // [B][kPmHo] hand-off state of the instances that enter the restoration phases
                            // (device workspace of the handle; nullptr: the restoration solve starts over)
    const double* x0;       // [B][6]   device
    const double* ref;      // [B][6]
    const double* prm;      // [B][6]  mu, Qp, Qv, R, u_lo, u_hi
    const double* w_warm;   // [B][nw] or nullptr
    double* u0;             // [B][2]
    double* f;              // [B]
    double* w_out;          // [B][nw] or nullptr
    int32_t* status;        // [B]
    int32_t* iters;         // [B]
    // host-pointer entry only: completion word per instance in mapped host memory, set to `seq`
    // after every other output of the instance is visible system-wide (the host polls it instead of
    // waiting for the stream); nullptr on the device entry
    uint32_t* done;         // [B] or nullptr
    uint32_t seq;           // wraps modulo 2^32 (defined unsigned arithmetic); never 0 (0 = cleared word)
};

// resident-server mailbox (mapped host memory): one 64-bit request word,
// sequence | batch << 32 | flags << 48 | stop << 56
struct PmpcServe {
    const uint32_t* mailbox;
    unsigned long long idle_ticks;   // s_memrealtime ticks (100 MHz) without a request before the waves exit
};

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_pmpc(const dartmpc::PmpcArgs* args, hipStream_t stream);
extern "C" hipError_t dartmpc_launch_pmpc_serve(const dartmpc::PmpcArgs* args, const dartmpc::PmpcServe* sv,
                                               hipStream_t stream);
extern "C" hipError_t dartmpc_launch_pmpc_resto(const dartmpc::PmpcArgs* args, hipStream_t stream);
extern "C" hipError_t dartmpc_wave_selftest(double* d_out, hipStream_t stream);
