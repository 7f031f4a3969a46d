// lmpc_policy.h -- launch arguments of the batched LMPC parameter-policy step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dartmpc {

// mean_net weights, fp32, stored input-major ([in][out]) so that lane j reads column j coalesced
struct PolicyWeights {
    const float* W1;        // [520][64]
    const float* b1;        // [64]
    const float* W2;        // [64][64]
    const float* b2;        // [64]
    const float* W3;        // [64][34]
    const float* b3;        // [34]
    const float* log_std;   // [34]
};

struct PolicyArgs {
    static constexpr int kHist = 10;
    int B;
    PolicyWeights w;
    const double* state;       // [B][8]
    const double* target;      // [B][8]
    const double* control;     // [B][2]
    const double* current_k;   // [B][34]  the worker's current_k (observation input)
    double* obs_mean;          // [B][52]  Welford state, in/out
    double* obs_M2;            // [B][52]
    int32_t* obs_count;        // [B]
    float* history;            // [B][10][52] normalised observations, oldest first, in/out
    int32_t* timestep;         // [B]  in/out
    const float* noise;        // [B][34]  standard-normal draws of Normal.rsample
    double* model_params;      // [B][34]  views["model_params"], in/out
    float* action_out;         // [B][34]  raw action, nullable
    int update_every;
    double max_delta, k_max, min_k, k_ceiling_margin, action_scale, smooth_alpha, log_std_min, log_std_max;
};

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_policy(const dartmpc::PolicyArgs* args, hipStream_t stream);
