// lmpc_policy.hip -- batched LMPC parameter policy step (inference + logit-space update), gfx950.
//
// Replaces the inference half of RLMPC._rl_worker (LMPC/src/controller/rlmpc2.py:537-769) for a
// batch of independent controllers, one wave64 per instance:
//   base = [state(8), target(8), control(2), current_k(34)]  (fp32 -> fp64, :648-653)
//   Welford running mean / M2 (fp64), std = sqrt(max(var, 1e-12)) (:656-665)
//   normalised = (base - mean) / (std + 1e-8) in fp32, 10-step history (:668-670)
//   mean_net: Linear(520, 64) - tanh - Linear(64, 64) - tanh - Linear(64, 34), fp32 (:33-80)
//   raw = mean + exp(clamp(log_std)) * eps  (Normal.rsample, eps given by the caller, :674-680)
//   every update_every-th step: k <- k_max sigmoid(logit(clamp(k / k_max)) + raw max_delta
//   action_scale) in fp32 (:742-756), then the EMA and the tanh soft clip of
//   write_params_to_shm (:606-616) in fp64.
// The weights are an input (the reference checkpoints are not loaded).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lmpc_policy.h"
#include "wave.h"

namespace dartmpc {

constexpr int PB = 52;              // base observation length
constexpr int PH = 64;              // hidden units
constexpr int PA = 34;              // action / parameter dimension

__global__ __launch_bounds__(kWave) void lmpc_policy_kernel(PolicyArgs a) {
    __shared__ float obs[PolicyArgs::kHist * PB];
    __shared__ float h1[PH], h2[PH];
    const int b = blockIdx.x;
    const int l = threadIdx.x;
    const int HL = PolicyArgs::kHist;
    const PolicyWeights& W = a.w;

    // ---- base vector, Welford update, normalisation (lanes 0..51) -------------------------
    const int64_t cnt = (int64_t)a.obs_count[b] + 1;
    float nv = 0.0f;
    if (l < PB) {
        double v;
        if (l < 8) v = (double)(float)a.state[8 * b + l];
        else if (l < 16) v = (double)(float)a.target[8 * b + l - 8];
        else if (l < 18) v = (double)(float)a.control[2 * b + l - 16];
        else v = (double)(float)a.current_k[PA * b + l - 18];
        double* mean = a.obs_mean + PB * b;
        double* M2 = a.obs_M2 + PB * b;
        const double d1 = v - mean[l];
        const double mn = mean[l] + d1 / (double)cnt;
        const double d2 = v - mn;
        const double m2 = M2[l] + d1 * d2;
        mean[l] = mn; M2[l] = m2;
        const double var = cnt > 1 ? m2 / (double)(cnt - 1) : 1e-6;
        const float sd = (float)sqrt(fmax(var, 1e-12));
        nv = ((float)v - (float)mn) / (sd + 1e-8f);
    }
    // ---- history: shift by one step, append (deque(maxlen=10), oldest first) -------------
    float* hist = a.history + (size_t)HL * PB * b;
    for (int e = l; e < (HL - 1) * PB; e += kWave) obs[e] = hist[e + PB];
    if (l < PB) obs[(HL - 1) * PB + l] = nv;
    __syncthreads();
    for (int e = l; e < HL * PB; e += kWave) hist[e] = obs[e];
    if (l == 0) a.obs_count[b] = (int32_t)cnt;

    // ---- mean_net (fp32): lane j owns hidden unit j -----------------------------------------
    {
        float s0 = W.b1[l], s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
        const int NI = HL * PB;
        int i = 0;
        for (; i + 3 < NI; i += 4) {
            s0 = fmaf(W.W1[(i + 0) * PH + l], obs[i + 0], s0);
            s1 = fmaf(W.W1[(i + 1) * PH + l], obs[i + 1], s1);
            s2 = fmaf(W.W1[(i + 2) * PH + l], obs[i + 2], s2);
            s3 = fmaf(W.W1[(i + 3) * PH + l], obs[i + 3], s3);
        }
        for (; i < NI; ++i) s0 = fmaf(W.W1[i * PH + l], obs[i], s0);
        h1[l] = tanhf((s0 + s1) + (s2 + s3));
    }
    __syncthreads();
    {
        float s0 = W.b2[l], s1 = 0.0f;
#pragma unroll 8
        for (int i = 0; i < PH; i += 2) {
            s0 = fmaf(W.W2[i * PH + l], h1[i], s0);
            s1 = fmaf(W.W2[(i + 1) * PH + l], h1[i + 1], s1);
        }
        h2[l] = tanhf(s0 + s1);
    }
    __syncthreads();
    if (l < PA) {
        float s0 = W.b3[l], s1 = 0.0f;
#pragma unroll 8
        for (int i = 0; i < PH; i += 2) {
            s0 = fmaf(W.W3[i * PA + l], h2[i], s0);
            s1 = fmaf(W.W3[(i + 1) * PA + l], h2[i + 1], s1);
        }
        const float mean = s0 + s1;
        const float lsd = fminf(fmaxf(W.log_std[l], (float)a.log_std_min), (float)a.log_std_max);
        const float raw = fmaf(expf(lsd), a.noise[PA * b + l], mean);
        if (a.action_out) a.action_out[PA * b + l] = raw;
        // ---- every update_every-th step: logit-space update (fp32) + EMA + soft clip (fp64) ----
        const int t = a.timestep[b];
        if (t % a.update_every == 0) {
            const float kmax = (float)a.k_max;
            const double prev = a.model_params[PA * b + l];
            const float minf = (float)(a.min_k / a.k_max);
            const float frac = fminf(fmaxf((float)prev / kmax, minf), 1.0f - 1e-6f);
            const float zp = logf(frac / (1.0f - frac));
            const float zn = zp + raw * (float)a.max_delta * (float)a.action_scale;
            const float kn = kmax * (1.0f / (1.0f + expf(-zn)));
            const double sm = a.smooth_alpha * (double)kn + (1.0 - a.smooth_alpha) * prev;
            const double lo = a.min_k, hi = a.k_max - a.k_ceiling_margin;
            const double c = 0.5 * (hi + lo), sc = 0.5 * (hi - lo) - 1e-3;
            a.model_params[PA * b + l] = c + sc * tanh((sm - c) / sc);
        }
    }
    if (l == 0) a.timestep[b] += 1;
}

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_policy(const dartmpc::PolicyArgs* args, hipStream_t stream) {
    if (args->B <= 0) return hipSuccess;
    hipLaunchKernelGGL(dartmpc::lmpc_policy_kernel, dim3(args->B), dim3(dartmpc::kWave), 0, stream, *args);
    return hipGetLastError();
}
