// lmpc_policy.h -- launch arguments and the per-wave body of the batched LMPC parameter-policy step.
//
// policy_step_wave is the inference half of RLMPC._rl_worker (LMPC/src/controller/rlmpc2.py:537-769)
// for one controller, run by one wave64; it serves the standalone policy kernel (lmpc_policy.hip)
// and the prologue of the fused policy + solve launch (lmpc_ipm.hip, C5 of BASELINE.json: the
// learned parameter net evaluated in the same launch as the shooting defects it parameterises).
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

constexpr int PB = 52;              // base observation length
constexpr int PH = 64;              // hidden units
constexpr int PA = 34;              // action / parameter dimension

// LDS of one policy step
struct PolicyLds {
    float obs[PolicyArgs::kHist * PB];
    float h1[PH], h2[PH];
    double pv[PA];                  // the parameter vector after the step (the solve's pvec)
};

// One policy step of controller b by the calling wave (64 lanes, all active):
//   base = [state(8), target(8), control(2), current_k(34)]  (fp32 -> fp64, :648-653)
//   Welford running mean / M2 (fp64), std = sqrt(max(var, 1e-12)) (:656-665)
//   normalised = (base - mean) / (std + 1e-8) in fp32, 10-step history (:668-670)
//   mean_net: Linear(520, 64) - tanh - Linear(64, 64) - tanh - Linear(64, 34), fp32 (:33-80)
//   raw = mean + exp(clamp(log_std)) * eps  (Normal.rsample, eps given by the caller, :674-680)
//   every update_every-th step: k <- k_max sigmoid(logit(clamp(k / k_max)) + raw max_delta
//   action_scale) in fp32 (:742-756), then the EMA and the tanh soft clip of
//   write_params_to_shm (:606-616) in fp64.
// On return L.pv holds views["model_params"] as the solver reads it next (:506); ends with a barrier.
__device__ __forceinline__ void policy_step_wave(const PolicyArgs& a, int b, PolicyLds& L) {
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
    for (int e = l; e < (HL - 1) * PB; e += 64) L.obs[e] = hist[e + PB];
    if (l < PB) L.obs[(HL - 1) * PB + l] = nv;
    __syncthreads();
    for (int e = l; e < HL * PB; e += 64) hist[e] = L.obs[e];
    if (l == 0) a.obs_count[b] = (int32_t)cnt;

    // ---- mean_net (fp32): lane j owns hidden unit j -----------------------------------------
    {
        float s0 = W.b1[l], s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
        const int NI = HL * PB;
        int i = 0;
        for (; i + 3 < NI; i += 4) {
            s0 = fmaf(W.W1[(i + 0) * PH + l], L.obs[i + 0], s0);
            s1 = fmaf(W.W1[(i + 1) * PH + l], L.obs[i + 1], s1);
            s2 = fmaf(W.W1[(i + 2) * PH + l], L.obs[i + 2], s2);
            s3 = fmaf(W.W1[(i + 3) * PH + l], L.obs[i + 3], s3);
        }
        for (; i < NI; ++i) s0 = fmaf(W.W1[i * PH + l], L.obs[i], s0);
        L.h1[l] = tanhf((s0 + s1) + (s2 + s3));
    }
    __syncthreads();
    {
        float s0 = W.b2[l], s1 = 0.0f;
#pragma unroll 8
        for (int i = 0; i < PH; i += 2) {
            s0 = fmaf(W.W2[i * PH + l], L.h1[i], s0);
            s1 = fmaf(W.W2[(i + 1) * PH + l], L.h1[i + 1], s1);
        }
        L.h2[l] = tanhf(s0 + s1);
    }
    __syncthreads();
    if (l < PA) {
        float s0 = W.b3[l], s1 = 0.0f;
#pragma unroll 8
        for (int i = 0; i < PH; i += 2) {
            s0 = fmaf(W.W3[i * PA + l], L.h2[i], s0);
            s1 = fmaf(W.W3[(i + 1) * PA + l], L.h2[i + 1], s1);
        }
        const float mean = s0 + s1;
        const float lsd = fminf(fmaxf(W.log_std[l], (float)a.log_std_min), (float)a.log_std_max);
        const float raw = fmaf(expf(lsd), a.noise[PA * b + l], mean);
        if (a.action_out) a.action_out[PA * b + l] = raw;
        // ---- every update_every-th step: logit-space update (fp32) + EMA + soft clip (fp64) ----
        const int t = a.timestep[b];
        double prm = a.model_params[PA * b + l];
        if (t % a.update_every == 0) {
            const float kmax = (float)a.k_max;
            const double prev = prm;
            const float minf = (float)(a.min_k / a.k_max);
            const float frac = fminf(fmaxf((float)prev / kmax, minf), 1.0f - 1e-6f);
            const float zp = logf(frac / (1.0f - frac));
            const float zn = zp + raw * (float)a.max_delta * (float)a.action_scale;
            const float kn = kmax * (1.0f / (1.0f + expf(-zn)));
            const double sm = a.smooth_alpha * (double)kn + (1.0 - a.smooth_alpha) * prev;
            const double lo = a.min_k, hi = a.k_max - a.k_ceiling_margin;
            const double c = 0.5 * (hi + lo), sc = 0.5 * (hi - lo) - 1e-3;
            prm = c + sc * tanh((sm - c) / sc);
            a.model_params[PA * b + l] = prm;
        }
        L.pv[l] = prm;
    }
    if (l == 0) a.timestep[b] += 1;
    __syncthreads();
}

}  // namespace dartmpc

extern "C" hipError_t dartmpc_launch_policy(const dartmpc::PolicyArgs* args, hipStream_t stream);
