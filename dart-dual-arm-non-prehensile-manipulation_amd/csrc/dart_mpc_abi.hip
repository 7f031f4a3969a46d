// dart_mpc_abi.hip -- the C ABI of include/dart_mpc.h (host side).
//
// Owns the device workspace for the host-pointer entry point and the
// per-handle stream; validates arguments the way PMPC.__init__/solve would
// fail (mpc_3d.py:12-138), then launches the batched kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "dart_mpc.h"
#include "pmpc_ipm.h"
#include "rmpc_ipm.h"
#include "lmpc_ipm.h"
#include "lmpc_policy.h"
#include "arm_qp.h"

#include <cmath>

struct dart_mpc_handle {
    dart_mpc_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    double* dbuf = nullptr;        // staged inputs/outputs for the host entry
    int32_t* ibuf = nullptr;
    size_t nd = 0, ni = 0;
    std::string err;
};

namespace {

int fail(dart_mpc_handle* h, int code, const char* what, hipError_t e = hipSuccess) {
    if (h) {
        char buf[256];
        if (e != hipSuccess) std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
        else std::snprintf(buf, sizeof buf, "%s", what);
        h->err = buf;
    }
    return code;
}

#define HIPCHK(h, call, what)                                          \
    do {                                                               \
        hipError_t e_ = (call);                                        \
        if (e_ != hipSuccess) return fail((h), DART_MPC_EHIP, (what), e_); \
    } while (0)

int check_cfg(const dart_mpc_config* c) {
    if (!c) return 0;
    if (c->variant != DART_MPC_PMPC && c->variant != DART_MPC_RMPC && c->variant != DART_MPC_LMPC) return 0;
    if (c->N < 1 || c->N > (c->variant == DART_MPC_PMPC ? 63 : 31)) return 0;
    if (!(c->Ts > 0.0) || !(c->tol > 0.0) || !(c->gravity == c->gravity) || c->max_iter < 1 || c->B_max < 1) return 0;
    if (c->acceptable_iter < 0 || (c->acceptable_iter > 0 && !(c->acceptable_tol > 0.0))) return 0;
    if (c->max_soc < 0 || c->max_soc > 8) return 0;
    return 1;
}

int launch(dart_mpc_handle* h, int B, const double* x0, const double* ref, const double* prm, const double* w_warm,
           double* u0, double* f, double* w_out, int32_t* status, int32_t* iters, hipStream_t s) {
    dartmpc::PmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.max_iter = h->cfg.max_iter; a.g = h->cfg.gravity;
    a.x0 = x0; a.ref = ref; a.prm = prm; a.w_warm = w_warm;
    a.u0 = u0; a.f = f; a.w_out = w_out; a.status = status; a.iters = iters;
    HIPCHK(h, dartmpc_launch_pmpc(&a, s), "kernel launch");
    return DART_MPC_OK;
}

}  // namespace

extern "C" {

void dart_mpc_config_default(dart_mpc_config* c) {
    if (!c) return;
    c->variant = DART_MPC_PMPC;
    c->N = 20;
    c->Ts = 0.002;
    c->tol = 1e-8;
    c->max_iter = 3000;
    c->B_max = 1024;
    c->gravity = -9.81;
    c->acceptable_tol = 1e-6;      // IPOPT defaults
    c->acceptable_iter = 15;
    c->max_soc = 4;
}

int dart_mpc_nw(int N) { return 6 * (N + 1) + 2 * N; }

int dart_rmpc_nw(int N) { return 4 * (N + 1) + 2 * N; }

int dart_lmpc_nw(int N) { return 8 * (N + 1) + 2 * N; }

int dart_mpc_abi_version(void) { return DART_MPC_ABI_VERSION; }

int dart_mpc_create(const dart_mpc_config* cfg, int device, dart_mpc_handle** out) {
    if (!out || !check_cfg(cfg)) return DART_MPC_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return DART_MPC_ENODEV;
    dart_mpc_handle* h = new dart_mpc_handle();
    h->cfg = *cfg;
    h->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    const size_t B = (size_t)cfg->B_max;
    if (cfg->variant == DART_MPC_LMPC) {
        const size_t nw = (size_t)dart_lmpc_nw(cfg->N);
        h->nd = B * (8 + 2 + dartmpc::LM_NPV + 8 + dartmpc::LM_NPRM + nw + 2 + 1 + nw);
    } else if (cfg->variant == DART_MPC_RMPC) {
        const size_t nw = (size_t)dart_rmpc_nw(cfg->N);
        h->nd = B * (4 + 2 + 14 + 98 + 7 + 2 + 4 * (cfg->N + 1) + 10 + nw + 2 + 1 + nw);
    } else {
        const size_t nw = (size_t)dart_mpc_nw(cfg->N);
        h->nd = B * (6 + 6 + 6 + nw + 2 + 1 + nw);
    }
    h->ni = B * 2;
    if (e == hipSuccess) e = hipMalloc(&h->dbuf, h->nd * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&h->ibuf, h->ni * sizeof(int32_t));
    if (e != hipSuccess) {
        dart_mpc_destroy(h);
        return DART_MPC_EHIP;
    }
    *out = h;
    return DART_MPC_OK;
}

int dart_mpc_solve_batch_dev(dart_mpc_handle* h, int B, const double* x0, const double* ref, const double* prm,
                             const double* w_warm, double* u0, double* f, double* w_out, int32_t* status,
                             int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    if (h->cfg.variant != DART_MPC_PMPC) return fail(h, DART_MPC_EINVAL, "handle is not a PMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !ref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    return launch(h, B, x0, ref, prm, w_warm, u0, f, w_out, status, iters, s);
}

int dart_mpc_solve_batch(dart_mpc_handle* h, int B, const double* x0, const double* ref, const double* prm,
                         const double* w_warm, double* u0, double* f, double* w_out, int32_t* status,
                         int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    if (h->cfg.variant != DART_MPC_PMPC) return fail(h, DART_MPC_EINVAL, "handle is not a PMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !ref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B > h->cfg.B_max) return fail(h, DART_MPC_EINVAL, "batch larger than B_max");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t nw = (size_t)dart_mpc_nw(h->cfg.N), Bm = (size_t)h->cfg.B_max;
    double* d_x0 = h->dbuf;
    double* d_ref = d_x0 + Bm * 6;
    double* d_prm = d_ref + Bm * 6;
    double* d_ww = d_prm + Bm * 6;
    double* d_u0 = d_ww + Bm * nw;
    double* d_f = d_u0 + Bm * 2;
    double* d_wo = d_f + Bm;
    int32_t* d_st = h->ibuf;
    int32_t* d_it = d_st + Bm;
    HIPCHK(h, hipMemcpyAsync(d_x0, x0, sizeof(double) * 6 * B, hipMemcpyHostToDevice, s), "copy x0");
    HIPCHK(h, hipMemcpyAsync(d_ref, ref, sizeof(double) * 6 * B, hipMemcpyHostToDevice, s), "copy ref");
    HIPCHK(h, hipMemcpyAsync(d_prm, prm, sizeof(double) * 6 * B, hipMemcpyHostToDevice, s), "copy prm");
    if (w_warm) HIPCHK(h, hipMemcpyAsync(d_ww, w_warm, sizeof(double) * nw * B, hipMemcpyHostToDevice, s), "copy w_warm");
    int rc = launch(h, B, d_x0, d_ref, d_prm, w_warm ? d_ww : nullptr, d_u0, d_f, w_out ? d_wo : nullptr, d_st, d_it, s);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(u0, d_u0, sizeof(double) * 2 * B, hipMemcpyDeviceToHost, s), "copy u0");
    HIPCHK(h, hipMemcpyAsync(f, d_f, sizeof(double) * B, hipMemcpyDeviceToHost, s), "copy f");
    if (w_out) HIPCHK(h, hipMemcpyAsync(w_out, d_wo, sizeof(double) * nw * B, hipMemcpyDeviceToHost, s), "copy w_out");
    HIPCHK(h, hipMemcpyAsync(status, d_st, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s), "copy status");
    HIPCHK(h, hipMemcpyAsync(iters, d_it, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s), "copy iters");
    HIPCHK(h, hipStreamSynchronize(s), "hipStreamSynchronize");
    return DART_MPC_OK;
}

int dart_rmpc_solve_batch_dev(dart_mpc_handle* h, int B, const double* x0, const double* u_prev, double* theta,
                              double* rls_P, const double* rls_phi, const double* rls_y, double rls_lambda,
                              const double* Rref, const double* prm, const double* w_warm, double* u0, double* f,
                              double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    if (h->cfg.variant != DART_MPC_RMPC) return fail(h, DART_MPC_EINVAL, "handle is not an RMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !u_prev || !theta || !Rref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (rls_P && (!rls_phi || !rls_y || !(rls_lambda > 0.0))) return fail(h, DART_MPC_EINVAL, "RLS inputs incomplete");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    dartmpc::RmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.g = h->cfg.gravity; a.max_iter = h->cfg.max_iter;
    a.x0 = x0; a.u_prev = u_prev; a.theta = theta; a.rls_P = rls_P; a.rls_phi = rls_phi; a.rls_y = rls_y;
    a.rls_lambda = rls_lambda; a.Rref = Rref; a.prm = prm; a.w_warm = w_warm;
    a.u0 = u0; a.f = f; a.w_out = w_out; a.status = status; a.iters = iters;
    HIPCHK(h, dartmpc_launch_rmpc(&a, stream ? (hipStream_t)stream : h->stream), "kernel launch");
    return DART_MPC_OK;
}

int dart_rmpc_solve_batch(dart_mpc_handle* h, int B, const double* x0, const double* u_prev, double* theta,
                          double* rls_P, const double* rls_phi, const double* rls_y, double rls_lambda,
                          const double* Rref, const double* prm, const double* w_warm, double* u0, double* f,
                          double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    if (h->cfg.variant != DART_MPC_RMPC) return fail(h, DART_MPC_EINVAL, "handle is not an RMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !u_prev || !theta || !Rref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (rls_P && (!rls_phi || !rls_y || !(rls_lambda > 0.0))) return fail(h, DART_MPC_EINVAL, "RLS inputs incomplete");
    if (B > h->cfg.B_max) return fail(h, DART_MPC_EINVAL, "batch larger than B_max");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t N = (size_t)h->cfg.N, nw = (size_t)dart_rmpc_nw(h->cfg.N), Bm = (size_t)h->cfg.B_max;
    double* p = h->dbuf;
    double* d_x0 = p; p += Bm * 4;
    double* d_up = p; p += Bm * 2;
    double* d_th = p; p += Bm * 14;
    double* d_P = p; p += Bm * 98;
    double* d_phi = p; p += Bm * 7;
    double* d_y = p; p += Bm * 2;
    double* d_R = p; p += Bm * 4 * (N + 1);
    double* d_prm = p; p += Bm * 10;
    double* d_ww = p; p += Bm * nw;
    double* d_u0 = p; p += Bm * 2;
    double* d_f = p; p += Bm;
    double* d_wo = p;
    int32_t* d_st = h->ibuf;
    int32_t* d_it = d_st + Bm;
    auto up = [&](double* d, const double* hsrc, size_t n) { return hipMemcpyAsync(d, hsrc, sizeof(double) * n, hipMemcpyHostToDevice, s); };
    HIPCHK(h, up(d_x0, x0, 4 * B), "copy x0");
    HIPCHK(h, up(d_up, u_prev, 2 * B), "copy u_prev");
    HIPCHK(h, up(d_th, theta, 14 * B), "copy theta");
    if (rls_P) {
        HIPCHK(h, up(d_P, rls_P, 98 * B), "copy rls_P");
        HIPCHK(h, up(d_phi, rls_phi, 7 * B), "copy rls_phi");
        HIPCHK(h, up(d_y, rls_y, 2 * B), "copy rls_y");
    }
    HIPCHK(h, up(d_R, Rref, 4 * (N + 1) * B), "copy Rref");
    HIPCHK(h, up(d_prm, prm, 10 * B), "copy prm");
    if (w_warm) HIPCHK(h, up(d_ww, w_warm, nw * B), "copy w_warm");
    int rc = dart_rmpc_solve_batch_dev(h, B, d_x0, d_up, d_th, rls_P ? d_P : nullptr, d_phi, d_y, rls_lambda, d_R, d_prm,
                                       w_warm ? d_ww : nullptr, d_u0, d_f, w_out ? d_wo : nullptr, d_st, d_it, s);
    if (rc) return rc;
    auto dn = [&](void* hdst, const void* d, size_t bytes) { return hipMemcpyAsync(hdst, d, bytes, hipMemcpyDeviceToHost, s); };
    HIPCHK(h, dn(u0, d_u0, sizeof(double) * 2 * B), "copy u0");
    HIPCHK(h, dn(f, d_f, sizeof(double) * B), "copy f");
    if (w_out) HIPCHK(h, dn(w_out, d_wo, sizeof(double) * nw * B), "copy w_out");
    if (rls_P) {
        HIPCHK(h, dn(theta, d_th, sizeof(double) * 14 * B), "copy theta");
        HIPCHK(h, dn(rls_P, d_P, sizeof(double) * 98 * B), "copy rls_P");
    }
    HIPCHK(h, dn(status, d_st, sizeof(int32_t) * B), "copy status");
    HIPCHK(h, dn(iters, d_it, sizeof(int32_t) * B), "copy iters");
    HIPCHK(h, hipStreamSynchronize(s), "hipStreamSynchronize");
    return DART_MPC_OK;
}

int dart_lmpc_solve_batch_dev(dart_mpc_handle* h, int B, const double* state, const double* u_prev,
                              const double* pvec, const double* target, const double* prm, const double* w_warm,
                              double* u0, double* f, double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    if (h->cfg.variant != DART_MPC_LMPC) return fail(h, DART_MPC_EINVAL, "handle is not an LMPC handle");
    if (B < 0 || (B > 0 && (!state || !u_prev || !pvec || !target || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    dartmpc::LmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.max_iter = h->cfg.max_iter;
    a.acc_tol = h->cfg.acceptable_tol; a.acc_iter = h->cfg.acceptable_iter; a.max_soc = h->cfg.max_soc;
    a.state = state; a.u_prev = u_prev; a.pvec = pvec; a.target = target; a.prm = prm; a.w_warm = w_warm;
    a.u0 = u0; a.f = f; a.w_out = w_out; a.status = status; a.iters = iters;
    HIPCHK(h, dartmpc_launch_lmpc(&a, stream ? (hipStream_t)stream : h->stream), "kernel launch");
    return DART_MPC_OK;
}

int dart_lmpc_solve_batch(dart_mpc_handle* h, int B, const double* state, const double* u_prev, const double* pvec,
                          const double* target, const double* prm, const double* w_warm, double* u0, double* f,
                          double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    if (h->cfg.variant != DART_MPC_LMPC) return fail(h, DART_MPC_EINVAL, "handle is not an LMPC handle");
    if (B < 0 || (B > 0 && (!state || !u_prev || !pvec || !target || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B > h->cfg.B_max) return fail(h, DART_MPC_EINVAL, "batch larger than B_max");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t nw = (size_t)dart_lmpc_nw(h->cfg.N), Bm = (size_t)h->cfg.B_max;
    double* p = h->dbuf;
    double* d_st0 = p; p += Bm * 8;
    double* d_up = p; p += Bm * 2;
    double* d_pv = p; p += Bm * dartmpc::LM_NPV;
    double* d_tg = p; p += Bm * 8;
    double* d_prm = p; p += Bm * dartmpc::LM_NPRM;
    double* d_ww = p; p += Bm * nw;
    double* d_u0 = p; p += Bm * 2;
    double* d_f = p; p += Bm;
    double* d_wo = p;
    int32_t* d_st = h->ibuf;
    int32_t* d_it = d_st + Bm;
    auto up = [&](double* d, const double* hsrc, size_t n) { return hipMemcpyAsync(d, hsrc, sizeof(double) * n, hipMemcpyHostToDevice, s); };
    HIPCHK(h, up(d_st0, state, 8 * B), "copy state");
    HIPCHK(h, up(d_up, u_prev, 2 * B), "copy u_prev");
    HIPCHK(h, up(d_pv, pvec, dartmpc::LM_NPV * B), "copy pvec");
    HIPCHK(h, up(d_tg, target, 8 * B), "copy target");
    HIPCHK(h, up(d_prm, prm, dartmpc::LM_NPRM * B), "copy prm");
    if (w_warm) HIPCHK(h, up(d_ww, w_warm, nw * B), "copy w_warm");
    int rc = dart_lmpc_solve_batch_dev(h, B, d_st0, d_up, d_pv, d_tg, d_prm, w_warm ? d_ww : nullptr, d_u0, d_f,
                                       w_out ? d_wo : nullptr, d_st, d_it, s);
    if (rc) return rc;
    auto dn = [&](void* hdst, const void* d, size_t bytes) { return hipMemcpyAsync(hdst, d, bytes, hipMemcpyDeviceToHost, s); };
    HIPCHK(h, dn(u0, d_u0, sizeof(double) * 2 * B), "copy u0");
    HIPCHK(h, dn(f, d_f, sizeof(double) * B), "copy f");
    if (w_out) HIPCHK(h, dn(w_out, d_wo, sizeof(double) * nw * B), "copy w_out");
    HIPCHK(h, dn(status, d_st, sizeof(int32_t) * B), "copy status");
    HIPCHK(h, dn(iters, d_it, sizeof(int32_t) * B), "copy iters");
    HIPCHK(h, hipStreamSynchronize(s), "hipStreamSynchronize");
    return DART_MPC_OK;
}

void dart_lmpc_policy_config_default(dart_lmpc_policy_config* c) {
    if (!c) return;
    c->update_every = 8;
    c->reserved = 0;
    c->max_delta = 0.02;
    c->k_max = 2.0;
    c->min_k = 1e-2;
    c->k_ceiling_margin = std::fmax(1e-3, 0.05 * c->k_max);
    c->action_scale = 1.0;
    c->smooth_alpha = 0.5;
    c->log_std_min = std::log(1e-2);
    c->log_std_max = std::log(2.0);
}

static int policy_args(const dart_lmpc_policy_config* c, int B, const float* w, dartmpc::PolicyArgs& a) {
    if (!c || B < 0 || !w || c->update_every < 1 || !(c->k_max > c->min_k) || !(c->min_k > 0.0)) return DART_MPC_EINVAL;
    a.B = B;
    a.w.W1 = w; a.w.b1 = w + 520 * 64; a.w.W2 = a.w.b1 + 64; a.w.b2 = a.w.W2 + 64 * 64;
    a.w.W3 = a.w.b2 + 64; a.w.b3 = a.w.W3 + 64 * 34; a.w.log_std = a.w.b3 + 34;
    a.update_every = c->update_every;
    a.max_delta = c->max_delta; a.k_max = c->k_max; a.min_k = c->min_k; a.k_ceiling_margin = c->k_ceiling_margin;
    a.action_scale = c->action_scale; a.smooth_alpha = c->smooth_alpha;
    a.log_std_min = c->log_std_min; a.log_std_max = c->log_std_max;
    return DART_MPC_OK;
}

int dart_lmpc_policy_step_dev(const dart_lmpc_policy_config* cfg, int B, const float* weights, const double* state,
                              const double* target, const double* control, const double* current_k, double* obs_mean,
                              double* obs_M2, int32_t* obs_count, float* history, int32_t* timestep, const float* noise,
                              double* model_params, float* action_out, void* stream) {
    dartmpc::PolicyArgs a;
    if (policy_args(cfg, B, weights, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B > 0 && (!state || !target || !control || !current_k || !obs_mean || !obs_M2 || !obs_count || !history ||
                  !timestep || !noise || !model_params)) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    a.state = state; a.target = target; a.control = control; a.current_k = current_k; a.obs_mean = obs_mean;
    a.obs_M2 = obs_M2; a.obs_count = obs_count; a.history = history; a.timestep = timestep; a.noise = noise;
    a.model_params = model_params; a.action_out = action_out;
    return dartmpc_launch_policy(&a, (hipStream_t)stream) == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_lmpc_policy_step(const dart_lmpc_policy_config* cfg, int B, const float* weights, const double* state,
                          const double* target, const double* control, const double* current_k, double* obs_mean,
                          double* obs_M2, int32_t* obs_count, float* history, int32_t* timestep, const float* noise,
                          double* model_params, float* action_out) {
    dartmpc::PolicyArgs a;
    if (policy_args(cfg, B, weights, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B > 0 && (!state || !target || !control || !current_k || !obs_mean || !obs_M2 || !obs_count || !history ||
                  !timestep || !noise || !model_params)) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    const size_t nd = (size_t)B * (8 + 8 + 2 + 34 + 52 + 52 + 34);
    const size_t nf = (size_t)DART_LMPC_POLICY_NWEIGHTS + (size_t)B * (10 * 52 + 34 + 34);
    double* d = nullptr; float* fl = nullptr; int32_t* iv = nullptr;
    hipError_t e = hipMalloc(&d, nd * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&fl, nf * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&iv, (size_t)2 * B * sizeof(int32_t));
    double *d_st = d, *d_tg = d_st + 8 * B, *d_ct = d_tg + 8 * B, *d_ck = d_ct + 2 * B, *d_mn = d_ck + 34 * B,
           *d_m2 = d_mn + 52 * B, *d_mp = d_m2 + 52 * B;
    float *d_w = fl, *d_h = d_w + DART_LMPC_POLICY_NWEIGHTS, *d_nz = d_h + 520 * B, *d_ao = d_nz + 34 * B;
    int32_t *d_cnt = iv, *d_ts = iv + B;
    auto up = [&](void* dst, const void* src, size_t bytes) {
        if (e == hipSuccess) e = hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
    };
    auto dn = [&](void* dst, const void* src, size_t bytes) {
        if (e == hipSuccess) e = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
    };
    up(d_w, weights, sizeof(float) * DART_LMPC_POLICY_NWEIGHTS);
    up(d_st, state, sizeof(double) * 8 * B); up(d_tg, target, sizeof(double) * 8 * B);
    up(d_ct, control, sizeof(double) * 2 * B); up(d_ck, current_k, sizeof(double) * 34 * B);
    up(d_mn, obs_mean, sizeof(double) * 52 * B); up(d_m2, obs_M2, sizeof(double) * 52 * B);
    up(d_mp, model_params, sizeof(double) * 34 * B); up(d_h, history, sizeof(float) * 520 * B);
    up(d_nz, noise, sizeof(float) * 34 * B); up(d_cnt, obs_count, sizeof(int32_t) * B);
    up(d_ts, timestep, sizeof(int32_t) * B);
    if (e == hipSuccess) {
        a.w.W1 = d_w; a.w.b1 = d_w + 520 * 64; a.w.W2 = a.w.b1 + 64; a.w.b2 = a.w.W2 + 64 * 64;
        a.w.W3 = a.w.b2 + 64; a.w.b3 = a.w.W3 + 64 * 34; a.w.log_std = a.w.b3 + 34;
        a.state = d_st; a.target = d_tg; a.control = d_ct; a.current_k = d_ck; a.obs_mean = d_mn; a.obs_M2 = d_m2;
        a.obs_count = d_cnt; a.history = d_h; a.timestep = d_ts; a.noise = d_nz; a.model_params = d_mp;
        a.action_out = d_ao;
        e = dartmpc_launch_policy(&a, nullptr);
    }
    dn(obs_mean, d_mn, sizeof(double) * 52 * B); dn(obs_M2, d_m2, sizeof(double) * 52 * B);
    dn(model_params, d_mp, sizeof(double) * 34 * B); dn(history, d_h, sizeof(float) * 520 * B);
    dn(obs_count, d_cnt, sizeof(int32_t) * B); dn(timestep, d_ts, sizeof(int32_t) * B);
    if (action_out) dn(action_out, d_ao, sizeof(float) * 34 * B);
    if (d) (void)hipFree(d);
    if (fl) (void)hipFree(fl);
    if (iv) (void)hipFree(iv);
    return e == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_rls_update_batch_dev(int B, double* theta, double* P, const double* phi, const double* y, double lambda,
                              void* stream) {
    if (B < 0 || (B > 0 && (!theta || !P || !phi || !y)) || !(lambda > 0.0)) return DART_MPC_EINVAL;
    return dartmpc_launch_rls(B, theta, P, phi, y, lambda, (hipStream_t)stream) == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_rls_update_batch(int B, double* theta, double* P, const double* phi, const double* y, double lambda) {
    if (B < 0 || (B > 0 && (!theta || !P || !phi || !y)) || !(lambda > 0.0)) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    double* d = nullptr;
    const size_t n = (size_t)B * (7 + 49 + 7 + 1);
    if (hipMalloc(&d, n * sizeof(double)) != hipSuccess) return DART_MPC_EHIP;
    double *dt = d, *dP = dt + 7 * B, *dphi = dP + 49 * B, *dy = dphi + 7 * B;
    hipError_t e = hipMemcpy(dt, theta, sizeof(double) * 7 * B, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dP, P, sizeof(double) * 49 * B, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dphi, phi, sizeof(double) * 7 * B, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dy, y, sizeof(double) * B, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = dartmpc_launch_rls(B, dt, dP, dphi, dy, lambda, nullptr);
    if (e == hipSuccess) e = hipMemcpy(theta, dt, sizeof(double) * 7 * B, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(P, dP, sizeof(double) * 49 * B, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_mpc_sync(dart_mpc_handle* h) {
    if (!h) return DART_MPC_EINVAL;
    HIPCHK(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    return DART_MPC_OK;
}

// internal self-test of the wave primitives (not in include/dart_mpc.h): host_out[195]
int dartmpc_selftest(double* host_out) {
    double* d = nullptr;
    if (hipMalloc(&d, 195 * sizeof(double)) != hipSuccess) return DART_MPC_EHIP;
    hipError_t e = dartmpc_wave_selftest(d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(host_out, d, 195 * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

const char* dart_mpc_last_error(const dart_mpc_handle* h) { return h ? h->err.c_str() : "null handle"; }

void dart_mpc_destroy(dart_mpc_handle* h) {
    if (!h) return;
    if (h->dbuf) (void)hipFree(h->dbuf);
    if (h->ibuf) (void)hipFree(h->ibuf);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// per-arm impedance QP (ARMCONTROL.solver_worker, PMPC/src/controller/arm.py:266-457)
void dart_arm_config_default(dart_arm_config* c) {
    if (!c) return;
    c->tol = 1e-10;
    c->acceptable_tol = 1e-7;
    c->max_iter = 60;
    c->reserved = 0;
}

int dart_arm_snapshot_len(int n) { return (n >= 1 && n <= DART_ARM_NMAX) ? dartmpc::arm_snap_len(n) : DART_MPC_EINVAL; }
int dart_arm_param_len(int n) { return (n >= 1 && n <= DART_ARM_NMAX) ? dartmpc::arm_prm_len(n) : DART_MPC_EINVAL; }

static int arm_args(const dart_arm_config* c, int B, int n, int prm_stride, dartmpc::ArmArgs& a) {
    if (!c || B < 0 || n < 1 || n > DART_ARM_NMAX) return DART_MPC_EINVAL;
    if (prm_stride != 0 && prm_stride != dartmpc::arm_prm_len(n)) return DART_MPC_EINVAL;
    if (!(c->tol > 0.0) || !(c->acceptable_tol >= c->tol) || c->max_iter < 1 || c->max_iter > 100000) return DART_MPC_EINVAL;
    a = dartmpc::ArmArgs{};
    a.B = B; a.n = n; a.prm_stride = prm_stride; a.max_iter = c->max_iter;
    a.tol = c->tol; a.acc_tol = c->acceptable_tol;
    return DART_MPC_OK;
}

int dart_arm_solve_batch_dev(const dart_arm_config* cfg, int B, int n, const double* snap, const double* prm,
                             int prm_stride, double* qdd, double* tau, double* loss, int32_t* status, int32_t* iters,
                             void* stream) {
    dartmpc::ArmArgs a;
    if (arm_args(cfg, B, n, prm_stride, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    if (!snap || !prm || !qdd || !tau || !loss || !status || !iters) return DART_MPC_EINVAL;
    a.snap = snap; a.prm = prm; a.qdd = qdd; a.tau = tau; a.loss = loss; a.status = status; a.iters = iters;
    return dartmpc_launch_arm(&a, (hipStream_t)stream) == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_arm_solve_batch(const dart_arm_config* cfg, int B, int n, const double* snap, const double* prm,
                         int prm_stride, double* qdd, double* tau, double* loss, int32_t* status, int32_t* iters) {
    dartmpc::ArmArgs a;
    if (arm_args(cfg, B, n, prm_stride, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    if (!snap || !prm || !qdd || !tau || !loss || !status || !iters) return DART_MPC_EINVAL;
    const size_t SL = (size_t)dartmpc::arm_snap_len(n), PL = (size_t)dartmpc::arm_prm_len(n);
    const size_t np = prm_stride ? PL * B : PL;
    const size_t nd = SL * B + np + (size_t)B * (2 * n + 1);
    double* d = nullptr;
    int32_t* iv = nullptr;
    hipError_t e = hipMalloc(&d, nd * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&iv, (size_t)2 * B * sizeof(int32_t));
    double *d_s = d, *d_p = d_s + SL * B, *d_q = d_p + np, *d_t = d_q + (size_t)n * B, *d_l = d_t + (size_t)n * B;
    if (e == hipSuccess) e = hipMemcpy(d_s, snap, sizeof(double) * SL * B, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_p, prm, sizeof(double) * np, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        a.snap = d_s; a.prm = d_p; a.qdd = d_q; a.tau = d_t; a.loss = d_l; a.status = iv; a.iters = iv + B;
        e = dartmpc_launch_arm(&a, nullptr);
    }
    if (e == hipSuccess) e = hipMemcpy(qdd, d_q, sizeof(double) * n * B, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(tau, d_t, sizeof(double) * n * B, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(loss, d_l, sizeof(double) * B, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(status, iv, sizeof(int32_t) * B, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(iters, iv + B, sizeof(int32_t) * B, hipMemcpyDeviceToHost);
    if (d) (void)hipFree(d);
    if (iv) (void)hipFree(iv);
    return e == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}
