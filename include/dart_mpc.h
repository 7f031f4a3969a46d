/*
 * dart_mpc.h -- C ABI of the MI355X-native batched tray-tilt NMPC solver.
 *
 * This is the drop-in boundary for DART's per-timestep MPC solve.  Each entry
 * point replaces one reference interface (paths relative to the reference root):
 *
 *   dart_mpc_create        <- PMPC.__init__ building the CasADi NLP and
 *                             ca.nlpsol('solver','ipopt',...)
 *                             PMPC/src/controller/mpc_3d.py:12-85 (:82)
 *   dart_mpc_solve_batch   <- PMPC.solve(target) -> (U_opt[0], loss), one call
 *                             per instance today: mpc_3d.py:115-138, called from
 *                             the worker loop PMPC/main_parallel_enhanced.py:51-53
 *   dart_mpc_solve_batch_dev  same, with device-resident inputs/outputs
 *   dart_rmpc_solve_batch(_dev) <- AdaptiveNPMPCSmooth.solve + the driver's RLS updates
 *                             RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py
 *                             :212-222 (RLS :10-30), RMPC/dev_dual/rob_ctrl.py:335-352
 *   dart_lmpc_solve_batch(_dev) <- the solve of RLMPC._solver_worker
 *                             LMPC/src/controller/rlmpc2.py:229-533 (NLP :239-491, solver call
 *                             and warm start :510-520), fed by RLMPC.solve :986-1021
 *   dart_lmpc_policy_step(_dev) <- the inference / parameter-write half of RLMPC._rl_worker
 *                             rlmpc2.py:537-769 (Policy :33-80, write_params_to_shm :606-616)
 *   dart_lmpc_policy_solve_batch(_dev) <- one control step of the LMPC stack: the policy step
 *                             above, then the solve with the parameters it wrote
 *                             (views["model_params"], rlmpc2.py:506-515), in ONE launch
 *   dart_arm_solve_batch(_dev) <- ARMCONTROL.solver_worker, the per-arm impedance QP
 *                             PMPC/src/controller/arm.py:266-457 (same code in
 *                             RMPC/dev_dual/controller/parallel.py, LMPC/src/controller/parallel.py),
 *                             fed by ARMCONTROL.compute_torque / compute_dynamics :111-231
 *   dart_mpc_sync / dart_mpc_last_error / dart_mpc_destroy
 *                           <- process-lifetime handling of the solver object in
 *                             mpc_worker (main_parallel_enhanced.py:22-55)
 *
 * Plain C types only: no torch, no HIP types in signatures (streams are void*).
 *
 * Layouts (row-major, fp64):
 *   x0  [B][6]  state  [px, vx, py, vy, pz, vz]             (mpc_3d.py:106-113)
 *   ref [B][6]  target [px, vx, py, vy, pz, vz]             (mpc_3d.py:34, P[nx:])
 *   prm [B][6]  [mu, Qp, Qv, R, u_lo, u_hi]                 (mpc_3d.py:12 ctor args)
 *   w   [B][nw] decision vector in the reference order: x_0..x_N (6 each) then
 *               u_0..u_{N-1} (2 each), nw = 6(N+1) + 2N     (mpc_3d.py:69)
 *   u0  [B][2]  first control U_opt[0] = [theta_x, theta_y] (mpc_3d.py:137-138)
 *   f   [B]     objective value at the solution ("loss")    (mpc_3d.py:134)
 *   status[B]   DART_MPC_SOLVED (0), DART_MPC_MAXITER (-1), DART_MPC_LS_FAIL (-2),
 *               DART_MPC_INERTIA_FAIL (-3), DART_MPC_MAXTIME (-4, LMPC's max_cpu_time),
 *               DART_MPC_INFEASIBLE (2, RMPC / LMPC: the restoration phase converged to local
 *               infeasibility, e.g. an RMPC start with a measured |v| above vmax at the pinned node 0).
 *               As in the reference (which never
 *               checks IPOPT's status, mpc_3d.py:133-138) u0 is written anyway.
 *   iters[B]    interior-point iterations taken.
 *
 * Errors: every int-returning call returns 0 on success or a negative
 * DART_MPC_E* code; dart_mpc_last_error() describes the last failure.
 * Threading: every entry taking a handle locks the handle's mutex, so several
 * host threads may share one handle (the reference calls its controllers from
 * background threads, RMPC/dev_dual/controller/convimp.py:435): their calls
 * take turns on the handle's staging buffers and stream.  For calls that run
 * side by side, give each thread its own handle.  The stateless entries (RLS,
 * arm QP, policy step) lock a per-device stage the same way.
 */
#ifndef DART_MPC_H
#define DART_MPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DART_MPC_ABI_VERSION 8

enum dart_mpc_variant {
    DART_MPC_PMPC = 0,      /* PMPC/src/controller/mpc_3d.py, N <= 63 */
    DART_MPC_RMPC = 1,      /* RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py, N <= 63 */
    DART_MPC_LMPC = 2       /* LMPC/src/controller/rlmpc2.py, N <= 63 */
};

enum dart_mpc_status {
    DART_MPC_SOLVED = 0,
    DART_MPC_ACCEPTABLE = 1,       /* IPOPT "Solved To Acceptable Level" (LMPC: acceptable_tol / _iter) */
    DART_MPC_INFEASIBLE = 2,       /* IPOPT "Infeasible Problem Detected" (RMPC / LMPC: the restoration phase converged) */
    DART_MPC_MAXITER = -1,
    DART_MPC_LS_FAIL = -2,         /* IPOPT "Restoration Failed" (or the failed line search, restoration = 0) */
    DART_MPC_INERTIA_FAIL = -3,
    DART_MPC_MAXTIME = -4          /* IPOPT "Maximum CpuTime Exceeded" (LMPC: dart_mpc_config.max_cpu_time, ABI 7) */
};

enum dart_mpc_error {
    DART_MPC_OK = 0,
    DART_MPC_EINVAL = -1,     /* bad argument (null pointer, N out of range, B > B_max) */
    DART_MPC_EHIP = -2,       /* HIP runtime error (message in dart_mpc_last_error) */
    DART_MPC_ENODEV = -3      /* no usable gfx950 device */
};

/* Solver configuration.  Defaults (dart_mpc_config_default) follow the
 * reference: N = 20 (mpc_3d.py:12), Ts = 0.002 (MuJoCo default timestep),
 * IPOPT tol = 1e-8 and max_iter = 3000 (IPOPT defaults; mpc_3d.py:82 sets
 * neither), gravity = -9.81 (world xml line 5). */
typedef struct dart_mpc_config {
    int32_t variant;    /* enum dart_mpc_variant */
    int32_t N;          /* horizon, 1 <= N <= 63 */
    double Ts;          /* sampling time [s] */
    double tol;         /* IPOPT-style scaled optimality tolerance */
    int32_t max_iter;   /* interior-point iteration cap */
    int32_t B_max;      /* largest batch the handle's device workspace serves */
    double gravity;     /* model.opt.gravity[2] (mpc_3d.py:23), default -9.81 */
    double acceptable_tol;   /* IPOPT acceptable_tol; used by LMPC (rlmpc2.py:487: 1e-3) */
    int32_t acceptable_iter; /* IPOPT acceptable_iter, 0 = off; used by LMPC (rlmpc2.py:488: 5) */
    int32_t max_soc;    /* IPOPT max_soc (second-order corrections per line search), default 4, 0 = off,
                           <= 8; used by PMPC, LMPC and RMPC's restoration phase (the reference leaves
                           IPOPT's default, mpc_3d.py:82, np_mpc...:158-162, rlmpc2.py:480-489) */
    int32_t pmpc_path;  /* PMPC only (ABI 5): 0 = IPOPT's path on the full 6-state NLP (default; the z
                           defect rows of mpc_3d.py:37, :48 in theta, the filter, the error measures and
                           the second-order correction); 1 = the reduced (x, y) path, opt-in: same KKT
                           point to the tolerance, fewer iterations, but not IPOPT's iterates */
    int32_t restoration;  /* LMPC (ABI 6), RMPC and PMPC (ABI 8): 1 = IPOPT's soft restoration and
                           restoration phases after a failed filter line search (default;
                           MinC_1NrmRestorationPhase, the fallback of every nlpsol call, mpc_3d.py:82,
                           np_mpc...:158-162, rlmpc2.py:480-489); 0 = stop with status -2 there.  PMPC and
                           LMPC batches of at most 32 with N <= 31 run them in the solving wave (unless the
                           environment sets DART_RESTO_FUSE=0); larger batches, N > 31 (the two-wave builds)
                           and RMPC hand the failed instances to a second kernel queued on the same stream.
                           PMPC: on
                           IPOPT's path; for N > 31 the soft phase only (the restoration phase proper and the
                           reduced path keep -2).  RMPC / LMPC: at every N */
    double constr_mult_init_max;  /* IPOPT constr_mult_init_max (default 1000): the starting equality
                           multipliers are IPOPT's least-square estimate unless its max norm exceeds this
                           (then 0); 0 = always start from 0.  Used by PMPC, RMPC and LMPC */
    double max_cpu_time;  /* LMPC (ABI 7): IPOPT max_cpu_time [s], default 0.05 (rlmpc2.py:485): a solve
                           that is still running when this much wall-clock time has passed since its
                           instance started ends with status -4 (Maximum_CpuTime_Exceeded) and the current
                           iterate, checked where IPOPT checks it (after max_iter, each iteration and each
                           restoration iteration); measured on the GPU's 100 MHz constant clock; 0 = off */
} dart_mpc_config;

typedef struct dart_mpc_handle dart_mpc_handle;

void dart_mpc_config_default(dart_mpc_config *cfg);

int dart_mpc_create(const dart_mpc_config *cfg, int device, dart_mpc_handle **out);

/* Host-pointer entry: stages inputs to HBM, solves, copies results back and
 * blocks until they are in host memory.  It returns as soon as every
 * instance's results are visible in host memory, which can be a moment before
 * the stream retires the kernel; the next entry on the handle (or
 * dart_mpc_sync) settles that stream first and reports a late stream error as
 * the previous call's.  w_warm (nullable) is an initial
 * guess in the w layout; NULL = the reference's cold start (mpc_3d.py:123).
 * w_out is nullable. */
int dart_mpc_solve_batch(dart_mpc_handle *h, int B,
                         const double *x0, const double *ref, const double *prm,
                         const double *w_warm,
                         double *u0, double *f, double *w_out,
                         int32_t *status, int32_t *iters, void *hip_stream);

/* Resident solver (ABI 5, PMPC with pmpc_path 0 and N <= 31): dart_mpc_serve_start launches one
 * long-lived grid of B_serve waves on a stream of its own; every later dart_mpc_solve_batch on the
 * handle with B <= B_serve and a NULL stream is then served by it through a mailbox in mapped host
 * memory (inputs and outputs at fixed mapped addresses, completion words as before): no kernel
 * launch, no dispatch and a warm instruction cache per call; the results are bit-identical to a
 * launch.  Replaces nothing in the reference; it is the low-latency form of PMPC.solve's per-step
 * call (mpc_3d.py:115-138, main_parallel_enhanced.py:22-55).  The waves leave when
 * dart_mpc_serve_stop (or dart_mpc_destroy) is called, or after idle_timeout_s seconds without a
 * request (the next call then restarts the grid transparently).  dart_mpc_serve_running reports
 * whether the grid is resident.  Larger batches, caller streams and the _dev entry still launch. */
int dart_mpc_serve_start(dart_mpc_handle *h, int B_serve, double idle_timeout_s);

/* In-place I/O (ABI 5, PMPC): dart_mpc_bind returns host pointers into the handle's mapped, pinned
 * I/O area for B_max instances (any argument may be NULL): inputs x0 / ref / prm [B_max][6] and
 * w_warm [B_max][nw], outputs u0 [B_max][2], f, w_out [B_max][nw], status, iters.  A caller writes
 * the first B rows of the inputs in place and calls dart_mpc_solve_bound(h, B, flags); the results
 * are in the output views when it returns (blocking, like dart_mpc_solve_batch, served by the resident
 * solver when it runs).  No copy on either side of the call.  flags: DART_MPC_BOUND_W_WARM (use w_warm),
 * DART_MPC_BOUND_W_OUT (fill w_out).  The pointers stay valid until dart_mpc_destroy. */
#define DART_MPC_BOUND_W_WARM 1
#define DART_MPC_BOUND_W_OUT 2
int dart_mpc_bind(dart_mpc_handle *h, double **x0, double **ref, double **prm, double **w_warm,
                  double **u0, double **f, double **w_out, int32_t **status, int32_t **iters);
int dart_mpc_solve_bound(dart_mpc_handle *h, int B, int flags);
int dart_mpc_serve_stop(dart_mpc_handle *h);
int dart_mpc_serve_running(dart_mpc_handle *h);

/* Device-pointer entry: all pointers are device memory; asynchronous on
 * hip_stream (NULL = the handle's own stream).  Call dart_mpc_sync or
 * synchronise the stream before reading results. */
int dart_mpc_solve_batch_dev(dart_mpc_handle *h, int B,
                             const double *x0, const double *ref, const double *prm,
                             const double *w_warm,
                             double *u0, double *f, double *w_out,
                             int32_t *status, int32_t *iters, void *hip_stream);

/* RMPC (handle created with variant DART_MPC_RMPC).  Replaces
 * AdaptiveNPMPCSmooth.solve(x0, u_prev, theta_hat, Rref_flat)
 * (RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py:212-222) and, when
 * rls_P != NULL, the two RLS.update calls that precede it in the driver
 * (RMPC/dev_dual/rob_ctrl.py:335-343; RLS :10-30), fused into the same launch.
 *   x0 [B][4], u_prev [B][2]
 *   theta [B][14]   theta_hat = [theta_x(7); theta_y(7)]; with rls_P != NULL it is the RLS
 *                   estimate, updated in place before the solve
 *   rls_P [B][2][7][7] (nullable, in/out), rls_phi [B][7] = phi(prev state), rls_y [B][2] =
 *                   measured accelerations, rls_lambda = forgetting factor (0.995 in the driver)
 *   Rref [B][4(N+1)] staged reference (np_mpc...:201-210)
 *   prm [B][10] = [Qp, Qv, Ru, Rdu, u_lo, u_hi, du_lo, du_hi, vmax, v_eps]
 *   w_warm [B][4(N+1)+2N] (nullable: zeros, the reference's first call :168), w_out same layout
 *   (x_0..x_N then u_0..u_{N-1}, :144). */
int dart_rmpc_solve_batch(dart_mpc_handle *h, int B,
                          const double *x0, const double *u_prev, double *theta,
                          double *rls_P, const double *rls_phi, const double *rls_y, double rls_lambda,
                          const double *Rref, const double *prm, const double *w_warm,
                          double *u0, double *f, double *w_out,
                          int32_t *status, int32_t *iters, void *hip_stream);

int dart_rmpc_solve_batch_dev(dart_mpc_handle *h, int B,
                              const double *x0, const double *u_prev, double *theta,
                              double *rls_P, const double *rls_phi, const double *rls_y, double rls_lambda,
                              const double *Rref, const double *prm, const double *w_warm,
                              double *u0, double *f, double *w_out,
                              int32_t *status, int32_t *iters, void *hip_stream);

/* Number of fp64 entries of the RMPC w for horizon N: 4(N+1) + 2N. */
int dart_rmpc_nw(int N);

/* LMPC (handle created with variant DART_MPC_LMPC).  Replaces the solver call of
 * RLMPC._solver_worker (LMPC/src/controller/rlmpc2.py:510-520): one NLP per instance with
 *   state [B][8] = [px, vx, py, vy, theta_x, omega_x, theta_y, omega_y] (views["state"], :503)
 *   u_prev [B][2] (views["control"], the last applied control, :505)
 *   pvec [B][34] (views["model_params"], :506; squashed inside as |p| + 1e-6 where the
 *                 reference does, :296-344)
 *   target [B][8] (views["target"], :504)
 *   prm [B][22] = [Q(8), Qt(8), R(4), u_lo, u_hi]   (LMPC/src/run.py:118-121)
 *   w_warm [B][8(N+1)+2N] nullable (the worker's w0 <- w_opt, :492, :519), w_out same layout.
 * Termination follows IPOPT with the handle's tol, max_iter, acceptable_tol and acceptable_iter
 * (the reference: 1e-4, 50, 1e-3, 5); status DART_MPC_ACCEPTABLE when the acceptable test ends it. */
int dart_lmpc_solve_batch(dart_mpc_handle *h, int B,
                          const double *state, const double *u_prev, const double *pvec, const double *target,
                          const double *prm, const double *w_warm,
                          double *u0, double *f, double *w_out,
                          int32_t *status, int32_t *iters, void *hip_stream);

int dart_lmpc_solve_batch_dev(dart_mpc_handle *h, int B,
                              const double *state, const double *u_prev, const double *pvec, const double *target,
                              const double *prm, const double *w_warm,
                              double *u0, double *f, double *w_out,
                              int32_t *status, int32_t *iters, void *hip_stream);

/* Number of fp64 entries of the LMPC w for horizon N: 8(N+1) + 2N. */
int dart_lmpc_nw(int N);

/* LMPC parameter policy: the inference half of RLMPC._rl_worker
 * (LMPC/src/controller/rlmpc2.py:537-769) for B independent controllers, producing the
 * 34-vector model parameters the next solve reads (views["model_params"]).  Per call:
 * Welford-normalised observation [state, target, control, current_k] (:648-666), 10-step
 * history (:668-670), mean_net MLP 520 -> 64 -> 64 -> 34 with tanh (Policy :33-80, fp32),
 * raw action = mean + exp(clamp(log_std)) * noise (Normal.rsample, :674-680; noise [B][34] are
 * the standard-normal draws), and every update_every-th step the logit-space update
 * (:742-756, fp32) followed by the EMA + tanh soft clip of write_params_to_shm (:606-616).
 * Weights (fp32) are given input-major: W1[520][64], b1[64], W2[64][64], b2[64], W3[64][34],
 * b3[34], log_std[34] packed in this order (39748 floats); nn.Linear stores W transposed. */
typedef struct dart_lmpc_policy_config {
    int32_t update_every;      /* 8 (:742) */
    int32_t reserved;
    double max_delta;          /* max_delta_abs, 0.02 (LMPC/src/run.py:140) */
    double k_max;              /* max_param_abs, 2.0 (run.py:139) */
    double min_k;              /* 1e-2 (:560) */
    double k_ceiling_margin;   /* max(1e-3, 0.05 k_max) (:563) */
    double action_scale;       /* 1.0 (:564) */
    double smooth_alpha;       /* shm_smooth_alpha, 0.5 (:609) */
    double log_std_min;        /* log(policy_std_min = 1e-2) (:60) */
    double log_std_max;        /* log(policy_std_max = 2.0) (:61) */
} dart_lmpc_policy_config;

#define DART_LMPC_POLICY_NWEIGHTS 39748

void dart_lmpc_policy_config_default(dart_lmpc_policy_config *cfg);

/* Device pointers, asynchronous on hip_stream.  In/out: obs_mean[B][52], obs_M2[B][52],
 * obs_count[B], history[B][10][52] (fp32), timestep[B], model_params[B][34]; action_out
 * [B][34] (fp32) nullable. */
int dart_lmpc_policy_step_dev(const dart_lmpc_policy_config *cfg, int B, const float *weights,
                              const double *state, const double *target, const double *control,
                              const double *current_k, double *obs_mean, double *obs_M2, int32_t *obs_count,
                              float *history, int32_t *timestep, const float *noise, double *model_params,
                              float *action_out, void *hip_stream);

/* Host pointers (stages through device memory and blocks). */
int dart_lmpc_policy_step(const dart_lmpc_policy_config *cfg, int B, const float *weights,
                          const double *state, const double *target, const double *control,
                          const double *current_k, double *obs_mean, double *obs_M2, int32_t *obs_count,
                          float *history, int32_t *timestep, const float *noise, double *model_params,
                          float *action_out);

/* Fused LMPC control step (handle of variant DART_MPC_LMPC): for every instance, the policy
 * step of dart_lmpc_policy_step with control = u_prev (views["control"] is both the policy's
 * observation input, rlmpc2.py:650, and the solver's u_prev, :505), then the LMPC solve of
 * dart_lmpc_solve_batch with pvec = the model_params the step leaves behind (:506) -- one
 * kernel launch; the learned parameter net runs in the prologue of the kernel that evaluates the
 * shooting defects it parameterises (BASELINE.json config C5).  Results equal a policy step
 * followed by a solve.  Policy state arrays (obs_mean, obs_M2, obs_count, history, timestep,
 * model_params) are in/out as in dart_lmpc_policy_step; action_out nullable. */
int dart_lmpc_policy_solve_batch_dev(dart_mpc_handle *h, const dart_lmpc_policy_config *pcfg, int B,
                                     const float *weights, const double *state, const double *u_prev,
                                     const double *target, const double *current_k, double *obs_mean,
                                     double *obs_M2, int32_t *obs_count, float *history, int32_t *timestep,
                                     const float *noise, double *model_params, float *action_out,
                                     const double *prm, const double *w_warm,
                                     double *u0, double *f, double *w_out,
                                     int32_t *status, int32_t *iters, void *hip_stream);

/* Host pointers (stages through the handle's pinned buffers and blocks). */
int dart_lmpc_policy_solve_batch(dart_mpc_handle *h, const dart_lmpc_policy_config *pcfg, int B,
                                 const float *weights, const double *state, const double *u_prev,
                                 const double *target, const double *current_k, double *obs_mean,
                                 double *obs_M2, int32_t *obs_count, float *history, int32_t *timestep,
                                 const float *noise, double *model_params, float *action_out,
                                 const double *prm, const double *w_warm,
                                 double *u0, double *f, double *w_out,
                                 int32_t *status, int32_t *iters, void *hip_stream);

/* Batched standalone RLS.update (np_mpc...:17-27) for B independent p = 7 filters:
 * theta [B][7] and P [B][7][7] updated in place with regressors phi [B][7], targets y [B],
 * forgetting factor lambda.  The host entry stages through device memory and blocks. */
int dart_rls_update_batch(int B, double *theta, double *P, const double *phi, const double *y, double lambda);

/* Device of the stateless entries (dart_rls_update_batch*, dart_lmpc_policy_step*, dart_arm_solve_batch*)
 * for the calling thread: they run on the HIP current device.  Returns DART_MPC_ENODEV for a device
 * that does not exist.  (Handles carry their own device.) */
int dart_set_device(int device);
int dart_rls_update_batch_dev(int B, double *theta, double *P, const double *phi, const double *y, double lambda,
                              void *hip_stream);

/* Per-arm impedance QP: the body of ARMCONTROL.solver_worker (PMPC/src/controller/arm.py:266-457)
 * for B independent arm snapshots (two per dual-arm simulation step).  Stateless (no handle).
 *   snap [B][dart_arm_snapshot_len(n)] = the shared-memory fields the worker reads (:314-324):
 *        q[n] qd[n] qdd_prev[n] mocap_pos[3] ee_pos[3] rotvec[3] jac[6][n] jacDot[6][n] M[n][n]
 *        h[n] Mx_inv[6][6]
 *   prm  [B or 1][dart_arm_param_len(n)] = the worker's params (:290-302):
 *        Wimp[6][6] Wpos[n][n] Wsmooth[n][n] Qmin[n] Qmax[n] Qdotmin[n] Qdotmax[n] taumin[n]
 *        taumax[n] K[6][6] K_null[n][n] dt;   prm_stride = 0 shares one row across the batch,
 *        else dart_arm_param_len(n)
 *   qdd [B][n] the optimal joint accelerations (the next qdd_prev, :431), tau [B][n] = M qdd + h
 *   (torque_out, :424/:432), loss [B] = the objective value (loss_out, :425/:433),
 *   status [B] (DART_ARM_*), iters [B] interior-point iterations.
 * The QP is strictly convex (Wpos > 0); IPOPT's answer is its unique KKT point with the bounds
 * relaxed by bound_relax_factor = 1e-8, which is what the solver returns (scaled KKT error <= tol).
 * n <= DART_ARM_NMAX; bounds with |value| >= 1e19 are treated as absent (IPOPT's convention). */
#define DART_ARM_NMAX 8

enum dart_arm_status {
    DART_ARM_SOLVED = 0,
    DART_ARM_ACCEPTABLE = 1,     /* normal matrix lost definiteness with the KKT error <= acceptable_tol */
    DART_ARM_MAXITER = -1,
    DART_ARM_BREAKDOWN = -2,
    DART_ARM_INFEASIBLE = -3     /* multipliers diverging: the bounds admit no qdd */
};

typedef struct dart_arm_config {
    double tol;                  /* scaled KKT tolerance, default 1e-10 */
    double acceptable_tol;       /* default 1e-7 */
    int32_t max_iter;            /* default 60 */
    int32_t reserved;
} dart_arm_config;

void dart_arm_config_default(dart_arm_config *cfg);
int dart_arm_snapshot_len(int n);
int dart_arm_param_len(int n);

/* Device pointers, asynchronous on hip_stream. */
int dart_arm_solve_batch_dev(const dart_arm_config *cfg, int B, int n, const double *snap, const double *prm,
                             int prm_stride, double *qdd, double *tau, double *loss, int32_t *status,
                             int32_t *iters, void *hip_stream);

/* Host pointers (stages through device memory and blocks). */
int dart_arm_solve_batch(const dart_arm_config *cfg, int B, int n, const double *snap, const double *prm,
                         int prm_stride, double *qdd, double *tau, double *loss, int32_t *status, int32_t *iters);

int dart_mpc_sync(dart_mpc_handle *h);

const char *dart_mpc_last_error(const dart_mpc_handle *h);

void dart_mpc_destroy(dart_mpc_handle *h);

/* Number of fp64 entries of w for horizon N: 6(N+1) + 2N. */
int dart_mpc_nw(int N);

/* ABI version (DART_MPC_ABI_VERSION) of the loaded library. */
int dart_mpc_abi_version(void);

/* Build identity (round 6): the first 16 hex digits of the SHA-1 of the sources the library was compiled from
 * (the Makefile's SRC then HDR lists, concatenated), and the diagnostic flavour of the build: "" for the product
 * library, "stamps" / "trace" for the phase-stamp and restoration-trace builds.  The Python binding refuses a
 * library whose identity is not that of the sources beside it (a stale build). */
const char *dart_mpc_build_id(void);
const char *dart_mpc_build_flavor(void);

#ifdef __cplusplus
}
#endif

#endif /* DART_MPC_H */
