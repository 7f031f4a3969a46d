// pmpc_model.h -- the PMPC tray model pieces shared by the register kernel (pmpc_ipm.hip) and the
// restoration kernel (pmpc_resto.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace dartmpc {

// hand-off of an instance whose filter line search failed to pmpc_resto_kernel (internal status)
constexpr int kPmNeedResto = -100;

// The state the register kernel hands over with such an instance (PmpcArgs::resto_buf, kPmHo doubles per
// instance): the iterate of the iteration whose line search failed -- per node k (< 32) the full state
// x[6] = [px vx py vy pz vz], the tilts u[2], the defect-row multipliers lam[6] (the z rows' are 0 on IPOPT's
// path: cost-free states), the bound multipliers zl[2], zu[2] -- the filter entries (theta, phi) and mu, the
// last inertia shift, the iteration and filter counters.  pmpc_resto_solve resumes from it: the failed
// iteration is repeated (its direction up to rounding) and the restoration phases follow, instead of solving
// the instance again from its start.
constexpr int kPmHoRow = 18;                          // x 0..5, u 6..7, lam 8..13, zl 14..15, zu 16..17
constexpr int kPmHoFilt = 32 * kPmHoRow;             // 64 entries (theta, phi)
constexpr int kPmHoScal = kPmHoFilt + 2 * 64;        // mu, delta_last, it, nfilt
constexpr int kPmHo = kPmHoScal + 4;

// mpc_3d.py:87-97, one axis:  pdot = v,  vdot = g sin(theta) - mu v
__device__ __forceinline__ void axis_rhs(double g, double mu, double s, double v, double& dp, double& dv) {
    dp = v;
    dv = g * s - mu * v;
}
// mpc_3d.py:99-104 on one axis with s = sin(theta) held constant
__device__ __forceinline__ void axis_rk4(double h, double g, double mu, double s, double p, double v,
                                         double& pn, double& vn) {
    double k1p, k1v, k2p, k2v, k3p, k3v, k4p, k4v;
    axis_rhs(g, mu, s, v, k1p, k1v);
    axis_rhs(g, mu, s, v + h / 2 * k1v, k2p, k2v);
    axis_rhs(g, mu, s, v + h / 2 * k2v, k3p, k3v);
    axis_rhs(g, mu, s, v + h * k3v, k4p, k4v);
    pn = p + h / 6 * (k1p + 2 * k2p + 2 * k3p + k4p);
    vn = v + h / 6 * (k1v + 2 * k2v + 2 * k3v + k4v);
}
// z sub-state (mpc_3d.py:93-97): pzdot = vz_new, vzdot = (vz_new - vz)/Ts, literal RK4
__device__ __forceinline__ void z_rk4(double h, double w, double pz, double vz, double& pzn, double& vzn) {
    const double k1v = (w - vz) / h;
    const double k2v = (w - (vz + h / 2 * k1v)) / h;
    const double k3v = (w - (vz + h / 2 * k2v)) / h;
    const double k4v = (w - (vz + h * k3v)) / h;
    pzn = pz + h / 6 * (w + 2 * w + 2 * w + w);
    vzn = vz + h / 6 * (k1v + 2 * k2v + 2 * k3v + k4v);
}

}  // namespace dartmpc
