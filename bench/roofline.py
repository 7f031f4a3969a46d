"""Roofline constants of the benchmark, frozen here so the figures in bench.py can be recomputed.

Unit of work: one interior-point iteration of one instance.  F_ITER counts the
algorithmic FP64 FLOP of one iteration on the reference's NLP (full-dimension Riccati step,
dynamics / Jacobian / Hessian evaluation, line search, barrier terms), not the kernels' own,
smaller operation counts (the PMPC kernel solves the separable 2 x (2-state) problem):
  F_stage = 2 nx^3 [A'PA] + 2 nx^3 [PA] + 4 nx^2 nu [PB, B'PA] + 2 nu^2 nx [B'PB] + nu^3 / 3
            + 2 nu^2 nx [K] + 2 nx^2 nu [S'K] + 6 (nx^2 + nx nu) [vectors]
            + (1 + nx + nu) C_rk4 [dynamics + Jacobian] + C_H [Hessian] + 2 C_rk4 [line search] + 8 nu
  F_iter  = N F_stage + F_terminal
PMPC (nx 6, nu 2, C_rk4 ~ 90, C_H ~ 300): ~3.0 kFLOP per stage -> 6.0e4 at N = 20.
RMPC (augmented nx 6, nu 2, C_rk4 ~ 150 with tanh): ~3.66 kFLOP -> 7.3e4 at N = 20.
LMPC (nx 8, nu 2, C_rk4 ~ 600): ~12.4 kFLOP -> 2.5e5 at N = 20, 3.7e5 at N = 30.

Algorithmic HBM bytes per solve: the fp64 inputs read and the outputs written once
(PMPC: state 6 + target 6 + params 6 in, u0 2 + f + status / iterations out = 176 B).
"""

FP64_PEAK_TFLOPS = 78.6       # MI355X FP64 vector (= FP64 matrix) peak, spec
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E, spec

F_ITER = {"pmpc_n20": 6.0e4, "rmpc_n20": 7.3e4, "lmpc_n20": 2.5e5, "lmpc_n30": 3.7e5}

BYTES_PER_SOLVE = {
    "pmpc": 176,                                                    # 18 fp64 in, u0[2] + f + status + iters out
    "rmpc": (4 + 2 + 14 + 98 + 7 + 2 + 84 + 10 + 14 + 98 + 4) * 8,  # x0, u_prev, theta, P, phi, y, Rref, prm in; theta, P, u0, f out
    "lmpc": (8 + 2 + 34 + 8 + 22 + 4) * 8,                          # state, u_prev, pvec, target, prm in; u0, f, status out
}


def achieved_tflops(iters_sum: float, f_iter: float, seconds: float) -> float:
    """Algorithmic FP64 TFLOP/s of a launch that ran iters_sum instance-iterations in `seconds`."""
    return iters_sum * f_iter / seconds / 1e12


def roofline(iters_sum: float, f_iter: float, seconds: float, **extra) -> dict:
    a = achieved_tflops(iters_sum, f_iter, seconds)
    return dict(bound="fp64-valu", achieved=a, peak=FP64_PEAK_TFLOPS, unit="TFLOP/s", frac=a / FP64_PEAK_TFLOPS, **extra)
