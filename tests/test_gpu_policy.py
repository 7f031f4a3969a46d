"""GPU parity of the LMPC parameter-policy kernel (row L5) against oracle/lmpc_policy.py.

Tolerances: the MLP is fp32 (as the reference's torch Policy), so raw actions agree to 1e-5
relative; Welford statistics are fp64 (1e-12); the parameter vectors after the fp32 logit update
and the fp64 EMA / soft clip agree to 1e-6."""
import numpy as np
import pytest

import lmpc_policy as lp
import oracle_lib

pytestmark = pytest.mark.gpu


def test_policy_kernel_matches_oracle_over_steps():
    import dart_mpc
    B, T = 6, 20
    rng = np.random.default_rng(5)
    pol = dart_mpc.LmpcPolicy(B, seed=11)
    orc = [lp.PolicyState(pol.current_k[b]) for b in range(B)]
    for t in range(T):
        s, g, c = rng.normal(size=(B, 8)) * 0.1, rng.normal(size=(B, 8)) * 0.1, rng.uniform(-0.4, 0.4, (B, 2))
        eps = rng.standard_normal((B, 34)).astype(np.float32)
        act = pol.step(s, g, c, noise=eps)
        ref = np.stack([lp.policy_step(orc[b], pol.weights, s[b], g[b], c[b], eps[b]) for b in range(B)])
        assert np.allclose(act, ref, rtol=1e-5, atol=1e-5), t
        assert np.allclose(pol.obs_mean, np.stack([o.obs_mean for o in orc]), rtol=1e-12, atol=1e-12)
        assert np.allclose(pol.model_params, np.stack([o.model_params for o in orc]), rtol=0, atol=1e-6), t
        assert np.array_equal(pol.timestep, np.full(B, t + 1))
    hist = np.stack([np.stack(list(o.history)) for o in orc])
    assert np.allclose(pol.history, hist, rtol=1e-5, atol=1e-6)


def test_rlmpc_front_end_step():
    """RLMPC.solve (rlmpc2.py:986-1021) on an explicit state: policy step -> pvec -> warm-started solve,
    against the oracle chain (restated policy + C solver, IPOPT's default second-order correction on,
    as in the kernel)."""
    import dart_mpc
    ctl = dart_mpc.RLMPC(None, None, dict(N=20), seed=4)
    st = lp.PolicyState(ctl.policy.current_k[0])
    rng = np.random.default_rng(9)
    state = np.array([0.02, 0.0, -0.01, 0.0, 0.0, 0.0, 0.0, 0.0]); target = np.array([0.1, 0, -0.05, 0, 0, 0, 0, 0])
    w0 = np.zeros(8 * 21 + 40); uprev = np.zeros(2)
    for k in range(4):
        eps = rng.standard_normal(34).astype(np.float32)
        ctl._rng = np.random.default_rng(0)
        ctl.policy.step(state, target, ctl.last_control, noise=eps[None])
        out = ctl.solver.solve_batch(state[None], ctl.last_control[None], ctl.policy.model_params, target[None],
                                     ctl.prm, w_warm=ctl.w0[None], want_w=True)
        ctl.w0 = out["w"][0]; ctl.last_control = out["u0"][0]
        lp.policy_step(st, ctl.policy.weights, state, target, uprev, eps)
        o = oracle_lib.lmpc_solve_batch(state[None], uprev[None], st.model_params[None], target[None], N=20,
                                        w_init=w0[None], soc=True)
        w0 = o["w"][0]; uprev = o["u0"][0]
        assert np.allclose(ctl.policy.model_params[0], st.model_params, atol=1e-6)
        assert np.max(np.abs(out["u0"][0] - o["u0"][0])) <= 1e-6, k


def test_fused_policy_solve_equals_policy_step_then_solve():
    """dart_lmpc_policy_solve_batch (policy step as the prologue of the solve launch, C5) against the
    two-launch chain on the same inputs over 10 steps (the logit update fires at steps 0 and 8):
    every output and every piece of policy state bit for bit."""
    import dart_mpc
    B, T, N = 6, 10, 20
    rng = np.random.default_rng(21)
    fa, fb = dart_mpc.LmpcPolicy(B, seed=3), dart_mpc.LmpcPolicy(B, seed=3)
    sa = dart_mpc.LmpcSolver(N=N, B_max=B)
    sb = dart_mpc.LmpcSolver(N=N, B_max=B)
    wa = wb = None
    up = np.zeros((B, 2))
    for t in range(T):
        state = np.concatenate([rng.uniform(-0.1, 0.1, (B, 4)), rng.uniform(-0.05, 0.05, (B, 4))], axis=1)
        target = np.zeros((B, 8)); target[:, 0] = rng.uniform(-0.1, 0.1, B); target[:, 2] = rng.uniform(-0.1, 0.1, B)
        eps = rng.standard_normal((B, 34)).astype(np.float32)
        oa = dart_mpc.policy_solve_batch(sa, fa, state, up, target, w_warm=wa, want_w=True, noise=eps)
        act = fb.step(state, target, up, noise=eps)
        ob = sb.solve_batch(state, up, fb.model_params, target, w_warm=wb, want_w=True)
        for k in ("u0", "f", "w", "status", "iters"):
            assert np.array_equal(oa[k], ob[k]), (t, k)
        assert np.array_equal(oa["action"], act), t
        for k in ("model_params", "obs_mean", "obs_M2", "obs_count", "history", "timestep"):
            assert np.array_equal(getattr(fa, k), getattr(fb, k)), (t, k)
        wa, wb, up = oa["w"], ob["w"], oa["u0"]


def test_rlmpc_fused_front_end_matches_oracle_chain():
    """RLMPC.solve with the fused launch (the default) against the restated policy + C solver chain."""
    import dart_mpc
    ctl = dart_mpc.RLMPC(None, None, dict(N=20), seed=4)
    assert ctl.fused
    st = lp.PolicyState(ctl.policy.current_k[0])
    rng = np.random.default_rng(9)
    state = np.array([0.02, 0.0, -0.01, 0.0, 0.0, 0.0, 0.0, 0.0]); target = np.array([0.1, 0, -0.05, 0, 0, 0, 0, 0])
    w0 = np.zeros(8 * 21 + 40); uprev = np.zeros(2)
    for k in range(4):
        eps = rng.standard_normal(34).astype(np.float32)
        ctl._rng = _FixedNormal(eps)
        u, loss = ctl.solve(target, state=state)
        lp.policy_step(st, ctl.policy.weights, state, target, uprev, eps)
        o = oracle_lib.lmpc_solve_batch(state[None], uprev[None], st.model_params[None], target[None], N=20,
                                        w_init=w0[None], soc=True)
        w0 = o["w"][0]; uprev = o["u0"][0]
        assert np.allclose(ctl.policy.model_params[0], st.model_params, atol=1e-6)
        assert np.max(np.abs(u - o["u0"][0])) <= 1e-6, k


class _FixedNormal:
    """Stand-in for the front-end's generator: hands out the given standard-normal draws."""

    def __init__(self, eps):
        self.eps = eps

    def standard_normal(self, shape):
        return np.asarray(self.eps, np.float32).reshape(shape)


def test_rlmpc_fused_and_two_launch_front_ends_agree():
    """RLMPC(fused=True) and RLMPC(fused=False) on the same states and draws: bit-identical controls,
    losses, plans and policy state over 9 steps (the logit update fires at steps 0 and 8)."""
    import dart_mpc
    ctl = [dart_mpc.RLMPC(None, None, dict(N=20), seed=7, fused=f) for f in (True, False)]
    rng = np.random.default_rng(31)
    for k in range(9):
        state = np.concatenate([rng.uniform(-0.08, 0.08, 4), rng.uniform(-0.03, 0.03, 4)])
        target = np.array([0.1, 0, -0.05, 0, 0, 0, 0, 0])
        eps = rng.standard_normal(34).astype(np.float32)
        outs = []
        for c in ctl:
            c._rng = _FixedNormal(eps)
            outs.append(c.solve(target, state=state))
        assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1]), k
        assert np.array_equal(ctl[0].w0, ctl[1].w0), k
        for a in ("model_params", "obs_mean", "obs_M2", "history", "timestep", "obs_count"):
            assert np.array_equal(getattr(ctl[0].policy, a), getattr(ctl[1].policy, a)), (k, a)


def test_c5_as_configured_fused_launch_matches_oracle_chain():
    """BASELINE.json C5 as configured: the policy step fused into the LMPC solve launch
    (dart_lmpc_policy_solve_batch), N = 30, B = 18, over 10 control steps (the logit update fires at
    steps 0 and 8), each solve warm-started from the previous plan (rlmpc2.py:510-520) with u_prev =
    the previous control, against the oracle chain: the restated policy step per instance
    (oracle/lmpc_policy.py) and the C oracle solve with the reference's IPOPT options (tol 1e-4,
    max_iter 50, acceptable 1e-3 x 5, max_soc 4).  The plant advances by the oracle's model RK4 under
    the oracle's control.  Every step: model_params within 1e-6, statuses equal, u0 within 1e-6."""
    import dart_mpc
    from dart_mpc.workload import lmpc_batch
    B, N, T = 18, 30, 10
    D = lmpc_batch(1, seed0=5)
    rng = np.random.default_rng(77)
    pol = dart_mpc.LmpcPolicy(B, seed=13)
    orc = [lp.PolicyState(pol.current_k[b]) for b in range(B)]
    s = dart_mpc.LmpcSolver(N=N, B_max=B)
    state, target = D["state"].copy(), D["target"]
    up_k, up_o = D["u_prev"].copy(), D["u_prev"].copy()
    wk = wo = None
    for t in range(T):
        eps = rng.standard_normal((B, 34)).astype(np.float32)
        out = dart_mpc.policy_solve_batch(s, pol, state, up_k, target, w_warm=wk, want_w=True, noise=eps)
        for b in range(B):
            lp.policy_step(orc[b], pol.weights, state[b], target[b], up_o[b], eps[b])
        mp_o = np.stack([o.model_params for o in orc])
        o = oracle_lib.lmpc_solve_batch(state, up_o, mp_o, target, N=N, w_init=wo, nthreads=8)
        assert np.max(np.abs(pol.model_params - mp_o)) <= 1e-6, t
        assert np.array_equal(out["status"], o["status"]), (t, out["status"], o["status"])
        assert np.max(np.abs(out["u0"] - o["u0"])) <= 1e-6, (t, np.max(np.abs(out["u0"] - o["u0"])))
        wk, wo, up_k, up_o = out["w"], o["w"], out["u0"], o["u0"]
        state = oracle_lib.lmpc_rk4(state, o["u0"], mp_o)
    s.close()
