"""Closed loops of the GPU controllers through dart_mpc.harness: every batched
solve of the loop succeeds, logged controls equal the oracle's for the logged states (spot checks,
tolerances as tests/test_gpu_pmpc.py and tests/test_gpu_rmpc.py), and the result files follow the
reference formats."""
import json

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu


def test_pmpc_closed_loop_matches_oracle_and_converges(tmp_path):
    from dart_mpc import harness
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(1, seed0=0)
    steps = 800
    logs, st = harness.run_pmpc(S, T, P, steps)
    assert np.all(st == 0)
    for k in (0, 300, steps - 1):
        X = np.stack([lg["X"][k] for lg in logs])
        U = np.stack([lg["U_cmd"][k] for lg in logs])
        ref = oracle_lib.solve_batch(X, T, P, N=20, Ts=0.002, tol=1e-8)
        assert np.max(np.abs(U - ref["u0"])) <= 1e-6, k
    e0 = np.linalg.norm(S[:, [0, 2]] - T[:, [0, 2]], axis=1)
    sse = np.array([lg["steady_state_error"] for lg in logs])
    assert np.all(sse <= np.maximum(e0, 0.01))                   # no experiment ends farther than it started
    assert np.mean(sse < 0.01) >= 0.5
    path = harness.save_npz(logs[0], {k: logs[0][k] for k in ("steady_state_error", "convergence_time",
                                                              "control_effort")}, tmp_path, "pmpc_gpu", "cube", 1.0, 0.05)
    assert set(harness.NPZ_KEYS) <= set(np.load(path).files)


def test_rmpc_closed_loop_first_step_and_episode_json(tmp_path):
    from dart_mpc import harness
    rng = np.random.default_rng(3)
    B = 4
    x0 = np.zeros((B, 4))
    tg = np.zeros((B, 4)); tg[:, 0] = rng.uniform(-0.08, 0.08, B); tg[:, 2] = rng.uniform(-0.08, 0.08, B)
    eps, st, done = harness.run_rmpc(x0, tg, 300)
    assert np.all(st == 0)
    # first step: RLS from theta = 0, P = 1e3 I with phi(x0) and zero measured acceleration, then the solve
    from dart_mpc import AdaptiveNPMPCSmooth
    from dart_mpc.rmpc import rls_features
    ctl = AdaptiveNPMPCSmooth(None, None, Ts=0.002, N=20, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0, u_bounds=(-0.6, 0.6),
                              du_bounds=(-0.06, 0.06), vmax=0.2, v_eps=0.1)
    th = np.zeros((B, 14)); Rref = np.zeros((B, 84))
    for b in range(B):
        phi = rls_features(x0[b], 0.1)
        for a in range(2):
            th[b, 7 * a:7 * a + 7], _ = oracle_lib.rls_update(np.zeros(7), np.eye(7) * 1e3, phi, 0.0, 0.995)
        r_v = 0.5 * np.clip(tg[b] - 0.0, -0.01, 0.01) * np.array([1.0, 0.0, 1.0, 0.0])
        Rref[b] = ctl.build_ref_traj(x0[b], r_v, tg[b], 20, 4, step_fraction=0.2)
    ref = oracle_lib.rmpc_solve_batch(x0, np.zeros((B, 2)), th, Rref, np.tile(ctl.params(), (B, 1)), N=20, tol=1e-8)
    u_first = np.stack([e["ep1"]["u_cmd"][0] for e in eps])
    assert np.max(np.abs(u_first - ref["u0"])) <= 1e-5
    harness.save_episodes_json(tmp_path / "ep.json", eps[0])
    d = json.loads((tmp_path / "ep.json").read_text())["data"]["ep1"]
    assert len(d["pos_err"]) == len(d["u_cmd"]) == len(d["timestep"]) == len(d["pos_err_norm"])
