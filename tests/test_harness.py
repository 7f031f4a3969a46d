"""CPU checks of the headless harness pieces: the stand-in plant against
the reference model, the AsyncLogger metrics (PMPC/src/logger.py:158-183), the npz layout
(:186-196) and the RMPC episode JSON (RMPC/dev_dual/rob_ctrl.py:51-86)."""
import json

import numpy as np

import pmpc_nlp


def test_plant_reduces_to_reference_model():
    """tau -> 0 and no Coulomb term: one plant step equals the reference RK4 (mpc_3d.py:87-104) on the
    x/y axes for the commanded tilt."""
    from dart_mpc.harness import TrayPlant
    rng = np.random.default_rng(0)
    x0 = rng.normal(0, 0.1, (5, 6)); u = rng.uniform(-0.5, 0.5, (5, 2)); mu = rng.uniform(0.05, 0.2, 5)
    pl = TrayPlant(x0, mu, tau=0.0, mu_c=0.0, dt=0.002)
    x1 = pl.step(u)
    for b in range(5):
        ref = pmpc_nlp.rk4_step(x0[b], u[b], mu[b], 0.002)
        assert np.allclose(x1[b, :4], ref[:4], rtol=0, atol=1e-15)


def test_logger_metrics_definitions():
    from dart_mpc.harness import logger_metrics
    t = np.arange(5) * 0.002
    X = np.zeros((5, 6)); X[:, 0] = [0.05, 0.03, 0.009, 0.004, 0.002]
    Xt = np.zeros((5, 6))
    U = np.tile([0.3, 0.4], (5, 1))                              # |u| = 0.5
    m = logger_metrics({"t": t, "X": X, "X_target": Xt, "U_cmd": U}, 0.002)
    assert m["steady_state_error"] == 0.002
    assert m["convergence_time"] == t[2]                          # first error < 1 cm
    assert abs(m["control_effort"] - 5 * 0.5 * 0.002) < 1e-15
    X[:, 0] = 0.5
    assert logger_metrics({"t": t, "X": X, "X_target": Xt, "U_cmd": U}, 0.002)["convergence_time"] == t[-1]


def test_npz_layout(tmp_path):
    from dart_mpc.harness import NPZ_KEYS, save_npz
    logs = {k: np.zeros((3, 2)) for k in NPZ_KEYS}
    path = save_npz(logs, {"steady_state_error": 0.1, "convergence_time": 0.2, "control_effort": 0.3}, tmp_path,
                    "exp", "cube", 1.0, 0.1)
    assert "cube/mass=1.0_friction=0.1/exp_" in path
    d = np.load(path)
    assert set(d.files) == set(NPZ_KEYS) | {"steady_state_error", "convergence_time", "control_effort"}


def test_episode_json_layout(tmp_path):
    from dart_mpc.harness import add_episode, save_episodes_json
    eps = {}
    add_episode(eps, "ep1", [[0.1, -0.2]], [np.float64(0.22)], [np.array([0.1, 0.2])], [np.zeros(2)], [float("nan")])
    save_episodes_json(tmp_path / "r.json", eps)
    d = json.loads((tmp_path / "r.json").read_text())
    assert list(d) == ["data"] and list(d["data"]["ep1"]) == ["pos_err", "pos_err_norm", "u_cmd", "torque", "timestep"]
    assert d["data"]["ep1"]["timestep"] == [None] and d["data"]["ep1"]["u_cmd"] == [[0.1, 0.2]]
