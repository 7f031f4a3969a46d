"""CPU tests of the LMPC parameter-policy restatement (row L5) and of the Python-side weight init."""
import numpy as np
import pytest

import lmpc_policy as lp


def _weights(seed=0):
    from dart_mpc.lmpc import init_policy_weights
    return init_policy_weights(seed)


def test_init_matches_policy_init_weights():
    """Policy._init_weights (rlmpc2.py:63-68): orthogonal rows/columns with gain sqrt(2), zero biases,
    log_std = log(0.1)."""
    W1, b1, W2, b2, W3, b3, ls = lp.unpack(_weights())
    for W in (W1, W2, W3):
        Wt = W.T.astype(np.float64)          # nn.Linear layout [out, in]
        G = Wt @ Wt.T if Wt.shape[0] <= Wt.shape[1] else Wt.T @ Wt
        assert np.allclose(G, 2.0 * np.eye(G.shape[0]), atol=1e-5)
    assert not b1.any() and not b2.any() and not b3.any()
    assert np.allclose(ls, np.log(0.1))


def test_mean_net_matches_torch_linear_stack():
    """fp32 reference of the kernel's MLP: torch nn.Sequential as Policy.mean_net builds it (:39-46)."""
    torch = pytest.importorskip("torch")
    W1, b1, W2, b2, W3, b3, _ = lp.unpack(_weights(3))
    net = torch.nn.Sequential(torch.nn.Linear(520, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64), torch.nn.Tanh(),
                              torch.nn.Linear(64, 34))
    with torch.no_grad():
        for lin, W, b in ((net[0], W1, b1), (net[2], W2, b2), (net[4], W3, b3)):
            lin.weight.copy_(torch.from_numpy(np.ascontiguousarray(W.T)))
            lin.bias.copy_(torch.from_numpy(b))
    obs = np.random.default_rng(0).standard_normal(520).astype(np.float32)
    ref = net(torch.from_numpy(obs)[None]).detach().numpy()[0]
    h1 = np.tanh(obs @ W1 + b1); h2 = np.tanh(h1 @ W2 + b2); mine = h2 @ W3 + b3
    assert np.allclose(mine, ref, rtol=1e-5, atol=1e-6)


def test_welford_history_and_update_cadence():
    rng = np.random.default_rng(1)
    st = lp.PolicyState(current_k=np.full(34, 1.0))
    w = _weights()
    bases = []
    for t in range(20):
        s, g, c = rng.normal(size=8), rng.normal(size=8), rng.normal(size=2) * 0.1
        prev = st.model_params.copy()
        lp.policy_step(st, w, s, g, c, rng.standard_normal(34))
        bases.append(np.concatenate([s, g, c, st.current_k]).astype(np.float32).astype(np.float64))
        B = np.array(bases)
        assert np.allclose(st.obs_mean, B.mean(0), rtol=1e-12, atol=1e-12)
        if t > 0:
            assert np.allclose(st.obs_M2 / t, B.var(0, ddof=1), rtol=1e-10, atol=1e-12)
        changed = not np.array_equal(prev, st.model_params)
        assert changed == (t % 8 == 0)
        assert np.all((st.model_params > 0.01) & (st.model_params < 1.9))
    assert len(st.history) == 10 and st.timestep == 20
