"""The MjData stand-in (dart_mpc.mjdata.BodyData) round-trips each controller's state through the
reference's get_state reads (mpc_3d.py:106-113, np_mpc...:195-198, rlmpc2.py:1034-1042)."""
from types import SimpleNamespace

import numpy as np


def test_pmpc_and_rmpc_state_roundtrip():
    import dart_mpc
    data = dart_mpc.BodyData("cube", "sphere")
    s_cube = np.array([0.05, -0.1, 0.02, 0.07, 0.43, 0.004])
    s_sphere = np.array([-0.12, 0.03, 0.09, -0.02, 0.41, -0.002])
    data.set_pmpc_state("cube", s_cube)
    data.set_pmpc_state("sphere", s_sphere)
    c = dart_mpc.PMPC(None, data, N=15)
    np.testing.assert_array_equal(c.get_state(), s_cube)
    c.target_body = "sphere"                      # main_parallel_enhanced.py:41
    np.testing.assert_array_equal(c.get_state(), s_sphere)
    r = dart_mpc.AdaptiveNPMPCSmooth(None, data, target_body="sphere")
    np.testing.assert_array_equal(r.get_state(), s_sphere[:4])


def test_lmpc_state_roundtrip_through_rotation_matrix():
    import dart_mpc
    data = dart_mpc.BodyData()
    rng = np.random.default_rng(3)
    for _ in range(20):
        s = rng.uniform(-0.3, 0.3, 8)
        data.set_lmpc_state("cube2", s)
        fake = SimpleNamespace(data=data, params={"body_name": "cube2"})
        np.testing.assert_allclose(dart_mpc.RLMPC.get_state(fake), s, atol=1e-14)
