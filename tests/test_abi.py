"""The C-ABI library loads and exports every symbol include/dart_mpc.h declares (no compute)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "dart_mpc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dart_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from dart_mpc import _lib
    L = _lib.lib()
    names = _declared_functions()
    assert len(names) >= 9
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.EXPORTS)


def test_defaults_follow_reference():
    from dart_mpc import _lib
    c = _lib.default_config()
    assert (c.variant, c.N, c.Ts, c.tol, c.max_iter, c.gravity) == (0, 20, 0.002, 1e-8, 3000, -9.81)
    assert _lib.lib().dart_mpc_nw(20) == 166 and _lib.lib().dart_mpc_nw(15) == 126
    assert _lib.lib().dart_mpc_abi_version() == 8
    assert c.restoration == 1      # IPOPT's restoration phases on by default (RMPC, LMPC)
    assert c.max_cpu_time == 0.05  # rlmpc2.py:485
    assert (c.acceptable_tol, c.acceptable_iter) == (1e-6, 15)                              # IPOPT defaults
    assert _lib.lib().dart_rmpc_nw(20) == 124 and _lib.lib().dart_rmpc_nw(1) == 10      # 4(N+1) + 2N
    assert _lib.lib().dart_lmpc_nw(20) == 208 and _lib.lib().dart_lmpc_nw(30) == 308


def test_create_rejects_bad_config_without_touching_a_gpu():
    from dart_mpc import _lib
    h = ctypes.c_void_p()
    for over in (dict(N=0), dict(N=64), dict(Ts=0.0), dict(tol=-1.0), dict(B_max=0), dict(variant=7),
                 dict(max_cpu_time=-1.0)):
        c = _lib.default_config(**over)
        assert _lib.lib().dart_mpc_create(ctypes.byref(c), 0, ctypes.byref(h)) == -1
    for over in (dict(variant=1, N=64), dict(variant=1, N=0), dict(variant=2, N=64),   # RMPC, LMPC: N <= 63
                 dict(variant=2, acceptable_iter=-1), dict(variant=2, acceptable_iter=5, acceptable_tol=0.0)):
        c = _lib.default_config(**over)
        assert _lib.lib().dart_mpc_create(ctypes.byref(c), 0, ctypes.byref(h)) == -1
    assert _lib.lib().dart_mpc_solve_batch(None, 1, *([None] * 10)) == -1
    assert _lib.lib().dart_rmpc_solve_batch(None, 1, *([None] * 6), 0.995, *([None] * 9)) == -1
    assert _lib.lib().dart_rls_update_batch(-1, None, None, None, None, 0.995) == -1
    assert _lib.lib().dart_lmpc_solve_batch(None, 1, *([None] * 12)) == -1
    # the fused LMPC control step: no handle, then a handle-free config check (both before any GPU work)
    assert _lib.lib().dart_lmpc_policy_solve_batch(None, None, 1, *([None] * 21)) == -1
    assert _lib.lib().dart_lmpc_policy_solve_batch_dev(None, None, 1, *([None] * 21)) == -1


def test_rmpc_shim_validates_like_reference():
    import dart_mpc
    with pytest.raises(ValueError):
        dart_mpc.AdaptiveNPMPCSmooth(None, None, nx=6)
    with pytest.raises(ValueError):
        dart_mpc.AdaptiveNPMPCSmooth(None, None, N=64)
    c = dart_mpc.AdaptiveNPMPCSmooth(None, None, Ts=0.002, N=20, Qp=80.0, Qv=2.0, Ru=0.02, Rdu=1.0,
                                     u_bounds=(-0.6, 0.6), du_bounds=(-0.06, 0.06), vmax=0.2, v_eps=0.1)
    assert c.w0.shape == (124,) and c.gz == -9.81
    np.testing.assert_array_equal(c.params(), [80, 2, 0.02, 1.0, -0.6, 0.6, -0.06, 0.06, 0.2, 0.1])
    with pytest.raises(RuntimeError):
        c.get_state()
    with pytest.raises(ValueError):
        dart_mpc.RLS(5)


def test_pmpc_shim_validates_like_reference():
    import dart_mpc
    with pytest.raises(ValueError):
        dart_mpc.PMPC(None, None, nx=4)
    with pytest.raises(ValueError):
        dart_mpc.PMPC(None, None, N=0)
    c = dart_mpc.PMPC(None, None, Ts=0.002, N=15, Qp=600, Qv=5, R=0.1, mu=0.1, u_bounds=(-0.6, 0.6))
    assert c.target_body == "cube" and c.w0.shape == (126,) and len(c.lbx) == 126
    np.testing.assert_array_equal(c.params(), [0.1, 600, 5, 0.1, -0.6, 0.6])
    with pytest.raises(RuntimeError):
        c.get_state()


def test_tilt_to_quat_matches_reference_formula():
    from scipy.spatial.transform import Rotation as Rot
    from dart_mpc import tilt_to_quat
    for u in ([0.1, -0.2], [0.6, 0.6], [0.0, 0.0]):
        q = Rot.from_euler("xyz", [u[1], -u[0], 0.0]).as_quat()          # main.py:107-116
        np.testing.assert_allclose(tilt_to_quat(u), [q[3], q[0], q[1], q[2]], atol=1e-15)


def test_arm_qp_abi_lengths_and_validation():
    """dart_arm_* (ARMCONTROL.solver_worker boundary): row lengths, defaults, argument checks that
    return before any device work."""
    import ctypes
    import dart_mpc
    from dart_mpc.arm import ArmConfig, arm_config
    L = dart_mpc.lib()
    assert L.dart_arm_snapshot_len(7) == 206 and L.dart_arm_param_len(7) == 262
    assert L.dart_arm_snapshot_len(0) < 0 and L.dart_arm_snapshot_len(9) < 0 and L.dart_arm_param_len(9) < 0
    c = arm_config()
    assert c.tol == 1e-10 and c.acceptable_tol == 1e-7 and c.max_iter == 60
    z = ctypes.c_void_p(0)
    args = lambda cfg, B, n, stride: (ctypes.byref(cfg), B, n, z, z, stride, z, z, z, z, z)  # noqa: E731
    assert L.dart_arm_solve_batch(*args(c, 0, 7, 0)) == 0                      # empty batch
    assert L.dart_arm_solve_batch(*args(c, 0, 9, 0)) == -1                     # n > DART_ARM_NMAX
    assert L.dart_arm_solve_batch(*args(c, 0, 7, 17)) == -1                    # bad parameter stride
    assert L.dart_arm_solve_batch(*args(c, 4, 7, 0)) == -1                     # null buffers
    bad = ArmConfig(tol=0.0, acceptable_tol=1e-7, max_iter=60)
    assert L.dart_arm_solve_batch(*args(bad, 0, 7, 0)) == -1
    bad = ArmConfig(tol=1e-6, acceptable_tol=1e-8, max_iter=60)              # acceptable < tol
    assert L.dart_arm_solve_batch(*args(bad, 0, 7, 0)) == -1
    assert L.dart_arm_solve_batch_dev(*(args(c, 0, 7, 262) + (z,))) == 0


def test_library_is_built_from_the_sources_beside_it(monkeypatch):
    """The product path refuses a stale library (hygiene): the build identity compiled into
    libdartmpc.so equals the SHA-1 of the sources, and a mismatch -- or an A/B library name without
    DART_MPC_AB=1 -- raises instead of loading."""
    from dart_mpc import _lib
    L = _lib.lib()
    assert L.dart_mpc_build_id().decode() == _lib.source_build_id()
    assert L.dart_mpc_build_flavor().decode() == ""
    monkeypatch.setattr(_lib, "source_build_id", lambda: "0" * 16)
    monkeypatch.delenv("DART_MPC_AB", raising=False)
    with pytest.raises(_lib.DartMPCError, match="stale build"):
        _lib._check_build(L)
    monkeypatch.setenv("DART_MPC_AB", "1")
    _lib._check_build(L)            # the A/B tools' explicit escape hatch
