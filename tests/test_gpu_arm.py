"""GPU parity of the per-arm impedance QP kernel (ARMCONTROL.solver_worker,
PMPC/src/controller/arm.py:266-457) against oracle/arm_qp.py.

The kernel and the oracle run the same Mehrotra IPM on the same QP (built by Jacobi eigen-
decompositions on the GPU, by numpy's pinv / inv / eigh in the oracle, as the reference does), so
statuses agree and the solutions agree to the QP's conditioning times rounding: qdd, tau within
1e-6 (1 + |.|) and loss within 1e-8 relative.  Iteration counts agree on >= 95 % of instances
(rounding can move a borderline convergence test by one iteration).  Parity against reference-run
numbers is unpinned (no casadi / MuJoCo here)."""
import numpy as np
import pytest

import arm_qp

pytestmark = pytest.mark.gpu

QDD_TOL = 1e-6
LOSS_RTOL = 1e-8


def _cmp(out, ref, ok_only=True, iters_frac=0.95):
    st, rs = out["status"], np.asarray(ref["status"])
    assert np.array_equal(st, rs), (st, rs)
    ok = (rs >= 0) if ok_only else np.ones_like(rs, dtype=bool)
    dq = np.abs(out["qdd"] - ref["qdd"])[ok] / (1.0 + np.abs(ref["qdd"][ok]))
    dt = np.abs(out["tau"] - ref["tau"])[ok] / (1.0 + np.abs(ref["tau"][ok]))
    dl = np.abs(out["loss"] - ref["loss"])[ok] / (1.0 + np.abs(ref["loss"][ok]))
    assert dq.max() <= QDD_TOL, dq.max()
    assert dt.max() <= QDD_TOL, dt.max()
    assert dl.max() <= LOSS_RTOL, dl.max()
    assert np.mean(out["iters"] == np.asarray(ref["iters"])) >= iters_frac
    return dq.max(), dl.max()


def test_goldens():
    import os
    import dart_mpc
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "arm_goldens.npz"))
    s = dart_mpc.ArmSolver(7)
    out = s.solve_batch(g["snap"], g["prm"])
    _cmp(out, {k: g[k] for k in ("qdd", "tau", "loss", "status", "iters")})


def test_fresh_batch_vs_oracle_shared_params():
    import dart_mpc
    from dart_mpc.arm import pack_params, pack_snapshot
    from dart_mpc.workload import arm_batch
    S, kinds = arm_batch(6, seed0=77)
    prm = arm_qp.default_params()
    out = dart_mpc.ArmSolver(7).solve_batch(pack_snapshot(S), pack_params(prm))
    ref = arm_qp.solve_batch(S, prm)
    _cmp(out, ref)


def test_device_path_and_per_instance_params():
    import torch
    import dart_mpc
    from dart_mpc.arm import pack_params, pack_snapshot
    from dart_mpc.workload import arm_batch
    S, _ = arm_batch(2, seed0=5)
    B = S["q"].shape[0]
    prm = arm_qp.default_params()
    rows, prow = pack_snapshot(S), pack_params(prm)
    host = dart_mpc.ArmSolver(7).solve_batch(rows, np.tile(prow, (B, 1)))
    dev = torch.device("cuda", 0)
    ds, dp = torch.tensor(rows, device=dev), torch.tensor(prow, device=dev)
    q, t = torch.empty((B, 7), dtype=torch.float64, device=dev), torch.empty((B, 7), dtype=torch.float64, device=dev)
    f = torch.empty(B, dtype=torch.float64, device=dev)
    st, it = torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev)
    dart_mpc.ArmSolver(7).solve_batch_dev(B, ds.data_ptr(), dp.data_ptr(), True, q.data_ptr(), t.data_ptr(),
                                          f.data_ptr(), st.data_ptr(), it.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(q.cpu().numpy(), host["qdd"])        # same kernel, same inputs: bit-identical
    assert np.array_equal(f.cpu().numpy(), host["loss"])
    assert np.array_equal(st.cpu().numpy(), host["status"])


def test_six_joint_arm_generic_params():
    import dart_mpc
    from dart_mpc.arm import pack_params, pack_snapshot
    from dart_mpc.workload import arm_batch
    S, _ = arm_batch(1, seed0=31, n=6)
    rng = np.random.default_rng(2)
    W = rng.normal(size=(6, 6))
    prm = {"Wimp": np.diag([5.0, 5, 5, 0.5, 0.5, 0.5]), "Wpos": W @ W.T * 0.01 + 0.05 * np.eye(6),
           "Wsmooth": np.eye(6) * 1e-8, "Qmin": np.full(6, -3.0), "Qmax": np.full(6, 3.0),
           "Qdotmin": np.full(6, -10.0), "Qdotmax": np.full(6, 10.0), "taumin": np.full(6, -25.0),
           "taumax": np.full(6, 25.0), "K": np.diag([3000.0, 3000, 3000, 30, 30, 30]),
           "K_null": np.diag(rng.uniform(0.5, 2.0, 6)), "dt": 0.002}
    out = dart_mpc.ArmSolver(6).solve_batch(pack_snapshot(S), pack_params(prm))
    ref = arm_qp.solve_batch(S, prm)
    _cmp(out, ref)


def test_arm_control_closed_loop():
    """ARMCONTROL.compute_torque over consecutive steps (qdd_prev fed back, arm.py:431) against the
    oracle fed the same dynamics snapshots."""
    import dart_mpc
    from dart_mpc.workload import arm_batch
    S, _ = arm_batch(1, seed0=3)
    prm = arm_qp.default_params()
    ctl = dart_mpc.ArmControl(prm)
    snap = {k: v[0].copy() for k, v in S.items()}
    snap.pop("qdd_prev")
    qdd_prev = np.zeros(7)
    for step in range(15):
        tau, loss = ctl.compute_torque(snap)
        r = arm_qp.solve_arm(dict(snap, qdd_prev=qdd_prev), prm)
        assert ctl.last_status == r["status"] == 0
        assert np.max(np.abs(tau - r["tau"]) / (1 + np.abs(r["tau"]))) <= QDD_TOL, step
        assert abs(loss - r["loss"]) <= LOSS_RTOL * (1 + abs(r["loss"])), step
        qdd_prev = r["qdd"]
        # integrate the synthetic joint state with the oracle's acceleration (shared by both loops)
        snap["qd"] = snap["qd"] + 0.002 * qdd_prev
        snap["q"] = snap["q"] + 0.002 * snap["qd"]
        snap["ee_pos"] = snap["ee_pos"] + 0.002 * (snap["jac"][:3] @ snap["qd"])
