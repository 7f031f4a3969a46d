"""CPU checks of the per-arm impedance QP oracle (oracle/arm_qp.py; SURVEY §8f rank 1,
ARMCONTROL.solver_worker PMPC/src/controller/arm.py:266-457) and of the arm front-end's packing.

Parity status: unpinned against reference-run numbers (casadi / MuJoCo absent, no stored outputs);
the oracle is pinned by the KKT certificate of the reference's own NLP and by SLSQP
(tests/golden/make_arm_goldens.py)."""
import numpy as np
import pytest

import arm_qp


@pytest.fixture(scope="module")
def arm_goldens():
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "arm_goldens.npz"))
    return {k: d[k] for k in d.files}


def _unpack(row, prow, n=7):
    from dart_mpc.arm import PARAM_FIELDS, SNAP_FIELDS, _width
    s, p, o = {}, {}, 0
    for k, w in SNAP_FIELDS:
        m = _width(w, n)
        v = row[o:o + m]
        s[k] = v.reshape(6, n) if k in ("jac", "jacDot") else v.reshape(n, n) if k == "M" else \
            v.reshape(6, 6) if k == "Mx_inv" else v
        o += m
    o = 0
    for k, w in PARAM_FIELDS:
        m = _width(w, n)
        v = prow[o:o + m]
        p[k] = v.reshape(6, 6) if k in ("Wimp", "K") else v.reshape(n, n) if k in ("Wpos", "Wsmooth", "K_null") \
            else float(v[0]) if k == "dt" else v
        o += m
    return s, p


def test_goldens_reproduce(arm_goldens):
    g = arm_goldens
    for i in range(len(g["kinds"])):
        s, p = _unpack(g["snap"][i], g["prm"][i])
        r = arm_qp.solve_arm(s, p)
        assert r["status"] == g["status"][i] and r["iters"] == g["iters"][i], i
        assert np.allclose(r["qdd"], g["qdd"][i], rtol=1e-12, atol=1e-12)
        assert abs(r["loss"] - g["loss"][i]) <= 1e-12 * (1 + abs(g["loss"][i]))


def test_goldens_cover_the_reference_branches(arm_goldens):
    g = arm_goldens
    dets, kinds = [], list(g["kinds"])
    for i in range(len(kinds)):
        s, _ = _unpack(g["snap"][i], g["prm"][i])
        dets.append(abs(np.linalg.det(s["Mx_inv"])))
    dets = np.array(dets)
    assert (dets > 1e-8).any() and (dets <= 1e-8).any()      # inv and pinv(rcond=1e-3) paths, arm.py:346-350
    assert -3 in g["status"] and "unbounded" in kinds and "smooth_nonsym" in kinds
    act = 0
    for i in range(len(kinds)):
        if g["status"][i] != 0:
            continue
        s, p = _unpack(g["snap"][i], g["prm"][i])
        H, c, const, A, b, lo, hi, _ = arm_qp.build_qp(s, p)
        r = A @ g["qdd"][i] + b
        act += int(np.any(np.isclose(r, hi, rtol=0, atol=1e-6) | np.isclose(r, lo, rtol=0, atol=1e-6)))
    assert act >= 10                                          # active torque / position bounds


def test_quadratic_form_equals_reference_cost(arm_goldens):
    """1/2 x'Hx + c'x + const is the reference objective (arm.py:377-388) for any x."""
    g = arm_goldens
    rng = np.random.default_rng(0)
    for i in range(0, len(g["kinds"]), 7):
        s, p = _unpack(g["snap"][i], g["prm"][i])
        H, c, const, A, b, lo, hi, aux = arm_qp.build_qp(s, p)
        for _ in range(3):
            x = rng.normal(0, 5, 7)
            f = 0.5 * x @ H @ x + c @ x + const
            assert abs(f - arm_qp.reference_cost(x, s, p, aux)) <= 1e-9 * (1 + abs(f))


def test_kkt_certificates(arm_goldens):
    g = arm_goldens
    ok = g["status"] >= 0
    assert ok.sum() >= len(ok) - 1
    assert np.max(g["kkt_stat"][ok]) <= 1e-9


def test_pack_roundtrip(arm_goldens):
    from dart_mpc.arm import pack_params, pack_snapshot
    g = arm_goldens
    s, p = _unpack(g["snap"][3], g["prm"][3])
    assert np.array_equal(pack_snapshot({k: np.asarray(v)[None] for k, v in s.items()})[0], g["snap"][3])
    assert np.array_equal(pack_params(p), g["prm"][3])
    assert g["snap"].shape[1] == 7 * 7 + 16 * 7 + 45 and g["prm"].shape[1] == 3 * 49 + 42 + 73
