"""LMPC with the reference's process topology: shared-memory arrays, Events, two GPU workers.

The reference LMPC controller (LMPC/src/controller/rlmpc2.py) is three processes around
``multiprocessing.shared_memory`` arrays (keys and shapes :115-128) and five Events (:143-149):

  * the simulation process calls ``RLMPC.solve(target)`` (:986-1021): it writes state and target,
    sets ``state_ready`` and, without waiting, takes the newest solution when ``ctrl_ready`` is set;
    otherwise it shifts the previous plan by one node (:1013-1018) or holds the last control;
  * ``RLMPC._solver_worker`` (:229-533) waits on ``state_ready`` with a 10 ms timeout (:496), reads
    state, control, model_params and target, solves the NLP warm-started from its previous solution
    (:508-519) and publishes ``w_opt``, ``loss`` and ``ctrl_ready`` (:521-524);
  * ``RLMPC._rl_worker`` (:537-769) reads the same arrays on the same event, runs the parameter
    policy and every 8th step writes a new ``model_params`` vector (:742-759, :606-616).

``RLMPCAsync`` keeps that protocol message for message.  What runs inside the two workers is new:
``lmpc_solver_worker`` calls the LMPC kernel of libdartmpc (``LmpcSolver``, the reference's IPOPT
options) and ``lmpc_policy_worker`` the policy kernel (``LmpcPolicy``; inference and parameter
write only -- PPO training stays out of scope).  Each worker creates its own GPU
context after the ``spawn`` start.  The synchronous one-process variant is ``dart_mpc.RLMPC``.
"""
from __future__ import annotations

import multiprocessing as mp
from multiprocessing import shared_memory

import numpy as np

N_PARAMS = 34                                 # rlmpc2.py:178
EVENT_NAMES = ("state_ready", "ctrl_ready", "data_ready", "terminate", "reset")    # :143-149
DEFAULTS = dict(Ts=0.002, nx=8, nu=2, N=20, g=-9.81, body_name="cube2",
                Q=[200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0],        # LMPC/src/run.py:118-126
                Qt=[200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0],
                R=[0.1, 0.1, 1.0, 1.0], u_bounds=(-0.4, 0.4),
                max_param_abs=2.0, max_delta_abs=0.02)                 # run.py:139-140


def shm_shapes(nx: int, nu: int, N: int) -> dict:
    """Shared arrays of rlmpc2.py:115-128 (all float64)."""
    return {"state": (nx,), "state_next": (nx,), "target": (nx,), "w_opt": (nx * (N + 1) + nu * N,),
            "loss": (1,), "control": (nu,), "model_params": (N_PARAMS,), "state_deriv": (nx,),
            "in_contact": (1,), "RLstatus": (1,)}


def _attach(shm_names, shapes):
    shms, views = {}, {}
    for key, shape in shapes.items():
        shm = shared_memory.SharedMemory(name=shm_names[key])
        shms[key] = shm
        views[key] = np.ndarray(shape, dtype=np.float64, buffer=shm.buf)
    return shms, views


def _detach(shms):
    for shm in shms.values():
        try:
            shm.close()
        except Exception:       # pragma: no cover - views may still reference the buffer
            pass


def write_params(prev, k_new, min_k, k_max, k_ceiling_margin, alpha=0.5):
    """write_params_to_shm (:606-616): EMA with the shared vector, then the tanh soft clip."""
    sm = alpha * np.asarray(k_new, np.float64) + (1 - alpha) * np.asarray(prev, np.float64)
    lo, hi = min_k, k_max - k_ceiling_margin
    c, s = (hi + lo) / 2, (hi - lo) / 2 - 1e-3
    return c + s * np.tanh((sm - c) / s)


def lmpc_solver_worker(shm_names, events, packet, shapes):
    """Replaces RLMPC._solver_worker (:229-533): same loop, the solve runs on the GPU."""
    shms, views = _attach(shm_names, shapes)
    try:
        from ._lib import LmpcSolver
        solver = LmpcSolver(N=int(packet["N"]), Ts=float(packet["Ts"]), B_max=1, device=int(packet.get("device", 0)))
        prm = np.concatenate([packet["Q"], packet["Qt"], packet["R"], packet["u_bounds"]]).astype(np.float64)[None]
        w0 = np.zeros(shapes["w_opt"])                                 # :492
        while True:
            events["state_ready"].wait(timeout=0.01)                   # :496
            if events["terminate"].is_set():
                break
            events["state_ready"].clear()
            state = views["state"].copy()
            target = views["target"].copy()
            control = views["control"].copy()
            pvec = views["model_params"].copy()
            out = solver.solve_batch(state[None], control[None], pvec[None], target[None], prm, w_warm=w0[None],
                                     want_w=True)                      # :508-519, warm start x0 = w0
            w0 = out["w"][0]
            views["w_opt"][:] = w0
            views["loss"][:] = out["f"]
            events["ctrl_ready"].set()                                 # :524
        solver.close()
    finally:
        _detach(shms)


def lmpc_policy_worker(shm_names, events, packet, shapes):
    """Replaces the inference / parameter-write half of RLMPC._rl_worker (:537-769)."""
    shms, views = _attach(shm_names, shapes)
    try:
        from ._lib import set_device
        set_device(int(packet.get("device", 0)))    # the stateless policy entry runs on the current device
        from .lmpc import LmpcPolicy
        k_max = float(packet.get("max_param_abs", DEFAULTS["max_param_abs"]))
        margin = float(packet.get("k_ceiling_margin", max(1e-3, 0.05 * k_max)))             # :589
        min_k = float(packet.get("min_k", 1e-2))
        pol = LmpcPolicy(1, weights=packet.get("policy_weights"), seed=int(packet.get("seed", 0)), k_max=k_max,
                         max_delta=float(packet.get("max_delta_abs", DEFAULTS["max_delta_abs"])),
                         k_ceiling_margin=margin, min_k=min_k)
        # :618-623: current_k at mid-range with jitter, written through the EMA + soft clip
        views["model_params"][:] = write_params(views["model_params"], pol.current_k[0], min_k, k_max, margin)
        rng = np.random.default_rng(packet.get("noise_seed"))
        while True:
            if events["terminate"].is_set():                           # :635-639
                break
            events["state_ready"].wait(timeout=0.01)
            if events["terminate"].is_set():
                break
            state = views["state"].copy()
            target = views["target"].copy()
            control = views["control"].copy()
            pol.model_params[0] = views["model_params"]                # the shared vector is the truth (:746)
            pol.step(state, target, control, noise=rng.standard_normal((1, N_PARAMS)))
            views["model_params"][:] = pol.model_params[0]
    finally:
        _detach(shms)


class RLMPCAsync:
    """RLMPC (:110-226, :986-1021) with its solver and policy processes on the GPU.

    ``params`` takes the reference's keys (Ts, nx, nu, N, Q, Qt, R, u_bounds, max_param_abs,
    max_delta_abs, body_name, ...); the defaults are those of LMPC/src/run.py.  ``solve(target)``
    never blocks: it returns the newest plan's first control, the shifted previous plan, or the last
    control, exactly as the reference front-end does."""

    def __init__(self, model=None, data=None, params=None, *, policy=True, policy_weights=None, seed=0, device=0,
                 solver_worker=None, policy_worker=None):
        p = dict(DEFAULTS)
        p.update(params or {})
        if int(p["nx"]) != 8 or int(p["nu"]) != 2:
            raise ValueError("the LMPC model is defined for nx=8, nu=2 (rlmpc2.py:260-429)")
        self.model, self.data, self.params = model, data, p
        self.N, self.nx, self.nu = int(p["N"]), int(p["nx"]), int(p["nu"])
        self.shapes = shm_shapes(self.nx, self.nu, self.N)
        self.shms, self.views = {}, {}
        for key, shape in self.shapes.items():
            shm = shared_memory.SharedMemory(create=True, size=int(np.prod(shape)) * 8)
            self.shms[key] = shm
            self.views[key] = np.ndarray(shape, dtype=np.float64, buffer=shm.buf)
            self.views[key][:] = 0.0
        self.shm_names = {k: v.name for k, v in self.shms.items()}
        rng = np.random.default_rng(seed)
        self.views["control"][:] = 0.0                                                      # :139
        self.views["model_params"][:] = rng.uniform(0, float(p["max_param_abs"]) / 2, N_PARAMS)   # :140
        self.last_control = np.zeros(self.nu)
        self.loss = 0.0
        ctx = mp.get_context("spawn")
        self.events = {name: ctx.Event() for name in EVENT_NAMES}
        packet = dict(p, device=int(device), seed=int(seed), noise_seed=int(seed) + 2, policy_weights=policy_weights)
        self.procs = [ctx.Process(target=solver_worker or lmpc_solver_worker,
                                  args=(self.shm_names, self.events, packet, self.shapes), daemon=True)]
        if policy:
            self.procs.append(ctx.Process(target=policy_worker or lmpc_policy_worker,
                                          args=(self.shm_names, self.events, packet, self.shapes), daemon=True))
        for pr in self.procs:
            pr.start()

    def get_state(self):
        """[px, vx, py, vy, theta_x, omega_x, theta_y, omega_y] from MjData (:1034-1042)."""
        if self.data is None:
            raise RuntimeError("get_state() needs MuJoCo data; pass state= to solve()")
        from scipy.spatial.transform import Rotation as Rot
        b = self.data.body(self.params["body_name"])
        th = Rot.from_matrix(np.asarray(b.xmat).reshape(3, 3)).as_euler("xyz", degrees=False)[:2]
        return np.array([b.xpos[0], b.cvel[3], b.xpos[1], b.cvel[4], th[0], b.cvel[0], th[1], b.cvel[1]])

    def _check_workers(self):
        """A worker that died (an exception in its loop, a failed device selection) would leave solve()
        shifting or holding the last plan forever: raise instead."""
        for pr in self.procs:
            if not pr.is_alive():
                from ._lib import DartMPCError
                raise DartMPCError(f"LMPC worker process {pr.name} exited (code {pr.exitcode})")

    def solve(self, target, state=None):
        """Non-blocking control step (:986-1021); returns (control[2], loss).  Raises DartMPCError when a
        worker process has died."""
        self._check_workers()
        state = self.get_state() if state is None else np.asarray(state, float)
        self.views["state"][:] = state
        self.views["target"][:] = target
        self.events["state_ready"].set()
        if self.events["ctrl_ready"].is_set():
            self.events["ctrl_ready"].clear()
            w_opt = self.views["w_opt"].copy()
            self.loss = self.views["loss"].copy()
            nX = self.nx * (self.N + 1)
            self.X_plan = w_opt[:nX].reshape(self.N + 1, self.nx)
            self.U_plan = w_opt[nX:].reshape(self.N, self.nu)
            if self.U_plan.size > 0:
                self.last_control = self.U_plan[0].astype(np.float64)
        elif hasattr(self, "U_plan") and self.U_plan.shape[0] > 1:        # shift the old plan
            self.last_control = self.U_plan[1]
            self.U_plan = self.U_plan[1:]
        self.views["control"][:] = self.last_control
        return self.last_control.copy(), self.loss

    def measure(self, state, state_deriv=None, contact=1.0):
        """The shared-array writes of RLMPC.measure (:1055-1065), with the values supplied."""
        self.views["state"][:] = state
        if state_deriv is not None:
            self.views["state_deriv"][:] = state_deriv
        self.views["in_contact"][:] = contact

    def wait_solution(self, timeout=5.0) -> bool:
        """Test / driver helper (not in the reference): block until the solver has published (raises
        DartMPCError if a worker died meanwhile)."""
        import time
        t_end = time.monotonic() + timeout
        while True:
            self._check_workers()
            left = t_end - time.monotonic()
            if self.events["ctrl_ready"].wait(min(0.05, max(0.0, left))):
                return True
            if left <= 0.0:
                return False

    def close(self):
        if not self.shms:
            return
        self.events["terminate"].set()
        for pr in self.procs:
            pr.join(timeout=10)
            if pr.is_alive():     # pragma: no cover - a hung worker
                pr.terminate()
                pr.join(timeout=5)
        self.views = {}
        for shm in self.shms.values():
            try:
                shm.close()
                shm.unlink()
            except FileNotFoundError:
                pass
        self.shms = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
