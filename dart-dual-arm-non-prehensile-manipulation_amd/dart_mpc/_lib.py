"""ctypes binding of libdartmpc.so (the C ABI declared in include/dart_mpc.h).

The product path has exactly one implementation: the HIP kernel in this
library.  There is no CPU fallback -- if the library or a GPU is missing,
every solve raises ``DartMPCError``.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import subprocess
import threading
import weakref

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
# DART_MPC_LIB: file name of an alternative in-tree build.  The product path loads only a library built from the
# sources beside it (build_id below): the product library itself, or a diagnostic build of the same sources
# (phase stamps, restoration trace).  A/B timing of two different builds (tools/ab_lib.sh) must say so with
# DART_MPC_AB=1, which only the A/B tools set.
LIB_NAME = os.path.basename(os.environ.get("DART_MPC_LIB", "libdartmpc.so"))
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)

SOLVED, ACCEPTABLE, INFEASIBLE, MAXITER, LS_FAIL, INERTIA_FAIL, MAXTIME = 0, 1, 2, -1, -2, -3, -4
STATUS_NAMES = {SOLVED: "Solve_Succeeded", ACCEPTABLE: "Solved_To_Acceptable_Level", INFEASIBLE: "Infeasible_Problem_Detected",
                MAXITER: "Maximum_Iterations_Exceeded", LS_FAIL: "Restoration_Failed",
                INERTIA_FAIL: "Error_In_Step_Computation", MAXTIME: "Maximum_CpuTime_Exceeded"}

# exported symbols of include/dart_mpc.h (tests check every one is present)
EXPORTS = ("dart_mpc_config_default", "dart_mpc_create", "dart_mpc_solve_batch", "dart_mpc_solve_batch_dev",
           "dart_mpc_sync", "dart_mpc_last_error", "dart_mpc_destroy", "dart_mpc_nw", "dart_mpc_abi_version",
           "dart_rmpc_solve_batch", "dart_rmpc_solve_batch_dev", "dart_rmpc_nw",
           "dart_rls_update_batch", "dart_rls_update_batch_dev",
           "dart_lmpc_solve_batch", "dart_lmpc_solve_batch_dev", "dart_lmpc_nw",
           "dart_lmpc_policy_config_default", "dart_lmpc_policy_step", "dart_lmpc_policy_step_dev",
           "dart_lmpc_policy_solve_batch", "dart_lmpc_policy_solve_batch_dev",
           "dart_arm_config_default", "dart_arm_snapshot_len", "dart_arm_param_len", "dart_arm_solve_batch",
           "dart_arm_solve_batch_dev", "dart_set_device", "dart_mpc_serve_start", "dart_mpc_serve_stop",
           "dart_mpc_serve_running", "dart_mpc_bind", "dart_mpc_solve_bound", "dart_mpc_build_id",
           "dart_mpc_build_flavor")
VARIANT_PMPC, VARIANT_RMPC, VARIANT_LMPC = 0, 1, 2
ABI_VERSION = 8


class DartMPCError(RuntimeError):
    pass


class Config(ctypes.Structure):
    """Mirror of ``struct dart_mpc_config``."""
    _fields_ = [("variant", ctypes.c_int32), ("N", ctypes.c_int32), ("Ts", ctypes.c_double),
                ("tol", ctypes.c_double), ("max_iter", ctypes.c_int32), ("B_max", ctypes.c_int32),
                ("gravity", ctypes.c_double), ("acceptable_tol", ctypes.c_double),
                ("acceptable_iter", ctypes.c_int32), ("max_soc", ctypes.c_int32), ("pmpc_path", ctypes.c_int32),
                ("restoration", ctypes.c_int32), ("constr_mult_init_max", ctypes.c_double),
                ("max_cpu_time", ctypes.c_double)]


_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)
_lib = None


def build(verbose: bool = False) -> str:
    """Compile libdartmpc.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    r = subprocess.run(["make", "-j6", "-C", CSRC_DIR], capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise DartMPCError("building libdartmpc.so failed:\n" + (r.stdout or "") + (r.stderr or ""))
    return LIB_PATH


def source_build_id() -> str:
    """SHA-1 (first 16 hex digits) of the library's sources as the Makefile computes it: the SRC then HDR files."""
    import hashlib
    import re
    mk = open(os.path.join(CSRC_DIR, "Makefile")).read()
    files = []
    for var in ("SRC", "HDR"):
        m = re.search(r"^%s := (.*)$" % var, mk, re.M)
        files += m.group(1).split()
    h = hashlib.sha1()
    for f in files:
        with open(os.path.join(CSRC_DIR, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _check_build(L):
    """Refuse a library that was not built from the sources beside it (unless an A/B run says otherwise)."""
    if not hasattr(L, "dart_mpc_build_id"):
        if os.environ.get("DART_MPC_AB") == "1":
            return
        raise DartMPCError(f"{LIB_PATH} predates the build identity: rebuild it (make -C {CSRC_DIR})")
    L.dart_mpc_build_id.restype = ctypes.c_char_p
    L.dart_mpc_build_flavor.restype = ctypes.c_char_p
    got, want = L.dart_mpc_build_id().decode(), source_build_id()
    flavor = L.dart_mpc_build_flavor().decode()
    if os.path.basename(LIB_PATH) == "libdartmpc.so" and flavor:
        raise DartMPCError(f"{LIB_PATH} is a diagnostic ({flavor}) build, not the product library")
    if got != want and os.environ.get("DART_MPC_AB") != "1":
        raise DartMPCError(f"{LIB_PATH} was built from other sources (build id {got}, sources {want}): "
                           f"stale build, run __graft_entry__.build() or `make -C {CSRC_DIR}`")


def lib():
    """Load the library (no compute).  Raises if it is missing or stale."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DartMPCError(f"{LIB_PATH} not built: run __graft_entry__.build() or `make -C {CSRC_DIR}`")
    # One HIP runtime per process: libamdhip64.so.7 is the SONAME of both the system ROCm runtime and
    # the one torch bundles, and the first one loaded serves both.  torch only works on its own, so
    # load torch first when it is installed (it is the device-memory / stream plumbing of the
    # package); our library then binds to the same runtime.
    # (DART_MPC_NO_TORCH=1: a process that never uses torch -- a controller worker -- skips it)
    if os.environ.get("DART_MPC_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:     # pragma: no cover - the C ABI works without torch
            pass
    L = ctypes.CDLL(LIB_PATH)
    L.dart_mpc_config_default.argtypes = [ctypes.POINTER(Config)]
    L.dart_mpc_config_default.restype = None
    L.dart_mpc_create.argtypes = [ctypes.POINTER(Config), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.dart_mpc_create.restype = ctypes.c_int
    sig = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.dart_mpc_solve_batch.argtypes = sig
    L.dart_mpc_solve_batch.restype = ctypes.c_int
    L.dart_mpc_solve_batch_dev.argtypes = sig
    L.dart_mpc_solve_batch_dev.restype = ctypes.c_int
    L.dart_mpc_sync.argtypes = [ctypes.c_void_p]
    L.dart_mpc_sync.restype = ctypes.c_int
    L.dart_mpc_last_error.argtypes = [ctypes.c_void_p]
    L.dart_mpc_last_error.restype = ctypes.c_char_p
    L.dart_mpc_destroy.argtypes = [ctypes.c_void_p]
    L.dart_mpc_destroy.restype = None
    L.dart_mpc_nw.argtypes = [ctypes.c_int]
    L.dart_mpc_nw.restype = ctypes.c_int
    L.dart_mpc_abi_version.argtypes = []
    L.dart_mpc_abi_version.restype = ctypes.c_int
    rsig = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_double] + [ctypes.c_void_p] * 9
    L.dart_rmpc_solve_batch.argtypes = rsig
    L.dart_rmpc_solve_batch.restype = ctypes.c_int
    L.dart_rmpc_solve_batch_dev.argtypes = rsig
    L.dart_rmpc_solve_batch_dev.restype = ctypes.c_int
    L.dart_rmpc_nw.argtypes = [ctypes.c_int]
    L.dart_rmpc_nw.restype = ctypes.c_int
    lsig = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 12
    L.dart_lmpc_solve_batch.argtypes = lsig
    L.dart_lmpc_solve_batch.restype = ctypes.c_int
    L.dart_lmpc_solve_batch_dev.argtypes = lsig
    L.dart_lmpc_solve_batch_dev.restype = ctypes.c_int
    L.dart_lmpc_nw.argtypes = [ctypes.c_int]
    L.dart_lmpc_nw.restype = ctypes.c_int
    L.dart_lmpc_policy_config_default.argtypes = [ctypes.c_void_p]
    L.dart_lmpc_policy_config_default.restype = None
    L.dart_lmpc_policy_step.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 13
    L.dart_lmpc_policy_step.restype = ctypes.c_int
    L.dart_lmpc_policy_step_dev.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 14
    L.dart_lmpc_policy_step_dev.restype = ctypes.c_int
    psig = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 21
    L.dart_lmpc_policy_solve_batch.argtypes = psig
    L.dart_lmpc_policy_solve_batch.restype = ctypes.c_int
    L.dart_lmpc_policy_solve_batch_dev.argtypes = psig
    L.dart_lmpc_policy_solve_batch_dev.restype = ctypes.c_int
    L.dart_rls_update_batch.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_double]
    L.dart_rls_update_batch.restype = ctypes.c_int
    L.dart_rls_update_batch_dev.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_double, ctypes.c_void_p]
    L.dart_rls_update_batch_dev.restype = ctypes.c_int
    L.dart_arm_config_default.argtypes = [ctypes.c_void_p]
    L.dart_arm_config_default.restype = None
    L.dart_arm_snapshot_len.argtypes = [ctypes.c_int]
    L.dart_arm_snapshot_len.restype = ctypes.c_int
    L.dart_arm_param_len.argtypes = [ctypes.c_int]
    L.dart_arm_param_len.restype = ctypes.c_int
    L.dart_arm_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int] + [ctypes.c_void_p] * 5
    L.dart_arm_solve_batch.restype = ctypes.c_int
    L.dart_arm_solve_batch_dev.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 6
    L.dart_arm_solve_batch_dev.restype = ctypes.c_int
    if hasattr(L, "dart_mpc_bind"):         # (absent only in older in-tree builds used for A/B timing)
        L.dart_mpc_bind.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 9
        L.dart_mpc_bind.restype = ctypes.c_int
        L.dart_mpc_solve_bound.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.dart_mpc_solve_bound.restype = ctypes.c_int
    if hasattr(L, "dart_mpc_serve_start"):  # (absent only in older in-tree builds used for A/B timing)
        L.dart_mpc_serve_start.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double]
        L.dart_mpc_serve_start.restype = ctypes.c_int
        L.dart_mpc_serve_stop.argtypes = [ctypes.c_void_p]
        L.dart_mpc_serve_stop.restype = ctypes.c_int
        L.dart_mpc_serve_running.argtypes = [ctypes.c_void_p]
        L.dart_mpc_serve_running.restype = ctypes.c_int
    if hasattr(L, "dart_set_device"):       # (absent only in older in-tree builds used for A/B timing)
        L.dart_set_device.argtypes = [ctypes.c_int]
        L.dart_set_device.restype = ctypes.c_int
    if L.dart_mpc_abi_version() != ABI_VERSION:
        raise DartMPCError("libdartmpc.so ABI version mismatch")
    _check_build(L)
    _lib = L
    return L


def set_device(device: int):
    """Select the device of the stateless entries (RLS, policy step, arm QP) for this thread."""
    rc = lib().dart_set_device(int(device))
    if rc != 0:
        raise DartMPCError(f"dart_set_device({device}) failed ({rc})")


def wave_selftest():
    """Run the internal wave-primitive self-test kernel (DPP shifts and reductions) on device 0."""
    L = lib()
    L.dartmpc_selftest.argtypes = [ctypes.c_void_p]
    L.dartmpc_selftest.restype = ctypes.c_int
    out = np.zeros(265)
    rc = L.dartmpc_selftest(ctypes.c_void_p(out.ctypes.data))
    if rc != 0:
        raise DartMPCError(f"dartmpc_selftest failed ({rc})")
    return out


def default_config(**over) -> Config:
    c = Config()
    lib().dart_mpc_config_default(ctypes.byref(c))
    for k, v in over.items():
        setattr(c, k, v)
    return c


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


# Handles still open at interpreter exit are destroyed by an atexit hook, before the HIP runtime's own teardown:
# a handle freed later, from a finaliser, would free device memory through a runtime that is already gone.
_LIVE = weakref.WeakSet()


@atexit.register
def _close_live_handles():
    for s in list(_LIVE):
        try:
            s.close()
        except Exception:
            pass


class Solver:
    """Owns one ``dart_mpc_handle`` (device workspace + stream) for a fixed N/Ts/tol.  ``max_soc`` is
    IPOPT's second-order-correction count (default 4, as ``mpc_3d.py:82`` leaves it; 0 = off).
    ``path``: "ipopt" (default) follows IPOPT's iterates on the full 6-state NLP; "reduced" is the
    faster opt-in that solves the (x, y) problem and rolls z out afterwards (same KKT point).
    ``restoration``: IPOPT's soft restoration and restoration phases after a failed filter line search
    (IPOPT's path, N <= 31; pmpc_resto.hip); off, or on the reduced path or beyond N = 31, such an instance
    ends at status -2."""

    PATHS = {"ipopt": 0, "reduced": 1}

    def __init__(self, N=20, Ts=0.002, tol=1e-8, max_iter=3000, B_max=1024, device=0, gravity=-9.81, max_soc=4,
                 path="ipopt", constr_mult_init_max=1000.0, restoration=True):
        self._h = ctypes.c_void_p()
        if path not in self.PATHS:
            raise DartMPCError(f"unknown PMPC path {path!r} (expected one of {sorted(self.PATHS)})")
        self.cfg = default_config(N=int(N), Ts=float(Ts), tol=float(tol), max_iter=int(max_iter), B_max=int(B_max),
                                  gravity=float(gravity), max_soc=int(max_soc), pmpc_path=self.PATHS[path],
                                  constr_mult_init_max=float(constr_mult_init_max),
                                  restoration=int(bool(restoration)))
        rc = lib().dart_mpc_create(ctypes.byref(self.cfg), int(device), ctypes.byref(self._h))
        _LIVE.add(self)
        if rc != 0:
            raise DartMPCError(f"dart_mpc_create failed with code {rc} (no gfx950 device or bad config)")
        self.N = int(N)
        self.nw = lib().dart_mpc_nw(self.N)

    def _err(self, rc, what):
        msg = lib().dart_mpc_last_error(self._h)
        raise DartMPCError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def solve_batch(self, x0, ref, prm, w_warm=None, want_w=False, out=None):
        """Host arrays in, host arrays out (blocking).  Returns dict(u0, f, w, status, iters).
        ``out``: a dict of preallocated u0[B,2], f[B], status[B] (int32), iters[B] (int32) and, with
        want_w, w[B,nw] arrays that are filled and returned instead of fresh ones."""
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 6)
        B = x0.shape[0]
        if out is not None:
            self._check_out(out, B, want_w)
        if w_warm is None and not want_w and B > 0:
            return self._solve_staged(B, x0, ref, prm, out)
        ref = np.ascontiguousarray(ref, np.float64).reshape(B, 6)
        prm = np.ascontiguousarray(prm, np.float64).reshape(B, 6)
        ww = None if w_warm is None else np.ascontiguousarray(w_warm, np.float64).reshape(B, self.nw)
        if out is not None:
            u0, f, st, it = out["u0"], out["f"], out["status"], out["iters"]
            w = out.get("w") if want_w else None
        else:
            u0 = np.empty((B, 2)); f = np.empty(B)
            w = np.empty((B, self.nw)) if want_w else None
            st = np.empty(B, np.int32); it = np.empty(B, np.int32)
        rc = lib().dart_mpc_solve_batch(self._h, B, _ptr(x0), _ptr(ref), _ptr(prm), _ptr(ww), _ptr(u0), _ptr(f),
                                        _ptr(w), _ptr(st), _ptr(it), None)
        if rc != 0:
            self._err(rc, "dart_mpc_solve_batch")
        return dict(u0=u0, f=f, w=w, status=st, iters=it)

    def _check_out(self, out, B, want_w):
        """out= arrays: shapes of the batch, float64 u0 / f (/ w), int32 status / iters, C-contiguous."""
        u0, f, st, it = out["u0"], out["f"], out["status"], out["iters"]
        if (u0.shape != (B, 2) or f.shape != (B,) or st.shape != (B,) or it.shape != (B,) or u0.dtype != np.float64
                or f.dtype != np.float64 or st.dtype != np.int32 or it.dtype != np.int32
                or not all(a.flags.c_contiguous for a in (u0, f, st, it))):
            raise DartMPCError("out= arrays do not match the batch")
        if want_w:
            w = out.get("w")
            if w is None or w.shape != (B, self.nw) or w.dtype != np.float64 or not w.flags.c_contiguous:
                raise DartMPCError("out['w'] must be a C-contiguous float64 [B, nw] array when want_w")

    def _solve_staged(self, B, x0, ref, prm, out):
        """Cold-start call without w: inputs copied into per-batch-size buffers whose pointers are
        cached (building ctypes pointers costs ~1 us each, a third of the Python side of a call)."""
        cache = self.__dict__.setdefault("_staged", {})
        st_ = cache.get(B)
        if st_ is None:
            if len(cache) >= 8:
                cache.clear()
            bufs = (np.empty((B, 6)), np.empty((B, 6)), np.empty((B, 6)), np.empty((B, 2)), np.empty(B),
                    np.empty(B, np.int32), np.empty(B, np.int32))
            st_ = cache[B] = (bufs, tuple(b.ctypes.data for b in bufs), threading.Lock())
        (bx, br, bp, bu, bf, bs, bi), (px, pr, pp, pu, pf, ps, pi), lock = st_
        with lock:
            np.copyto(bx, x0)
            np.copyto(br, np.reshape(ref, (B, 6)))
            np.copyto(bp, np.reshape(prm, (B, 6)))
            rc = lib().dart_mpc_solve_batch(self._h, B, px, pr, pp, None, pu, pf, None, ps, pi, None)
            if rc != 0:
                self._err(rc, "dart_mpc_solve_batch")
            if out is not None:
                for k, src in (("u0", bu), ("f", bf), ("status", bs), ("iters", bi)):
                    np.copyto(out[k], src)
                return dict(u0=out["u0"], f=out["f"], w=None, status=out["status"], iters=out["iters"])
            return dict(u0=bu.copy(), f=bf.copy(), w=None, status=bs.copy(), iters=bi.copy())

    def solve_one(self, x0, ref, prm, want_w=False):
        """One instance (the per-control-step call of PMPC.solve / mpc_worker): the rows are copied
        into buffers allocated once, whose pointers are cached, so the Python side of a call is a few
        slice copies and one ctypes call.  Returns (u0[2], f, status, iters, w or None); the arrays
        are fresh copies."""
        one = getattr(self, "_one", None)
        if one is None:
            bufs = [np.empty(6), np.empty(6), np.empty(6), np.empty(2), np.empty(1), np.empty(self.nw),
                    np.empty(1, np.int32), np.empty(1, np.int32)]
            one = self._one = (threading.Lock(), bufs, [_ptr(b) for b in bufs])
        lock, (bx, br, bp, bu, bf, bw, bs, bi), ptrs = one
        with lock:
            bx[:] = x0; br[:] = ref; bp[:] = prm
            rc = lib().dart_mpc_solve_batch(self._h, 1, ptrs[0], ptrs[1], ptrs[2], None, ptrs[3], ptrs[4],
                                            ptrs[5] if want_w else None, ptrs[6], ptrs[7], None)
            if rc != 0:
                self._err(rc, "dart_mpc_solve_batch")
            return bu.copy(), float(bf[0]), int(bs[0]), int(bi[0]), (bw.copy() if want_w else None)

    def solve_batch_dev(self, B, x0, ref, prm, u0, f, status, iters, w_warm=0, w_out=0, stream=0):
        """Device pointers (ints) in/out, asynchronous on ``stream`` (an int hipStream_t, 0 = own)."""
        rc = lib().dart_mpc_solve_batch_dev(self._h, int(B), x0, ref, prm, w_warm or None, u0, f, w_out or None,
                                            status, iters, stream or None)
        if rc != 0:
            self._err(rc, "dart_mpc_solve_batch_dev")

    def sync(self):
        rc = lib().dart_mpc_sync(self._h)
        if rc != 0:
            self._err(rc, "dart_mpc_sync")

    # -- resident solver (PMPC, IPOPT's path, N <= 31): dart_mpc_serve_start / _stop / _running ----
    def serve_start(self, B_serve=18, idle_timeout=1.0):
        """Keep a grid of ``B_serve`` waves resident; later ``solve_batch`` / ``solve_one`` calls with
        B <= B_serve are served without a kernel launch (bit-identical results)."""
        rc = lib().dart_mpc_serve_start(self._h, int(B_serve), float(idle_timeout))
        if rc != 0:
            self._err(rc, "dart_mpc_serve_start")
        return self

    def serve_stop(self):
        rc = lib().dart_mpc_serve_stop(self._h)
        if rc != 0:
            self._err(rc, "dart_mpc_serve_stop")

    def serving(self):
        return bool(lib().dart_mpc_serve_running(self._h))

    def bind(self):
        """In-place I/O (dart_mpc_bind): a ``Bound`` whose numpy views live in the handle's mapped, pinned
        I/O area.  Write the inputs of the first B rows, call ``bound.solve(B)``, read the outputs: no
        copies and a two-argument ctypes call per solve."""
        b = getattr(self, "_bound", None)
        if b is None:
            b = self._bound = Bound(self)
        return b

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        if self._h:
            lib().dart_mpc_destroy(self._h)      # stops a resident grid first
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Bound:
    """Views of a PMPC handle's in-place I/O area for B_max instances (Solver.bind)."""

    def __init__(self, solver):
        ptrs = [ctypes.c_void_p() for _ in range(9)]
        rc = lib().dart_mpc_bind(solver._h, *[ctypes.byref(p) for p in ptrs])
        if rc != 0:
            solver._err(rc, "dart_mpc_bind")
        Bm, nw = int(solver.cfg.B_max), solver.nw

        def view(p, shape, ct):
            n = int(np.prod(shape))
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ct)), shape=(n,)).reshape(shape)

        d = ctypes.c_double
        self.x0, self.ref, self.prm = view(ptrs[0], (Bm, 6), d), view(ptrs[1], (Bm, 6), d), view(ptrs[2], (Bm, 6), d)
        self.w_warm = view(ptrs[3], (Bm, nw), d)
        self.u0, self.f, self.w_out = view(ptrs[4], (Bm, 2), d), view(ptrs[5], (Bm,), d), view(ptrs[6], (Bm, nw), d)
        self.status, self.iters = view(ptrs[7], (Bm,), ctypes.c_int32), view(ptrs[8], (Bm,), ctypes.c_int32)
        self._solver = solver
        self._fn = lib().dart_mpc_solve_bound
        self._h = solver._h

    def solve(self, B, w_warm=False, want_w=False):
        rc = self._fn(self._h, B, (1 if w_warm else 0) | (2 if want_w else 0))
        if rc != 0:
            self._solver._err(rc, "dart_mpc_solve_bound")


class RmpcSolver(Solver):
    """``dart_mpc_handle`` of variant RMPC (regressor NMPC + fused RLS), N <= 63 (N > 31: the two-wave build).  Defaults are the
    reference's options (np_mpc...:158-162: max_iter 200) and IPOPT's: constr_mult_init_max 1000, its soft
    restoration / restoration phases after a failed line search (restoration=False: status -2 there; a measured
    |v| above vmax at the pinned node 0 ends at status 2 with them) and max_soc 4 in the restoration phase."""

    def __init__(self, N=20, Ts=0.002, tol=1e-8, max_iter=200, B_max=1024, device=0, gravity=-9.81,
                 constr_mult_init_max=1000.0, restoration=True, max_soc=4):
        self._h = ctypes.c_void_p()
        self.cfg = default_config(variant=VARIANT_RMPC, N=int(N), Ts=float(Ts), tol=float(tol),
                                  max_iter=int(max_iter), B_max=int(B_max), gravity=float(gravity),
                                  constr_mult_init_max=float(constr_mult_init_max),
                                  restoration=int(bool(restoration)), max_soc=int(max_soc))
        rc = lib().dart_mpc_create(ctypes.byref(self.cfg), int(device), ctypes.byref(self._h))
        _LIVE.add(self)
        if rc != 0:
            raise DartMPCError(f"dart_mpc_create(RMPC) failed with code {rc} (no gfx950 device or bad config)")
        self.N = int(N)
        self.nw = lib().dart_rmpc_nw(self.N)

    def solve_batch(self, x0, u_prev, theta, Rref, prm, w_warm=None, want_w=False, rls_P=None, rls_phi=None,
                    rls_y=None, rls_lambda=0.995):
        """Host arrays in/out (blocking).  With ``rls_P`` the RLS update is fused: ``theta`` and
        ``rls_P`` are updated in place (returned in the dict as well)."""
        c = lambda a, n: np.ascontiguousarray(a, np.float64).reshape(-1, n)
        x0 = c(x0, 4)
        B = x0.shape[0]
        u_prev, theta, Rref, prm = c(u_prev, 2), c(theta, 14).copy(), c(Rref, 4 * (self.N + 1)), c(prm, 10)
        ww = None if w_warm is None else c(w_warm, self.nw)
        P = phi = y = None
        if rls_P is not None:
            P = np.ascontiguousarray(rls_P, np.float64).reshape(B, 2, 7, 7).copy()
            phi, y = c(rls_phi, 7), c(rls_y, 2)
        u0 = np.empty((B, 2)); f = np.empty(B)
        w = np.empty((B, self.nw)) if want_w else None
        st = np.empty(B, np.int32); it = np.empty(B, np.int32)
        rc = lib().dart_rmpc_solve_batch(self._h, B, _ptr(x0), _ptr(u_prev), _ptr(theta), _ptr(P), _ptr(phi), _ptr(y),
                                         float(rls_lambda), _ptr(Rref), _ptr(prm), _ptr(ww), _ptr(u0), _ptr(f),
                                         _ptr(w), _ptr(st), _ptr(it), None)
        if rc != 0:
            self._err(rc, "dart_rmpc_solve_batch")
        return dict(u0=u0, f=f, w=w, status=st, iters=it, theta=theta, rls_P=P)

    def solve_batch_dev(self, B, x0, u_prev, theta, Rref, prm, u0, f, status, iters, w_warm=0, w_out=0,
                        rls_P=0, rls_phi=0, rls_y=0, rls_lambda=0.995, stream=0):
        rc = lib().dart_rmpc_solve_batch_dev(self._h, int(B), x0, u_prev, theta, rls_P or None, rls_phi or None,
                                             rls_y or None, float(rls_lambda), Rref, prm, w_warm or None, u0, f,
                                             w_out or None, status, iters, stream or None)
        if rc != 0:
            self._err(rc, "dart_rmpc_solve_batch_dev")


LMPC_PRM_DEFAULT = np.array([200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0,     # Q   LMPC/src/run.py:118
                             200.0, 2.0, 200.0, 2.0, 0.0, 0.0, 0.0, 0.0,     # Qt  :119
                             0.1, 0.1, 1.0, 1.0,                             # R   :120
                             -0.4, 0.4])                                     # u_bounds :121


class LmpcSolver(Solver):
    """``dart_mpc_handle`` of variant LMPC, N <= 63 (N > 31: the two-wave build).  Defaults are the reference's IPOPT options
    (LMPC/src/controller/rlmpc2.py:480-489): max_iter 50, tol 1e-4, acceptable_tol 1e-3,
    acceptable_iter 5, and IPOPT's defaults max_soc 4 (second-order correction; 0 = off),
    constr_mult_init_max 1000 (least-square starting multipliers; 0 = start from 0) and its soft
    restoration / restoration phases after a failed line search (restoration=False: status -2 there);
    max_cpu_time 0.05 s (rlmpc2.py:485; status -4 past it, measured per instance on the GPU clock; 0 = off)."""

    def __init__(self, N=20, Ts=0.002, tol=1e-4, max_iter=50, acceptable_tol=1e-3, acceptable_iter=5,
                 B_max=1024, device=0, max_soc=4, constr_mult_init_max=1000.0, restoration=True, max_cpu_time=0.05):
        self._h = ctypes.c_void_p()
        self.cfg = default_config(variant=VARIANT_LMPC, N=int(N), Ts=float(Ts), tol=float(tol), max_iter=int(max_iter),
                                  B_max=int(B_max), acceptable_tol=float(acceptable_tol),
                                  acceptable_iter=int(acceptable_iter), max_soc=int(max_soc),
                                  constr_mult_init_max=float(constr_mult_init_max),
                                  restoration=int(bool(restoration)), max_cpu_time=float(max_cpu_time))
        rc = lib().dart_mpc_create(ctypes.byref(self.cfg), int(device), ctypes.byref(self._h))
        _LIVE.add(self)
        if rc != 0:
            raise DartMPCError(f"dart_mpc_create(LMPC) failed with code {rc} (no gfx950 device or bad config)")
        self.N = int(N)
        self.nw = lib().dart_lmpc_nw(self.N)

    def solve_batch(self, state, u_prev, pvec, target, prm=None, w_warm=None, want_w=False):
        c = lambda a, n: np.ascontiguousarray(a, np.float64).reshape(-1, n)
        state = c(state, 8)
        B = state.shape[0]
        u_prev, pvec, target = c(u_prev, 2), c(pvec, 34), c(target, 8)
        prm = c(np.tile(LMPC_PRM_DEFAULT, (B, 1)) if prm is None else prm, 22)
        ww = None if w_warm is None else c(w_warm, self.nw)
        u0 = np.empty((B, 2)); f = np.empty(B)
        w = np.empty((B, self.nw)) if want_w else None
        st = np.empty(B, np.int32); it = np.empty(B, np.int32)
        rc = lib().dart_lmpc_solve_batch(self._h, B, _ptr(state), _ptr(u_prev), _ptr(pvec), _ptr(target), _ptr(prm),
                                         _ptr(ww), _ptr(u0), _ptr(f), _ptr(w), _ptr(st), _ptr(it), None)
        if rc != 0:
            self._err(rc, "dart_lmpc_solve_batch")
        return dict(u0=u0, f=f, w=w, status=st, iters=it)

    def solve_batch_dev(self, B, state, u_prev, pvec, target, prm, u0, f, status, iters, w_warm=0, w_out=0, stream=0):
        rc = lib().dart_lmpc_solve_batch_dev(self._h, int(B), state, u_prev, pvec, target, prm, w_warm or None, u0, f,
                                             w_out or None, status, iters, stream or None)
        if rc != 0:
            self._err(rc, "dart_lmpc_solve_batch_dev")

    def policy_solve_batch_dev(self, pcfg, B, weights, state, u_prev, target, current_k, obs_mean, obs_M2, obs_count,
                               history, timestep, noise, model_params, prm, u0, f, status, iters, action_out=0,
                               w_warm=0, w_out=0, stream=0):
        """Fused policy step + solve (dart_lmpc_policy_solve_batch_dev), device pointers, asynchronous;
        ``pcfg`` is a ``dart_mpc.lmpc.PolicyConfig``."""
        rc = lib().dart_lmpc_policy_solve_batch_dev(
            self._h, ctypes.byref(pcfg), int(B), weights, state, u_prev, target, current_k, obs_mean, obs_M2, obs_count,
            history, timestep, noise, model_params, action_out or None, prm, w_warm or None, u0, f, w_out or None,
            status, iters, stream or None)
        if rc != 0:
            self._err(rc, "dart_lmpc_policy_solve_batch_dev")


def rls_update_batch(theta, P, phi, y, lam=0.995):
    """Batched RLS.update on the GPU (B filters of p = 7).  Returns updated (theta[B,7], P[B,7,7])."""
    th = np.ascontiguousarray(theta, np.float64).reshape(-1, 7).copy()
    B = th.shape[0]
    Pm = np.ascontiguousarray(P, np.float64).reshape(B, 7, 7).copy()
    ph = np.ascontiguousarray(phi, np.float64).reshape(B, 7)
    yy = np.ascontiguousarray(y, np.float64).reshape(B)
    rc = lib().dart_rls_update_batch(B, _ptr(th), _ptr(Pm), _ptr(ph), _ptr(yy), float(lam))
    if rc != 0:
        raise DartMPCError(f"dart_rls_update_batch failed ({rc})")
    return th, Pm
