"""Benchmark: MPC solves/sec of the batched PMPC solve (BASELINE.json metric).

Workload (BASELINE.json configs[1]): PMPC, batch = 18 object
configs (3 shapes x 2 masses x 3 frictions), horizon N = 20, Ts = 0.002, fp64,
cold start, IPOPT tol 1e-8.  One step = one batched solve of 18 fresh seeded
instances whose inputs are already resident in HBM.  With --gpus N (one process
per GPU, torchrun) every rank solves its own 18-instance batch per step
(different seeds): weak scaling, no collective on the data path.

Reported roofline: the kernel is FP64-VALU / latency bound (one wave per
instance, 176 B of HBM traffic per solve); `achieved` is algorithmic FP64
FLOP/s = sum(iters) * F_iter / mean kernel time, F_iter = 6.0e4 FLOP per
IPM iteration per instance, against the 78.6 TFLOP/s FP64 peak.

cpu_baseline: the C oracle (oracle/pmpc_ipm.c: IPOPT-style filter IPM on the
full 6-state NLP), timed on rank 0 over a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))

sys.path.insert(0, ROOT)
from bench import roofline as RL   # noqa: E402  frozen roofline constants

F_ITER_PMPC = RL.F_ITER["pmpc_n20"]          # FLOP per IPM iteration per instance, PMPC N=20
BYTES_PER_SOLVE = RL.BYTES_PER_SOLVE["pmpc"]  # 18 fp64 in + u0, f, status, iters out
FP64_PEAK_TFLOPS = RL.FP64_PEAK_TFLOPS       # MI355X FP64 (vector = matrix), spec
METRIC = "MPC solves/sec (horizon N=20, batch=18 objects) at 1/2/4/8 GPUs; max |u−u_ref|"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Under torchrun it must equal WORLD_SIZE; without torchrun and > 1, "
                         "bench.py starts the N rank processes itself (default: WORLD_SIZE, else 1)")
    ap.add_argument("--plumbing-only", action="store_true",
                    help="run the multi-rank plumbing (process group, barrier + max-over-ranks timing, the C4 "
                         "shard / gather) on the CPU without solving: a launcher self-test")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=18, help="instances per step per GPU (18 = the metric's config)")
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--tol", type=float, default=1e-8)
    ap.add_argument("--pmpc-path", default="ipopt", choices=("ipopt", "reduced"),
                    help="PMPC path: IPOPT's iterates on the full NLP (default, the drop-in) or the reduced opt-in")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-calls", type=int, default=200, help="calls of the host-pointer (PCIe-inclusive) path")
    ap.add_argument("--rmpc-steps", type=int, default=200, help="launches of the supplementary C3 RMPC line (0 = skip)")
    ap.add_argument("--lmpc-steps", type=int, default=300,
                    help="launches of the supplementary C5 stress line (0 = skip; its rate is set by the few batches with a restoration instance, so it needs a few hundred)")
    ap.add_argument("--lmpc-policy-steps", type=int, default=100,
                    help="launches of the supplementary C5 line with the policy step fused into the launch (0 = skip)")
    ap.add_argument("--arm-steps", type=int, default=200, help="launches of the supplementary arm-QP line (0 = skip)")
    ap.add_argument("--n15-steps", type=int, default=200,
                    help="launches of the supplementary PMPC line at the driver's horizon N=15 (0 = skip)")
    ap.add_argument("--resto-steps", type=int, default=10,
                    help="launches per line of the supplementary PMPC restoration lines (0 = skip)")
    ap.add_argument("--long-steps", type=int, default=10,
                    help="batches per line of the supplementary long-horizon lines (N = 40, 63; 0 = skip)")
    ap.add_argument("--c4-steps", type=int, default=50,
                    help="steps of the supplementary C4 line (1152 instances sharded over the ranks + gather; 0 = skip)")
    ap.add_argument("--dist-backend", default=None,
                    help="torch.distributed backend for N > 1 (default nccl = RCCL over xGMI); 'gloo' with every rank "
                         "on the card(s) present rehearses the multi-rank path on a one-GPU box")
    ap.add_argument("--saturation-batch", type=int, default=18 * 1024,
                    help="supplementary single-launch batch for the saturated rate (0 = skip)")
    return ap.parse_args()


def bench_rmpc(args, torch, dev, stream, dart_mpc):
    """C3: RMPC batch=18 (N=20), fused RLS + warm-start-free solve per launch, inputs in HBM."""
    from dart_mpc.workload import rmpc_batch
    B, K, N = 18, args.rmpc_steps, 20
    D = [rmpc_batch(1, seed0=9000 + i) for i in range(K + 5)]
    T = lambda k, dt=torch.float64: torch.tensor(np.stack([d[k] for d in D]), dtype=dt, device=dev).contiguous()
    X0, UP, TH, RR, PR, PP, PH, YY = (T("x0"), T("u_prev"), T("rls_theta"), T("Rref"), T("prm"), T("rls_P"),
                                      T("phi_prev"), T("y"))
    U0 = torch.empty((K + 5, B, 2), dtype=torch.float64, device=dev)
    FV = torch.empty((K + 5, B), dtype=torch.float64, device=dev)
    ST = torch.empty((K + 5, B), dtype=torch.int32, device=dev)
    IT = torch.empty((K + 5, B), dtype=torch.int32, device=dev)
    s = dart_mpc.RmpcSolver(N=N, tol=args.tol, B_max=B, device=dev.index)
    sp = stream.cuda_stream

    def launch(i):
        s.solve_batch_dev(B, X0[i].data_ptr(), UP[i].data_ptr(), TH[i].data_ptr(), RR[i].data_ptr(), PR[i].data_ptr(),
                          U0[i].data_ptr(), FV[i].data_ptr(), ST[i].data_ptr(), IT[i].data_ptr(),
                          rls_P=PP[i].data_ptr(), rls_phi=PH[i].data_ptr(), rls_y=YY[i].data_ptr(), rls_lambda=0.995,
                          stream=sp)

    for i in range(5):
        launch(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for j in range(K):
            launch(5 + j)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st, its = ST[5:].cpu().numpy(), IT[5:].cpu().numpy()
    u0_first = U0[5].cpu().numpy()
    kern_ms = _event_ms(torch, stream, lambda j: launch(5 + j), K)     # (re-applies the fused RLS update)
    # accuracy on the first timed launch: the oracle with the same (host-updated) RLS estimate, tol 1e-11
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib   # checker + CPU baseline only
    d = D[5]
    th = np.zeros((B, 14))
    for b in range(B):
        for a in range(2):
            th[b, 7 * a:7 * a + 7], _ = oracle_lib.rls_update(d["rls_theta"][b, 7 * a:7 * a + 7], d["rls_P"][b, a],
                                                              d["phi_prev"][b], d["y"][b, a], 0.995)
    ref = oracle_lib.rmpc_solve_batch(d["x0"], d["u_prev"], th, d["Rref"], d["prm"], N=N, tol=1e-11, max_iter=500,
                                      nthreads=4, want_w=False)
    max_du = float(np.max(np.abs(u0_first - ref["u0"])))
    out = {"workload": "C3: RMPC batch=18, N=20, Ts=0.002, RLS update (2 filters, p=7) fused, cold start, tol "
                       f"{args.tol:g}", "solves_per_s": B * K / dt, "ms_per_step": dt / K * 1e3, "kernel_ms": kern_ms,
           "status_ok_frac": float(np.mean(st == 0)), "iters_mean": float(its.mean()),
           "max_abs_u0_err_vs_exact_optimum": max_du,
           "roofline": RL.roofline(float(its.sum(axis=1).mean()), RL.F_ITER["rmpc_n20"], kern_ms * 1e-3,
                                   note="sum(iters) x 7.3e4 FLOP per launch / mean kernel time")}
    if not args.no_cpu_baseline:
        try:
            ncores = len(os.sched_getaffinity(0))
        except AttributeError:
            ncores = os.cpu_count() or 1
        nt = max(1, min(16, ncores))
        Db = rmpc_batch(max(1, nt // 2), seed0=4242)
        solved, c0 = 0, time.perf_counter()
        while time.perf_counter() - c0 < min(6.0, args.cpu_seconds):
            oracle_lib.rmpc_solve_batch(Db["x0"], Db["u_prev"], Db["theta"], Db["Rref"], Db["prm"], N=N, tol=args.tol,
                                        nthreads=nt, want_w=False)
            solved += Db["x0"].shape[0]
        cdt = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": solved / cdt, "unit": "solves/s", "cores": nt, "kind": "port",
                               "sample": f"C oracle (oracle/rmpc_ipm.c), {solved} cold-start C3 solves in {cdt:.1f} s"}
    # the infeasible-start regime: measured velocities 3x the C3 spread put |v| above vmax at the pinned node 0 on
    # most instances, and IPOPT's restoration phases end those at status 2 (the oracle's), whose point the next
    # step warm-starts from (np_mpc...:214-217).  Same shape as C3 (batch 18, N = 20), without the RLS update.
    K2 = max(1, min(K, 100))
    Dv = [rmpc_batch(1, seed0=200000 + i) for i in range(K2 + 1)]
    for d in Dv:
        d["x0"] = d["x0"].copy()
        d["x0"][:, [1, 3]] *= 3.0
    Tv = lambda k: torch.tensor(np.stack([d[k] for d in Dv]), dtype=torch.float64, device=dev).contiguous()
    VX0, VUP, VTH, VRR, VPR = Tv("x0"), Tv("u_prev"), Tv("theta"), Tv("Rref"), Tv("prm")

    def vlaunch(i):
        s.solve_batch_dev(B, VX0[i].data_ptr(), VUP[i].data_ptr(), VTH[i].data_ptr(), VRR[i].data_ptr(),
                          VPR[i].data_ptr(), U0[i].data_ptr(), FV[i].data_ptr(), ST[i].data_ptr(), IT[i].data_ptr(),
                          stream=sp)

    vlaunch(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for i in range(1, K2 + 1):
            vlaunch(i)
    torch.cuda.synchronize()
    dtv = time.perf_counter() - t0
    stv, u0v = ST[1:K2 + 1].cpu().numpy(), U0[1].cpu().numpy()
    d = Dv[1]
    ov = oracle_lib.rmpc_solve_batch(d["x0"], d["u_prev"], d["theta"], d["Rref"], d["prm"], N=N, tol=args.tol,
                                     nthreads=4, want_w=False)
    out["infeasible_start"] = {
        "workload": "C3 shape with measured velocities x3 (|v| > vmax at node 0), restoration phases on, no RLS",
        "solves_per_s": B * K2 / dtv, "ms_per_step": dtv / K2 * 1e3,
        "status_infeasible_frac": float(np.mean(stv == 2)), "status_ok_frac": float(np.mean(stv == 0)),
        "iters_mean": float(IT[1:K2 + 1].float().mean().item()), "batch_max_iters_mean":
            float(IT[1:K2 + 1].max(dim=1).values.float().mean().item()),
        "first_batch_status_equal_to_oracle": bool(np.array_equal(stv[0], ov["status"])),
        "first_batch_max_abs_u0_err_vs_oracle": float(np.max(np.abs(u0v - ov["u0"])))}
    if not args.no_cpu_baseline:
        # the same infeasible-start batches on the C oracle (restoration phases included), bounded sample
        nt = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1))
        solved, c0, i = 0, time.perf_counter(), 1
        while time.perf_counter() - c0 < min(6.0, args.cpu_seconds) and i <= K2:
            dd = Dv[i]
            oracle_lib.rmpc_solve_batch(dd["x0"], dd["u_prev"], dd["theta"], dd["Rref"], dd["prm"], N=N, tol=args.tol,
                                        nthreads=nt, want_w=False)
            solved += B
            i += 1
        cdt = time.perf_counter() - c0
        out["infeasible_start"]["cpu_baseline"] = {
            "value": solved / cdt, "unit": "solves/s", "cores": nt, "kind": "port",
            "sample": f"C oracle (oracle/rmpc_ipm.c, IPOPT's restoration phases), {solved} solves of the bench's own "
                      f"infeasible-start batches in {cdt:.1f} s"}
    # SURVEY 8(d), host to host: the reference's RMPC step is synchronous (rob_ctrl.py:351-352) -- host arrays in,
    # the fused RLS update and the solve, theta / P / u0 back in host memory, per call
    if args.host_calls > 0:
        Kh = max(20, min(args.host_calls, K))
        hs = dart_mpc.RmpcSolver(N=N, tol=args.tol, B_max=B, device=dev.index)

        def hcall(i):
            d = D[i % len(D)]
            th, Pm = d["rls_theta"].copy(), d["rls_P"].copy()
            hs.solve_batch(d["x0"], d["u_prev"], th, d["Rref"], d["prm"], rls_P=Pm, rls_phi=d["phi_prev"], rls_y=d["y"],
                           rls_lambda=0.995)
        h = _host_line(hcall, Kh)
        hs.close()
        out["host_inclusive_8d"] = {"value": B / (h["ms_per_call"] * 1e-3), "unit": "solves/s", **h,
                                    "median_solves_per_s": B / (h["median_ms_per_call"] * 1e-3),
                                    "note": "dart_rmpc_solve_batch from Python: host inputs (x0, u_prev, theta, Rref, prm, "
                                            "RLS P / phi / y) in, RLS update + solve, theta, P, u0, f back in host "
                                            "memory; value = B / mean call time"}
    # saturated lines: C3-type batches of 18 x 64 and 18 x 1024 in one launch each (the object-config sweep x
    # Monte-Carlo seeds of north_star, np_mpc...:212-222)
    sat = {}
    for ns in (64, 1024):
        Dd = rmpc_batch(ns, seed0=600000)
        Bs = 18 * ns
        t_ = lambda k: torch.tensor(Dd[k], dtype=torch.float64, device=dev).contiguous()
        a_ = [t_(k) for k in ("x0", "u_prev", "theta", "Rref", "prm")]
        su = torch.empty((Bs, 2), dtype=torch.float64, device=dev); sf = torch.empty(Bs, dtype=torch.float64, device=dev)
        ss = torch.empty(Bs, dtype=torch.int32, device=dev); si = torch.empty(Bs, dtype=torch.int32, device=dev)
        big = dart_mpc.RmpcSolver(N=N, tol=args.tol, B_max=Bs, device=dev.index)
        line = _saturated(torch, stream, lambda: big.solve_batch_dev(
            Bs, *[x.data_ptr() for x in a_], su.data_ptr(), sf.data_ptr(), ss.data_ptr(), si.data_ptr(), stream=sp),
            Bs, ss, si, RL.F_ITER["rmpc_n20"], int(dart_mpc._lib.lib().dartmpc_rmpc_blocks_per_cu()))
        big.close()
        sat[f"b{Bs}"] = line
    sat["note"] = ("C3-type inputs (no RLS update), cold start, tol 1e-8, one launch per batch; rmpc_ipm_kernel<false> "
                   "takes 70.6 KB of LDS and 256 VGPRs + 240 AGPRs per instance")
    out["saturation"] = sat
    s.close()
    return out


def bench_long_horizons(args, dart_mpc):
    """Horizons beyond the one-wave kernels (N = 40 and 63; the reference takes N as a free constructor argument,
    mpc_3d.py:12, np_mpc...:35, rlmpc2.py): per variant a batch of 18 fresh instances per call through the host
    entry (inputs copied in, outputs out: PCIe-inclusive), statuses and iterations of the first batch against
    the C oracle.  N > 31 runs the two-wave builds of all three variants (PMPC: the scan build, pmpc_wg2.o)."""
    from dart_mpc.workload import lmpc_batch, pmpc_batch, rmpc_batch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib   # checker only
    K = args.long_steps
    out = {"note": "host entry (PCIe-inclusive), batch 18, fresh instances per call; *_equal: the first batch "
                   "against the C oracle at the same options"}
    for N in (40, 63):
        P = [pmpc_batch(1, seed0=700000 + 1000 * i) for i in range(K + 1)]
        R = [rmpc_batch(1, seed0=9500 + i, N=N) for i in range(K + 1)]
        L = [lmpc_batch(1, seed0=7500 + i) for i in range(K + 1)]
        line = {}
        s = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=18)
        first = s.solve_batch(*P[0])
        t0 = time.perf_counter()
        for i in range(1, K + 1):
            s.solve_batch(*P[i])
        dt = time.perf_counter() - t0
        s.close()
        o = oracle_lib.solve_batch(*P[0], N=N, Ts=0.002, tol=args.tol, nthreads=8, want_w=False)
        line["pmpc"] = {"solves_per_s": 18 * K / dt, "status_equal": bool(np.array_equal(first["status"], o["status"])),
                        "iters_equal_frac": float(np.mean(first["iters"] == o["iters"]))}
        s = dart_mpc.RmpcSolver(N=N, tol=args.tol, B_max=18)
        k5 = ("x0", "u_prev", "theta", "Rref", "prm")
        first = s.solve_batch(*(R[0][k] for k in k5))
        t0 = time.perf_counter()
        for i in range(1, K + 1):
            s.solve_batch(*(R[i][k] for k in k5))
        dt = time.perf_counter() - t0
        s.close()
        o = oracle_lib.rmpc_solve_batch(*(R[0][k] for k in k5), N=N, tol=args.tol, nthreads=8, want_w=False)
        line["rmpc"] = {"solves_per_s": 18 * K / dt, "status_equal": bool(np.array_equal(first["status"], o["status"])),
                        "iters_equal_frac": float(np.mean(first["iters"] == o["iters"]))}
        s = dart_mpc.LmpcSolver(N=N, B_max=18)
        k4 = ("state", "u_prev", "pvec", "target")
        first = s.solve_batch(*(L[0][k] for k in k4))
        t0 = time.perf_counter()
        for i in range(1, K + 1):
            s.solve_batch(*(L[i][k] for k in k4))
        dt = time.perf_counter() - t0
        s.close()
        o = oracle_lib.lmpc_solve_batch(*(L[0][k] for k in k4), N=N, nthreads=8, want_w=False)
        line["lmpc"] = {"solves_per_s": 18 * K / dt, "status_equal": bool(np.array_equal(first["status"], o["status"])),
                        "iters_equal_frac": float(np.mean(first["iters"] == o["iters"])),
                        "options": "reference (tol 1e-4, acceptable 1e-3 x 5, max_iter 50)"}
        out[f"N{N}"] = line
    return out


def bench_pmpc_driver_horizon(args, torch, dev, stream, dart_mpc, N=15):
    """PMPC at the DART driver's own horizon (N = 15 for every object, main_parallel_enhanced.py:171-196),
    batch 18, fresh instances per launch, inputs in HBM.  At N <= 15 each axis fits one 16-lane DPP row
    and the scans skip their cross-row steps."""
    from dart_mpc.workload import pmpc_batch
    B, K = 18, args.n15_steps
    steps = [pmpc_batch(1, seed0=600000 + 1000 * i) for i in range(K + 5)]
    T = lambda j: torch.tensor(np.stack([st[j] for st in steps]), dtype=torch.float64, device=dev).contiguous()
    X0, RF, PR = T(0), T(1), T(2)
    U0 = torch.empty((K + 5, B, 2), dtype=torch.float64, device=dev)
    FV = torch.empty((K + 5, B), dtype=torch.float64, device=dev)
    ST = torch.empty((K + 5, B), dtype=torch.int32, device=dev)
    IT = torch.empty((K + 5, B), dtype=torch.int32, device=dev)
    s = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=B, device=dev.index, path=args.pmpc_path)
    sp = stream.cuda_stream

    def launch(i):
        s.solve_batch_dev(B, X0[i].data_ptr(), RF[i].data_ptr(), PR[i].data_ptr(), U0[i].data_ptr(), FV[i].data_ptr(),
                          ST[i].data_ptr(), IT[i].data_ptr(), stream=sp)

    for i in range(5):
        launch(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for j in range(K):
            launch(5 + j)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = ST[5:].cpu().numpy()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib   # checker only
    S0, T0, P0 = steps[5]
    ref = oracle_lib.solve_batch(S0, T0, P0, N=N, Ts=0.002, tol=1e-11, nthreads=4, want_w=False)
    s.close()
    return {"workload": f"PMPC batch=18, N={N} (the DART driver's horizon), tol {args.tol:g}, cold start",
            "solves_per_s": B * K / dt, "ms_per_step": dt / K * 1e3, "status_ok_frac": float(np.mean(st == 0)),
            "max_abs_u0_err_vs_exact_optimum": float(np.max(np.abs(U0[5].cpu().numpy() - ref["u0"])))}


def _event_ms(torch, stream, launch, K):
    """Mean kernel duration from HIP events around each of K launches, in a pass of its own after the
    timed loop (same inputs; the timed loop carries no events, so its wall clock is the bare rate)."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    with torch.cuda.stream(stream):
        for j in range(K):
            ev[j][0].record(stream)
            launch(j)
            ev[j][1].record(stream)
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def _host_line(call, n_calls, warm=3):
    """SURVEY 8(d) host-to-host rate of one batch per call: host arrays in, results back in host memory, blocking;
    median of n_calls timed calls (fresh inputs each) after `warm` untimed ones.  call(i) runs call i."""
    for i in range(warm):
        call(i)
    per = np.empty(n_calls)
    t0 = time.perf_counter()
    for j in range(n_calls):
        c0 = time.perf_counter()
        call(warm + j)
        per[j] = time.perf_counter() - c0
    tot = time.perf_counter() - t0
    return {"calls": n_calls, "ms_per_call": tot / n_calls * 1e3, "median_ms_per_call": float(np.median(per)) * 1e3}


def _saturated(torch, stream, launch, B, ST, IT, f_iter, blocks_per_cu, reps=3):
    """One launch over a large batch (inputs resident in HBM), timed by HIP events on the launch stream: the
    median of `reps` launches after one untimed.  Residency: instances of the kernel the runtime keeps per CU."""
    launch()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launch()
        e1.record(stream)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    m = float(np.median(ms))
    st, it = ST.cpu().numpy(), IT.cpu().numpy()
    ncu = torch.cuda.get_device_properties(stream.device).multi_processor_count
    return {"batch": B, "ms_per_launch": m, "solves_per_s": B / (m * 1e-3), "iters_mean": float(it.mean()),
            "status_ok_frac": float(np.mean(np.isin(st, (0, 1)))),
            "residency": {"instances_per_cu": blocks_per_cu, "cus": ncu,
                          "instances_in_flight": blocks_per_cu * ncu if blocks_per_cu > 0 else None,
                          "source": "hipOccupancyMaxActiveBlocksPerMultiprocessor of the solve kernel (one wave per "
                                    "instance; its registers and LDS)"},
            "roofline": RL.roofline(float(it.sum()), f_iter, m * 1e-3,
                                    note=f"sum(iters) x {f_iter:.1e} FLOP / launch time; the chip holds "
                                         f"{blocks_per_cu} instance(s) per CU")}


def _max_over_ranks(vals, dev, host_coll):
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64, device="cpu" if host_coll else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def bench_c4(args, torch, dev, stream, dart_mpc, world, rank, host_coll=False, coll=None):
    """C4 (BASELINE.json configs[3]): PMPC 18 configs x 64 seeds = 1152 instances, N=20, sharded over the
    ranks in contiguous blocks (dart_mpc.parallel.shard_bounds).  One step = every rank solves its block,
    packs [u0, f, status] and joins one all_gather_into_tensor (RCCL over xGMI) of the padded blocks.
    The global batch is fixed as ranks are added (strong scaling); the gather is inside the timed region
    of `solves_per_s`; `solves_per_s_without_gather` times the solves alone."""
    import torch.distributed as dist
    from dart_mpc.parallel import RESULT_COLS, shard_bounds
    from dart_mpc.workload import pmpc_batch
    # the collective runs whenever a process group exists -- also at N = 1 with --dist-backend nccl, where
    # the gather is one RCCL all_gather_into_tensor over a world of one
    coll = (world > 1) if coll is None else coll
    Bg, K, N = 18 * 64, args.c4_steps, args.N
    S, T, P = pmpc_batch(n_seeds=64, seed0=300000)
    lo, hi = shard_bounds(Bg, world, rank)
    per, n = -(-Bg // world), hi - lo
    dt64 = torch.float64
    X0 = torch.tensor(S[lo:hi], dtype=dt64, device=dev).contiguous()
    RF = torch.tensor(T[lo:hi], dtype=dt64, device=dev).contiguous()
    PR = torch.tensor(P[lo:hi], dtype=dt64, device=dev).contiguous()
    U0 = torch.empty((n, 2), dtype=dt64, device=dev)
    FV = torch.empty(n, dtype=dt64, device=dev)
    ST = torch.empty(n, dtype=torch.int32, device=dev)
    IT = torch.empty(n, dtype=torch.int32, device=dev)
    block = torch.zeros((per, RESULT_COLS), dtype=dt64, device=dev)
    # without a collective the gathered result of one rank is its block: the same buffer
    full = torch.zeros((world * per, RESULT_COLS), dtype=dt64, device=dev) if coll else block
    solver = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=max(1, n), device=dev.index, path=args.pmpc_path)
    sp = stream.cuda_stream

    def step(gather=True):
        solver.solve_batch_dev(n, X0.data_ptr(), RF.data_ptr(), PR.data_ptr(), U0.data_ptr(), FV.data_ptr(),
                               ST.data_ptr(), IT.data_ptr(), stream=sp)
        if not gather:
            return
        with torch.cuda.stream(stream):
            # [u0, f, status] rows in one kernel
            torch.cat((U0, FV.unsqueeze(1), ST.unsqueeze(1).to(dt64)), dim=1, out=block[:n])
            if coll and host_coll:
                fh = full.cpu()     # gloo rehearsal: the gather runs on host copies
                dist.all_gather_into_tensor(fh, block.cpu())
                full.copy_(fh)
            elif coll:
                dist.all_gather_into_tensor(full, block)

    def timed(gather):
        for _ in range(3):
            step(gather)
        torch.cuda.synchronize()
        if coll:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step(gather)
        torch.cuda.synchronize()
        if coll:
            dist.barrier()
        t = time.perf_counter() - t0
        return _max_over_ranks([t], dev, host_coll)[0] if coll else t

    dt_solve = timed(False)      # the solves alone (with and without the gather)
    dt = timed(True)
    res = full.cpu().numpy()[:Bg]
    # every rank finds its own block, bit for bit, at its offset of the gathered result
    mine = bool(np.array_equal(res[lo:hi], block[:n].cpu().numpy()))
    if coll:
        mine = _max_over_ranks([0.0 if mine else 1.0], dev, host_coll)[0] == 0.0
    solver.close()
    if rank != 0:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib   # checker only
    ref = oracle_lib.solve_batch(S[:36], T[:36], P[:36], N=N, Ts=0.002, tol=1e-11, nthreads=4, want_w=False)
    # the same path at the same tolerance: every one of the 1152 gathered controls against the oracle at tol 1e-8
    same = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=args.tol, nthreads=8, want_w=False)
    return {"workload": "C4: PMPC 18 configs x 64 seeds = 1152 instances, N=20, tol 1e-8, cold start, contiguous "
                        "blocks over the ranks + all_gather_into_tensor of [u0, f, status] (RCCL)",
            "global_batch": Bg, "per_rank": per, "n_gpus": world, "scaling": "strong", "steps": K,
            "solves_per_s": Bg * K / dt, "ms_per_step": dt / K * 1e3, "gather_in_timed_region": coll,
            "gather": ("RCCL all_gather_into_tensor on device tensors" if coll and not host_coll
                       else "gloo all_gather_into_tensor on host copies" if coll else "none: one rank, its packed block is the result"),
            "solves_per_s_without_gather": Bg * K / dt_solve, "ms_per_step_without_gather": dt_solve / K * 1e3,
            "status_ok_frac": float(np.mean(res[:, 3] == 0)), "rank_blocks_consistent": mine,
            "max_abs_u0_err_vs_oracle_same_tol": float(np.max(np.abs(res[:, 0:2] - same["u0"]))),
            "status_equal_to_oracle": bool(np.array_equal(res[:, 3].astype(np.int32), same["status"])),
            "max_abs_u0_err_vs_exact_optimum_first36": float(np.max(np.abs(res[:36, 0:2] - ref["u0"]))),
            "note_exact_optimum": "IPOPT's own stopping point at tol 1e-8 sits ~mu/z inside weakly active bounds: "
                                  "the oracle at tol 1e-8 is as far from the tol-1e-11 optimum"}


def bench_pmpc_restoration(args, torch, dev, stream, dart_mpc):
    """PMPC launches that contain instances needing IPOPT's restoration phases (pmpc_resto.h): C4's 1152
    instances at N = 31 with the default options (a few fail the filter line search) and at N = 20 with
    max_soc = 0 (about one in ten), against the same launches with the phases off (restoration = False: those
    instances stop at -2, the cost of a launch without restoration); and C2-size batches of 18 that hold one such
    instance (the restoration runs in the solving wave).  The restored controls are checked against the oracle."""
    from dart_mpc.workload import pmpc_batch
    K = args.resto_steps
    S, T, P = pmpc_batch(n_seeds=64, seed0=300000)
    B = S.shape[0]
    dt64 = torch.float64
    X0, RF, PR = (torch.tensor(a, dtype=dt64, device=dev).contiguous() for a in (S, T, P))
    U0 = torch.empty((B, 2), dtype=dt64, device=dev); FV = torch.empty(B, dtype=dt64, device=dev)
    ST = torch.empty(B, dtype=torch.int32, device=dev); IT = torch.empty(B, dtype=torch.int32, device=dev)
    sp = stream.cuda_stream
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib   # checker only

    def timed(solver, n, k):
        def launch():
            solver.solve_batch_dev(n, X0.data_ptr(), RF.data_ptr(), PR.data_ptr(), U0.data_ptr(), FV.data_ptr(),
                                   ST.data_ptr(), IT.data_ptr(), stream=sp)
        launch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            launch()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k

    out = {}
    for name, N, soc in (("c4_n31_default", 31, 4), ("c4_n20_max_soc0", 20, 0)):
        on = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=B, device=dev.index, max_soc=soc)
        off = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=B, device=dev.index, max_soc=soc, restoration=False)
        t_off = timed(off, B, K)
        rest = ST.cpu().numpy() == -2
        t_on = timed(on, B, K)
        st, u0, it = ST.cpu().numpy(), U0.cpu().numpy(), IT.cpu().numpy()
        idx = np.flatnonzero(rest)
        o = oracle_lib.solve_batch(S[idx], T[idx], P[idx], N=N, Ts=0.002, tol=args.tol, max_iter=3000, nthreads=8,
                                   want_w=False, soc=soc)
        line = {"instances": B, "restored": int(rest.sum()), "ms_per_launch": t_on * 1e3,
                "ms_per_launch_restoration_off": t_off * 1e3, "ratio_to_restoration_off": t_on / t_off,
                "status_ok_frac": float(np.mean(st == 0)), "restored_iters_mean": float(it[idx].mean()),
                "restored_status_equal_to_oracle": bool(np.array_equal(st[idx], o["status"])),
                "restored_max_abs_u0_err_vs_oracle": float(np.max(np.abs(u0[idx] - o["u0"])))}
        # a C2-size batch of 18 holding one such instance (the restoration in the solving wave)
        if idx.size:
            sel = np.concatenate([idx[:1], np.flatnonzero(~rest)[:17]])
            for a, src in ((X0, S), (RF, T), (PR, P)):
                a[:18].copy_(torch.tensor(src[sel], dtype=dt64, device=dev))
            s18 = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=18, device=dev.index, max_soc=soc)
            o18 = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=18, device=dev.index, max_soc=soc,
                                  restoration=False)
            line["b18_one_restored_ms"] = timed(s18, 18, K) * 1e3
            line["b18_one_restored_status"] = int(ST[0].item())
            line["b18_restoration_off_ms"] = timed(o18, 18, K) * 1e3
            s18.close(); o18.close()
            for a, src in ((X0, S), (RF, T), (PR, P)):
                a.copy_(torch.tensor(src, dtype=dt64, device=dev))
        out[name] = line
        on.close(); off.close()
    out["note"] = ("one launch per call, inputs resident in HBM; a launch lasts as long as its slowest instance, and a "
                   "restored instance is solved again from its start on the LDS Riccati engine (pmpc_resto.h)")
    return out


def bench_lmpc(args, torch, dev, stream, dart_mpc):
    """C5: LMPC batch=18, N=30 (the reference runs N=20), the reference's IPOPT options
    (tol 1e-4, max_iter 50, acceptable 1e-3 x 5), cold start, inputs resident in HBM."""
    from dart_mpc.workload import lmpc_batch
    from dart_mpc._lib import LMPC_PRM_DEFAULT
    B, K, N = 18, args.lmpc_steps, 30
    D = [lmpc_batch(1, seed0=7000 + i) for i in range(K + 3)]
    T = lambda k: torch.tensor(np.stack([d[k] for d in D]), dtype=torch.float64, device=dev).contiguous()
    ST0, UP, PV, TG = T("state"), T("u_prev"), T("pvec"), T("target")
    PR = torch.tensor(np.tile(LMPC_PRM_DEFAULT, (B, 1)), dtype=torch.float64, device=dev)
    U0 = torch.empty((K + 3, B, 2), dtype=torch.float64, device=dev)
    FV = torch.empty((K + 3, B), dtype=torch.float64, device=dev)
    ST = torch.empty((K + 3, B), dtype=torch.int32, device=dev)
    IT = torch.empty((K + 3, B), dtype=torch.int32, device=dev)
    s = dart_mpc.LmpcSolver(N=N, B_max=B, device=dev.index)
    sp = stream.cuda_stream

    def launch(i):
        s.solve_batch_dev(B, ST0[i].data_ptr(), UP[i].data_ptr(), PV[i].data_ptr(), TG[i].data_ptr(), PR.data_ptr(),
                          U0[i].data_ptr(), FV[i].data_ptr(), ST[i].data_ptr(), IT[i].data_ptr(), stream=sp)

    for i in range(3):
        launch(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for j in range(K):
            launch(3 + j)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ref_out = (U0[3:].clone(), ST[3:].clone(), IT[3:].clone())
    kern_ms = _event_ms(torch, stream, lambda j: launch(3 + j), K)
    st, its = ST[3:].cpu().numpy(), IT[3:].cpu().numpy()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib   # checker + CPU baseline only
    d = D[3]
    ref = oracle_lib.lmpc_solve_batch(d["state"], d["u_prev"], d["pvec"], d["target"], N=N, nthreads=4, want_w=False)
    exact = oracle_lib.lmpc_solve_batch(d["state"], d["u_prev"], d["pvec"], d["target"], N=N, tol=1e-11, acc_iter=0,
                                        max_iter=500, nthreads=4, want_w=False)
    u0 = U0[3].cpu().numpy()
    ok = (exact["status"] == 0) & np.isin(st[0], (0, 1))
    # the same launches with IPOPT's restoration phases off (a failed line search ends with status -2, as
    # in rounds 1-2): the cost of the restoration tail
    s_off = dart_mpc.LmpcSolver(N=N, B_max=B, device=dev.index, restoration=False)

    def launch_off(i):
        s_off.solve_batch_dev(B, ST0[i].data_ptr(), UP[i].data_ptr(), PV[i].data_ptr(), TG[i].data_ptr(), PR.data_ptr(),
                              U0[i].data_ptr(), FV[i].data_ptr(), ST[i].data_ptr(), IT[i].data_ptr(), stream=sp)
    launch_off(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for j in range(K):
            launch_off(3 + j)
    torch.cuda.synchronize()
    dt_off = time.perf_counter() - t0
    st_off = ST[3:].cpu().numpy()
    s_off.close()
    # the same K independent batches with several in flight: launch j on stream j mod S (each stream its own
    # restoration hand-off area), so a batch held up by a restoration instance overlaps the next batches --
    # as the reference's controllers, each with its own solver process, do not wait for one another
    # (rlmpc2.py:494-524).  Same outputs bit for bit as one stream.
    inflight = {}
    for n_str in (2, 4):
        streams = [torch.cuda.Stream(device=dev) for _ in range(n_str)]

        def launch_s(i, st_):
            s.solve_batch_dev(B, ST0[i].data_ptr(), UP[i].data_ptr(), PV[i].data_ptr(), TG[i].data_ptr(),
                              PR.data_ptr(), U0[i].data_ptr(), FV[i].data_ptr(), ST[i].data_ptr(), IT[i].data_ptr(),
                              stream=st_.cuda_stream)
        for q in range(n_str):
            launch_s(q % 3, streams[q])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(K):
            launch_s(3 + j, streams[j % n_str])
        torch.cuda.synchronize()
        dt_s = time.perf_counter() - t0
        same = bool(torch.equal(U0[3:], ref_out[0]) and torch.equal(ST[3:], ref_out[1]) and torch.equal(IT[3:], ref_out[2]))
        inflight[f"streams_{n_str}"] = {"solves_per_s": B * K / dt_s, "ms_per_step": dt_s / K * 1e3,
                                        "outputs_equal_to_one_stream": same}
    inflight["note"] = ("the same K batches of 18 with 2 / 4 of them in flight on as many streams (a batch lasts as "
                        "long as its slowest instance; in flight, the batches behind a restoration instance proceed)")
    out = {"workload": "C5 stress: LMPC batch=18, N=30, Ts=0.002, pvec~U(0.01,1.9)^34 input (SURVEY 8d; random "
                       "physical parameters, harsher than the policy's), reference IPOPT options (tol 1e-4, max_iter 50, "
                       "acceptable 1e-3 x 5), cold start, IPOPT's restoration phases on.  C5 as BASELINE.json configures "
                       "it (the learned net inlined into the launch) is `policy_fused`",
           "solves_per_s": B * K / dt, "ms_per_step": dt / K * 1e3, "kernel_ms": kern_ms,
           "status_ok_frac": float(np.mean(np.isin(st, (0, 1)))), "status_optimal_frac": float(np.mean(st == 0)),
           "status_acceptable_frac": float(np.mean(st == 1)), "status_maxiter_frac": float(np.mean(st == -1)),
           "status_infeasible_frac": float(np.mean(st == 2)), "status_failed_frac": float(np.mean(st <= -2)),
           "iters_mean": float(its.mean()),
           "restoration_off": {"solves_per_s": B * K / dt_off, "ms_per_step": dt_off / K * 1e3,
                               "status_ok_frac": float(np.mean(st_off >= 0)),
                               "note": "the same launches, restoration=False: a failed filter line search ends the "
                                       "solve with status -2 (rounds 1-2); the difference is IPOPT's restoration tail "
                                       "(~1 % of the instances, up to max_iter 50 iterations each)"},
           "batches_in_flight": inflight,
           "roofline": RL.roofline(float(its.sum(axis=1).mean()), RL.F_ITER["lmpc_n30"], kern_ms * 1e-3,
                                   note="sum(iters) x 3.7e5 FLOP per launch / mean kernel time"),
           "max_abs_u0_err_vs_oracle_same_options": float(np.max(np.abs(u0 - ref["u0"]))),
           "max_abs_u0_err_vs_exact_optimum": float(np.max(np.abs(u0[ok] - exact["u0"][ok]))) if ok.any() else None}
    if not args.no_cpu_baseline:
        try:
            ncores = len(os.sched_getaffinity(0))
        except AttributeError:
            ncores = os.cpu_count() or 1
        nt = max(1, min(16, ncores))
        Db = lmpc_batch(max(1, nt // 2), seed0=4242)
        solved, c0 = 0, time.perf_counter()
        while time.perf_counter() - c0 < min(6.0, args.cpu_seconds):
            oracle_lib.lmpc_solve_batch(Db["state"], Db["u_prev"], Db["pvec"], Db["target"], N=N, nthreads=nt,
                                        want_w=False)
            solved += Db["state"].shape[0]
        cdt = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": solved / cdt, "unit": "solves/s", "cores": nt, "kind": "port",
                               "sample": f"C oracle (oracle/lmpc_ipm.c, exact jet Hessian), {solved} cold-start C5 "
                                         f"solves in {cdt:.1f} s"}
    # SURVEY 8(d), host to host: one C5 batch per call from host arrays (the solver worker's shared-memory inputs,
    # rlmpc2.py:508-515), u0 / f / status back in host memory
    if args.host_calls > 0:
        Kh = max(20, min(args.host_calls, K))
        hs = dart_mpc.LmpcSolver(N=N, B_max=B, device=dev.index)

        def hcall(i):
            d = D[i % len(D)]
            hs.solve_batch(d["state"], d["u_prev"], d["pvec"], d["target"])
        h = _host_line(hcall, Kh)
        hs.close()
        out["host_inclusive_8d"] = {"value": B / (h["ms_per_call"] * 1e-3), "unit": "solves/s", **h,
                                    "median_solves_per_s": B / (h["median_ms_per_call"] * 1e-3),
                                    "note": "dart_lmpc_solve_batch from Python: host inputs in, u0, f, status back in "
                                            "host memory; value = B / mean call time (restoration tails included; the "
                                            "median call is the typical step)"}
    sat = {}
    for ns in (64, 1024):
        Dd = lmpc_batch(ns, seed0=600000)
        Bs = 18 * ns
        t_ = lambda k: torch.tensor(Dd[k], dtype=torch.float64, device=dev).contiguous()
        a_ = [t_(k) for k in ("state", "u_prev", "pvec", "target")]
        pr_ = torch.tensor(np.tile(LMPC_PRM_DEFAULT, (Bs, 1)), dtype=torch.float64, device=dev)
        su = torch.empty((Bs, 2), dtype=torch.float64, device=dev); sf = torch.empty(Bs, dtype=torch.float64, device=dev)
        ss = torch.empty(Bs, dtype=torch.int32, device=dev); si = torch.empty(Bs, dtype=torch.int32, device=dev)
        big = dart_mpc.LmpcSolver(N=N, B_max=Bs, device=dev.index)
        line = _saturated(torch, stream, lambda: big.solve_batch_dev(
            Bs, *[x.data_ptr() for x in a_], pr_.data_ptr(), su.data_ptr(), sf.data_ptr(), ss.data_ptr(), si.data_ptr(),
            stream=sp), Bs, ss, si, RL.F_ITER["lmpc_n30"], int(dart_mpc._lib.lib().dartmpc_lmpc_blocks_per_cu()))
        big.close()
        sat[f"b{Bs}"] = line
    sat["note"] = ("C5 stress inputs, reference options, restoration phases on (queued kernel for batches above 32), "
                   "one launch per batch; lmpc_ipm_kernel<false> takes LmShared of LDS per instance")
    out["saturation"] = sat
    s.close()
    return out


def bench_lmpc_policy(args, torch, dev, stream, dart_mpc):
    """C5 with the learned parameter net in the launch (BASELINE.json configs[4]): 18 LMPC controllers,
    N=30; one step = the policy step of every controller (Welford-normalised 10-step history, MLP
    520-64-64-34 fp32, rsample, logit update every 8th step, EMA + soft clip) and the solve with the
    parameters it wrote, as ONE launch (dart_lmpc_policy_solve_batch_dev).  Also timed: the same step
    as two launches (policy kernel, then solve), and the check that both give identical results."""
    from dart_mpc.lmpc import init_policy_weights, policy_config
    from dart_mpc.workload import lmpc_batch
    from dart_mpc._lib import LMPC_PRM_DEFAULT, lib
    B, K, N = 18, args.lmpc_policy_steps, 30
    D = [lmpc_batch(1, seed0=7000 + i) for i in range(K + 3)]
    f64 = lambda a: torch.tensor(np.asarray(a), dtype=torch.float64, device=dev).contiguous()
    ST0 = f64(np.stack([d["state"] for d in D])); TG = f64(np.stack([d["target"] for d in D]))
    UP = f64(np.stack([d["u_prev"] for d in D]))
    rng = np.random.default_rng(17)
    NZ = torch.tensor(rng.standard_normal((K + 3, B, 34)), dtype=torch.float32, device=dev)
    PR = f64(np.tile(LMPC_PRM_DEFAULT, (B, 1)))
    W = torch.tensor(init_policy_weights(0), dtype=torch.float32, device=dev)
    cfg = policy_config()
    k0 = np.clip(0.5 * cfg.k_max + np.random.default_rng(1).uniform(-0.05, 0.05, (B, 34)) * cfg.k_max, cfg.min_k,
                 cfg.k_max - cfg.k_ceiling_margin)

    def state():
        return dict(ck=f64(k0), mean=torch.zeros((B, 52), dtype=torch.float64, device=dev),
                    M2=torch.zeros((B, 52), dtype=torch.float64, device=dev),
                    cnt=torch.zeros(B, dtype=torch.int32, device=dev),
                    hist=torch.zeros((B, 10, 52), dtype=torch.float32, device=dev),
                    ts=torch.zeros(B, dtype=torch.int32, device=dev), mp=f64(k0))

    out = {k: torch.empty((K + 3, B, 2), dtype=torch.float64, device=dev) for k in ("u0_f", "u0_s")}
    FV = torch.empty((K + 3, B), dtype=torch.float64, device=dev)
    SS = torch.empty((K + 3, B), dtype=torch.int32, device=dev)
    IT = torch.empty((K + 3, B), dtype=torch.int32, device=dev)
    s = dart_mpc.LmpcSolver(N=N, B_max=B, device=dev.index)
    sp = stream.cuda_stream
    A, Bst = state(), state()

    def fused(i, P=A):
        s.policy_solve_batch_dev(cfg, B, W.data_ptr(), ST0[i].data_ptr(), UP[i].data_ptr(), TG[i].data_ptr(),
                                 P["ck"].data_ptr(), P["mean"].data_ptr(), P["M2"].data_ptr(), P["cnt"].data_ptr(),
                                 P["hist"].data_ptr(), P["ts"].data_ptr(), NZ[i].data_ptr(), P["mp"].data_ptr(),
                                 PR.data_ptr(), out["u0_f"][i].data_ptr(), FV[i].data_ptr(), SS[i].data_ptr(),
                                 IT[i].data_ptr(), stream=sp)

    def two_launch(i, P=Bst):
        rc = lib().dart_lmpc_policy_step_dev(ctypes.byref(cfg), B, W.data_ptr(), ST0[i].data_ptr(), TG[i].data_ptr(),
                                             UP[i].data_ptr(), P["ck"].data_ptr(), P["mean"].data_ptr(),
                                             P["M2"].data_ptr(), P["cnt"].data_ptr(), P["hist"].data_ptr(),
                                             P["ts"].data_ptr(), NZ[i].data_ptr(), P["mp"].data_ptr(), None, sp)
        assert rc == 0
        s.solve_batch_dev(B, ST0[i].data_ptr(), UP[i].data_ptr(), P["mp"].data_ptr(), TG[i].data_ptr(), PR.data_ptr(),
                          out["u0_s"][i].data_ptr(), FV[i].data_ptr(), SS[i].data_ptr(), IT[i].data_ptr(), stream=sp)

    res = {}
    for name, fn in (("fused", fused), ("two_launch", two_launch)):
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            for j in range(K):
                fn(3 + j)
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / K
    same = bool(torch.equal(out["u0_f"], out["u0_s"])) and all(torch.equal(A[k], Bst[k]) for k in A)
    kern_ms = _event_ms(torch, stream, lambda j: fused(3 + j), min(K, 50))
    s.close()
    cpu = None
    if not args.no_cpu_baseline:
        # the same step on the host: the numpy restatement of the policy step per controller, then the C oracle's
        # solves of the 18 NLPs with the parameters it wrote (fresh states every step, as the timed GPU loop)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_lib   # CPU baseline only
        import lmpc_policy as lp
        try:
            ncores = len(os.sched_getaffinity(0))
        except AttributeError:
            ncores = os.cpu_count() or 1
        nt = max(1, min(16, ncores))
        wts = init_policy_weights(0)
        orc = [lp.PolicyState(k0[b]) for b in range(B)]
        nzh = NZ.cpu().numpy()
        steps, c0 = 0, time.perf_counter()
        while time.perf_counter() - c0 < min(6.0, args.cpu_seconds):
            d = D[steps % len(D)]
            for b in range(B):
                lp.policy_step(orc[b], wts, d["state"][b], d["target"][b], d["u_prev"][b], nzh[steps % len(D), b])
            mp = np.stack([o.model_params for o in orc])
            oracle_lib.lmpc_solve_batch(d["state"], d["u_prev"], mp, d["target"], N=N, nthreads=nt, want_w=False)
            steps += 1
        cdt = time.perf_counter() - c0
        cpu = {"value": steps * B / cdt, "unit": "solves/s", "cores": nt, "kind": "port",
               "sample": f"{steps} steps of 18 controllers in {cdt:.1f} s: oracle/lmpc_policy.py policy step per "
                         f"controller (numpy, one core) + the C oracle's 18 solves (oracle/lmpc_ipm.c, {nt} threads)"}
    return {"workload": "C5 with the parameter policy in the launch: 18 LMPC controllers, N=30, reference IPOPT "
                        "options, policy step (MLP 520-64-64-34 fp32, logit update every 8th step) as the prologue "
                        "of the solve kernel, fresh states every step, weights = Policy._init_weights (checkpoints "
                        "not loaded)",
            "solves_per_s": B / res["fused"], "ms_per_step": res["fused"] * 1e3, "kernel_ms": kern_ms,
            "two_launch_ms_per_step": res["two_launch"] * 1e3,
            "status_ok_frac": float(((SS[3:] == 0) | (SS[3:] == 1)).float().mean()), "iters_mean": float(IT[3:].double().mean()),
            "fused_equals_two_launch": same, "cpu_baseline": cpu,
            "note": "pvec comes from the policy (current_k mid-range +-5 %, then logit updates), not from the "
                    "U(0.01, 1.9) draws of the plain C5 line, so these NLPs are easier (fewer iterations)"}


def bench_arm(args, torch, dev, stream, dart_mpc):
    """Per-arm impedance QP (ARMCONTROL.solver_worker): 36 arm snapshots per launch
    (18 object configs x 2 arms = one dual-arm simulation step of the C2 batch), fresh synthetic
    snapshots every launch, resident in HBM; plus one saturated launch."""
    from dart_mpc.arm import pack_params, pack_snapshot
    from dart_mpc.workload import arm_batch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import arm_qp   # checker + CPU baseline only
    K, n = args.arm_steps, 7
    snaps = [arm_batch(1, seed0=5000 + i)[0] for i in range(K + 3)]
    B = snaps[0]["q"].shape[0]
    prm = arm_qp.default_params()
    SR = torch.tensor(np.stack([pack_snapshot(x) for x in snaps]), dtype=torch.float64, device=dev).contiguous()
    PR = torch.tensor(pack_params(prm), dtype=torch.float64, device=dev)
    QD = torch.empty((K + 3, B, n), dtype=torch.float64, device=dev)
    TQ = torch.empty((K + 3, B, n), dtype=torch.float64, device=dev)
    LS = torch.empty((K + 3, B), dtype=torch.float64, device=dev)
    ST = torch.empty((K + 3, B), dtype=torch.int32, device=dev)
    IT = torch.empty((K + 3, B), dtype=torch.int32, device=dev)
    s = dart_mpc.ArmSolver(n)
    sp = stream.cuda_stream

    def launch(i):
        s.solve_batch_dev(B, SR[i].data_ptr(), PR.data_ptr(), True, QD[i].data_ptr(), TQ[i].data_ptr(),
                          LS[i].data_ptr(), ST[i].data_ptr(), IT[i].data_ptr(), stream=sp)

    for i in range(3):
        launch(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for j in range(K):
            launch(3 + j)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_ms = _event_ms(torch, stream, lambda j: launch(3 + j), K)
    st, its = ST[3:].cpu().numpy(), IT[3:].cpu().numpy()
    ref = arm_qp.solve_batch(snaps[3], prm)
    ok = ref["status"] >= 0
    dq = np.abs(QD[3].cpu().numpy() - ref["qdd"])[ok] / (1 + np.abs(ref["qdd"][ok]))
    out = {"workload": "arm QP: 36 arm snapshots per launch (18 configs x 2 arms), n=7, reference parameters "
                       "(rob_ctrl.py:232-275), synthetic dynamics, qdd_prev warm start, scaled KKT tol 1e-10",
           "solves_per_s": B * K / dt, "ms_per_step": dt / K * 1e3, "kernel_ms": kern_ms,
           "status_ok_frac": float(np.mean(st >= 0)), "iters_mean": float(its.mean()),
           "status_equal_to_oracle": bool(np.array_equal(st[0], ref["status"])),
           "max_rel_qdd_err_vs_oracle": float(dq.max()) if ok.any() else None}
    if args.saturation_batch > 0:
        nb = max(1, args.saturation_batch // B)
        big = arm_batch(nb, seed0=90000)[0]
        Bs = big["q"].shape[0]
        bs = torch.tensor(pack_snapshot(big), device=dev)
        bo = [torch.empty((Bs, n), dtype=torch.float64, device=dev) for _ in range(2)] + \
             [torch.empty(Bs, dtype=torch.float64, device=dev)] + [torch.empty(Bs, dtype=torch.int32, device=dev) for _ in range(2)]
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            s.solve_batch_dev(Bs, bs.data_ptr(), PR.data_ptr(), True, *[t.data_ptr() for t in bo], stream=sp)
            e1.record(stream)
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        out["saturation"] = {"batch": Bs, "ms_per_launch": ms, "solves_per_s": Bs / (ms * 1e-3),
                             "ok_frac": float((bo[3] >= 0).float().mean())}
    if not args.no_cpu_baseline:
        Sb = arm_batch(4, seed0=4242)[0]
        solved, c0 = 0, time.perf_counter()
        while time.perf_counter() - c0 < min(5.0, args.cpu_seconds):
            arm_qp.solve_batch(Sb, prm)
            solved += Sb["q"].shape[0]
        cdt = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": solved / cdt, "unit": "solves/s", "cores": 1, "kind": "port",
                               "sample": f"numpy oracle (oracle/arm_qp.py: numpy pinv/inv/eigh QP build + Mehrotra "
                                         f"IPM), {solved} solves in {cdt:.1f} s; the reference additionally rebuilds "
                                         f"the CasADi nlpsol every step (arm.py:407-408)"}
    return out


def _spawn_ranks(n):
    """`--gpus N` (N > 1) without torchrun: start the N rank processes here, in the environment torchrun
    gives them (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT), and return the
    exit status.  This parent never imports torch, so nothing has touched a GPU when the children start;
    rank r takes GPU r (LOCAL_RANK).  If a rank fails, the others (which may wait in a collective) are
    stopped by their PIDs.  The rank-0 JSON line reaches stdout from rank 0 itself.  This replaces
    PMPC/main_parallel_enhanced.py:200-207's one-worker Process spawn with one process per GPU."""
    import signal
    import socket
    import subprocess
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGTERM)
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(0.05)
    for p in procs:
        if rc == 0 and p.returncode:
            rc = p.returncode
    return rc


def _world_from_env(args):
    """(world, rank) of this process; spawns the ranks itself for `--gpus N > 1` outside torchrun (returns
    None after they finished, with the exit status in the second slot)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        return None, _spawn_ranks(args.gpus)
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (torchrun --nproc-per-node must "
                         f"equal --gpus)\n")
        return None, 2
    return world, int(os.environ.get("RANK", "0"))


def plumbing_main(args, world, rank, json_fd):
    """--plumbing-only: the multi-rank path without a GPU or a solve.  Every rank joins a gloo process group,
    fills its C4 block (contiguous ceil(1152 / world) instances, dart_mpc.parallel.shard_bounds) with rows that
    are a function of the global instance index, all-gathers the blocks and checks that every rank's rows sit
    at its offset bit for bit; timing is barrier + max over ranks, as in main()."""
    import torch
    import torch.distributed as dist
    from dart_mpc.parallel import RESULT_COLS, shard_bounds
    if world > 1:
        dist.init_process_group("gloo")
    Bg = 18 * 64
    lo, hi = shard_bounds(Bg, world, rank)
    per, n = -(-Bg // world), hi - lo
    block = torch.zeros((per, RESULT_COLS), dtype=torch.float64)
    idx = torch.arange(lo, hi, dtype=torch.float64)
    for c in range(RESULT_COLS):
        block[:n, c] = idx * (c + 1) + 0.25 * c
    full = torch.zeros((world * per, RESULT_COLS), dtype=torch.float64)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if world > 1:
        dist.all_gather_into_tensor(full, block)
        dist.barrier()
    else:
        full.copy_(block)
    t = time.perf_counter() - t0
    res = full[:Bg].numpy()
    mine = bool(np.array_equal(res[lo:hi], block[:n].numpy()))
    want = np.stack([np.arange(Bg) * (c + 1) + 0.25 * c for c in range(RESULT_COLS)], axis=1)
    every = bool(np.array_equal(res, want))
    if world > 1:
        t, bad = _max_over_ranks([t, 0.0 if (mine and every) else 1.0], "cpu", True)
        mine = every = bad == 0.0
        dist.destroy_process_group()
    if rank == 0:
        line = {"metric": METRIC, "value": None, "unit": "solves/s", "n_gpus": world, "plumbing_only": True,
                "pmpc_c4": {"global_batch": Bg, "per_rank": per, "n_gpus": world, "gather_s": t,
                            "rank_blocks_consistent": mine, "gathered_equals_global_rows": every,
                            "gather": "gloo all_gather_into_tensor on host tensors"}}
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    return 0


def main():
    args = parse()
    world, rank = _world_from_env(args)
    if world is None:
        sys.exit(rank)
    # stdout carries exactly one JSON line (rank 0): everything else written to fd 1 -- Python prints and the
    # libraries' own output (RCCL prints a version banner there when a communicator starts) -- goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.plumbing_only:
        sys.exit(plumbing_main(args, world, rank, json_fd))
    import torch
    import torch.distributed as dist
    import dart_mpc
    from dart_mpc.workload import pmpc_batch
    # the CPU baselines are timed on rank 0 of a one-GPU run only (the N > 1 runs report GPU rates)
    args.no_cpu_baseline = args.no_cpu_baseline or world > 1
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = args.dist_backend or ("nccl" if torch.cuda.is_available() else "gloo")
    host_coll = backend == "gloo"
    # a process group for N > 1, and at N = 1 when --dist-backend is given (bench_c4's RCCL gather then runs
    # over a world of one: the collective path exercised on a one-GPU box)
    coll = world > 1 or args.dist_backend is not None
    if coll:
        if world == 1:
            import socket
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                so = socket.socket(); so.bind(("127.0.0.1", 0)); os.environ["MASTER_PORT"] = str(so.getsockname()[1]); so.close()
            os.environ.setdefault("RANK", "0"); os.environ.setdefault("WORLD_SIZE", "1")
    # one rank per GPU; a gloo rehearsal with more ranks than cards shares them round robin
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev if host_coll else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if coll:
        # RCCL: the rank's device named explicitly (a guessed rank -> GPU mapping can hang)
        dist.init_process_group(backend, **({} if host_coll else {"device_id": dev}))

    B, N, K, W = args.batch, args.N, args.steps, args.warmup
    n_seeds_step = max(1, -(-B // 18))
    # fresh seeded inputs for every step, all resident in HBM before timing
    steps_in = []
    for i in range(W + K):
        S, T, P = pmpc_batch(n_seeds=n_seeds_step, seed0=100000 * rank + n_seeds_step * i)
        steps_in.append((S[:B], T[:B], P[:B]))
    X0 = torch.tensor(np.stack([s[0] for s in steps_in]), dtype=torch.float64, device=dev).contiguous()
    RF = torch.tensor(np.stack([s[1] for s in steps_in]), dtype=torch.float64, device=dev).contiguous()
    PR = torch.tensor(np.stack([s[2] for s in steps_in]), dtype=torch.float64, device=dev).contiguous()
    U0 = torch.empty((W + K, B, 2), dtype=torch.float64, device=dev)
    FV = torch.empty((W + K, B), dtype=torch.float64, device=dev)
    ST = torch.empty((W + K, B), dtype=torch.int32, device=dev)
    IT = torch.empty((W + K, B), dtype=torch.int32, device=dev)

    solver = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=B, device=local, path=args.pmpc_path)
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream

    # every step's device pointers formed before the timed region (tensor indexing costs the host ~5 us per view;
    # at 20 steps the first launch's share of that sat in the timed region before the GPU started)
    ptrs = [(X0[i].data_ptr(), RF[i].data_ptr(), PR[i].data_ptr(), U0[i].data_ptr(), FV[i].data_ptr(),
             ST[i].data_ptr(), IT[i].data_ptr()) for i in range(W + K)]

    def launch(i):
        solver.solve_batch_dev(B, *ptrs[i], stream=sp)

    # kernel time base of the roofline: ONE event pair on the launch stream around the whole timed
    # loop of back-to-back launches, divided by K -- the mean launch duration including the (~0-2 us)
    # gaps between launches, so it can never exceed ms_per_step and `frac` is a lower bound; the
    # rocprofv3 average of the same launches is committed under profiles/ (tools/profile_round.sh).
    # The events are created and recorded once in the warm-up (a first record creates the HIP event
    # and once cost the timed loop ~2 ms of wall clock)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for i in range(W):
        launch(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    ev0.elapsed_time(ev1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the start event goes on the stream just before the timed region: its host cost (~10 us of torch + HIP event
    # record) is not the hot path's, and the event span then also covers the host's first launch (kernel_ms a
    # slight overestimate: roofline.frac stays a lower bound)
    with torch.cuda.stream(stream):
        ev0.record(stream)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for j in range(K):
            launch(W + j)
        ev1.record(stream)
    # the host notices the end of the last launch by polling its event (hipEventQuery) rather than by the blocking
    # wait alone, whose wake-up latency (tens of us) would otherwise count against a 20-step run; the
    # synchronize that brackets the timed region follows and returns at once
    while not ev1.query():
        pass
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / K
    if world > 1:
        elapsed, kern_ms = _max_over_ranks([elapsed, kern_ms], dev, host_coll)

    st = ST[W:].cpu().numpy()
    its = IT[W:].cpu().numpy()
    u0 = U0[W:].cpu().numpy()
    ok_frac = float(np.mean(st == 0))
    iters_sum_per_launch = float(its.sum(axis=1).mean())

    # accuracy: max |u0 - u0_ref| against the C oracle on the first timed step (rank 0)
    max_du = None
    cpu_baseline = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_lib   # checker + CPU baseline only
        S, T, P = steps_in[W]
        # u_ref = the exact KKT point (oracle driven to tol 1e-11 on the full 6-state NLP)
        ref = oracle_lib.solve_batch(S, T, P, N=N, Ts=0.002, tol=1e-11, nthreads=1, want_w=False)
        max_du = float(np.max(np.abs(u0[0] - ref["u0"])))
        if not args.no_cpu_baseline:
            try:
                ncores = len(os.sched_getaffinity(0))
            except AttributeError:
                ncores = os.cpu_count() or 1
            nthreads = max(1, min(16, ncores))
            Sb, Tb, Pb = pmpc_batch(n_seeds=4 * nthreads, seed0=777)
            oracle_lib.solve_batch(Sb[:18], Tb[:18], Pb[:18], N=N, tol=args.tol, nthreads=1, want_w=False)
            solved, c0 = 0, time.perf_counter()
            while time.perf_counter() - c0 < args.cpu_seconds:
                oracle_lib.solve_batch(Sb, Tb, Pb, N=N, Ts=0.002, tol=args.tol, nthreads=nthreads, want_w=False)
                solved += Sb.shape[0]
            cdt = time.perf_counter() - c0
            # the same oracle on one core (cores used and the 1-core rate), a fifth of the time
            solved1, c1 = 0, time.perf_counter()
            while time.perf_counter() - c1 < args.cpu_seconds / 5:
                oracle_lib.solve_batch(Sb[:18], Tb[:18], Pb[:18], N=N, Ts=0.002, tol=args.tol, nthreads=1, want_w=False)
                solved1 += 18
            cdt1 = time.perf_counter() - c1
            cpu_baseline = {"value": solved / cdt, "unit": "solves/s", "cores": nthreads, "kind": "port",
                            "sample": f"CPU restatement, not CasADi/IPOPT (neither is installed): C oracle IPM "
                                      f"(oracle/pmpc_ipm.c, IPOPT's algorithm on the full 6-state NLP, filter line search, "
                                      f"tol {args.tol:g}), {solved} cold-start solves of seeded 18-config batches "
                                      f"(N={N}) in {cdt:.1f} s on {nthreads} OpenMP threads",
                            "one_core": {"value": solved1 / cdt1, "unit": "solves/s", "cores": 1,
                                         "sample": f"{solved1} solves of the first 18-config batch in {cdt1:.1f} s"}}

    # supplementary saturated rate: one launch over a large batch (not the headline value)
    saturation = None
    if args.saturation_batch > 0:
        Bs = args.saturation_batch
        S, T, P = pmpc_batch(n_seeds=-(-Bs // 18), seed0=500000 + 1000 * rank)
        sx = torch.tensor(S[:Bs], device=dev); st_ = torch.tensor(T[:Bs], device=dev); spr = torch.tensor(P[:Bs], device=dev)
        su = torch.empty((Bs, 2), dtype=torch.float64, device=dev); sf = torch.empty(Bs, dtype=torch.float64, device=dev)
        ss = torch.empty(Bs, dtype=torch.int32, device=dev); si = torch.empty(Bs, dtype=torch.int32, device=dev)
        big = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=Bs, device=local, path=args.pmpc_path)
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            big.solve_batch_dev(Bs, sx.data_ptr(), st_.data_ptr(), spr.data_ptr(), su.data_ptr(), sf.data_ptr(),
                                ss.data_ptr(), si.data_ptr(), stream=sp)
            e1.record(stream)
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        sat_tflops = float(si.double().sum()) * F_ITER_PMPC / (ms * 1e-3) / 1e12
        saturation = {"batch": Bs, "ms_per_launch": ms, "solves_per_s": Bs / (ms * 1e-3),
                      "ok_frac": float((ss == 0).float().mean()), "iters_mean": float(si.double().mean()),
                      "roofline": {"bound": "fp64-valu", "achieved": sat_tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                   "frac": sat_tflops / FP64_PEAK_TFLOPS,
                                   "note": "same algorithmic FLOP count as the headline; the chip filled with "
                                           f"{Bs} waves instead of 18"}}

    # SURVEY 8(d)'s definition of the metric: B / wall time of dart_mpc_solve_batch, host arrays in
    # (host -> device), u0 back in host memory, every rank on its own GPU, barrier + max over ranks.
    # The task's bench contract makes `value` the device-resident rate (inputs in HBM when the timed
    # region starts), so this is reported beside it as `value_host_inclusive_8d`.
    host_incl = None
    if args.host_calls > 0:
        Kh = min(K, args.host_calls)
        bufs = dict(u0=np.empty((B, 2)), f=np.empty(B), status=np.empty(B, np.int32), iters=np.empty(B, np.int32))

        def host_leg(serve, bound=False):
            hs = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=B, device=local, path=args.pmpc_path)
            if serve:
                hs.serve_start(B_serve=B, idle_timeout=10.0)
            bd = hs.bind() if bound else None

            def call(S_, T_, P_):
                if bd is None:
                    hs.solve_batch(S_, T_, P_, out=bufs)
                else:           # inputs written in place into the mapped I/O area, u0 read from it
                    bd.x0[:B] = S_; bd.ref[:B] = T_; bd.prm[:B] = P_
                    bd.solve(B)
            for i in range(min(W, 10)):
                call(*steps_in[i])
            per_call = np.empty(Kh)
            if world > 1:
                dist.barrier()
            th0 = time.perf_counter()
            for j in range(Kh):
                c0 = time.perf_counter()
                call(*steps_in[W + j])
                per_call[j] = time.perf_counter() - c0
            th1 = time.perf_counter()
            if world > 1:
                dist.barrier()
            hs.close()
            hel, med = th1 - th0, float(np.median(per_call))
            if world > 1:
                hel, med = _max_over_ranks([hel, med], dev, host_coll)
            return {"value": world * B * Kh / hel, "unit": "solves/s", "calls": Kh, "ms_per_call": hel / Kh * 1e3,
                    "median_ms_per_call": med * 1e3, "median_solves_per_s": world * B / med}

        launched = host_leg(False)
        can_serve = args.pmpc_path == "ipopt" and N <= 31
        served = host_leg(True) if can_serve else None
        bound = host_leg(True, bound=True) if can_serve else host_leg(False, bound=True)
        host_incl = dict(bound)
        host_incl["mode"] = ("resident solver (dart_mpc_serve_start) + in-place I/O (dart_mpc_bind / "
                             "dart_mpc_solve_bound)" if can_serve else "in-place I/O, kernel launch per call")
        host_incl["solve_batch_served"] = served
        host_incl["solve_batch_launch_per_call"] = launched
        host_incl["note"] = ("SURVEY 8(d): host inputs in, u0 back in host memory, per call, from Python; barrier + "
                             "max over ranks.  `value`: fresh inputs written into the mapped I/O area, one "
                             "two-argument call, results read in place, served by the resident solver (one "
                             "long-lived grid takes each call from a mailbox: no launch, no dispatch).  Also "
                             "dart_mpc_solve_batch (host arrays copied in and out) served and with one kernel "
                             "launch per call")

    # supplementary host-pointer path (dart_mpc_solve_batch): H2D copies + solve + D2H + sync per call
    host_path = None
    if rank == 0 and args.host_calls > 0:
        hs = dart_mpc.Solver(N=N, Ts=0.002, tol=args.tol, B_max=B, device=local, path=args.pmpc_path)
        S, T, P = steps_in[W]
        for _ in range(5):
            hs.solve_batch(S, T, P)
        h0 = time.perf_counter()
        for _ in range(args.host_calls):
            hs.solve_batch(S, T, P)
        hdt = (time.perf_counter() - h0) / args.host_calls
        # one instance per call: the latency PMPC.solve / mpc_worker sees per control step
        for _ in range(5):
            hs.solve_batch(S[:1], T[:1], P[:1])
        h1 = time.perf_counter()
        for _ in range(args.host_calls):
            hs.solve_batch(S[:1], T[:1], P[:1])
        h1dt = (time.perf_counter() - h1) / args.host_calls
        host_path = {"batch": B, "ms_per_call": hdt * 1e3, "solves_per_s": B / hdt,
                     "single_instance_ms_per_call": h1dt * 1e3,
                     "note": "dart_mpc_solve_batch through the Python Solver: inputs packed into mapped, coherent "
                             "pinned host memory that the kernel reads zero-copy at its start (no DMA copy on the "
                             "call path), outputs written by the kernel into mapped pinned memory, stream sync"}
        hs.close()

    # supplementary C4 (BASELINE.json configs[3]): 1152 instances sharded over the ranks + result gather
    c4 = bench_c4(args, torch, dev, stream, dart_mpc, world, rank, host_coll, coll) if args.c4_steps > 0 else None

    # supplementary: PMPC launches holding instances that need IPOPT's restoration phases
    pmpc_resto = None
    if rank == 0 and args.resto_steps > 0:
        pmpc_resto = bench_pmpc_restoration(args, torch, dev, stream, dart_mpc)

    # supplementary: horizons beyond 31 on all three variants
    long_h = None
    if rank == 0 and args.long_steps > 0:
        long_h = bench_long_horizons(args, dart_mpc)

    # supplementary PMPC line at the DART driver's horizon (N = 15)
    n15 = None
    if rank == 0 and args.n15_steps > 0:
        n15 = bench_pmpc_driver_horizon(args, torch, dev, stream, dart_mpc)

    # supplementary C3 (BASELINE.json configs[2]): RMPC batch=18 with the RLS update fused into the launch
    rmpc = None
    if rank == 0 and args.rmpc_steps > 0:
        rmpc = bench_rmpc(args, torch, dev, stream, dart_mpc)

    # supplementary C5 (BASELINE.json configs[4]): LMPC batch=18, N=30, pvec as input
    lmpc = None
    if rank == 0 and args.lmpc_steps > 0:
        lmpc = bench_lmpc(args, torch, dev, stream, dart_mpc)
        if args.lmpc_policy_steps > 0:
            lmpc["policy_fused"] = bench_lmpc_policy(args, torch, dev, stream, dart_mpc)

    # supplementary: per-arm impedance QP
    arm = None
    if rank == 0 and args.arm_steps > 0:
        arm = bench_arm(args, torch, dev, stream, dart_mpc)

    # HBM traffic per launch from the committed rocprofv3 PMC passes of this build (tools/profile_round.sh)
    traffic = None
    pmc = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary.json")))
    if pmc:
        with open(pmc[-1]) as fh:
            traffic = json.load(fh).get("traffic_bytes_per_launch")
    # latency regime: with one wave per instance the launch is bound by the wave's own instruction
    # issue; the committed SQ counters of this build (tools/pmc_sq.sh) give the busy fraction
    issue = None
    sq = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "sq_summary.json")))
    if sq:
        with open(sq[-1]) as fh:
            pi = json.load(fh)["kernels"]["PMPC C2"]["per_instance"]
        issue = {"bound": "VALU issue of one wave per instance", "valu_busy_frac": pi["valu_busy_frac"],
                 "valu_insts_per_solve": pi["valu_insts"], "cycles_per_valu_inst": pi["cycles_per_valu_inst"],
                 "mfma_busy_frac": pi.get("mfma_busy_frac"), "source": os.path.relpath(sq[-1], ROOT)}

    if rank == 0:
        value = world * B * K / elapsed
        achieved_tflops = iters_sum_per_launch * F_ITER_PMPC / (kern_ms * 1e-3) / 1e12
        # north_star's target (>= 100x the CPU baseline's solves/s) is stated on "the 18-object x N-seed
        # batch at horizon N=20": C4's 18 x 64 instances, gather included; C2's 18 instances beside it
        ratio = None
        if cpu_baseline and cpu_baseline.get("value"):
            cb = cpu_baseline["value"]
            ratio = {"target": 100.0, "cpu_baseline_solves_per_s": cb, "cpu_cores": cpu_baseline.get("cores"),
                     "c4_18x64_vs_cpu": (c4["solves_per_s"] / cb) if c4 else None,
                     "c2_18_vs_cpu": value / cb,
                     "saturated_vs_cpu": (saturation["solves_per_s"] / cb) if saturation else None,
                     "note": "CPU baseline = the C restatement of IPOPT's algorithm (cpu_baseline.sample), "
                             "not CasADi+IPOPT (not installed); C4 is the batch north_star names"}
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "value_host_inclusive_8d": host_incl["value"] if host_incl else None,
            "dtype": "f64",
            "data": "synthetic (seeded SURVEY §8d workload, fresh instances every step)",
            "config": {"workload": "C2: PMPC batch=18 object configs (3 shapes x 2 masses x 3 frictions), "
                                   "N=20, Ts=0.002, cold start, IPOPT tol 1e-8; one rank per GPU",
                       "batch_per_gpu": B, "N": N, "parallelism": f"instance-sharded x{world}",
                       **({"dist_backend": backend} if coll else {})},
            "roofline": {"bound": "fp64-valu", "achieved": achieved_tflops, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved_tflops / FP64_PEAK_TFLOPS, "traffic": traffic,
                         "kernel": "pmpc_ipm_kernel", "kernel_ms": kern_ms, "issue": issue,
                         "note": "FP64 vector compute roof (78.6 TFLOP/s; the FP64 MFMA rate is the same on gfx950 "
                                 "and no MFMA instruction is issued: issue.mfma_busy_frac, SQ_VALU_MFMA_BUSY_CYCLES); "
                                 "algorithmic FLOP = sum(iters) x 6.0e4 per launch; time = one HIP event pair around "
                                 "the K back-to-back launches of the timed loop / K; algorithmic HBM bytes = 176 per "
                                 "solve"},
            "cpu_baseline": cpu_baseline,
            "north_star_ratio": ratio,
            "max_abs_u0_err_vs_exact_optimum": max_du,
            "status_ok_frac": ok_frac,
            "iters_mean": float(its.mean()),
            "saturation": saturation,
            "host_path_pcie_inclusive": host_path,
            "host_inclusive_8d": host_incl,
            "pmpc_c4": c4,
            "pmpc_restoration": pmpc_resto,
            "pmpc_n15": n15,
            "long_horizons": long_h,
            "rmpc_c3": rmpc,
            "lmpc_c5": lmpc,
            "arm_qp": arm,
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if coll:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
