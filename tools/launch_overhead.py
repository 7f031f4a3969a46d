"""Diagnostic: where the fixed overhead of a K-step timed loop goes (C2 launches, inputs in HBM): host timestamps around
the event record, the first launch, the loop and the wait, against the events' GPU span; then the same K launches
captured once in a HIP graph (torch.cuda.CUDAGraph on the launch stream) and replayed.  Usage: python
tools/launch_overhead.py [K]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))
import torch  # noqa: E402
import dart_mpc  # noqa: E402
from dart_mpc.workload import pmpc_batch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W = 5
dev = torch.device("cuda", 0)
B = 18
ins = [pmpc_batch(1, seed0=i) for i in range(W + K)]
f64 = lambda a: torch.tensor(np.stack(a), dtype=torch.float64, device=dev).contiguous()
X0, RF, PR = f64([s[0] for s in ins]), f64([s[1] for s in ins]), f64([s[2] for s in ins])
U0 = torch.empty((W + K, B, 2), dtype=torch.float64, device=dev); FV = torch.empty((W + K, B), dtype=torch.float64, device=dev)
ST = torch.empty((W + K, B), dtype=torch.int32, device=dev); IT = torch.empty((W + K, B), dtype=torch.int32, device=dev)
solver = dart_mpc.Solver(N=20, Ts=0.002, tol=1e-8, B_max=B, device=0)
stream = torch.cuda.Stream(device=dev)
sp = stream.cuda_stream
ptrs = [(X0[i].data_ptr(), RF[i].data_ptr(), PR[i].data_ptr(), U0[i].data_ptr(), FV[i].data_ptr(), ST[i].data_ptr(),
         IT[i].data_ptr()) for i in range(W + K)]
launch = lambda i: solver.solve_batch_dev(B, *ptrs[i], stream=sp)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(5):
    for i in range(W):
        launch(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev0.record(stream)
        ta = time.perf_counter()
        launch(W)
        tb = time.perf_counter()
        for j in range(1, K):
            launch(W + j)
        ev1.record(stream)
    tc = time.perf_counter()
    while not ev1.query():
        pass
    td = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gpu = ev0.elapsed_time(ev1) * 1e3
    print(f"rep {rep}: wall {1e6 * (t1 - t0):7.1f} us  GPU events {gpu:7.1f} us  overhead {1e6 * (t1 - t0) - gpu:6.1f} us | "
          f"record {1e6 * (ta - t0):5.1f}  first launch {1e6 * (tb - ta):5.1f}  rest {1e6 * (tc - tb):6.1f}  "
          f"wait {1e6 * (td - tc):6.1f}  sync {1e6 * (t1 - td):5.1f} us", flush=True)
ref = U0[W:].clone()
# the same K launches in a HIP graph
g = torch.cuda.CUDAGraph()
try:
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=stream):
        for j in range(K):
            launch(W + j)
    ok = True
except Exception as e:      # capture not possible: report and stop
    print("graph capture failed:", repr(e))
    ok = False
def upload(graph):
    """hipGraphUpload of the instantiated graph on the launch stream (no execution)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return hip.hipGraphUpload(ctypes.c_void_p(graph.raw_cuda_graph_exec()), ctypes.c_void_p(sp))


if ok:
    # a W-step warmup graph replayed first: does it warm the first replay of a separate K-step graph?
    gw, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(gw, stream=stream):
        for i in range(W):
            launch(i)
    with torch.cuda.graph(g3, stream=stream):
        for j in range(K):
            launch(W + j)
    gw.replay()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        ev0.record(stream)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        g3.replay()
        ev1.record(stream)
    while not ev1.query():
        pass
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"warmup graph, then the K-step graph's first replay: wall {1e6 * (t1 - t0):7.1f} us", flush=True)
    # launches with the start event recorded before the timed region
    for rep in range(3):
        for i in range(W):
            launch(i)
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            ev0.record(stream)
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            for j in range(K):
                launch(W + j)
            ev1.record(stream)
        while not ev1.query():
            pass
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        print(f"launches, start event before t0: wall {1e6 * (t1 - t0):7.1f} us  events {ev0.elapsed_time(ev1) * 1e3:7.1f} us",
              flush=True)
    # a second graph of the same K launches, uploaded but never replayed before its timed replay
    g2 = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g2, stream=stream):
        for j in range(K):
            launch(W + j)
    rc = upload(g2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        g2.replay()
    while not ev1.query():
        pass
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"uploaded graph (rc {rc}), first replay: wall {1e6 * (t1 - t0):7.1f} us", flush=True)
    U0.zero_()
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            ev0.record(stream)
            g.replay()
            ev1.record(stream)
        while not ev1.query():
            pass
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        gpu = ev0.elapsed_time(ev1) * 1e3
        print(f"graph rep {rep}: wall {1e6 * (t1 - t0):7.1f} us  GPU events {gpu:7.1f} us  per step {1e6 * (t1 - t0) / K:6.2f} us",
              flush=True)
    print("graph outputs equal to the launches:", bool(torch.equal(U0[W:], ref)))
solver.close()
