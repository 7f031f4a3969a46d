"""A/B timing of one solver variant on the GPU box (run once per library, DART_MPC_LIB + DART_MPC_AB=1).

Usage: python tools/ab_variant.py <rmpc|lmpc|pmpc|rmpc_inf> <launches> <out.npz>
Times <launches> back-to-back launches of the variant's bench workload (inputs resident in HBM, batch 18) by one
HIP event pair and prints the mean launch time; saves every launch's u0 / status / iters so that two builds can be
compared bit for bit (tools/ab_compare.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"))
import torch  # noqa: E402
import dart_mpc  # noqa: E402
from dart_mpc import workload as W  # noqa: E402

kind, K, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
dev = torch.device("cuda", 0)
f64 = lambda a: torch.tensor(np.asarray(a), dtype=torch.float64, device=dev).contiguous()
B = 18
nb = min(K, 200)                 # distinct input batches, cycled
if kind in ("rmpc", "rmpc_inf"):
    D = [W.rmpc_batch(1, seed0=9000 + i) for i in range(nb)]
    if kind == "rmpc_inf":
        for d in D:
            d["x0"] = d["x0"].copy(); d["x0"][:, [1, 3]] *= 3.0
    X = [f64(np.stack([d[k] for d in D])) for k in ("x0", "u_prev", "theta", "Rref", "prm")]
    s = dart_mpc.RmpcSolver(N=20, tol=1e-8, B_max=B, device=0)
    call = lambda i, o: s.solve_batch_dev(B, *[x[i % nb].data_ptr() for x in X], *o, stream=sp)
elif kind == "lmpc":
    from dart_mpc._lib import LMPC_PRM_DEFAULT
    D = [W.lmpc_batch(1, seed0=7000 + i) for i in range(nb)]
    X = [f64(np.stack([d[k] for d in D])) for k in ("state", "u_prev", "pvec", "target")]
    PR = f64(np.tile(LMPC_PRM_DEFAULT, (B, 1)))
    s = dart_mpc.LmpcSolver(N=30, B_max=B, device=0)
    call = lambda i, o: s.solve_batch_dev(B, *[x[i % nb].data_ptr() for x in X], PR.data_ptr(), *o, stream=sp)
elif kind == "arm":
    # the bench's arm QP line: 36 arm snapshots per launch (18 configs x 2 arms), n = 7, reference parameters
    from dart_mpc.arm import pack_params, pack_snapshot
    from dart_mpc.workload import arm_batch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import arm_qp   # (the reference parameters only)
    snaps = [arm_batch(1, seed0=5000 + i)[0] for i in range(nb)]
    B = snaps[0]["q"].shape[0]
    SR = f64(np.stack([pack_snapshot(x) for x in snaps]))
    PR = f64(pack_params(arm_qp.default_params()))
    s = dart_mpc.ArmSolver(7)
    TQ = torch.empty((K, B, 7), dtype=torch.float64, device=dev)
    call = lambda i, o: s.solve_batch_dev(B, SR[i % nb].data_ptr(), PR.data_ptr(), True, o[0], TQ[i].data_ptr(),
                                          o[1], o[2], o[3], stream=sp)
elif kind in ("pmpc_resto", "pmpc_soc0"):
    # C4's 1152 instances with IPOPT's restoration phases in play: N = 31 (a few restored), or N = 20 with
    # max_soc = 0 (about one in ten restored); one launch per call, the same inputs every call
    B, nb = 1152, 1
    S_, T_, P_ = W.pmpc_batch(64, seed0=300000)
    X = [f64(a)[None] for a in (S_, T_, P_)]
    s = dart_mpc.Solver(N=31 if kind == "pmpc_resto" else 20, tol=1e-8, B_max=B, device=0,
                        max_soc=4 if kind == "pmpc_resto" else 0)
    call = lambda i, o: s.solve_batch_dev(B, *[x[0].data_ptr() for x in X], *o, stream=sp)
else:
    Ds = [W.pmpc_batch(1, seed0=i) for i in range(nb)]
    X = [f64(np.stack([d[j] for d in Ds])) for j in range(3)]
    s = dart_mpc.Solver(N=20, tol=1e-8, B_max=B, device=0)
    call = lambda i, o: s.solve_batch_dev(B, *[x[i % nb].data_ptr() for x in X], *o, stream=sp)
stream = torch.cuda.Stream(device=dev)
sp = stream.cuda_stream
U0 = torch.empty((K, B, 7 if kind == "arm" else 2), dtype=torch.float64, device=dev)
ST = torch.empty((K, B), dtype=torch.int32, device=dev)
IT = torch.empty((K, B), dtype=torch.int32, device=dev)
FV = torch.empty((K, B), dtype=torch.float64, device=dev)
outs = lambda i: (U0[i].data_ptr(), FV[i].data_ptr(), ST[i].data_ptr(), IT[i].data_ptr())
for i in range(10):
    call(i, outs(i))
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(stream):
    e0.record(stream)
    for i in range(K):
        call(i, outs(i))
    e1.record(stream)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
np.savez(out, u0=U0.cpu().numpy(), st=ST.cpu().numpy(), it=IT.cpu().numpy(), f=FV.cpu().numpy())
print(f"{os.environ.get('DART_MPC_LIB', 'libdartmpc.so')} {kind} {ms * 1e3:.2f} us/launch {B / ms * 1e3:.0f} solves/s")
