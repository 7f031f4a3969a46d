"""CPU side of the RMPC status-2 investigation: whose iterate is off where the kernel and
the oracle both end an infeasible start at status 2 (IPOPT's Infeasible_Problem_Detected) with different u0.

Input: gpurun_out/rmpc_status2_kernel.npz (tools/rmpc_dump_status2.py on the GPU box).  For every case and every
instance both solvers end at status 2 it computes, solver-independently (oracle/rmpc_nlp.py):
  * V(w): the l1 constraint violation of the reference NLP (np_mpc...:103-127: x0 pinning, RK4 defects, du rows,
    velocity caps; U box kept) at the kernel's and at the oracle's point -- the quantity IPOPT's restoration phase
    minimises (MinC_1NrmRestorationPhase);
  * the l1-stationarity certificate (no decrease of the linearised violation within |d| <= 1e-4) at both;
  * V along the segment between the two points: flat means both lie on one face of l1 minimisers, where the
    restoration problem fixes the point only through its proximity term eta/2 |D_R (x - x_R)|^2, eta = sqrt(mu);
  * both points re-solved by the oracle at tol 1e-10 from their own w (IPOPT warm start), and the oracle cold at
    tol 1e-10: which of the two tol-1e-8 points is nearer the tighter answers.
Usage: [DART_S2_CASES=... DART_S2_OUT=...] python tools/rmpc_status2_analysis.py [top_k]  (default profiles/r05/rmpc_status2.txt)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd"),
                os.path.join(ROOT, "tools")]
import oracle_lib  # noqa: E402  (checker)
import rmpc_nlp  # noqa: E402
from rmpc_dump_status2 import CASES, batch  # noqa: E402

N = 20
NX = 4 * (N + 1)


violation = rmpc_nlp.l1_violation


def main():
    top_k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    K = np.load(os.path.join(ROOT, "gpurun_out", "rmpc_status2_kernel.npz"))
    lines = []
    pr = lambda s="": (print(s, flush=True), lines.append(s))
    keys = ("x0", "u_prev", "theta", "Rref", "prm")
    for name, (n, seed0, spread) in CASES.items():
        D = batch(n, seed0, spread)
        args = tuple(D[k] for k in keys)
        o = oracle_lib.rmpc_solve_batch(*args, N=N, tol=1e-8, nthreads=8)
        g = {k: K[f"{name}/{k}"] for k in ("u0", "w", "status", "iters")}
        b18 = {k: K[f"{name}/b18_{k}"] for k in ("u0", "w", "status", "iters")}
        inf = (g["status"] == 2) & (o["status"] == 2)
        idx = np.flatnonzero(inf)
        du = np.abs(g["u0"] - o["u0"]).max(axis=1)
        pr(f"== {name}: {len(g['status'])} instances, status equal {np.mean(g['status'] == o['status']):.4f}, "
           f"status 2 by both {idx.size}; batches of 18 = one launch bit for bit: "
           f"{all(np.array_equal(g[k], b18[k]) for k in g)}")
        pr(f"   |du0| on status 2: median {np.median(du[idx]):.2e}, 99 % {np.quantile(du[idx], 0.99):.2e}, "
           f"max {du[idx].max():.2e}; iterations equal {np.mean(g['iters'][idx] == o['iters'][idx]):.4f}")
        # the certificate and the violation on every status-2 instance
        Vk = np.array([violation(g["w"][i], D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i]) for i in idx])
        Vo = np.array([violation(o["w"][i], D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i]) for i in idx])
        dec_k = np.array([rmpc_nlp.l1_stationarity(g["w"][i], D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i])[0]
                          for i in idx])
        dec_o = np.array([rmpc_nlp.l1_stationarity(o["w"][i], D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i])[0]
                          for i in idx])
        rel = np.abs(Vk - Vo) / np.maximum(Vo, 1e-300)
        pr(f"   l1 violation V: kernel - oracle relative median {np.median(rel):.1e}, max {rel.max():.1e} "
           f"(kernel lower on {int(np.sum(Vk < Vo))}, higher on {int(np.sum(Vk > Vo))}); l1-stationarity decrease "
           f"within |d| <= 1e-4: kernel max {dec_k.max():.1e}, oracle max {dec_o.max():.1e}")
        # the instances with the largest |du0|
        worst = idx[np.argsort(-du[idx])[:top_k]]
        wk = g["w"][worst]
        wo = o["w"][worst]
        sub = tuple(a[worst] for a in args)
        rk = oracle_lib.rmpc_solve_batch(*sub, N=N, tol=1e-10, w_init=wk, nthreads=8)
        ro = oracle_lib.rmpc_solve_batch(*sub, N=N, tol=1e-10, w_init=wo, nthreads=8)
        rc = oracle_lib.rmpc_solve_batch(*sub, N=N, tol=1e-10, nthreads=8)
        for j, i in enumerate(worst):
            a = (D["x0"][i], D["u_prev"][i], D["theta"][i], D["prm"][i])
            seg = [violation(wo[j] + t * (wk[j] - wo[j]), *a) for t in (0.0, 0.25, 0.5, 0.75, 1.0)]
            flat = (max(seg) - min(seg)) / max(seg)
            vk, vo = violation(wk[j], *a), violation(wo[j], *a)
            d_res = lambda w1, w2: np.abs(w1[NX:NX + 2] - w2[NX:NX + 2]).max()
            pr(f"   #{i}: |du0| {du[i]:.2e}, iterations kernel {g['iters'][i]} oracle {o['iters'][i]}; "
               f"V kernel {vk:.10e} oracle {vo:.10e}; V on the segment flat to {flat:.1e}")
            pr(f"       oracle tol 1e-10 from the kernel's w: status {rk['status'][j]}, u0 moves {d_res(rk['w'][j], wk[j]):.2e}; "
               f"from the oracle's w: status {ro['status'][j]}, u0 moves {d_res(ro['w'][j], wo[j]):.2e}; "
               f"cold tol 1e-10: status {rc['status'][j]}, u0 from kernel {d_res(rc['w'][j], wk[j]):.2e} / from oracle "
               f"{d_res(rc['w'][j], wo[j]):.2e}; the two re-solved points {d_res(rk['w'][j], ro['w'][j]):.2e} apart")
    out = os.environ.get("DART_S2_OUT", os.path.join(ROOT, "profiles", "r05", "rmpc_status2.txt"))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
