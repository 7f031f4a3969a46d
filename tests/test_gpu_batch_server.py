"""mpc_batch_server on the GPU: six spawned fake-sim clients, each with its own
object parameters (one C2 configuration apiece) and the reference's queue protocol, are served by
one process through the resident solver and in-place I/O.  Every reply must be bit-equal to a
launched solve of the same instance and within 1e-6 of the oracle (the tolerance of the other PMPC
parity tests), in the client's request order."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _client(cid, rows, pipelined, sq, cq, out):
    import numpy as np
    S, T = rows
    replies = []
    if pipelined:
        for s, t in zip(S, T):
            sq.put((s, t))
        replies = [cq.get(timeout=120) for _ in range(len(S))]
    else:
        for s, t in zip(S, T):
            sq.put((s, t))
            replies.append(cq.get(timeout=120))
    sq.put("STOP")
    out.put((cid, [r[0] for r in replies], np.concatenate([r[1] for r in replies]), [r[2] for r in replies]))


def test_batch_server_replies_equal_launch_and_oracle():
    import multiprocessing as mp
    import dart_mpc
    import oracle_lib
    from dart_mpc.workload import pmpc_batch
    S, T, P = pmpc_batch(4)            # 18 configurations x 4 seeds, seed-major (row 18 s + config)
    n, K = 6, 4
    order = np.array([18 * s + c for c in range(n) for s in range(K)])    # client c <- config c's seeds
    S, T, P = S[order], T[order], P[order]
    ctx = mp.get_context("spawn")
    sqs, cqs = [ctx.Queue() for _ in range(n)], [ctx.Queue() for _ in range(n)]
    out = ctx.Queue()
    rows = {c: (S[c * K:(c + 1) * K], T[c * K:(c + 1) * K]) for c in range(n)}
    procs = [ctx.Process(target=_client, args=(c, rows[c], c % 2 == 0, sqs[c], cqs[c], out)) for c in range(n)]
    for p in procs:
        p.start()
    clients = []
    for c in range(n):
        mu, qp, qv, r, lo, hi = P[c * K]
        clients.append(("cube", dict(Ts=0.002, nx=6, nu=2, N=15, Qp=qp, Qv=qv, R=r, u_bounds=(lo, hi), mu=mu),
                        sqs[c], cqs[c]))
    sizes = dart_mpc.mpc_batch_server("unused.xml", clients)
    got = {}
    for _ in range(n):
        cid, u, f, dt = out.get(timeout=120)
        got[cid] = (np.stack(u), f, dt)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(sizes) == n * K and max(sizes) <= n
    B = n * K
    launch = dart_mpc.Solver(N=15, Ts=0.002, tol=1e-8, max_iter=3000, B_max=B)
    one = launch.solve_batch(S[:B], T[:B], P[:B])
    launch.close()
    ref = oracle_lib.solve_batch(S[:B], T[:B], P[:B], N=15, tol=1e-8, max_iter=3000)
    for c in range(n):
        u, f, dt = got[c]
        sl = slice(c * K, (c + 1) * K)
        np.testing.assert_array_equal(u, one["u0"][sl])
        np.testing.assert_array_equal(f, one["f"][sl])
        assert np.max(np.abs(u - ref["u0"][sl])) <= 1e-6
        assert all(t >= 0.0 for t in dt)
