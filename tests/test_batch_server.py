"""mpc_batch_server's host logic (no GPU): several spawned fake-sim clients speak the reference's
queue protocol (main_parallel_enhanced.py:22-55 -- ``(state, target)`` / ``"STOP"`` in, ``(u_cmd, loss,
solve_time)`` out); the server batches their pending requests and must route every reply to its own
client in request order, group clients by horizon, and return once all clients stopped.  The GPU
handle is replaced by a numpy stand-in whose output is a fixed function of each row's inputs, so a
misrouted or reordered reply shows up as a wrong value."""
import numpy as np


def fake_u0(x0, ref, prm):
    return np.array([x0 @ prm + ref[0], x0[2] - 3.0 * ref[4]])


class _FakeBound:
    def __init__(self, B_max, N, log):
        self.x0, self.ref, self.prm = np.zeros((B_max, 6)), np.zeros((B_max, 6)), np.zeros((B_max, 6))
        self.u0, self.f = np.zeros((B_max, 2)), np.zeros(B_max)
        self.N, self.log = N, log

    def solve(self, B):
        self.log.append((self.N, B))
        for r in range(B):
            self.u0[r] = fake_u0(self.x0[r], self.ref[r], self.prm[r])
            self.f[r] = self.ref[r].sum() + self.N


class _FakeSolver:
    def __init__(self, N, Ts, B_max, log):
        self.bound = _FakeBound(B_max, N, log)
        self.closed = False

    def bind(self):
        return self.bound

    def close(self):
        self.closed = True


def _client(cid, K, pipelined, sq, cq, out):
    rng = np.random.default_rng(100 + cid)
    reqs = [(rng.uniform(-0.2, 0.2, 6), rng.uniform(-0.2, 0.2, 6)) for _ in range(K)]
    replies = []
    if pipelined:                   # all requests queued before the first reply is read
        for r in reqs:
            sq.put(r)
        replies = [cq.get(timeout=60) for _ in reqs]
    else:                           # the reference driver: one request, wait for its reply
        for r in reqs:
            sq.put(r)
            replies.append(cq.get(timeout=60))
    sq.put("STOP")
    out.put((cid, reqs, replies))


def _params(cid):
    return dict(Ts=0.002, nx=6, nu=2, N=15 if cid % 3 else 20, Qp=100.0 + 50 * cid, Qv=float(cid), R=0.1,
                u_bounds=(-0.5 - 0.01 * cid, 0.5), mu=0.1 + 0.05 * cid)


def test_batch_server_routes_fifo_replies_per_client():
    import multiprocessing as mp
    import dart_mpc
    from dart_mpc.batch_server import _prm_row
    ctx = mp.get_context("spawn")
    n, K = 5, 6
    sqs, cqs = [ctx.Queue() for _ in range(n)], [ctx.Queue() for _ in range(n)]
    out = ctx.Queue()
    procs = [ctx.Process(target=_client, args=(c, K, c % 2 == 1, sqs[c], cqs[c], out)) for c in range(n)]
    for p in procs:
        p.start()
    log, made = [], []

    def factory(N, Ts, B_max):
        s = _FakeSolver(N, Ts, B_max, log)
        made.append(s)
        return s

    clients = [("cube", _params(c), sqs[c], cqs[c]) for c in range(n)]
    sizes = dart_mpc.mpc_batch_server("unused.xml", clients, solver_factory=factory)
    res = {}
    for _ in range(n):
        cid, reqs, replies = out.get(timeout=60)
        res[cid] = (reqs, replies)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert sorted(res) == list(range(n))
    for cid, (reqs, replies) in res.items():
        prm = _prm_row(_params(cid))
        assert len(replies) == K
        for (x, t), (u, loss, dt) in zip(reqs, replies):
            np.testing.assert_allclose(u, fake_u0(np.asarray(x), np.asarray(t), prm), rtol=0, atol=1e-15)
            assert loss.shape == (1,) and loss[0] == t.sum() + _params(cid)["N"] and dt >= 0.0
    # two horizon groups (N=15 / N=20), every request solved exactly once, batches never exceed the group
    assert sorted(len([c for c in range(n) if _params(c)["N"] == N]) for N in (15, 20)) == [2, 3]
    assert sum(sizes) == n * K == sum(B for _, B in log)
    assert all(B <= 3 for _, B in log)
    assert len(made) == 2 and all(s.closed for s in made)


def test_batch_server_rejects_non_pmpc_dims():
    import queue
    import pytest
    import dart_mpc
    with pytest.raises(ValueError):
        dart_mpc.mpc_batch_server("x", [("cube", dict(nx=8, nu=2), queue.Queue(), queue.Queue())],
                                  solver_factory=lambda *a: None)
