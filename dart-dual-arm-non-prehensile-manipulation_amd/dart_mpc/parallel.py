"""Instance sharding across GPUs (one process per GPU) and the single result gather.

SURVEY.md §8e: MPC instances are independent, so a batch (object-config sweep
x Monte-Carlo seeds) is split into contiguous per-rank blocks of ceil(B/G)
instances.  Each rank builds or receives its own block and solves it locally;
the only collective is one ``all_gather_into_tensor`` of the packed results
``[u0_x, u0_y, f, status]`` (fp64, padded to the block size) -- RCCL over xGMI
with backend "nccl" on MI355X, gloo on CPU.  It is off the timed data path in
bench.py (weak scaling).
"""
from __future__ import annotations

import numpy as np

RESULT_COLS = 4     # u0[2], f, status


def shard_bounds(B: int, world: int, rank: int):
    """Half-open [lo, hi) of rank's contiguous block (ceil(B/world) per rank)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    per = -(-int(B) // world)
    lo = min(B, rank * per)
    return lo, min(B, lo + per)


def pack_results(u0, f, status, rows: int):
    """[rows, 4] fp64 block (zero padded) of one rank's results."""
    n = len(f)
    out = np.zeros((rows, RESULT_COLS))
    out[:n, 0:2] = np.asarray(u0).reshape(n, 2)
    out[:n, 2] = f
    out[:n, 3] = status
    return out


def gather_results(local_block, B: int, world: int, group=None, device=None):
    """All-gather the per-rank [ceil(B/world), 4] blocks; returns (u0[B,2], f[B], status[B]) on every rank."""
    import torch
    import torch.distributed as dist
    per = -(-int(B) // world)
    t = torch.as_tensor(np.ascontiguousarray(local_block), dtype=torch.float64)
    if device is not None:
        t = t.to(device)
    full = torch.empty((world * per, RESULT_COLS), dtype=torch.float64, device=t.device)
    dist.all_gather_into_tensor(full, t, group=group)
    a = full.cpu().numpy()[:B]
    return a[:, 0:2].copy(), a[:, 2].copy(), a[:, 3].astype(np.int32)


def solve_sharded(solve_fn, states, targets, params, world: int, rank: int, group=None, device=None):
    """Solve this rank's block with ``solve_fn(states, targets, params) -> dict(u0, f, status)``
    and gather every rank's results."""
    B = states.shape[0]
    lo, hi = shard_bounds(B, world, rank)
    out = solve_fn(states[lo:hi], targets[lo:hi], params[lo:hi])
    block = pack_results(out["u0"], out["f"], out["status"], -(-B // world))
    return gather_results(block, B, world, group=group, device=device)
