"""Row-sharded sqrt-PST commit across ranks.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on
MI355X, "gloo" on CPU for tests).  The 2^m_col row MSMs of
``Polynomial::commit`` (sqrt_pst.rs:121-125) are independent: rank g owns rows
[g*R, (g+1)*R), R = 2^m_col / world -- a contiguous block of *columns* of Z,
which the K1 kernel reads through the strided view with no data movement.

Exchange: C1 = all-gather of the 96-byte row commitments (RCCL moves bytes;
there is no elliptic-curve reduction op, so nothing is reduced in flight);
the IPP T = prod e(C_i, h_i) (sqrt_pst.rs:128-143) is then computed on rank 0
over the gathered list and broadcast (576 bytes).  The per-rank compute and
the IPP are injected, so the orchestration is testable on CPU with the
oracle standing in for the GPU (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np


def shard_rows(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    if n_rows % world:
        raise ValueError("row count %d not divisible by world size %d" % (n_rows, world))
    per = n_rows // world
    return rank * per, (rank + 1) * per


def sharded_commit(n: int, commit_rows: Callable[[int, int], np.ndarray], ipp: Callable[[np.ndarray], np.ndarray],
                   dist, device) -> Tuple[np.ndarray, np.ndarray]:
    """Returns (comm_list (2^m_col, 12) uint64, T (72,) uint64) on every rank."""
    import torch
    world = dist.get_world_size()
    rank = dist.get_rank()
    m_col = n // 2
    r0, r1 = shard_rows(1 << m_col, world, rank)
    local = np.ascontiguousarray(commit_rows(r0, r1), dtype=np.uint64).reshape(r1 - r0, 12)
    t = torch.from_numpy(local.view(np.int64).reshape(-1).copy()).to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)  # C1: row commitments, bytes only
    comms = torch.cat(parts).cpu().numpy().view(np.uint64).reshape(-1, 12)
    T = torch.zeros(72, dtype=torch.int64, device=device)
    if rank == 0:
        T.copy_(torch.from_numpy(np.ascontiguousarray(ipp(comms), dtype=np.uint64).view(np.int64)))
    dist.broadcast(T, src=0)
    return comms, T.cpu().numpy().view(np.uint64).copy()
