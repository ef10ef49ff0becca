"""Row-sharded sqrt-PST commit across ranks.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on
MI355X, "gloo" on CPU for tests).  The 2^m_col row MSMs of
``Polynomial::commit`` (sqrt_pst.rs:121-125) are independent: rank g owns rows
[g*R, (g+1)*R), R = 2^m_col / world -- a contiguous block of *columns* of Z,
which the K1 kernel reads through the strided view with no data movement.

Exchange: every rank also runs the Miller loops of its own rows' pairs
(C_i, h_i) and keeps their product f_g unreduced, so the IPP
T = prod e(C_i, h_i) (sqrt_pst.rs:128-143) is split by rows too.  One RCCL
all-gather moves each rank's [row commitments (96 B each) | f_g (576 B)] as
raw bytes (RCCL has no elliptic-curve or GT reduction op, so nothing is
reduced in flight); rank 0 multiplies the world's f_g and runs the single
final exponentiation, then broadcasts T (576 B).  The per-rank compute and
the finalisation are injected, so the orchestration is testable on CPU with
the C++ oracle standing in for the GPU (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np


def shard_rows(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    if n_rows % world:
        raise ValueError("row count %d not divisible by world size %d" % (n_rows, world))
    per = n_rows // world
    return rank * per, (rank + 1) * per


def sharded_commit(n: int, commit_rows_partial: Callable[[int, int], Tuple[np.ndarray, np.ndarray]],
                   finalize: Callable[[np.ndarray], np.ndarray], dist, device) -> Tuple[np.ndarray, np.ndarray]:
    """Returns (comm_list (2^m_col, 12) uint64, T (72,) uint64) on every rank.

    commit_rows_partial(r0, r1) -> (comms (r1-r0, 12), miller partial (72,));
    finalize(partials (world, 72)) -> T, run on rank 0 only."""
    import torch
    if dist.get_backend() == "gloo":  # gloo gathers host tensors only
        device = "cpu"
    world = dist.get_world_size()
    rank = dist.get_rank()
    m_col = n // 2
    r0, r1 = shard_rows(1 << m_col, world, rank)
    comms, ml = commit_rows_partial(r0, r1)
    local = np.concatenate([np.ascontiguousarray(comms, dtype=np.uint64).reshape(-1),
                            np.ascontiguousarray(ml, dtype=np.uint64).reshape(72)])
    t = torch.from_numpy(local.view(np.int64).copy()).to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)  # C1: row commitments + Miller partials, bytes only
    got = torch.stack(parts).cpu().numpy().view(np.uint64)
    R = r1 - r0
    comm_list = got[:, :12 * R].reshape(-1, 12).copy()
    T = torch.zeros(72, dtype=torch.int64, device=device)
    if rank == 0:
        T.copy_(torch.from_numpy(np.ascontiguousarray(finalize(got[:, 12 * R:]), dtype=np.uint64).view(np.int64)))
    dist.broadcast(T, src=0)
    return comm_list, T.cpu().numpy().view(np.uint64).copy()
