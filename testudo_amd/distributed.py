"""Row-sharded sqrt-PST commit and opening inputs across ranks.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on
MI355X, "gloo" on CPU for tests).  The 2^m_col row MSMs of
``Polynomial::commit`` (sqrt_pst.rs:121-125) are independent: rank g owns rows
[g*R, (g+1)*R), R = 2^m_col / world -- a contiguous block of *columns* of Z,
which the K1 kernel reads through the strided view with no data movement.

Commit exchange (C1/C2): every rank also runs the Miller loops of its own rows'
pairs (C_i, h_i) and keeps their product f_g unreduced, so the IPP
T = prod e(C_i, h_i) (sqrt_pst.rs:128-143) is split by rows too.  One
all-gather moves each rank's [row commitments (96 B each) | f_g (576 B)] as
raw bytes, device tensor to device tensor (RCCL has no elliptic-curve or GT
reduction op, so nothing is reduced in flight); rank 0 multiplies the world's
f_g and runs the single final exponentiation straight from the gathered
device buffer, then broadcasts T (576 B).

Opening exchange (C3): get_q's mat-vec z_q[j] = sum_i Z_i[j] chi_i(b)
(sqrt_pst.rs:92-95) and c_u = sum_i chi_i(b) C_i (sqrt_pst.rs:198) are sums
over rows, so each rank computes its rows' share of both; one all-gather of
[z_q share (2^m_row Fr) | c_u share (G1)] and a mod-r / G1 sum on rank 0 give
q and U, and rank 0 opens from q alone (no rank holds the whole Z).

Sharded opening (C4): the MIPP rounds (mipp.rs:58-120) run on every rank
over its rows i = rank mod W (tpst_poly_open_sharded): each round's cross
MSMs, folds, h preparations and look-ahead pairings on the rank's own rows,
one all-gather per product (cross partials as XYZZ, Miller partials before
the final exponentiation), every rank replaying the transcript; once a round
is shorter than 4W the folded vector moves to rank 0, which finishes the
rounds, the PST proof of q and the final folds.  The library calls back into
TorchExchange for each all-gather: an RCCL all_gather_into_tensor enqueued on
the library's comm stream (no host synchronisation), or, over gloo, a host
round trip.

Split MSM (strong scaling): one variable-base MSM (sqrt_pst.rs:198,
mipp.rs:393) over n points is cut into equal contiguous point ranges; each
rank computes its range's sum as a raw XYZZ point (192 B, no per-rank affine
inversion), one all-gather moves the shares as bytes and one device sums them
(tpst_g1_xyzz_sum_dev) -- the "single reduce of partial bucket sums", done as
a gather because RCCL has no elliptic-curve reduction.

The per-rank compute and the combines are injected, so the orchestration is
testable on CPU with the C++ oracle standing in for the GPU
(tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_rows(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    if n_rows % world:
        raise ValueError("row count %d not divisible by world size %d" % (n_rows, world))
    per = n_rows // world
    return rank * per, (rank + 1) * per


def _device(dist, device):
    return "cpu" if dist.get_backend() == "gloo" else device  # gloo moves host tensors only


def _all_gather(dist, t):
    """(world, *t.shape) tensor on t's device: one all-gather of equal-size shares."""
    import torch
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return torch.stack(parts)


def sharded_commit(n: int, commit_rows_partial_into: Callable, finalize: Callable, dist,
                   device) -> Tuple[Optional[np.ndarray], np.ndarray, np.ndarray]:
    """Row-sharded Polynomial::commit.

    commit_rows_partial_into(r0, r1, out) fills the int64 tensor ``out`` (on
    the rank's device, R * 12 + 72 words) with [row commitments (R, 12) |
    unreduced Miller partial (72)] as canonical u64 limbs;
    finalize(gathered) -> T (72,) uint64 runs on rank 0 over the gathered
    (world, R * 12 + 72) device tensor.

    Returns (comm_list (2^m_col, 12) uint64 on every rank, T (72,) on every
    rank, this rank's own row commitments (R, 12))."""
    import torch
    dev = _device(dist, device)
    world, rank = dist.get_world_size(), dist.get_rank()
    r0, r1 = shard_rows(1 << (n // 2), world, rank)
    R = r1 - r0
    buf = torch.empty(R * 12 + 72, dtype=torch.int64, device=dev)
    commit_rows_partial_into(r0, r1, buf)
    got = _all_gather(dist, buf)  # C1 + C2: bytes only
    own = buf[:12 * R].cpu().numpy().view(np.uint64).reshape(R, 12).copy()
    T = torch.zeros(72, dtype=torch.int64, device=dev)
    # every rank holds the gathered list (the sharded opening reads all of it)
    comm_list = got[:, :12 * R].cpu().numpy().view(np.uint64).reshape(-1, 12).copy()
    if rank == 0:
        T.copy_(torch.from_numpy(np.ascontiguousarray(finalize(got), dtype=np.uint64).view(np.int64)))
    dist.broadcast(T, src=0)
    return comm_list, T.cpu().numpy().view(np.uint64).copy(), own


def sharded_open_inputs(n: int, q_partial_into: Callable, cu_partial: Callable, combine_q: Callable,
                        combine_cu: Callable, dist, device):
    """C3: this rank's rows' share of z_q and of c_u, one all-gather, the
    combine on rank 0.

    q_partial_into(r0, r1, out) fills the int64 tensor ``out`` (2^m_row * 4
    words) with the share of z_q (canonical Fr); cu_partial(r0, r1) -> (12,)
    uint64 canonical affine share of c_u; combine_q(gathered (world, N * 4)
    tensor) -> z_q as an int64 tensor on the rank's device; combine_cu(shares
    (world, 12) uint64) -> U (12,).  Returns (z_q, U) on rank 0, (None, U)
    elsewhere (every rank combines U: the sharded opening absorbs it)."""
    import torch
    dev = _device(dist, device)
    world, rank = dist.get_world_size(), dist.get_rank()
    r0, r1 = shard_rows(1 << (n // 2), world, rank)
    N = 1 << (n - n // 2)
    buf = torch.empty(N * 4 + 12, dtype=torch.int64, device=dev)
    q_partial_into(r0, r1, buf[:N * 4])
    cu = np.ascontiguousarray(cu_partial(r0, r1), dtype=np.uint64).reshape(12)
    buf[N * 4:].copy_(torch.from_numpy(cu.view(np.int64)))
    got = _all_gather(dist, buf)
    U = np.ascontiguousarray(combine_cu(got[:, N * 4:].cpu().numpy().view(np.uint64).copy()),
                             dtype=np.uint64).reshape(12)
    if rank != 0:
        return None, U
    zq = combine_q(got[:, :N * 4].contiguous())
    return zq, U


def sharded_msm(n: int, msm_partial_into: Callable, combine: Callable, dist, device):
    """Strong-scaled MSM over n points split evenly across the ranks.

    msm_partial_into(i0, i1, out) fills the int64 tensor ``out`` (24 words on
    the rank's device) with the XYZZ sum of points [i0, i1);
    combine(gathered (world, 24) tensor) -> (12,) canonical affine, run on
    rank 0.  Returns the MSM on rank 0, None elsewhere."""
    import torch
    dev = _device(dist, device)
    i0, i1 = shard_rows(n, dist.get_world_size(), dist.get_rank())
    buf = torch.empty(24, dtype=torch.int64, device=dev)
    msm_partial_into(i0, i1, buf)
    got = _all_gather(dist, buf)
    return combine(got) if dist.get_rank() == 0 else None


class TorchExchange:
    """tpst_exchange over torch.distributed for tpst_poly_open_sharded.

    The arena (sized by tpst_open_sharded_arena_bytes) is a torch allocation
    on the rank's GPU; the library writes its send slots there and calls
    back for each all-gather with byte offsets and its comm stream.  "nccl"
    (RCCL): all_gather_into_tensor on uint8 views of the arena, issued with
    the library's stream as the current stream -- stream-ordered, no host
    synchronisation.  "gloo" (tests, shared-GPU rehearsals): the stream is
    synchronised, the slot goes through host memory."""

    def __init__(self, ctx, dist, device, n: int):
        import torch
        from . import _lib
        self.dist = dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.device = torch.device(device)
        nbytes = int(ctx.lib.tpst_open_sharded_arena_bytes(n, self.world))
        self.arena = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=self.device)
        self.nccl = dist.get_backend() == "nccl"
        self.calls = 0
        self.error = None
        self._cb = _lib.ALLGATHER_FN(self._gather)
        self.struct = _lib.Exchange(self.world, self.rank, self._cb, None, self.arena.data_ptr(), nbytes)

    def _gather(self, user, send_off, recv_off, nbytes, stream):
        import torch
        try:
            self.calls += 1
            send = self.arena[send_off:send_off + nbytes]
            recv = self.arena[recv_off:recv_off + self.world * nbytes]
            s = torch.cuda.ExternalStream(stream, device=self.device)
            if self.nccl:
                with torch.cuda.stream(s):
                    self.dist.all_gather_into_tensor(recv, send)
            else:
                s.synchronize()
                h = send.cpu()
                parts = [torch.empty_like(h) for _ in range(self.world)]
                self.dist.all_gather(parts, h)
                with torch.cuda.stream(s):
                    recv.copy_(torch.cat(parts))
                s.synchronize()
            return 0
        except Exception as e:  # reported by the library as TPST_E_STATE
            self.error = e
            return 1


def sharded_rounds(n: int, world: int) -> int:
    """The MIPP rounds tpst_poly_open_sharded splits across `world` ranks
    (length >= 4 world); rank 0 runs the remaining n // 2 - this alone."""
    r, C = 0, 1 << (n // 2)
    while r < n // 2 and (C >> r) >= 4 * world:
        r += 1
    return r


def sharded_open(ctx, n: int, handle, comm_list, point, U, transcript, dist, device, exchange=None):
    """C4: the MIPP rounds of Polynomial::open split over the ranks
    (tpst_poly_open_sharded).  Every rank passes the whole comm_list (as
    returned by sharded_commit), the point, U (sharded_open_inputs) and a
    fresh transcript; rank 0 passes its opening handle (from_q) and gets
    (U, pst_proof, MippProof), the others pass None and get None.
    `exchange` (a TorchExchange for this n) may be reused across calls."""
    from . import sqrt_pst as S
    x = exchange if exchange is not None else TorchExchange(ctx, dist, device, n)
    try:
        return S.open_sharded(ctx, handle if dist.get_rank() == 0 else None, transcript, n, comm_list, point, U, x)
    except Exception:
        if x.error is not None:
            raise RuntimeError("exchange all-gather failed: %r" % (x.error,)) from x.error
        raise
