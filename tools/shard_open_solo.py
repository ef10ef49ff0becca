"""Per-rank latency of the row-sharded opening at world W, measured on ONE GPU
by one process playing rank 0 with a loop-back exchange (every all-gather
returns W copies of this rank's own slot -- no communication).  The proof is
not the real one (the transcript absorbs the loop-back values), but every
kernel runs at its real per-rank size: the look-ahead folds and pairings over
len / W positions, the local h preparations, the gathered-partial products,
the hand-over and rank 0's last rounds.  What an N-GPU run adds on top is the
all-gathers' latency (2 per sharded round + 2; tens of microseconds each over
xGMI).  Also runs the unsharded open for reference.  JSON lines.

    python tools/shard_open_solo.py N_LOG W [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class LoopExchange:
    """tpst_exchange that copies the caller's slot into all W receive slots."""

    def __init__(self, ctx, W, n):
        import torch
        from testudo_amd import _lib
        self.W = W
        nbytes = int(ctx.lib.tpst_open_sharded_arena_bytes(n, W))
        self.arena = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=torch.device("cuda", 0))
        self.calls = 0
        self._cb = _lib.ALLGATHER_FN(self._gather)
        self.struct = _lib.Exchange(W, 0, self._cb, None, self.arena.data_ptr(), nbytes)

    def _gather(self, user, send_off, recv_off, nbytes, stream):
        import torch
        self.calls += 1
        s = torch.cuda.ExternalStream(stream, device=torch.device("cuda", 0))
        with torch.cuda.stream(s):
            src = self.arena[send_off:send_off + nbytes]
            for w in range(self.W):
                self.arena[recv_off + w * nbytes:recv_off + (w + 1) * nbytes].copy_(src)
        return 0


def main():
    n = int(sys.argv[1])
    W = int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    import numpy as np
    from testudo_amd import Context
    from testudo_amd import sqrt_pst as S
    ctx = Context(0)
    S.srs_setup(ctx, (n + 1) // 2, 0x7E57D1)
    Z, k = S.fr_stream(0x7E57D0, 1 << n)
    pt, _ = S.fr_stream(0x7E57D0, n, k)
    pl = S.Polynomial.from_evaluations(ctx, Z)
    del Z
    comms, T = pl.commit()
    pl.eval(pt)
    U = np.zeros(12, dtype=np.uint64)
    base = []
    for _ in range(reps):
        t = time.perf_counter()
        U, _, _ = pl.open(S.PoseidonTranscript(), comms, pt, T)
        base.append(time.perf_counter() - t)
    x = LoopExchange(ctx, W, n)
    solo = []
    for _ in range(reps):
        x.calls = 0
        t = time.perf_counter()
        S.open_sharded(ctx, pl, S.PoseidonTranscript(), n, comms, pt, U, x)
        solo.append(time.perf_counter() - t)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(json.dumps({"n": n, "world": W, "open_unsharded_s": round(med(base), 5),
                      "open_rank0_solo_s": round(med(solo), 5), "gathers": x.calls,
                      "note": "rank 0 of W on one GPU, loop-back exchange: per-rank kernel sizes, no communication"}),
          flush=True)


if __name__ == "__main__":
    main()
