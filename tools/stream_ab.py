"""A/B of the 2^n commit + open with and without a pipelined device MSM run
first in the same context (the MSM creates its own streams; the opening's
concurrency depends on how HIP maps streams onto hardware queues).

    python tools/stream_ab.py N_LOG {msm|none} [reps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1])
    mode = sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    import numpy as np
    import torch
    from testudo_amd import Context
    from testudo_amd import sqrt_pst as S
    ctx = Context(0)
    if mode == "msm":
        m = 1 << 17
        sc, _ = S.fr_stream(5, m)
        dev = torch.device("cuda", 0)
        d_s = torch.from_numpy(sc.view(np.int64)).to(dev)
        d_k = torch.from_numpy(sc.view(np.int64)).to(dev)
        d_b = torch.empty(m * 12, dtype=torch.int64, device=dev)
        d_o = torch.empty(12, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        ctx.g1_mul_generator_dev(d_k.data_ptr(), m, d_b.data_ptr())
        for _ in range(3):
            ctx.g1_msm_dev(d_b.data_ptr(), d_s.data_ptr(), m, d_o.data_ptr())
        ctx.synchronize()
    S.srs_setup(ctx, (n + 1) // 2, 0x7E57D1)
    Z, k = S.fr_stream(0x7E57D0, 1 << n)
    pt, _ = S.fr_stream(0x7E57D0, n, k)
    pl = S.Polynomial.from_evaluations(ctx, Z)
    pl.eval(pt)
    tc, to = [], []
    for _ in range(reps):
        t = time.perf_counter()
        comms, T = pl.commit()
        t1 = time.perf_counter()
        pl.open(S.PoseidonTranscript(), comms, pt, T)
        t2 = time.perf_counter()
        tc.append(t1 - t)
        to.append(t2 - t1)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(json.dumps({"n": n, "mode": mode, "commit_ms": round(med(tc) * 1e3, 3), "open_ms": round(med(to) * 1e3, 3)}),
          flush=True)


if __name__ == "__main__":
    main()
