"""Host-side timing of back-to-back pipelined tpst_g1_msm_dev calls: the
time each call takes to return (enqueue only, if nothing blocks the host)
and the wall time of K calls + one synchronize.  JSON line.

    python tools/msm_host_timing.py [log_n] [K]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import numpy as np
    import torch
    from testudo_amd import Context
    from testudo_amd.sqrt_pst import fr_stream
    n = 1 << lg
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    sc, _ = fr_stream(5, n)
    d_s = torch.from_numpy(sc.view(np.int64)).to(dev)
    d_b = torch.empty(n * 12, dtype=torch.int64, device=dev)
    d_o = torch.empty(12, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ctx.g1_mul_generator_dev(d_s.data_ptr(), n, d_b.data_ptr())
    for _ in range(3):
        ctx.g1_msm_dev(d_b.data_ptr(), d_s.data_ptr(), n, d_o.data_ptr())
    ctx.synchronize()
    calls = []
    t0 = time.perf_counter()
    for _ in range(K):
        a = time.perf_counter()
        ctx.g1_msm_dev(d_b.data_ptr(), d_s.data_ptr(), n, d_o.data_ptr())
        calls.append((time.perf_counter() - a) * 1e3)
    t1 = time.perf_counter()
    ctx.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"log_n": lg, "K": K, "call_ms": [round(x, 3) for x in calls],
                      "enqueue_ms": round((t1 - t0) * 1e3, 3), "wall_ms": round((t2 - t0) * 1e3, 3),
                      "ms_per_msm": round((t2 - t0) * 1e3 / K, 4)}), flush=True)


if __name__ == "__main__":
    main()
