"""2^20 G1 MSM time under skewed scalar distributions (the
sentinel bin and one-bucket windows): uniform, 90 % zero / 10 % one, all
ones, 16-bit scalars.  Each result checked by linearity against the
generator multiple of sum s_i b_i."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import Context  # noqa: E402
from testudo_amd.encoding import fr_array  # noqa: E402
from testudo_amd.sqrt_pst import fr_stream  # noqa: E402

R = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001
n = 1 << 20
ctx = Context(0)
dev = torch.device("cuda", 0)
bk, _ = fr_stream(5, n)
d_bk = torch.from_numpy(bk.view(np.int64)).to(dev)
d_b = torch.empty(n * 12, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
ctx.g1_mul_generator_dev(d_bk.data_ptr(), n, d_b.data_ptr())
ctx.synchronize()
rng = np.random.default_rng(9)
cases = {}
cases["uniform"] = fr_stream(6, n)[0]
s = np.zeros((n, 4), dtype=np.uint64)
s[:, 0] = (rng.random(n) < 0.1).astype(np.uint64)
cases["bool10"] = s
s = np.zeros((n, 4), dtype=np.uint64)
s[:, 0] = 1
cases["ones"] = s
s = np.zeros((n, 4), dtype=np.uint64)
s[:, 0] = rng.integers(0, 1 << 16, n, dtype=np.uint64)
cases["u16"] = s
b_int = bk.astype(object)
bv = b_int[:, 0] + (b_int[:, 1] << 64) + (b_int[:, 2] << 128) + (b_int[:, 3] << 192)
d_out = torch.empty(12, dtype=torch.int64, device=dev)
for name, sc in cases.items():
    d_s = torch.from_numpy(sc.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    for _ in range(2):
        ctx.g1_msm_dev(d_b.data_ptr(), d_s.data_ptr(), n, d_out.data_ptr())
    ctx.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        ctx.g1_msm_dev(d_b.data_ptr(), d_s.data_ptr(), n, d_out.data_ptr())
    ctx.synchronize()
    ms = (time.perf_counter() - t) / 5 * 1e3
    s_int = sc.astype(object)
    sv = s_int[:, 0] + (s_int[:, 1] << 64) + (s_int[:, 2] << 128) + (s_int[:, 3] << 192)
    tot = int(np.dot(sv, bv) % R)
    ok = bool(np.array_equal(d_out.cpu().numpy().view(np.uint64), ctx.g1_mul_generator(fr_array([tot]))[0]))
    print(json.dumps({"case": name, "ms": round(ms, 3), "ok": ok}), flush=True)
