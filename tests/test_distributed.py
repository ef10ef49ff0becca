"""world_size-2 gloo tests on CPU of the multi-rank paths:

* the row-sharded commit orchestration (testudo_amd/distributed.py) with the
  C++ oracle standing in for the per-rank GPU compute (row MSMs + unreduced
  Miller-loop partial per rank, one final exponentiation on rank 0) -- the
  gathered commitment list and T must equal the single-process commit bit for
  bit -- and the sharded opening inputs (C3: per-rank shares of get_q's z_q and
  of c_u, summed on rank 0) against the single-process q and U;
* the split (strong-scaled) MSM: shares of equal point ranges, one
  all-gather, the combine on rank 0, against the oracle MSM of all points;
* bench.py's timing aggregation (barrier + max over ranks).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle", "cpu"))
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import orc
        import pst as PY
        from testudo_amd.distributed import sharded_commit, sharded_open_inputs
        R_ = PY.R
        nv = (n + 1) // 2
        srs = orc.SRS(nv, 0x7E57D1)
        flat = srs.export()
        C, Rn = 1 << (n // 2), 1 << nv
        pg0 = flat[36:36 + Rn * 12].reshape(Rn, 12)
        # powers_of_h[odd]: skip g, h, level 0 (G1 + G2) when odd
        off = 36
        levels = []
        for i in range(nv):
            m = 1 << (nv - i)
            levels.append((off, off + m * 12))
            off += m * 12 + m * 24
        odd = n % 2
        hstart = levels[odd][1]
        hvec = flat[hstart:hstart + C * 24].reshape(C, 24)
        Z, k = orc.fr_stream(0x7E57D0, 1 << n)
        pt, _ = orc.fr_stream(0x7E57D0, n, k)

        def commit_rows_partial_into(r0, r1, out):
            cm = orc.g1_msm_batch(pg0, Z[r0:].reshape(-1), r1 - r0, 1, C)
            ml = orc.miller_product(cm, hvec[r0:r1])
            out.copy_(torch.from_numpy(np.concatenate([cm.reshape(-1), ml]).view(np.int64)))

        def finalize(got):
            Rr = C // world
            return orc.gt_final_exp_product(got[:, 12 * Rr:].numpy().view(np.uint64))

        comms, T, own = sharded_commit(n, commit_rows_partial_into, finalize, dist, torch.device("cpu"))
        # C3: shares of z_q and c_u (oracle/py restatement of the per-rank work)
        Zi = [int(v) for v in (Z[:, 0].astype(object) + (Z[:, 1].astype(object) << 64) +
                               (Z[:, 2].astype(object) << 128) + (Z[:, 3].astype(object) << 192))]
        pti = [int(a) + (int(b) << 64) + (int(c) << 128) + (int(d) << 192) for a, b, c, d in pt]
        m_col, m_row = n // 2, n - n // 2
        chis = [PY.get_chi_i(pti[m_row:], i) for i in range(C)]

        def fr_np(vals):
            return np.array([[(v >> (64 * t)) & (2 ** 64 - 1) for t in range(4)] for v in vals], dtype=np.uint64)

        def q_partial_into(r0, r1, out):
            share = [sum(Zi[(j << m_col) | i] * chis[i] for i in range(r0, r1)) % R_ for j in range(1 << m_row)]
            out.copy_(torch.from_numpy(fr_np(share).reshape(-1).view(np.int64)))

        def cu_partial(r0, r1):
            return orc.g1_msm(own, fr_np(chis[r0:r1]))

        def combine_q(got):
            a = got.numpy().view(np.uint64).reshape(world, -1, 4)
            tot = [sum(int(a[w, j, 0]) + (int(a[w, j, 1]) << 64) + (int(a[w, j, 2]) << 128) + (int(a[w, j, 3]) << 192)
                       for w in range(world)) % R_ for j in range(a.shape[1])]
            return torch.from_numpy(fr_np(tot).reshape(-1).view(np.int64))

        def combine_cu(shares):
            ones = np.zeros((len(shares), 4), dtype=np.uint64)
            ones[:, 0] = 1
            return orc.g1_msm(shares, ones)

        zq, U = sharded_open_inputs(n, q_partial_into, cu_partial, combine_q, combine_cu, dist, torch.device("cpu"))
        if rank == 0:
            c2, T2 = orc.pst_commit(srs, Z, n)
            ref = PY.Polynomial(Zi)
            ref.get_q(pti)
            pr = orc.pst_open(srs, Z, n, pt, c2)
            q.put((bool(np.array_equal(comms, c2)), bool(np.array_equal(T, T2)),
                   bool(np.array_equal(zq.numpy().view(np.uint64).reshape(-1, 4), fr_np(ref.q))),
                   bool(np.array_equal(U, pr["U"]))))
        else:
            q.put(None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [6, 7])
def test_sharded_commit_gloo_world2(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = [r for r in res if r is not None]
    assert res == [(True, True, True, True)]  # comm_list, T, combined z_q, combined c_u


def _msm_worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle", "cpu"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import orc
        from testudo_amd.distributed import sharded_msm
        k, _ = orc.fr_stream(0x7E57D6, n)
        s, _ = orc.fr_stream(0x7E57D5, n)
        bases = orc.g1_mul_gen(k)

        def partial_into(i0, i1, out):  # the oracle stands in for tpst_g1_msm_xyzz_dev
            share = np.zeros(24, dtype=np.uint64)
            share[:12] = orc.g1_msm(bases[i0:i1], s[i0:i1])
            out.copy_(torch.from_numpy(share.view(np.int64)))

        def combine(got):
            pts = got.numpy().view(np.uint64)[:, :12]
            ones = np.zeros((len(pts), 4), dtype=np.uint64)
            ones[:, 0] = 1
            return orc.g1_msm(np.ascontiguousarray(pts), ones)

        out = sharded_msm(n, partial_into, combine, dist, torch.device("cpu"))
        q.put(bool(np.array_equal(out, orc.g1_msm(bases, s))) if rank == 0 else None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 1 << 18])
def test_sharded_msm_gloo_world2(n):
    """Strong-scaled MSM orchestration: two ranks take halves of the points,
    one all-gather of the shares, the combine on rank 0 equals the oracle MSM
    of all points.  n = 2^18 gives each share exactly 2^17 points (the
    window-group boundary configs[1] hits at 8 GPUs)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_msm_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r in res if r is not None] == [True]


def _timing_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import time
        dist.barrier()
        t0 = time.perf_counter()
        time.sleep(0.05 * (rank + 1))  # rank 1 is the slow one
        dist.barrier()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, float(t.item())))
    finally:
        dist.destroy_process_group()


def test_bench_max_over_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timing_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == res[1] and res[0] >= 0.1


def test_bench_launcher_spawns_ranks_dry_run():
    """`python bench.py --gpus 2` (no WORLD_SIZE) starts torch.distributed.run
    with 2 ranks as a child process; with --dry-run the ranks rendezvous over
    gloo, time barrier-bracketed steps, take the max over ranks (rank 1 is the
    slower one) and rank 0 alone prints one JSON line."""
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "5",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] and d["steps"] == 5
    assert d["ms_per_step"] >= 2.0  # rank 1 sleeps 2 ms per step: the max over ranks is reported
