"""Row-sharded opening (mipp.rs:58-120 split across ranks)
on the GPU box: `world` processes share the one GPU, each with its own
context, joined by a gloo process group (RCCL refuses two ranks on one card;
tests/test_rccl.py runs the same path through a one-rank RCCL group).

Every rank runs the sharded commit on its column block (sqrt_pst.rs:121-143),
its z_q / c_u shares (sqrt_pst.rs:92-95, 198) and then
tpst_poly_open_sharded: the MIPP rounds on its rows i = rank mod world, one
all-gather per product through testudo_amd.distributed.TorchExchange (the
gloo host path), the hand-over of the folded vector to rank 0 once a round is
shorter than 4 world.  Rank 0's proof must equal, byte for byte, the
single-process tpst_poly_open of the same polynomial (n <= 13) or the
BASELINE configs[3] fixture (n = 24 at world 2, 4 and 8: the 1/2/4/8-GPU
splits north_star names), and verify.
"""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _arr(hexs, shape):
    return np.frombuffer(bytes.fromhex(hexs), dtype=np.uint64).reshape(shape)


def _worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from testudo_amd import Context
        from testudo_amd import sqrt_pst as S
        from testudo_amd.distributed import shard_rows, sharded_commit, sharded_open, sharded_open_inputs
        ctx = Context(0)
        dev = torch.device("cuda", 0)
        fixture = None
        if n == 24:
            import golden_io as G
            fixture = G.load("fullsize_n24.json")
            seed_srs, seed_z = fixture["seed_srs"], fixture["seed_z"]
        else:
            seed_srs, seed_z = 0x7E57D1, 0x7E57D0 + 11 * n
        nv = (n + 1) // 2
        S.srs_setup(ctx, nv, seed_srs)
        Z, k = S.fr_stream(seed_z, 1 << n)
        pt, _ = S.fr_stream(seed_z, n, k)
        C = 1 << (n // 2)
        r0, r1 = shard_rows(C, world, rank)
        R = r1 - r0
        shard = S.Polynomial.from_evaluations_cols(ctx, Z, r0, r1)
        comms, T, own = sharded_commit(n, shard.commit_rows_partial_into,
                                       lambda got: S.gt_final_exp_product_gathered(ctx, got, R), dist, dev)
        zq, U = sharded_open_inputs(n, lambda a, b, out: shard.get_q_partial_into(pt, a, b, out),
                                    lambda a, b: S.cu_partial(ctx, n, pt, a, b, own),
                                    lambda got: S.fr_sum(ctx, got), lambda sh: S.g1_sum(ctx, sh), dist, dev)
        del shard
        handle = S.Polynomial.from_q(ctx, n, pt, zq, U) if rank == 0 else None
        v = handle.eval(pt) if rank == 0 else None
        from testudo_amd.distributed import TorchExchange, sharded_rounds
        x = TorchExchange(ctx, dist, dev, n)
        out = sharded_open(ctx, n, handle, comms, pt, U, S.PoseidonTranscript(), dist, dev, exchange=x)
        # every sharded round: the cross partials and the look-ahead partials;
        # round 0's direct t_l / t_r; the hand-over of the folded vector
        rs = sharded_rounds(n, world)
        assert rs >= 1 and x.calls == 2 * rs + 2, (rs, x.calls)
        if n == 24:  # configs[3] at 2 / 4 / 8 GPUs
            assert x.calls == {2: 22, 4: 20, 8: 18}[world], (world, x.calls)
        if rank != 0:
            assert out is None
            q.put((rank, None))
            return
        U2, pst, mipp = out
        res = {"U": bool(np.array_equal(U2, U))}
        if fixture is not None:
            m_col, m_row = n // 2, n - n // 2
            d = fixture
            res["T"] = bool(np.array_equal(T, _arr(d["T"], (72,))))
            res["v"] = bool(np.array_equal(v, _arr(d["eval"], (4,))))
            res["U_fix"] = bool(np.array_equal(U2, _arr(d["U"], (12,))))
            res["pst"] = bool(np.array_equal(pst, _arr(d["pst_proof"], (m_row, 24))))
            res["comms_t"] = bool(np.array_equal(mipp.comms_t, _arr(d["comms_t"], (m_col, 2, 72))))
            res["comms_u"] = bool(np.array_equal(mipp.comms_u, _arr(d["comms_u"], (m_col, 2, 12))))
            res["final_a"] = bool(np.array_equal(mipp.final_a, _arr(d["final_a"], (12,))))
            res["final_h"] = bool(np.array_equal(mipp.final_h, _arr(d["final_h"], (24,))))
            res["pst_proof_h"] = bool(np.array_equal(mipp.pst_proof_h, _arr(d["pst_proof_h"], (m_col, 12))))
        else:
            full = S.Polynomial.from_evaluations(ctx, Z)
            c2, T2 = full.commit()
            res["comms"] = bool(np.array_equal(comms, c2))
            res["T"] = bool(np.array_equal(T, T2))
            res["v"] = bool(np.array_equal(v, full.eval(pt)))
            U3, pst3, mipp3 = full.open(S.PoseidonTranscript(), c2, pt, T2)
            res["U_single"] = bool(np.array_equal(U2, U3))
            res["pst"] = bool(np.array_equal(pst, pst3))
            for f in ("comms_t", "comms_u", "final_a", "final_h", "pst_proof_h"):
                res[f] = bool(np.array_equal(getattr(mipp, f), getattr(mipp3, f)))
        res["verified"] = bool(S.verify(ctx, S.PoseidonTranscript(), U2, pt, v, pst, mipp, T))
        q.put((rank, res))
    except Exception as e:  # surfaced in the parent
        import traceback
        q.put((rank, "error: %r\n%s" % (e, traceback.format_exc())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(11, 2), (12, 4), (13, 8), (24, 2), (24, 4), (24, 8)])
def test_sharded_open_matches_single_process(n, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    errs = {r: v for r, v in res.items() if isinstance(v, str)}
    assert not errs, errs
    for p in procs:
        assert p.exitcode == 0
    assert all(v is None for r, v in res.items() if r != 0)
    bad = {k: v for k, v in res[0].items() if not v}
    assert not bad, res[0]
