"""RCCL on the GPU box: the multi-GPU code paths of testudo_amd/distributed.py
run through a real `nccl` (= RCCL) process group, in a spawned child that
initialises the group before any other GPU work of its process -- the same
order bench.py's ranks use at N > 1.  A one-rank group is what a one-GPU box
can hold (RCCL refuses two ranks on one card); its all-gathers and broadcast
go through RCCL on device tensors exactly as the 8-GPU run's do.

Checked bit for bit against the single-process library on the same inputs:
the row-sharded commit (C1/C2: [row commitments | Miller partial] all-gather,
final exponentiation read from the gathered device buffer), the opening
inputs (C3: z_q / c_u shares, device mod-r sum of a non-contiguous gathered
view), the opening from q alone, the sharded opening (C4, all-gathers on the
library's comm stream through TorchExchange), and the split (strong-scaled) MSM with its
device combine of the gathered XYZZ shares.
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


def _child(port, n, n_msm, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)  # before any other GPU work
    try:
        from testudo_amd import Context
        from testudo_amd import sqrt_pst as S
        from testudo_amd.distributed import sharded_commit, sharded_msm, sharded_open_inputs
        res = {"backend": dist.get_backend()}
        ctx = Context(0)
        dev = torch.device("cuda", 0)
        nv = (n + 1) // 2
        S.srs_setup(ctx, nv, 0x7E57D1)
        Z, k = S.fr_stream(0x7E57D0 + 7 * n, 1 << n)
        pt, _ = S.fr_stream(0x7E57D0 + 7 * n, n, k)
        C = 1 << (n // 2)
        shard = S.Polynomial.from_evaluations_cols(ctx, Z, 0, C)
        comms, T, own = sharded_commit(n, shard.commit_rows_partial_into,
                                       lambda got: S.gt_final_exp_product_gathered(ctx, got, C), dist, dev)
        zq, U = sharded_open_inputs(n, lambda a, b, out: shard.get_q_partial_into(pt, a, b, out),
                                    lambda a, b: S.cu_partial(ctx, n, pt, a, b, own),
                                    lambda got: S.fr_sum(ctx, got), lambda sh: S.g1_sum(ctx, sh), dist, dev)
        pq = S.Polynomial.from_q(ctx, n, pt, zq, U)
        vq = pq.eval(pt)
        Uq, pstq, mippq = pq.open(S.PoseidonTranscript(), comms, pt, T)
        # single process, same inputs
        full = S.Polynomial.from_evaluations(ctx, Z)
        c2, T2 = full.commit()
        v = full.eval(pt)
        U2, pst2, mipp2 = full.open(S.PoseidonTranscript(), c2, pt, T2)
        res["comms"] = bool(np.array_equal(comms, c2))
        res["T"] = bool(np.array_equal(T, T2))
        res["own"] = bool(np.array_equal(own, c2))
        res["zq"] = bool(np.array_equal(zq.cpu().numpy().view(np.uint64).reshape(-1, 4),
                                        full.get_q_partial(pt, 0, C)))
        res["U"] = bool(np.array_equal(U, U2))
        res["eval"] = bool(np.array_equal(vq, v))
        res["proof"] = bool(np.array_equal(Uq, U2) and np.array_equal(pstq, pst2) and all(
            np.array_equal(getattr(mippq, f), getattr(mipp2, f))
            for f in ("comms_t", "comms_u", "final_a", "final_h", "pst_proof_h")))
        res["verified"] = bool(S.verify(ctx, S.PoseidonTranscript(), Uq, pt, vq, pstq, mippq, T))
        # the sharded opening (C4) with its all-gathers through RCCL on the
        # library's comm stream: a one-rank group runs every sharded round
        # (len >= 4) and the hand-over to rank 0 at len = 2
        from testudo_amd.distributed import sharded_open
        pq2 = S.Polynomial.from_q(ctx, n, pt, zq, U)
        Us, psts, mipps = sharded_open(ctx, n, pq2, comms, pt, U, S.PoseidonTranscript(), dist, dev)
        res["sharded_open"] = bool(np.array_equal(Us, U2) and np.array_equal(psts, pst2) and all(
            np.array_equal(getattr(mipps, f), getattr(mipp2, f))
            for f in ("comms_t", "comms_u", "final_a", "final_h", "pst_proof_h")))
        # split MSM over the group, combined on the device
        sc, _ = S.fr_stream(0x7E57D5, n_msm)
        bk, _ = S.fr_stream(0x7E57D6, n_msm)
        d_s = torch.from_numpy(sc.view(np.int64)).to(dev)
        d_k = torch.from_numpy(bk.view(np.int64)).to(dev)
        d_b = torch.empty(n_msm * 12, dtype=torch.int64, device=dev)
        ctx.torch_to_lib()
        ctx.g1_mul_generator_dev(d_k.data_ptr(), n_msm, d_b.data_ptr())
        out = sharded_msm(n_msm, lambda a, b, o: S.g1_msm_partial_into(ctx, d_b.data_ptr(), d_s.data_ptr(), a, b, o),
                          lambda got: S.g1_xyzz_combine(ctx, got), dist, dev)
        ref = ctx.g1_msm(ctx.g1_mul_generator(bk), sc)
        res["split_msm"] = bool(np.array_equal(out.cpu().numpy().view(np.uint64), ref))
        q.put(res)
    except Exception as e:  # report, never hang the parent
        q.put({"error": repr(e)})
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_sharded_commit_open_and_split_msm():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), 11, 1 << 16, q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=120)
    assert "error" not in res, res
    assert p.exitcode == 0
    assert res.pop("backend") == "nccl"
    assert all(res.values()), res
