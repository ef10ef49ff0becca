"""Host-side mirror of Testudo's sqrt-PST surface over libtpst.

Reference: ``src/sqrt_pst.rs:14-265`` (``Polynomial``), ``src/mipp.rs``
(``MippProof``) and ``src/poseidon_transcript.rs`` (``PoseidonTranscript``).
Names and argument meaning follow the reference; every computation runs in
libtpst (HIP on gfx950) -- this module only marshals arrays:

* field elements are numpy ``uint64`` arrays of canonical little-endian limbs
  (Fr: 4, Fq: 6), G1 affine 12 limbs, G2 affine 24, GT 72 (include/tpst.h);
* errors raise ``TpstError``; ``verify`` returns ``False`` on an invalid proof
  where the reference would ``assert!`` (sqrt_pst.rs:250, mipp.rs:308-317).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .encoding import ptr
from .engine import Context, TpstError


def _torch_ready() -> bool:
    """True when torch is importable with a GPU (stream ordering applies)."""
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


def _u64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return a if shape is None else a.reshape(shape)


class PoseidonTranscript:
    """PoseidonTranscript<Fq> with get_bls12377_fq_params (parameters.rs:309-338)."""

    def __init__(self):
        self.lib = _lib.load()
        self.t = _lib.Transcript()
        self.lib.tpst_transcript_init(C.byref(self.t))

    def append_g1(self, p):
        self.lib.tpst_transcript_append_g1(C.byref(self.t), ptr(_u64(p, (12,))))

    def append_gt(self, f):
        self.lib.tpst_transcript_append_gt(C.byref(self.t), ptr(_u64(f, (72,))))

    def append_bytes(self, b: bytes):
        """append_bytes (poseidon_transcript.rs:67-69); ``append`` of a value
        is this over its Compress::No serialisation."""
        b = bytes(b)
        self.lib.tpst_transcript_append_bytes(C.byref(self.t), b, len(b))

    def challenge_scalar(self) -> np.ndarray:
        out = np.zeros(4, dtype=np.uint64)
        self.lib.tpst_transcript_challenge(C.byref(self.t), ptr(out))
        return out

    def state(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.t.state).reshape(18).copy()


@dataclass
class MippProof:
    """mipp.rs:21-28."""
    comms_t: np.ndarray      # (m_col, 2, 72) GT
    comms_u: np.ndarray      # (m_col, 2, 12) G1
    final_a: np.ndarray      # (12,)
    final_h: np.ndarray      # (24,)
    pst_proof_h: np.ndarray  # (m_col, 12) ProofG1


def srs_setup(ctx: Context, nv: int, seed: int):
    """MultilinearPC::setup + trim to nv variables, trapdoor from ``seed``."""
    ctx.check(ctx.lib.tpst_srs_setup(ctx.h, nv, seed), "tpst_srs_setup")


def srs_load(ctx: Context, nv: int, flat: np.ndarray):
    flat = _u64(flat)
    if len(flat) != ctx.lib.tpst_srs_flat_len(nv):
        raise TpstError("SRS flat length mismatch")
    ctx.check(ctx.lib.tpst_srs_load(ctx.h, nv, ptr(flat)), "tpst_srs_load")


def srs_export(ctx: Context, nv: int) -> np.ndarray:
    out = np.zeros(ctx.lib.tpst_srs_flat_len(nv), dtype=np.uint64)
    ctx.check(ctx.lib.tpst_srs_export(ctx.h, ptr(out)), "tpst_srs_export")
    return out


def fr_stream(seed: int, n: int, start: int = 0):
    lib = _lib.load()
    out = np.zeros((n, 4), dtype=np.uint64)
    nxt = lib.tpst_fr_stream(seed, n, start, ptr(out))
    return out, nxt


def _nv(evals) -> int:
    """log2 of the evaluation count; a non-power-of-two vector is an error
    (the reference's MultilinearExtension always has 2^nv evaluations)."""
    nv = len(evals).bit_length() - 1
    if len(evals) == 0 or 1 << nv != len(evals):
        raise TpstError("evaluation count must be a power of two")
    return nv


class MultilinearPC:
    """The ark-poly-commit fork's MultilinearPC<Bls12_377> calls the reference
    makes, against the SRS loaded in ``ctx``.  Points are
    LSB-first (MultilinearPC's order); ``check``/``check_2`` return bool."""

    @staticmethod
    def commit(ctx: Context, evals) -> np.ndarray:
        """sqrt_pst.rs:124 -> g_product (12,)."""
        evals = _u64(evals).reshape(-1, 4)
        nv = _nv(evals)
        out = np.zeros(12, dtype=np.uint64)
        ctx.check(ctx.lib.tpst_mlpc_commit(ctx.h, ptr(evals), nv, ptr(out)), "MultilinearPC::commit")
        return out

    @staticmethod
    def commit_g2(ctx: Context, evals) -> np.ndarray:
        """mipp.rs:133 -> h_product (24,)."""
        evals = _u64(evals).reshape(-1, 4)
        nv = _nv(evals)
        out = np.zeros(24, dtype=np.uint64)
        ctx.check(ctx.lib.tpst_mlpc_commit_g2(ctx.h, ptr(evals), nv, ptr(out)), "MultilinearPC::commit_g2")
        return out

    @staticmethod
    def open(ctx: Context, evals, point) -> np.ndarray:
        """sqrt_pst.rs:225 -> Proof (nv, 24) G2."""
        evals = _u64(evals).reshape(-1, 4)
        nv = _nv(evals)
        point = _u64(point, (nv, 4))
        out = np.zeros((nv, 24), dtype=np.uint64)
        ctx.check(ctx.lib.tpst_mlpc_open(ctx.h, ptr(evals), nv, ptr(point), ptr(out)), "MultilinearPC::open")
        return out

    @staticmethod
    def open_g1(ctx: Context, evals, point) -> np.ndarray:
        """mipp.rs:144 -> ProofG1 (nv, 12)."""
        evals = _u64(evals).reshape(-1, 4)
        nv = _nv(evals)
        point = _u64(point, (nv, 4))
        out = np.zeros((nv, 12), dtype=np.uint64)
        ctx.check(ctx.lib.tpst_mlpc_open_g1(ctx.h, ptr(evals), nv, ptr(point), ptr(out)), "MultilinearPC::open_g1")
        return out

    @staticmethod
    def _chk(ctx, fn, nv, comm, point, value, proofs, what):
        rc = fn(ctx.h, nv, ptr(comm), ptr(point), ptr(value), ptr(proofs))
        if rc == -5:
            return False
        ctx.check(rc, what)
        return True

    @staticmethod
    def check(ctx: Context, comm, point, value, proofs) -> bool:
        """sqrt_pst.rs:261."""
        point = _u64(point).reshape(-1, 4)
        nv = len(point)
        return MultilinearPC._chk(ctx, ctx.lib.tpst_mlpc_check, nv, _u64(comm, (12,)), point, _u64(value, (4,)),
                                  _u64(proofs, (nv, 24)) if nv else np.zeros(24, np.uint64),
                                  "MultilinearPC::check")

    @staticmethod
    def check_2(ctx: Context, comm_h, point, value, proofs) -> bool:
        """mipp.rs:307."""
        point = _u64(point).reshape(-1, 4)
        nv = len(point)
        return MultilinearPC._chk(ctx, ctx.lib.tpst_mlpc_check_2, nv, _u64(comm_h, (24,)), point, _u64(value, (4,)),
                                  _u64(proofs, (nv, 12)) if nv else np.zeros(12, np.uint64), "MultilinearPC::check_2")


class Polynomial:
    """sqrt_pst.rs:14-20 -- 2^n evaluations viewed as 2^m_col rows of 2^m_row."""

    def __init__(self, ctx: Context, handle, n: int, keep=None):
        self.ctx = ctx
        self.h = handle
        self.n = n
        self.m_col = n // 2
        self.m_row = n - self.m_col
        self.odd = n % 2
        self._keep = keep

    @classmethod
    def from_evaluations(cls, ctx: Context, Z: np.ndarray) -> "Polynomial":
        """sqrt_pst.rs:32-75."""
        Z = _u64(Z).reshape(-1, 4)
        n = int(len(Z)).bit_length() - 1
        if 1 << n != len(Z):
            raise TpstError("evaluation count must be a power of two")
        h = C.c_void_p()
        ctx.check(ctx.lib.tpst_poly_from_evaluations(ctx.h, ptr(Z), n, C.byref(h)), "from_evaluations")
        return cls(ctx, h, n)

    @classmethod
    def from_evaluations_cols(cls, ctx: Context, Z: np.ndarray, c0: int, c1: int) -> "Polynomial":
        """This rank's column block [c0, c1) of the strided view only (one 2D
        copy); serves commit_rows / commit_rows_partial for rows in [c0, c1)."""
        Z = _u64(Z).reshape(-1, 4)
        n = int(len(Z)).bit_length() - 1
        if 1 << n != len(Z):
            raise TpstError("evaluation count must be a power of two")
        h = C.c_void_p()
        ctx.check(ctx.lib.tpst_poly_from_evaluations_cols(ctx.h, ptr(Z), n, c0, c1, C.byref(h)),
                  "from_evaluations_cols")
        return cls(ctx, h, n)

    @classmethod
    def from_device(cls, ctx: Context, d_ptr: int, n: int, keep=None) -> "Polynomial":
        h = C.c_void_p()
        if _torch_ready():
            ctx.torch_to_lib()  # d_ptr may be a torch tensor written on torch's stream
        ctx.check(ctx.lib.tpst_poly_from_evaluations_dev(ctx.h, C.c_void_p(d_ptr), n, C.byref(h)),
                  "from_evaluations_dev")
        return cls(ctx, h, n, keep)

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.tpst_poly_free(self.h)
                self.h = None
        except Exception:
            pass

    def eval(self, point) -> np.ndarray:
        """sqrt_pst.rs:105-115 (computes and caches q on first use)."""
        point = _u64(point, (self.n, 4))
        out = np.zeros(4, dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_poly_eval(self.ctx.h, self.h, ptr(point), ptr(out)), "eval")
        return out

    def commit(self):
        """sqrt_pst.rs:117-149 -> (comm_list (2^m_col, 12), T (72,))."""
        comms = np.zeros((1 << self.m_col, 12), dtype=np.uint64)
        T = np.zeros(72, dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_poly_commit(self.ctx.h, self.h, ptr(comms), ptr(T)), "commit")
        return comms, T

    def commit_rows(self, r0: int, r1: int) -> np.ndarray:
        """Row MSMs of rows [r0, r1) only (one rank's shard of sqrt_pst.rs:121-125)."""
        out = np.zeros((r1 - r0, 12), dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_poly_commit_rows(self.ctx.h, self.h, r0, r1, ptr(out)), "commit_rows")
        return out

    def commit_rows_partial(self, r0: int, r1: int):
        """Rows [r0, r1) of sqrt_pst.rs:121-125 plus their share of the IPP
        (sqrt_pst.rs:128-143) as an unreduced Miller-loop product (72,)."""
        out = np.zeros((r1 - r0, 12), dtype=np.uint64)
        ml = np.zeros(72, dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_poly_commit_rows_partial(self.ctx.h, self.h, r0, r1, ptr(out), ptr(ml)),
                       "commit_rows_partial")
        return out, ml

    def commit_rows_partial_into(self, r0: int, r1: int, out) -> None:
        """commit_rows_partial written into the int64 tensor ``out`` (R * 12 +
        72 words, [comms | Miller partial]): straight from device memory when
        ``out`` is a GPU tensor (the RCCL all-gather buffer), else via host."""
        if out.is_cuda:
            self.ctx.torch_to_lib()  # `out` may come from torch's caching allocator
            self.ctx.check(self.ctx.lib.tpst_poly_commit_rows_partial_dev(self.ctx.h, self.h, r0, r1,
                                                                          C.c_void_p(out.data_ptr())),
                           "commit_rows_partial_dev")
            self.ctx.lib_to_torch()  # the all-gather reads it on torch's stream
            return
        import torch
        cm, ml = self.commit_rows_partial(r0, r1)
        out.copy_(torch.from_numpy(np.concatenate([cm.reshape(-1), ml]).view(np.int64)))

    def get_q_partial(self, point, r0: int, r1: int) -> np.ndarray:
        """Rows [r0, r1)'s share of get_q (sqrt_pst.rs:92-95): (2^m_row, 4) canonical Fr."""
        point = _u64(point, (self.n, 4))
        out = np.zeros((1 << self.m_row, 4), dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_poly_get_q_partial(self.ctx.h, self.h, ptr(point), r0, r1, ptr(out)),
                       "get_q_partial")
        return out

    def get_q_partial_into(self, point, r0: int, r1: int, out) -> None:
        """get_q_partial into the int64 tensor ``out`` (device-side when it is a GPU tensor)."""
        if out.is_cuda:
            point = _u64(point, (self.n, 4))
            self.ctx.torch_to_lib()
            self.ctx.check(self.ctx.lib.tpst_poly_get_q_partial_dev(self.ctx.h, self.h, ptr(point), r0, r1,
                                                                    C.c_void_p(out.data_ptr())),
                           "get_q_partial_dev")
            self.ctx.lib_to_torch()
            return
        import torch
        out.copy_(torch.from_numpy(self.get_q_partial(point, r0, r1).reshape(-1).view(np.int64)))

    @classmethod
    def from_q(cls, ctx: Context, n: int, point, zq, U=None) -> "Polynomial":
        """Opening-only Polynomial from the combined q (an int64 tensor of 2^m_row
        canonical Fr, moved to the device if needed) and optionally the combined
        c_u: serves eval and open; no evaluations resident."""
        import torch
        point = _u64(point, (n, 4))
        if not zq.is_cuda:
            zq = zq.to(torch.device("cuda", ctx.device))
        zq = zq.contiguous()
        ctx.torch_to_lib()  # zq was produced on torch's stream
        Up = ptr(_u64(U, (12,))) if U is not None else None
        h = C.c_void_p()
        ctx.check(ctx.lib.tpst_poly_from_q_dev(ctx.h, n, ptr(point), C.c_void_p(zq.data_ptr()), Up, C.byref(h)),
                  "from_q")
        return cls(ctx, h, n, keep=zq)

    def commit_dev(self, d_comms: int, d_T: int):
        self.ctx.check(self.ctx.lib.tpst_poly_commit_dev(self.ctx.h, self.h, C.c_void_p(d_comms),
                                                         C.c_void_p(d_T)), "commit_dev")

    def open(self, transcript: PoseidonTranscript, comm_list, point, T):
        """sqrt_pst.rs:168-230 -> (U, pst_proof (m_row, 24), MippProof)."""
        comm_list = _u64(comm_list, (1 << self.m_col, 12))
        point = _u64(point, (self.n, 4))
        T = _u64(T, (72,))
        pr = _lib.OpenProof()
        self.ctx.check(self.ctx.lib.tpst_poly_open(self.ctx.h, self.h, C.byref(transcript.t), ptr(comm_list),
                                                   ptr(point), ptr(T), C.byref(pr)), "open")
        return _unpack(pr)


def open_sharded(ctx: Context, p, transcript: PoseidonTranscript, n: int, comm_list, point, U, exchange):
    """Row-sharded Polynomial::open (tpst_poly_open_sharded):
    every rank calls it with the whole comm_list, the point, c_u and its own
    transcript copy; rank 0 passes its opening handle `p` and gets (U,
    pst_proof, MippProof); the other ranks pass p = None and get None.
    `exchange` is a testudo_amd.distributed.TorchExchange (or any object with
    a ctypes `struct` attribute of type _lib.Exchange)."""
    comm_list = _u64(comm_list, (1 << (n // 2), 12))
    point = _u64(point, (n, 4))
    U = _u64(U, (12,))
    lead = exchange.struct.rank == 0
    pr = _lib.OpenProof() if lead else None
    if _torch_ready():
        ctx.torch_to_lib()  # the exchange arena is a torch allocation
    ctx.check(ctx.lib.tpst_poly_open_sharded(ctx.h, p.h if p is not None else None, C.byref(transcript.t), n,
                                             ptr(comm_list), ptr(point), ptr(U), C.byref(exchange.struct),
                                             C.byref(pr) if lead else None), "open_sharded")
    return _unpack(pr) if lead else None


def _unpack(pr):
    mc, mr = pr.m_col, pr.m_row
    arr = lambda x: np.ctypeslib.as_array(x).copy()  # noqa: E731
    U = arr(pr.U)
    pst = arr(pr.pst_proof)[:mr]
    mipp = MippProof(comms_t=arr(pr.comms_t)[:mc], comms_u=arr(pr.comms_u)[:mc], final_a=arr(pr.final_a),
                     final_h=arr(pr.final_h), pst_proof_h=arr(pr.pst_proof_h)[:mc])
    return U, pst, mipp


def pack_proof(n, U, pst_proof, mipp: MippProof):
    pr = _lib.OpenProof()
    pr.m_col, pr.m_row = n // 2, n - n // 2
    np.ctypeslib.as_array(pr.U)[:] = _u64(U, (12,))
    np.ctypeslib.as_array(pr.pst_proof)[:pr.m_row] = _u64(pst_proof, (pr.m_row, 24))
    np.ctypeslib.as_array(pr.comms_t)[:pr.m_col] = _u64(mipp.comms_t, (pr.m_col, 2, 72))
    np.ctypeslib.as_array(pr.comms_u)[:pr.m_col] = _u64(mipp.comms_u, (pr.m_col, 2, 12))
    np.ctypeslib.as_array(pr.final_a)[:] = _u64(mipp.final_a, (12,))
    np.ctypeslib.as_array(pr.final_h)[:] = _u64(mipp.final_h, (24,))
    np.ctypeslib.as_array(pr.pst_proof_h)[:pr.m_col] = _u64(mipp.pst_proof_h, (pr.m_col, 12))
    return pr


def ipp(ctx: Context, n: int, comms) -> np.ndarray:
    """T = prod e(C_i, h_i) for a full (gathered) commitment list."""
    T = np.zeros(72, dtype=np.uint64)
    ctx.check(ctx.lib.tpst_poly_ipp(ctx.h, n, ptr(_u64(comms, (-1, 12))), ptr(T)), "ipp")
    return T


def gt_final_exp_product_gathered(ctx: Context, gathered, R: int) -> np.ndarray:
    """T = FE(prod of the Miller partials) of an all-gathered (world, R * 12 +
    72) int64 tensor of commit_rows_partial shares, read in place on the device."""
    import torch
    if not gathered.is_cuda:
        gathered = gathered.to(torch.device("cuda", ctx.device))
    gathered = gathered.contiguous()
    ctx.torch_to_lib()  # the all-gather / copy wrote it on torch's stream
    k, w = gathered.shape
    T = np.zeros(72, dtype=np.uint64)
    ctx.check(ctx.lib.tpst_gt_final_exp_product_dev(ctx.h, C.c_void_p(gathered.data_ptr() + 96 * R), 8 * w, k,
                                                    ptr(T)), "gt_final_exp_product_dev")
    return T


def fr_sum(ctx: Context, gathered):
    """Mod-r sum of the rows of a (k, n * 4) int64 tensor of canonical Fr (the C3
    combine): an (n * 4,) int64 tensor on the context's device."""
    import torch
    if not gathered.is_cuda:
        gathered = gathered.to(torch.device("cuda", ctx.device))
    gathered = gathered.contiguous()
    k, w = gathered.shape
    out = torch.empty(w, dtype=torch.int64, device=gathered.device)
    ctx.torch_to_lib()  # gathered (all-gather / stack / contiguous) and out's previous users
    ctx.check(ctx.lib.tpst_fr_sum_dev(ctx.h, C.c_void_p(gathered.data_ptr()), k, w // 4, C.c_void_p(out.data_ptr())),
              "fr_sum_dev")
    ctx.lib_to_torch()
    return out


def cu_partial(ctx: Context, n: int, point, r0: int, r1: int, comms_rows) -> np.ndarray:
    """Rows [r0, r1)'s share of c_u = MSM(comm_list, chi(b)) (sqrt_pst.rs:198), (12,)."""
    point = _u64(point, (n, 4))
    comms_rows = _u64(comms_rows, (r1 - r0, 12)) if r1 > r0 else np.zeros((1, 12), dtype=np.uint64)
    out = np.zeros(12, dtype=np.uint64)
    ctx.check(ctx.lib.tpst_poly_cu_partial(ctx.h, n, ptr(point), r0, r1, ptr(comms_rows), ptr(out)), "cu_partial")
    return out


def g1_sum(ctx: Context, points) -> np.ndarray:
    """Sum of canonical affine G1 points (the c_u combine): an MSM with unit scalars."""
    points = _u64(points).reshape(-1, 12)
    ones = np.zeros((len(points), 4), dtype=np.uint64)
    ones[:, 0] = 1
    return ctx.g1_msm(points, ones)


def gt_final_exp_product(ctx: Context, partials) -> np.ndarray:
    """T = final_exponentiation(prod of the ranks' Miller-loop partials)."""
    partials = _u64(partials, (-1, 72))
    T = np.zeros(72, dtype=np.uint64)
    ctx.check(ctx.lib.tpst_gt_final_exp_product(ctx.h, ptr(partials), len(partials), ptr(T)), "gt_final_exp_product")
    return T


def verify(ctx: Context, transcript: PoseidonTranscript, U, point, v, pst_proof, mipp: MippProof, T) -> bool:
    """Polynomial::verify (sqrt_pst.rs:232-264)."""
    point = _u64(point).reshape(-1, 4)
    n = len(point)
    pr = pack_proof(n, U, pst_proof, mipp)
    rc = ctx.lib.tpst_pst_verify(ctx.h, C.byref(transcript.t), n, ptr(point), ptr(_u64(v, (4,))),
                                 ptr(_u64(T, (72,))), C.byref(pr))
    if rc == -5:
        return False
    ctx.check(rc, "verify")
    return True


def g1_msm_partial_into(ctx: Context, d_bases: int, d_scalars: int, i0: int, i1: int, out) -> None:
    """Points [i0, i1) of a device-resident MSM (Montgomery bases, canonical Fr
    scalars) summed into the int64 tensor ``out`` (24 words, raw XYZZ; a host
    tensor -- the gloo path -- is filled through a device staging tensor)."""
    import torch
    dst = out if out.is_cuda else torch.empty(24, dtype=torch.int64, device=torch.device("cuda", ctx.device))
    ctx.torch_to_lib()
    ctx.g1_msm_xyzz_dev(d_bases + 96 * i0, d_scalars + 32 * i0, i1 - i0, dst.data_ptr())
    ctx.lib_to_torch()
    if dst is not out:
        out.copy_(dst.cpu())


def g1_xyzz_combine(ctx: Context, gathered):
    """Sum of a gathered (k, 24) int64 tensor of XYZZ shares on the device ->
    (12,) canonical affine G1 as an int64 tensor."""
    import torch
    if not gathered.is_cuda:
        gathered = gathered.to(torch.device("cuda", ctx.device))
    gathered = gathered.contiguous()
    out = torch.empty(12, dtype=torch.int64, device=gathered.device)
    ctx.torch_to_lib()
    ctx.g1_xyzz_sum_dev(gathered.data_ptr(), gathered.shape[0], 8 * gathered.shape[1], out.data_ptr())
    ctx.lib_to_torch()
    return out
