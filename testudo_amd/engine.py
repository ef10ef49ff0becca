"""Python handle on a libtpst context (one per GPU / process).

Thin, typed wrappers over the C-ABI primitives; every call goes to the HIP
library.  Errors raise ``TpstError`` with the library's message.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .encoding import ptr


class TpstError(RuntimeError):
    pass


class Context:
    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = C.c_void_p()
        rc = self.lib.tpst_create(device, C.byref(h))
        if rc != 0:
            raise TpstError("tpst_create(%d) failed: %d" % (device, rc))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            self.lib.tpst_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.tpst_last_error(self.h)
            raise TpstError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    # ------------------------------------------------------------ MSM ----
    def g1_msm(self, bases: np.ndarray, scalars: np.ndarray) -> np.ndarray:
        bases = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, 12)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros(12, dtype=np.uint64)
        self.check(self.lib.tpst_g1_msm(self.h, ptr(bases), len(bases), ptr(scalars), len(scalars), ptr(out)),
                   "tpst_g1_msm")
        return out

    def g2_msm(self, bases: np.ndarray, scalars: np.ndarray) -> np.ndarray:
        bases = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, 24)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros(24, dtype=np.uint64)
        self.check(self.lib.tpst_g2_msm(self.h, ptr(bases), len(bases), ptr(scalars), len(scalars), ptr(out)),
                   "tpst_g2_msm")
        return out

    def multiexp(self, bases: np.ndarray, scalars: np.ndarray, g2: bool = False) -> np.ndarray:
        """mipp.rs:385-394 `multiexponentiation`: raises on a length mismatch
        (the reference's Err(InvalidIPVectorLength))."""
        w = 24 if g2 else 12
        bases = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, w)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros(w, dtype=np.uint64)
        fn = self.lib.tpst_g2_multiexp if g2 else self.lib.tpst_g1_multiexp
        self.check(fn(self.h, ptr(bases), len(bases), ptr(scalars), len(scalars), ptr(out)), "multiexponentiation")
        return out

    def msm_fixed(self, bases: np.ndarray, scalars: np.ndarray, L: int = 0, D: int = 0, g2: bool = False):
        """Grouped fixed-base MSM (include/tpst.h tpst_g*_msm_fixed): (L/D, 12|24)."""
        w = 24 if g2 else 12
        bases = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, w)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        n = len(bases)
        L = L or n
        D = D or L
        out = np.zeros((L // D, w), dtype=np.uint64)
        fn = self.lib.tpst_g2_msm_fixed if g2 else self.lib.tpst_g1_msm_fixed
        self.check(fn(self.h, ptr(bases), n, ptr(scalars), L, D, ptr(out)), "tpst_msm_fixed")
        return out

    def multi_pairing(self, g1: np.ndarray, g2: np.ndarray) -> np.ndarray:
        g1 = np.ascontiguousarray(g1, dtype=np.uint64).reshape(-1, 12)
        g2 = np.ascontiguousarray(g2, dtype=np.uint64).reshape(-1, 24)
        assert len(g1) == len(g2)
        out = np.zeros(72, dtype=np.uint64)
        self.check(self.lib.tpst_multi_pairing(self.h, ptr(g1), ptr(g2), len(g1), ptr(out)), "tpst_multi_pairing")
        return out

    def g1_mul_generator(self, scalars: np.ndarray) -> np.ndarray:
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros((len(scalars), 12), dtype=np.uint64)
        self.check(self.lib.tpst_g1_mul_generator(self.h, ptr(scalars), len(scalars), ptr(out)),
                   "tpst_g1_mul_generator")
        return out

    def g2_mul_generator(self, scalars: np.ndarray) -> np.ndarray:
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros((len(scalars), 24), dtype=np.uint64)
        self.check(self.lib.tpst_g2_mul_generator(self.h, ptr(scalars), len(scalars), ptr(out)),
                   "tpst_g2_mul_generator")
        return out

    # ------------------------------------------------------- profiling ---
    STAGES = ("decompose", "sort", "bounds", "bucket_acc", "reduce", "combine", "batch_sort",
              # sqrt-PST stages under the reference's Timer labels (sqrt_pst.rs:33-262), device spans
              "build_q", "sqrt_commit", "comm_list", "ipp", "sqrt_open", "msm", "mipp_prove", "pst_open")

    def profile(self, on: bool):
        self.check(self.lib.tpst_profile_enable(self.h, 1 if on else 0), "tpst_profile_enable")

    def profile_reset(self):
        self.check(self.lib.tpst_profile_reset(self.h), "tpst_profile_reset")

    def profile_read(self) -> dict:
        out = {}
        for i, name in enumerate(self.STAGES):
            ms, cnt = C.c_double(), C.c_uint64()
            self.check(self.lib.tpst_profile_read(self.h, i, C.byref(ms), C.byref(cnt)), "tpst_profile_read")
            out[name] = (ms.value, cnt.value)
        return out

    def synchronize(self):
        self.check(self.lib.tpst_synchronize(self.h), "tpst_synchronize")

    # ------------------------------------------- ordering against torch ---
    # The library runs on its own non-blocking stream.  A device buffer that
    # torch produced (all-gather output, a .contiguous() copy, torch.empty from
    # the caching allocator) is handed to a _dev call only after torch_to_lib();
    # a buffer the library filled is used by torch only after lib_to_torch().
    @staticmethod
    def _torch_stream(device):
        import torch
        return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)

    def torch_to_lib(self):
        """Library work queued from now on waits for torch's current stream."""
        self.check(self.lib.tpst_wait_stream(self.h, self._torch_stream(self.device)), "tpst_wait_stream")

    def lib_to_torch(self):
        """Torch work queued from now on (current stream) waits for the library."""
        self.check(self.lib.tpst_join_stream(self.h, self._torch_stream(self.device)), "tpst_join_stream")

    def g1_msm_dev(self, d_bases: int, d_scalars: int, n: int, d_out: int):
        """Stream-ordered device MSM: later work on the library stream sees d_out."""
        self.check(self.lib.tpst_g1_msm_dev(self.h, C.c_void_p(d_bases), C.c_void_p(d_scalars), n,
                                            C.c_void_p(d_out)), "tpst_g1_msm_dev")

    def g1_msm_dev_async(self, d_bases: int, d_scalars: int, n: int, d_out: int):
        """Pipelined device MSM (tpst_g1_msm_dev_async): consecutive calls overlap.
        The buffers must stay alive and untouched until synchronize() /
        lib_to_torch() or the next call of another entry point."""
        self.check(self.lib.tpst_g1_msm_dev_async(self.h, C.c_void_p(d_bases), C.c_void_p(d_scalars), n,
                                                  C.c_void_p(d_out)), "tpst_g1_msm_dev_async")

    def g1_msm_xyzz_dev(self, d_bases: int, d_scalars: int, n: int, d_out: int):
        """One rank's share of a split MSM: the raw XYZZ sum (24 u64, Montgomery) at d_out."""
        self.check(self.lib.tpst_g1_msm_xyzz_dev(self.h, C.c_void_p(d_bases), C.c_void_p(d_scalars), n,
                                                 C.c_void_p(d_out)), "tpst_g1_msm_xyzz_dev")

    def g1_xyzz_sum_dev(self, d_parts: int, k: int, stride_bytes: int, d_out: int):
        """Sum of k XYZZ shares (stride_bytes apart) -> one canonical affine G1 (12 u64) at d_out."""
        self.check(self.lib.tpst_g1_xyzz_sum_dev(self.h, C.c_void_p(d_parts), k, stride_bytes, C.c_void_p(d_out)),
                   "tpst_g1_xyzz_sum_dev")

    def g1_mul_generator_dev(self, d_scalars: int, n: int, d_out: int):
        self.check(self.lib.tpst_g1_mul_generator_dev(self.h, C.c_void_p(d_scalars), n, C.c_void_p(d_out)),
                   "tpst_g1_mul_generator_dev")

    def microbench(self, kind: int, threads: int, iters: int) -> float:
        ms = C.c_double()
        self.check(self.lib.tpst_microbench(self.h, kind, threads, iters, C.byref(ms)), "tpst_microbench")
        return ms.value

    def selftest_inv(self, vals: np.ndarray):
        """device Fq inverses of Montgomery-form values (n x 6 words) by the
        lone-lane and the wave-cooperative routine"""
        vals = np.ascontiguousarray(vals, dtype=np.uint64).reshape(-1, 6)
        ol = np.zeros_like(vals)
        ow = np.zeros_like(vals)
        self.check(self.lib.tpst_selftest_inv(self.h, len(vals), ptr(vals), ptr(ol), ptr(ow)), "tpst_selftest_inv")
        return ol, ow


class Gens:
    """MultiCommitGens {n, G, h} (commitments.rs:9-15) resident on the device,
    with PedersenCommit::commit_slice (commitments.rs:79-86), the Hyrax row
    commitments of DensePolynomial::commit_inner (dense_mlpoly.rs:314-329) and
    the strided shared-base batch MSM."""

    def __init__(self, ctx: Context, G: np.ndarray, h: np.ndarray = None):
        self.ctx = ctx
        G = np.ascontiguousarray(G, dtype=np.uint64).reshape(-1, 12)
        self.n = len(G)
        hh = None if h is None else np.ascontiguousarray(h, dtype=np.uint64).reshape(12)
        handle = C.c_void_p()
        ctx.check(ctx.lib.tpst_gens_load(ctx.h, ptr(G), self.n, ptr(hh) if hh is not None else None,
                                         C.byref(handle)), "tpst_gens_load")
        self.handle = handle

    @classmethod
    def new(cls, ctx: Context, n: int, label: bytes) -> "Gens":
        """MultiCommitGens::new (commitments.rs:17-39): the generators of a
        label, derived on the device (tpst_gens_new); .G (n, 12), .h (12,)."""
        G = np.zeros((n, 12), dtype=np.uint64)
        h = np.zeros(12, dtype=np.uint64)
        handle = C.c_void_p()
        ctx.check(ctx.lib.tpst_gens_new(ctx.h, n, bytes(label), len(label), ptr(G), ptr(h), C.byref(handle)),
                  "tpst_gens_new")
        obj = cls.__new__(cls)
        obj.ctx, obj.n, obj.handle, obj.G, obj.h = ctx, n, handle, G, h
        return obj

    def close(self):
        if self.handle:
            self.ctx.lib.tpst_gens_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def msm_batch(self, scalars: np.ndarray, rows: int, row_stride: int, col_stride: int) -> np.ndarray:
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros((rows, 12), dtype=np.uint64)
        if rows and self.n:
            need = (rows - 1) * row_stride + (self.n - 1) * col_stride + 1
            if len(scalars) < need:
                raise TpstError("scalar buffer shorter than the strided view")
        self.ctx.check(self.ctx.lib.tpst_g1_msm_batch(self.ctx.h, self.handle, ptr(scalars), rows, self.n,
                                                      row_stride, col_stride, ptr(out)), "tpst_g1_msm_batch")
        return out

    def commit_slice(self, scalars: np.ndarray, blind: np.ndarray) -> np.ndarray:
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        blind = np.ascontiguousarray(blind, dtype=np.uint64).reshape(4)
        out = np.zeros(12, dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_pedersen_commit_slice(self.ctx.h, self.handle, ptr(scalars), len(scalars),
                                                               ptr(blind), ptr(out)), "commit_slice")
        return out

    def commit_rows(self, Z: np.ndarray, blinds: np.ndarray) -> np.ndarray:
        Z = np.ascontiguousarray(Z, dtype=np.uint64).reshape(-1, 4)
        blinds = np.ascontiguousarray(blinds, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros((len(blinds), 12), dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_pedersen_commit_rows(self.ctx.h, self.handle, ptr(Z), len(Z), ptr(blinds),
                                                              len(blinds), ptr(out)), "commit_inner")
        return out


def dense_commit(gens: Gens, Z: np.ndarray, blinds: np.ndarray = None) -> np.ndarray:
    """DensePolynomial::commit (dense_mlpoly.rs:349-377), the Hyrax commitment:
    ell = log2 |Z|, L = 2^(ell/2) rows of R = 2^(ell - ell/2) contiguous
    evaluations, row i -> commit_slice(Z[R i .. R (i+1)], blinds[i]) with
    gens.n == R; blinds default to zero (random_blinds = false, as in
    Derefs::commit sparse_mlpoly.rs:75-81 and SparseMatPolynomial::multi_commit)."""
    Z = np.ascontiguousarray(Z, dtype=np.uint64).reshape(-1, 4)
    ell = len(Z).bit_length() - 1
    if len(Z) != 1 << ell:
        raise TpstError("|Z| must be a power of two")
    L, R = 1 << (ell // 2), 1 << (ell - ell // 2)
    if gens.n != R:
        raise TpstError("gens.n must be 2^(ell - ell/2)")
    if blinds is None:
        blinds = np.zeros((L, 4), dtype=np.uint64)
    return gens.commit_rows(Z, blinds)
