"""Spartan R1CS prover around the sqrt-PST commitment (csrc/r1cs.hip through
the C-ABI): the mirror of R1CSInstance / R1CSProof::prove (r1csinstance.rs,
r1csproof.rs:237-370), without the Groth16 `prove_verifier` step.

    inst, vars, inputs = R1CSInstance.produce_synthetic_r1cs(ctx, num_cons, num_vars, num_inputs, seed)
    sqrt_pst.srs_setup(ctx, (log2(num_vars) + 1) // 2, seed)
    proof, rx, ry = R1CSProof.prove(inst, vars, inputs, PoseidonTranscript())

No CPU fallback: every table and sum-check round runs on the device.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .encoding import ptr
from .engine import Context
from .sqrt_pst import MippProof, PoseidonTranscript, _unpack


def _fr(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return a.reshape(-1, 4) if n is None else a.reshape(n, 4)


def transcript_append_scalar(tr: PoseidonTranscript, fr) -> None:
    """PoseidonTranscript::append_scalar (poseidon_transcript.rs:83-85)."""
    rc = _lib.load().tpst_transcript_append_fr(C.byref(tr.t), ptr(_fr(fr, 1)))
    if rc != 0:
        raise ValueError("scalar >= r")


def transcript_new_from_state2(tr: PoseidonTranscript, fr) -> None:
    """PoseidonTranscript::new_from_state2 (poseidon_transcript.rs:55-60)."""
    rc = _lib.load().tpst_transcript_reset_fr(C.byref(tr.t), ptr(_fr(fr, 1)))
    if rc != 0:
        raise ValueError("scalar >= r")


class UniPoly:
    """UniPoly::from_evals (unipoly.rs:15-45): the round-polynomial encoding of
    the sum-checks (host C-ABI, the same routine the device rounds use)."""

    @staticmethod
    def from_evals(evals) -> np.ndarray:
        e = _fr(evals)
        out = np.zeros_like(e)
        if _lib.load().tpst_unipoly_from_evals(ptr(e), len(e), ptr(out)) != 0:
            raise ValueError("UniPoly::from_evals takes 3 or 4 evaluations < r")
        return out


class EqPolynomial:
    """EqPolynomial (dense_mlpoly.rs:221-250): ``evals`` is the MSB-first chi
    table of r, computed by the device kernel the phase-one sum-check uses."""

    def __init__(self, r):
        self.r = _fr(r)

    def evals(self, ctx: Context) -> np.ndarray:
        ell = len(self.r)
        out = np.zeros((1 << ell, 4), dtype=np.uint64)
        ctx.check(ctx.lib.tpst_eq_evals(ctx.h, ptr(self.r), ell, ptr(out)), "EqPolynomial::evals")
        return out


class R1CSInstance:
    """Device-resident R1CS instance (A, B, C as CSR + CSC)."""

    def __init__(self, ctx: Context, handle, num_cons, num_vars, num_inputs):
        self.ctx, self.h = ctx, handle
        self.num_cons, self.num_vars, self.num_inputs = num_cons, num_vars, num_inputs

    @classmethod
    def new(cls, ctx: Context, num_cons, num_vars, num_inputs, A, B, C_):
        """R1CSInstance::new (r1csinstance.rs:91-140): A, B, C lists of (row, col, Fr limbs)."""
        mats = []
        for M in (A, B, C_):
            rows = np.ascontiguousarray([e[0] for e in M], dtype=np.uint32)
            cols = np.ascontiguousarray([e[1] for e in M], dtype=np.uint32)
            vals = _fr(np.array([np.asarray(e[2], dtype=np.uint64) for e in M]).reshape(-1)) if M else \
                np.zeros((0, 4), dtype=np.uint64)
            mats.append((rows, cols, vals))
        nnz = (C.c_size_t * 3)(*[len(m[0]) for m in mats])
        rp = (C.c_void_p * 3)(*[m[0].ctypes.data for m in mats])
        cp = (C.c_void_p * 3)(*[m[1].ctypes.data for m in mats])
        vp = (C.c_void_p * 3)(*[m[2].ctypes.data for m in mats])
        h = C.c_void_p()
        ctx.check(ctx.lib.tpst_r1cs_load(ctx.h, num_cons, num_vars, num_inputs, nnz, rp, cp, vp, C.byref(h)),
                  "tpst_r1cs_load")
        return cls(ctx, h, num_cons, num_vars, num_inputs)

    @classmethod
    def produce_synthetic_r1cs(cls, ctx: Context, num_cons, num_vars, num_inputs, seed):
        """r1csinstance.rs:166-242 over the seeded Fr stream -> (inst, vars, inputs)."""
        vars_ = np.zeros((num_vars, 4), dtype=np.uint64)
        inputs = np.zeros((max(num_inputs, 1), 4), dtype=np.uint64)
        h = C.c_void_p()
        ctx.check(ctx.lib.tpst_r1cs_synthetic(ctx.h, num_cons, num_vars, num_inputs, seed, C.byref(h), ptr(vars_),
                                              ptr(inputs)), "tpst_r1cs_synthetic")
        return cls(ctx, h, num_cons, num_vars, num_inputs), vars_, inputs[:num_inputs]

    def commit(self, label: bytes):
        """R1CSInstance::commit (r1csinstance.rs:313-344): SparseMatPolynomial::
        multi_commit over (A, B, C) -> (comm_comb_ops, comm_comb_mem) G1 rows."""
        ctx = self.ctx
        n_ops, n_mem = C.c_size_t(0), C.c_size_t(0)
        ctx.check(ctx.lib.tpst_r1cs_commit(ctx.h, self.h, bytes(label), len(label), None, C.byref(n_ops), None,
                                           C.byref(n_mem)), "tpst_r1cs_commit")
        ops = np.zeros((n_ops.value, 12), dtype=np.uint64)
        mem = np.zeros((n_mem.value, 12), dtype=np.uint64)
        ctx.check(ctx.lib.tpst_r1cs_commit(ctx.h, self.h, bytes(label), len(label), ptr(ops), C.byref(n_ops),
                                           ptr(mem), C.byref(n_mem)), "tpst_r1cs_commit")
        return ops, mem

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.tpst_r1cs_free(self.h)
                self.h = None
        except Exception:
            pass


@dataclass
class R1CSProof:
    T: np.ndarray
    initial_state: np.ndarray
    sc_proof_phase1: np.ndarray      # (rounds_x, 4) Fr coefficients, constant first
    claims_phase2: np.ndarray        # (Az, Bz, Cz, Az Bz)(rx)
    sc_proof_phase2: np.ndarray      # (rounds_y, 3)
    claims_z_abc: np.ndarray         # phase-two finals (z(ry), ABC(ry))
    r_abc: np.ndarray
    rx: np.ndarray
    ry: np.ndarray
    transcript_sat_state: np.ndarray
    eval_vars_at_ry: np.ndarray
    comm: np.ndarray                 # U
    proof_eval_vars_at_ry: np.ndarray
    mipp_proof: MippProof

    @staticmethod
    def prove(inst: R1CSInstance, vars_, inputs, transcript: PoseidonTranscript):
        """r1csproof.rs:237-370 -> (proof, rx, ry)."""
        ctx = inst.ctx
        vars_ = _fr(vars_, inst.num_vars)
        inputs = _fr(inputs) if inst.num_inputs else np.zeros((1, 4), dtype=np.uint64)
        pr = _lib.R1CSProof()
        ctx.check(ctx.lib.tpst_r1cs_prove(ctx.h, inst.h, ptr(vars_), ptr(inputs), C.byref(transcript.t),
                                          C.byref(pr)), "tpst_r1cs_prove")
        a = lambda x: np.ctypeslib.as_array(x).copy()  # noqa: E731
        rxn, ryn = pr.rounds_x, pr.rounds_y
        U, pst, mipp = _unpack(pr.open)
        proof = R1CSProof(T=a(pr.T), initial_state=a(pr.initial_state), sc_proof_phase1=a(pr.sc1)[:rxn],
                          claims_phase2=a(pr.claims_phase2), sc_proof_phase2=a(pr.sc2)[:ryn],
                          claims_z_abc=a(pr.claims_phase2_z_abc), r_abc=a(pr.r_abc), rx=a(pr.rx)[:rxn],
                          ry=a(pr.ry)[:ryn], transcript_sat_state=a(pr.transcript_sat_state),
                          eval_vars_at_ry=a(pr.eval_vars_at_ry), comm=U, proof_eval_vars_at_ry=pst,
                          mipp_proof=mipp)
        return proof, proof.rx, proof.ry
