"""Groth16 over BLS12-377 for an R1CS instance (csrc/groth16.hip through the
C-ABI): the prover behind R1CSProof::prove_verifier (r1csproof.rs:374-434,
``Groth16::<E>::prove`` at :421) -- ark-groth16's LibsnarkReduction QAP
(NTTs on the device) and four device MSMs -- with the matching key generation
and the pairing-product verifier.

    inst, vars, inputs = R1CSInstance.produce_synthetic_r1cs(ctx, m, n, k, seed)
    pk = ProvingKey.setup(inst, toxic)          # toxic = (tau, alpha, beta, gamma, delta)
    proof = prove(pk, inst, vars, inputs, r, s)
    assert verify(ctx, pk.vk(), inputs, proof)

The reference draws the toxic waste and (r, s) from thread_rng; here they are
arguments so runs reproduce.  No CPU fallback: setup, witness map and MSMs
run on the device; verify is a device multi-pairing.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from .encoding import ptr
from .r1cs import R1CSInstance, _fr

_P = 0x01AE3A4617C510EAC63B05C06CA1493B1A22D9F300F5138F1EF3622FBA094800170B5D44300000008508C00000000001


@dataclass
class VerifyingKey:
    alpha_g1: np.ndarray      # (12,)
    beta_g2: np.ndarray       # (24,)
    gamma_g2: np.ndarray
    delta_g2: np.ndarray
    gamma_abc_g1: np.ndarray  # (num_inputs + 1, 12)


@dataclass
class Proof:
    a: np.ndarray  # G1 (12,)
    b: np.ndarray  # G2 (24,)
    c: np.ndarray  # G1 (12,)


class ProvingKey:
    """Device-resident proving key of one R1CS instance."""

    def __init__(self, inst: R1CSInstance, handle):
        self.inst, self.ctx, self.h = inst, inst.ctx, handle

    @classmethod
    def setup(cls, inst: R1CSInstance, toxic) -> "ProvingKey":
        """generate_random_parameters_with_reduction (ark-groth16 generator.rs)
        with the toxic waste (tau, alpha, beta, gamma, delta) given."""
        ctx = inst.ctx
        t = _fr(toxic, 5)
        h = C.c_void_p()
        ctx.check(ctx.lib.tpst_groth16_setup(ctx.h, inst.h, ptr(t), C.byref(h)), "tpst_groth16_setup")
        return cls(inst, h)

    @property
    def domain_size(self) -> int:
        n = C.c_size_t(0)
        self.ctx.check(self.ctx.lib.tpst_groth16_domain(self.h, C.byref(n)), "tpst_groth16_domain")
        return n.value

    def vk(self) -> VerifyingKey:
        ni = self.inst.num_inputs
        a, b, g, d = (np.zeros(w, dtype=np.uint64) for w in (12, 24, 24, 24))
        abc = np.zeros((ni + 1, 12), dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_groth16_vk(self.ctx.h, self.h, ptr(a), ptr(b), ptr(g), ptr(d), ptr(abc)),
                       "tpst_groth16_vk")
        return VerifyingKey(a, b, g, d, abc)

    def witness_map(self, vars_, inputs) -> np.ndarray:
        """LibsnarkReduction::witness_map: (n - 1, 4) canonical h coefficients."""
        inst = self.inst
        h = np.zeros((self.domain_size - 1, 4), dtype=np.uint64)
        self.ctx.check(self.ctx.lib.tpst_groth16_witness_map(self.ctx.h, self.h, inst.h, ptr(_fr(vars_, inst.num_vars)),
                                                             ptr(_inputs(inst, inputs)), ptr(h)),
                       "tpst_groth16_witness_map")
        return h

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.tpst_groth16_pk_free(self.h)
                self.h = None
        except Exception:
            pass


def _inputs(inst, inputs):
    return _fr(inputs) if inst.num_inputs else np.zeros((1, 4), dtype=np.uint64)


def prove(pk: ProvingKey, inst: R1CSInstance, vars_, inputs, r, s) -> Proof:
    """create_proof_with_reduction (ark-groth16 prover.rs) with (r, s) given."""
    ctx = pk.ctx
    rs = _fr(np.concatenate([_fr(r, 1), _fr(s, 1)]), 2)
    a, b, c = np.zeros(12, dtype=np.uint64), np.zeros(24, dtype=np.uint64), np.zeros(12, dtype=np.uint64)
    ctx.check(ctx.lib.tpst_groth16_prove(ctx.h, pk.h, inst.h, ptr(_fr(vars_, inst.num_vars)), ptr(_inputs(inst, inputs)),
                                         ptr(rs), ptr(a), ptr(b), ptr(c)), "tpst_groth16_prove")
    return Proof(a, b, c)


def verify(ctx, vk: VerifyingKey, inputs, proof: Proof) -> bool:
    """Groth16::verify_proof: e(A, B) == e(alpha, beta) e(IC, gamma) e(C, delta)
    with IC = gamma_abc[0] + sum inputs_i gamma_abc[i + 1] (tpst_groth16_verify:
    a device MSM and one device multi-pairing).  Every proof and key element
    is validated first (canonical, on the curve, in the subgroup; inputs < r),
    as arkworks' Validate::Yes deserialisation would: a malformed element is
    an invalid proof (False)."""
    inputs = np.ascontiguousarray(inputs, dtype=np.uint64).reshape(-1, 4)
    abc = np.ascontiguousarray(vk.gamma_abc_g1, dtype=np.uint64).reshape(-1, 12)
    if len(inputs) + 1 != len(abc):
        raise ValueError("wrong number of public inputs")
    u = lambda a, n: np.ascontiguousarray(a, dtype=np.uint64).reshape(n)  # noqa: E731
    rc = ctx.lib.tpst_groth16_verify(ctx.h, ptr(u(vk.alpha_g1, 12)), ptr(u(vk.beta_g2, 24)), ptr(u(vk.gamma_g2, 24)),
                                     ptr(u(vk.delta_g2, 24)), ptr(abc), len(abc),
                                     ptr(inputs if len(inputs) else np.zeros((1, 4), dtype=np.uint64)), len(inputs),
                                     ptr(u(proof.a, 12)), ptr(u(proof.b, 24)), ptr(u(proof.c, 12)))
    if rc == -5:
        return False
    ctx.check(rc, "Groth16::verify")
    return True
