"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Pure-Python restatement of the arkworks wire format (ark-serialize 0.4,
Compress::Yes) for the sqrt-PST objects, the byte strings measured by
benches/pst.rs:43-46 (commiter_key_size) and :64-74 (proof_size =
|Proof| + |MippProof|).  Independent of the C++ writer in
testudo_amd/csrc/serialize.hip; the tests compare the two byte for byte.

Rules restated from the published crates (not vendored in /root/reference):
  * Fp: canonical value, little endian, buffer_byte_size(modulus bits + flag
    bits) bytes (Fq 48, Fr 32); SWFlags in the top two bits of the last
    byte: 0x80 = YIsNegative (y > -y), 0x40 = PointAtInfinity.
  * Fq2 = c0 || c1, flags on c1; Fq2 order compares c1 first, then c0.
  * Fq12 = 12 Fq in tower order, no flags.
  * usize = u64 LE; Vec<T> = u64 LE length || items; structs in field order:
      Commitment { nv, g_product }                      (ark-poly-commit)
      Proof { proofs: Vec<G2Affine> }, ProofG1 { proofs: Vec<G1Affine> }
      MippProof { comms_t, comms_u, final_a, final_h, pst_proof_h }  (mipp.rs:21-28)
      CommitterKey { nv, powers_of_g, powers_of_h, g, h }
Parity unpinned against arkworks (no Rust toolchain, no reference fixture).
"""
from __future__ import annotations

import struct

from bls377 import G2_B, P, R, f2_mul, f2_neg, f2_sqr, g1_in_subgroup, g1_on_curve, g2_in_subgroup, g2_on_curve


def _le(v: int, n: int) -> bytes:
    return v.to_bytes(n, "little")


def _fq_neg_flag(y: int) -> bool:
    return y > (P - y) % P


def _fq2_neg_flag(y) -> bool:
    n = f2_neg(y)
    if y[1] != n[1]:
        return y[1] > n[1]
    return y[0] > n[0]


def ser_g1(p) -> bytes:
    if p is None:
        return bytes(47) + b"\x40"
    x, y = p
    b = bytearray(_le(x, 48))
    if _fq_neg_flag(y):
        b[47] |= 0x80
    return bytes(b)


def ser_g2(p) -> bytes:
    if p is None:
        return bytes(95) + b"\x40"
    (x0, x1), y = p
    b = bytearray(_le(x0, 48) + _le(x1, 48))
    if _fq2_neg_flag(y):
        b[95] |= 0x80
    return bytes(b)


def ser_gt(t) -> bytes:
    return b"".join(_le(c, 48) for c in t)


def _u64(v: int) -> bytes:
    return struct.pack("<Q", v)


def ser_commitment(nv: int, g1) -> bytes:
    return _u64(nv) + ser_g1(g1)


def ser_pst_proof(proofs) -> bytes:
    return _u64(len(proofs)) + b"".join(ser_g2(q) for q in proofs)


def ser_mipp_proof(comms_t, comms_u, final_a, final_h, pst_proof_h) -> bytes:
    out = _u64(len(comms_t)) + b"".join(ser_gt(a) + ser_gt(b) for a, b in comms_t)
    out += _u64(len(comms_u)) + b"".join(ser_g1(a) + ser_g1(b) for a, b in comms_u)
    out += ser_g1(final_a) + ser_g2(final_h)
    out += _u64(len(pst_proof_h)) + b"".join(ser_g1(q) for q in pst_proof_h)
    return out


def ser_committer_key(nv, powers_of_g, powers_of_h, g, h) -> bytes:
    out = _u64(nv)
    out += _u64(len(powers_of_g)) + b"".join(_u64(len(l)) + b"".join(ser_g1(q) for q in l) for l in powers_of_g)
    out += _u64(len(powers_of_h)) + b"".join(_u64(len(l)) + b"".join(ser_g2(q) for q in l) for l in powers_of_h)
    return out + ser_g1(g) + ser_g2(h)


# ---- deserialisation (Validate::Yes) ----
def _fq_sqrt(a: int):
    """Tonelli-Shanks (p - 1 = 2^46 q); None for a non-residue."""
    a %= P
    if a == 0:
        return 0
    if pow(a, (P - 1) // 2, P) != 1:
        return None
    s, q = 0, P - 1
    while q % 2 == 0:
        q //= 2
        s += 1
    z = 2
    while pow(z, (P - 1) // 2, P) != P - 1:
        z += 1
    m, c, t, r = s, pow(z, q, P), pow(a, q, P), pow(a, (q + 1) // 2, P)
    while t != 1:
        i, t2 = 0, t
        while t2 != 1:
            t2 = t2 * t2 % P
            i += 1
        b = pow(c, 1 << (m - i - 1), P)
        m, c, t, r = i, b * b % P, t * b * b % P, r * b % P
    return r


def _fq2_sqrt(a):
    a0, a1 = a
    if a1 == 0:
        s = _fq_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = _fq_sqrt(-a0 * pow(5, -1, P) % P)
        return None if s is None else (0, s)
    d = _fq_sqrt((a0 * a0 + 5 * a1 * a1) % P)
    if d is None:
        return None
    half = pow(2, -1, P)
    for x0 in ((a0 + d) * half % P, (a0 - d) * half % P):
        c0 = _fq_sqrt(x0)
        if c0 is not None and c0 != 0:
            r = (c0, a1 * pow(2 * c0, -1, P) % P)
            return r if f2_sqr(r) == (a0 % P, a1 % P) else None
    return None


def de_g1(b: bytes):
    fl = b[47] & 0xC0
    if fl == 0xC0:
        raise ValueError("both flags")
    x = int.from_bytes(b[:47] + bytes([b[47] & 0x3F]), "little")
    if x >= P:
        raise ValueError("x >= p")
    if fl == 0x40:
        return None
    y = _fq_sqrt((x * x * x + 1) % P)
    if y is None:
        raise ValueError("not on curve")
    if _fq_neg_flag(y) != (fl == 0x80):
        y = (P - y) % P
    pt = (x, y)
    if not (g1_on_curve(pt) and g1_in_subgroup(pt)):
        raise ValueError("not in G1")
    return pt


def de_g2(b: bytes):
    fl = b[95] & 0xC0
    if fl == 0xC0:
        raise ValueError("both flags")
    x0 = int.from_bytes(b[:48], "little")
    x1 = int.from_bytes(b[48:95] + bytes([b[95] & 0x3F]), "little")
    if x0 >= P or x1 >= P:
        raise ValueError("x >= p")
    if fl == 0x40:
        return None
    x = (x0, x1)
    rhs = f2_mul(f2_sqr(x), x)
    rhs = ((rhs[0] + G2_B[0]) % P, (rhs[1] + G2_B[1]) % P)
    y = _fq2_sqrt(rhs)
    if y is None:
        raise ValueError("not on curve")
    if _fq2_neg_flag(y) != (fl == 0x80):
        y = f2_neg(y)
    pt = (x, y)
    if not (g2_on_curve(pt) and g2_in_subgroup(pt)):
        raise ValueError("not in G2")
    return pt


__all__ = ["ser_g1", "ser_g2", "ser_gt", "ser_commitment", "ser_pst_proof", "ser_mipp_proof",
           "ser_committer_key", "de_g1", "de_g2", "R"]
