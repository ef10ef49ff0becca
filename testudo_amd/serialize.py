"""arkworks wire format of the sqrt-PST objects (Compress::Yes), through the
host-only C-ABI of csrc/serialize.hip (no GPU needed).

Mirrors the reference's serialisation calls: benches/pst.rs:43-46
(`ck.serialize_with_mode(.., Compress::Yes)` -> commiter_key_size) and
:64-74 (`pst_proof` and `mipp_proof` -> proof_size).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .sqrt_pst import MippProof, _unpack, pack_proof


class SerializationError(ValueError):
    """ark_serialize::SerializationError (InvalidData / NotEnoughSpace)."""


def _lib_():
    return _lib.load()


def _u64p(a):
    return np.ascontiguousarray(a, dtype=np.uint64).ctypes.data_as(C.POINTER(C.c_uint64))


def _write(fn, *args) -> bytes:
    n = C.c_size_t(0)
    if fn(*args, None, 0, C.byref(n)) != 0:
        raise SerializationError("element not serialisable (non-canonical limbs)")
    buf = C.create_string_buffer(n.value)
    if fn(*args, buf, n.value, C.byref(n)) != 0:
        raise SerializationError("serialisation failed")
    return buf.raw[:n.value]


def ser_g1(p) -> bytes:
    out = C.create_string_buffer(48)
    if _lib_().tpst_ser_g1(_u64p(np.asarray(p, dtype=np.uint64).reshape(12)), out) != 0:
        raise SerializationError("bad G1 limbs")
    return out.raw


def ser_g2(p) -> bytes:
    out = C.create_string_buffer(96)
    if _lib_().tpst_ser_g2(_u64p(np.asarray(p, dtype=np.uint64).reshape(24)), out) != 0:
        raise SerializationError("bad G2 limbs")
    return out.raw


def de_g1(b: bytes) -> np.ndarray:
    out = np.zeros(12, dtype=np.uint64)
    if len(b) != 48 or _lib_().tpst_de_g1(b, _u64p(out)) != 0:
        raise SerializationError("invalid G1 encoding")
    return out


def de_g2(b: bytes) -> np.ndarray:
    out = np.zeros(24, dtype=np.uint64)
    if len(b) != 96 or _lib_().tpst_de_g2(b, _u64p(out)) != 0:
        raise SerializationError("invalid G2 encoding")
    return out


def ser_commitment(nv: int, g1) -> bytes:
    """ark-poly-commit Commitment { nv, g_product } (U of sqrt_pst.rs:201)."""
    g1 = np.ascontiguousarray(g1, dtype=np.uint64).reshape(12)
    return _write(_lib_().tpst_ser_commitment, nv, _u64p(g1))


def _proof_struct(pst_proof, mipp: MippProof):
    m_row, m_col = len(pst_proof), len(mipp.comms_t)
    return pack_proof(m_col + m_row, np.zeros(12, dtype=np.uint64), pst_proof, mipp)


def ser_pst_proof(pst_proof, mipp: MippProof) -> bytes:
    pr = _proof_struct(pst_proof, mipp)
    return _write(_lib_().tpst_ser_pst_proof, C.byref(pr))


def ser_mipp_proof(pst_proof, mipp: MippProof) -> bytes:
    pr = _proof_struct(pst_proof, mipp)
    return _write(_lib_().tpst_ser_mipp_proof, C.byref(pr))


def proof_size(pst_proof, mipp: MippProof) -> int:
    """benches/pst.rs:64-74: |pst_proof| + |mipp_proof| compressed."""
    return len(ser_pst_proof(pst_proof, mipp)) + len(ser_mipp_proof(pst_proof, mipp))


def de_open_proof(pst_bytes: bytes, mipp_bytes: bytes):
    """-> (pst_proof (m_row, 24), MippProof); SerializationError if invalid."""
    pr = _lib.OpenProof()
    if _lib_().tpst_de_open_proof(pst_bytes, len(pst_bytes), mipp_bytes, len(mipp_bytes), C.byref(pr)) != 0:
        raise SerializationError("invalid proof encoding")
    _, pst, mipp = _unpack(pr)
    return pst, mipp


def ser_committer_key(nv: int, srs_flat) -> bytes:
    """CommitterKey { nv, powers_of_g, powers_of_h, g, h } of the flat SRS
    (tpst_srs_export layout) -- benches/pst.rs:43-46."""
    flat = np.ascontiguousarray(srs_flat, dtype=np.uint64)
    return _write(_lib_().tpst_ser_committer_key, nv, _u64p(flat), len(flat))
