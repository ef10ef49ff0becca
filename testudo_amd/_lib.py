"""ctypes binding of libtpst.so (include/tpst.h).

The library is built in-tree by testudo_amd/build.py.  There is no CPU
fallback: if the shared object is missing or cannot be loaded, importing the
product path raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TPST_LIB_PATH") or os.path.join(_HERE, "libtpst.so")  # override: A/B builds (experiments)

_u64p = C.POINTER(C.c_uint64)
_vp = C.c_void_p
_sz = C.c_size_t

# (name, restype, argtypes) -- mirrors include/tpst.h
PROTOTYPES = [
    ("tpst_device_count", C.c_int, []),
    ("tpst_create", C.c_int, [C.c_int, C.POINTER(_vp)]),
    ("tpst_destroy", None, [_vp]),
    ("tpst_last_error", C.c_char_p, [_vp]),
    ("tpst_stream", _vp, [_vp]),
    ("tpst_synchronize", C.c_int, [_vp]),
    ("tpst_wait_stream", C.c_int, [_vp, _vp]),
    ("tpst_join_stream", C.c_int, [_vp, _vp]),
    ("tpst_g1_msm", C.c_int, [_vp, _u64p, _sz, _u64p, _sz, _u64p]),
    ("tpst_g2_msm", C.c_int, [_vp, _u64p, _sz, _u64p, _sz, _u64p]),
    ("tpst_g1_msm_dev", C.c_int, [_vp, _vp, _vp, _sz, _vp]),
    ("tpst_g1_msm_dev_async", C.c_int, [_vp, _vp, _vp, _sz, _vp]),
    ("tpst_g1_msm_xyzz_dev", C.c_int, [_vp, _vp, _vp, _sz, _vp]),
    ("tpst_g1_xyzz_sum_dev", C.c_int, [_vp, _vp, _sz, _sz, _vp]),
    ("tpst_g1_multiexp", C.c_int, [_vp, _u64p, _sz, _u64p, _sz, _u64p]),
    ("tpst_g2_multiexp", C.c_int, [_vp, _u64p, _sz, _u64p, _sz, _u64p]),
    ("tpst_gens_load", C.c_int, [_vp, _u64p, _sz, _u64p, C.POINTER(_vp)]),
    ("tpst_gens_free", None, [_vp]),
    ("tpst_gens_new", C.c_int, [_vp, _sz, C.c_char_p, _sz, _u64p, _u64p, C.POINTER(_vp)]),
    ("tpst_gens_seeds", C.c_int, [_sz, C.c_char_p, _sz, C.c_char_p]),
    ("tpst_g1_msm_batch", C.c_int, [_vp, _vp, _u64p, _sz, _sz, _sz, _sz, _u64p]),
    ("tpst_g1_msm_batch_dev", C.c_int, [_vp, _vp, _vp, _sz, _sz, _sz, _sz, _vp]),
    ("tpst_pedersen_commit_slice", C.c_int, [_vp, _vp, _u64p, _sz, _u64p, _u64p]),
    ("tpst_pedersen_commit_rows", C.c_int, [_vp, _vp, _u64p, _sz, _u64p, _sz, _u64p]),
    ("tpst_g1_msm_fixed", C.c_int, [_vp, _u64p, _sz, _u64p, _sz, _sz, _u64p]),
    ("tpst_g2_msm_fixed", C.c_int, [_vp, _u64p, _sz, _u64p, _sz, _sz, _u64p]),
    ("tpst_multi_pairing", C.c_int, [_vp, _u64p, _u64p, _sz, _u64p]),
    ("tpst_g1_check", C.c_int, [_u64p]),
    ("tpst_g2_check", C.c_int, [_u64p]),
    ("tpst_g1_mul_generator", C.c_int, [_vp, _u64p, _sz, _u64p]),
    ("tpst_g2_mul_generator", C.c_int, [_vp, _u64p, _sz, _u64p]),
    ("tpst_g1_mul_generator_dev", C.c_int, [_vp, _vp, _sz, _vp]),
    ("tpst_microbench", C.c_int, [_vp, C.c_int, _sz, C.c_int, C.POINTER(C.c_double)]),
    ("tpst_microbench_wave_phases", C.c_int, [_vp, C.c_int, C.c_int, _u64p]),
    ("tpst_selftest_inv", C.c_int, [_vp, _sz, _u64p, _u64p, _u64p]),
    ("tpst_transcript_init", None, [_vp]),
    ("tpst_transcript_append_g1", C.c_int, [_vp, _u64p]),
    ("tpst_transcript_append_gt", C.c_int, [_vp, _u64p]),
    ("tpst_transcript_challenge", C.c_int, [_vp, _u64p]),
    ("tpst_srs_flat_len", _sz, [C.c_int]),
    ("tpst_srs_setup", C.c_int, [_vp, C.c_int, C.c_uint64]),
    ("tpst_srs_load", C.c_int, [_vp, C.c_int, _u64p]),
    ("tpst_srs_export", C.c_int, [_vp, _u64p]),
    ("tpst_fr_stream", C.c_uint64, [C.c_uint64, _sz, C.c_uint64, _u64p]),
    ("tpst_poly_from_evaluations", C.c_int, [_vp, _u64p, C.c_int, C.POINTER(_vp)]),
    ("tpst_poly_from_evaluations_dev", C.c_int, [_vp, _vp, C.c_int, C.POINTER(_vp)]),
    ("tpst_poly_from_evaluations_cols", C.c_int, [_vp, _u64p, C.c_int, _sz, _sz, C.POINTER(_vp)]),
    ("tpst_poly_free", None, [_vp]),
    ("tpst_poly_eval", C.c_int, [_vp, _vp, _u64p, _u64p]),
    ("tpst_poly_commit", C.c_int, [_vp, _vp, _u64p, _u64p]),
    ("tpst_poly_commit_dev", C.c_int, [_vp, _vp, _vp, _vp]),
    ("tpst_poly_commit_rows", C.c_int, [_vp, _vp, _sz, _sz, _u64p]),
    ("tpst_poly_ipp", C.c_int, [_vp, C.c_int, _u64p, _u64p]),
    ("tpst_poly_commit_rows_partial", C.c_int, [_vp, _vp, _sz, _sz, _u64p, _u64p]),
    ("tpst_gt_final_exp_product", C.c_int, [_vp, _u64p, _sz, _u64p]),
    ("tpst_poly_commit_rows_partial_dev", C.c_int, [_vp, _vp, _sz, _sz, _vp]),
    ("tpst_gt_final_exp_product_dev", C.c_int, [_vp, _vp, _sz, _sz, _u64p]),
    ("tpst_poly_get_q_partial", C.c_int, [_vp, _vp, _u64p, _sz, _sz, _u64p]),
    ("tpst_poly_get_q_partial_dev", C.c_int, [_vp, _vp, _u64p, _sz, _sz, _vp]),
    ("tpst_fr_sum_dev", C.c_int, [_vp, _vp, _sz, _sz, _vp]),
    ("tpst_poly_cu_partial", C.c_int, [_vp, C.c_int, _u64p, _sz, _sz, _u64p, _u64p]),
    ("tpst_poly_from_q_dev", C.c_int, [_vp, C.c_int, _u64p, _vp, _u64p, C.POINTER(_vp)]),
    ("tpst_poly_open", C.c_int, [_vp, _vp, _vp, _u64p, _u64p, _u64p, _vp]),
    ("tpst_open_sharded_arena_bytes", _sz, [C.c_int, C.c_int]),
    ("tpst_poly_open_sharded", C.c_int, [_vp, _vp, _vp, C.c_int, _u64p, _u64p, _u64p, _vp, _vp]),
    ("tpst_pst_verify", C.c_int, [_vp, _vp, C.c_int, _u64p, _u64p, _u64p, _vp]),
    ("tpst_mlpc_commit", C.c_int, [_vp, _u64p, C.c_int, _u64p]),
    ("tpst_mlpc_commit_g2", C.c_int, [_vp, _u64p, C.c_int, _u64p]),
    ("tpst_mlpc_open", C.c_int, [_vp, _u64p, C.c_int, _u64p, _u64p]),
    ("tpst_mlpc_open_g1", C.c_int, [_vp, _u64p, C.c_int, _u64p, _u64p]),
    ("tpst_mlpc_check", C.c_int, [_vp, C.c_int, _u64p, _u64p, _u64p, _u64p]),
    ("tpst_mlpc_check_2", C.c_int, [_vp, C.c_int, _u64p, _u64p, _u64p, _u64p]),
    ("tpst_transcript_append_fr", C.c_int, [_vp, _u64p]),
    ("tpst_transcript_reset_fr", C.c_int, [_vp, _u64p]),
    ("tpst_transcript_append_bytes", C.c_int, [_vp, C.c_char_p, _sz]),
    ("tpst_unipoly_from_evals", C.c_int, [_u64p, C.c_int, _u64p]),
    ("tpst_eq_evals", C.c_int, [_vp, _u64p, C.c_int, _u64p]),
    ("tpst_r1cs_load", C.c_int, [_vp, _sz, _sz, _sz, C.POINTER(_sz), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp),
                                 C.POINTER(_vp)]),
    ("tpst_r1cs_synthetic", C.c_int, [_vp, _sz, _sz, _sz, C.c_uint64, C.POINTER(_vp), _u64p, _u64p]),
    ("tpst_r1cs_free", None, [_vp]),
    ("tpst_r1cs_commit", C.c_int, [_vp, _vp, C.c_char_p, _sz, _u64p, C.POINTER(_sz), _u64p, C.POINTER(_sz)]),
    ("tpst_r1cs_prove", C.c_int, [_vp, _vp, _u64p, _u64p, _vp, _vp]),
    ("tpst_groth16_setup", C.c_int, [_vp, _vp, _u64p, C.POINTER(_vp)]),
    ("tpst_groth16_pk_free", None, [_vp]),
    ("tpst_groth16_domain", C.c_int, [_vp, C.POINTER(_sz)]),
    ("tpst_groth16_vk", C.c_int, [_vp, _vp, _u64p, _u64p, _u64p, _u64p, _u64p]),
    ("tpst_groth16_witness_map", C.c_int, [_vp, _vp, _vp, _u64p, _u64p, _u64p]),
    ("tpst_groth16_prove", C.c_int, [_vp, _vp, _vp, _u64p, _u64p, _u64p, _u64p, _u64p, _u64p]),
    ("tpst_groth16_verify", C.c_int, [_vp, _u64p, _u64p, _u64p, _u64p, _u64p, _sz, _u64p, _sz, _u64p, _u64p,
                                      _u64p]),
    ("tpst_ser_g1", C.c_int, [_u64p, C.c_char_p]),
    ("tpst_ser_g2", C.c_int, [_u64p, C.c_char_p]),
    ("tpst_de_g1", C.c_int, [C.c_char_p, _u64p]),
    ("tpst_de_g2", C.c_int, [C.c_char_p, _u64p]),
    ("tpst_ser_commitment", C.c_int, [C.c_int, _u64p, C.c_char_p, _sz, C.POINTER(_sz)]),
    ("tpst_ser_pst_proof", C.c_int, [_vp, C.c_char_p, _sz, C.POINTER(_sz)]),
    ("tpst_ser_mipp_proof", C.c_int, [_vp, C.c_char_p, _sz, C.POINTER(_sz)]),
    ("tpst_de_open_proof", C.c_int, [C.c_char_p, _sz, C.c_char_p, _sz, _vp]),
    ("tpst_ser_committer_key", C.c_int, [C.c_int, _u64p, _sz, C.c_char_p, _sz, C.POINTER(_sz)]),
    ("tpst_profile_enable", C.c_int, [_vp, C.c_int]),
    ("tpst_profile_reset", C.c_int, [_vp]),
    ("tpst_profile_read", C.c_int, [_vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
]

MAX_VARS = 20


class Transcript(C.Structure):
    """tpst_transcript: PoseidonTranscript<Fq> sponge state."""
    _fields_ = [("state", (C.c_uint64 * 6) * 3), ("squeezing", C.c_uint32), ("index", C.c_uint32)]


class OpenProof(C.Structure):
    """tpst_open_proof: (U, PST proof, MippProof) of Polynomial::open."""
    _fields_ = [
        ("m_col", C.c_int32), ("m_row", C.c_int32),
        ("U", C.c_uint64 * 12),
        ("pst_proof", (C.c_uint64 * 24) * MAX_VARS),
        ("comms_t", ((C.c_uint64 * 72) * 2) * MAX_VARS),
        ("comms_u", ((C.c_uint64 * 12) * 2) * MAX_VARS),
        ("final_a", C.c_uint64 * 12),
        ("final_h", C.c_uint64 * 24),
        ("pst_proof_h", (C.c_uint64 * 12) * MAX_VARS),
    ]

# tpst_allgather_fn(user, send_off, recv_off, bytes, stream) -> 0 on success
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, _vp, _sz, _sz, _sz, _vp)


class Exchange(C.Structure):
    """tpst_exchange: the caller's all-gather for tpst_poly_open_sharded."""
    _fields_ = [("world", C.c_int), ("rank", C.c_int), ("allgather", ALLGATHER_FN), ("user", _vp),
                ("d_arena", _vp), ("arena_bytes", _sz)]


R1CS_MAX_ROUNDS = 48


class R1CSProof(C.Structure):
    """tpst_r1cs_proof: R1CSProof (r1csproof.rs:24-38) without the Groth16 part."""
    _fields_ = [
        ("rounds_x", C.c_int32), ("rounds_y", C.c_int32), ("num_vars_log", C.c_int32), ("pad", C.c_int32),
        ("T", C.c_uint64 * 72),
        ("initial_state", C.c_uint64 * 4),
        ("sc1", ((C.c_uint64 * 4) * 4) * R1CS_MAX_ROUNDS),
        ("claims_phase2", (C.c_uint64 * 4) * 4),
        ("claims_phase2_z_abc", (C.c_uint64 * 4) * 2),
        ("r_abc", (C.c_uint64 * 4) * 3),
        ("sc2", ((C.c_uint64 * 4) * 3) * R1CS_MAX_ROUNDS),
        ("rx", (C.c_uint64 * 4) * R1CS_MAX_ROUNDS),
        ("ry", (C.c_uint64 * 4) * R1CS_MAX_ROUNDS),
        ("transcript_sat_state", C.c_uint64 * 4),
        ("eval_vars_at_ry", C.c_uint64 * 4),
        ("open", OpenProof),
    ]


_lib = None


def load() -> C.CDLL:
    """Load libtpst.so and bind every prototype; raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libtpst.so not built (%s); run testudo_amd/build.py" % LIB_PATH)
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 /
    # libhsa-runtime64.so.1.  Loaded first, it satisfies libtpst's
    # dependencies by soname; loaded after libtpst (which links /opt/rocm's),
    # both runtimes would initialise the device and torch finds no GPU --
    # and device pointers / streams could not be shared across the two.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return [p[0] for p in PROTOTYPES]
