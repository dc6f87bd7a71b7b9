"""ctypes binding of libstarkgpu.so (the C ABI in include/stark_gpu.h).

The library is built in-tree by `make -C zk-stark-tutor_amd` (or
`__graft_entry__.build()`).  There is no fallback: if the shared object is
missing or cannot be loaded, importing the product path raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SG_LIB_PATH: load a differently-built copy (plan experiments); default in-tree build
LIB_PATH = os.environ.get("SG_LIB_PATH") or os.path.join(_HERE, "libstarkgpu.so")


class StarkGpuError(RuntimeError):
    """A libstarkgpu call returned a negative status."""

    def __init__(self, code, msg):
        super().__init__(f"libstarkgpu error {code}: {msg}")
        self.code = code


SG_OK = 0
SG_ERR_INVALID = -1
SG_ERR_HIP = -2
SG_ERR_NONCANONICAL = -3
SG_ERR_CALLBACK = -4
SG_ERR_NOMEM = -5


class sg_fe(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


class sg_fri(ctypes.Structure):
    _fields_ = [("offset", sg_fe), ("omega", sg_fe), ("domain_length", ctypes.c_uint64),
                ("expansion_factor", ctypes.c_uint64), ("num_colinearity_tests", ctypes.c_uint64)]


PUSH_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint8, ctypes.POINTER(ctypes.c_uint8),
                           ctypes.c_size_t)
FS_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint8))


class sg_proof_stream(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("push", PUSH_CB), ("fiat_shamir_prover", FS_CB)]


A2A_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


ABORT_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class sg_dist_transport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("all_to_all", A2A_CB), ("all_gather", A2A_CB), ("abort", ABORT_CB)]


# name -> (restype, argtypes)
_P = ctypes.POINTER
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_u8p = _P(ctypes.c_uint8)
_fep = _P(sg_fe)
PROTOTYPES = {
    "sg_ctx_create": (ctypes.c_int, [ctypes.c_int, _P(_vp)]),
    "sg_ctx_destroy": (None, [_vp]),
    "sg_last_error": (ctypes.c_char_p, [_vp]),
    "sg_ctx_stream": (_vp, [_vp]),
    "sg_ctx_trim": (ctypes.c_int, [_vp]),
    "sg_ctx_cached_tables": (ctypes.c_int, [_vp, _P(_sz), _P(_sz)]),
    "sg_ctx_set_option": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int64]),
    "sg_ctx_memory": (ctypes.c_int, [_vp, _P(ctypes.c_uint64), _P(ctypes.c_uint64), _P(ctypes.c_uint64),
                                     _P(ctypes.c_uint64), _P(ctypes.c_uint64), ctypes.c_int]),
    "sg_hbm_copy_probe": (ctypes.c_int, [_vp, _sz, ctypes.c_int, ctypes.c_uint, _P(ctypes.c_double)]),
    "sg_ctx_set_async": (ctypes.c_int, [_vp, ctypes.c_int]),
    "sg_ctx_synchronize": (ctypes.c_int, [_vp]),
    "sg_ctx_profile": (ctypes.c_int, [_vp, ctypes.c_int]),
    "sg_ctx_profile_only": (ctypes.c_int, [_vp, ctypes.c_char_p]),
    "sg_ctx_profile_report": (ctypes.c_int, [_vp, ctypes.c_char_p, _sz, _P(_sz)]),
    "sg_field_prime": (sg_fe, []),
    "sg_field_generator": (sg_fe, []),
    "sg_primitive_nth_root": (ctypes.c_int, [ctypes.c_uint64, _fep]),
    "sg_field_sample": (sg_fe, [_u8p, _sz]),
    "sg_fe_mul": (sg_fe, [sg_fe, sg_fe]),
    "sg_fe_inverse": (sg_fe, [sg_fe]),
    "sg_fe_pow": (sg_fe, [sg_fe, ctypes.c_uint64]),
    "sg_ntt": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _vp]),
    "sg_intt": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _vp]),
    "sg_fast_coset_evaluate": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, sg_fe, _vp, _sz, _vp]),
    "sg_ntt_dev": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _vp]),
    "sg_intt_dev": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _vp]),
    "sg_fast_coset_evaluate_dev": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, sg_fe, _vp, _sz, _vp]),
    "sg_fast_coset_evaluate_batch_dev": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, sg_fe, _P(_vp), _sz, _P(_vp),
                                                        _sz]),
    "sg_merkle_commit": (ctypes.c_int, [_vp, _vp, _sz, _vp]),
    "sg_merkle_open": (ctypes.c_int, [_vp, _sz, _vp, _sz, _vp, _P(_sz)]),
    "sg_merkle_verify": (ctypes.c_int, [_vp, _sz, _vp, _sz, sg_fe]),
    "sg_merkle_build_dev": (ctypes.c_int, [_vp, _vp, _sz, _P(_vp)]),
    "sg_merkle_build_batch_dev": (ctypes.c_int, [_vp, _P(_vp), _sz, _sz, _P(_vp)]),
    "sg_tree_root": (ctypes.c_int, [_vp, _vp]),
    "sg_tree_leaves": (_sz, [_vp]),
    "sg_tree_open": (ctypes.c_int, [_vp, _vp, _sz, _vp, _P(_sz)]),
    "sg_tree_free": (None, [_vp, _vp]),
    "sg_stream_create": (_vp, []),
    "sg_stream_create_signature": (_vp, [_vp, _sz]),
    "sg_stream_destroy": (None, [_vp]),
    "sg_stream_callbacks": (sg_proof_stream, [_vp]),
    "sg_stream_push": (ctypes.c_int, [_vp, ctypes.c_uint8, _vp, _sz]),
    "sg_stream_count": (_sz, [_vp]),
    "sg_stream_digest": (ctypes.c_int, [_vp, _vp, _sz, _P(_sz)]),
    "sg_stream_fiat_shamir_prover": (ctypes.c_int, [_vp, _sz, _vp]),
    "sg_stream_fiat_shamir_verifier": (ctypes.c_int, [_vp, _sz, _vp]),
    "sg_stream_pull": (ctypes.c_int, [_vp, _P(ctypes.c_uint8), _P(_u8p), _P(_sz)]),
    "sg_stream_deserialize": (ctypes.c_int, [_vp, _sz, _P(_vp)]),
    "sg_fri_num_rounds": (_sz, [_P(sg_fri)]),
    "sg_fri_commit": (ctypes.c_int, [_vp, _P(sg_fri), _vp, _sz, _P(sg_proof_stream), _P(_vp)]),
    "sg_fri_commit_dev": (ctypes.c_int, [_vp, _P(sg_fri), _vp, _sz, _P(sg_proof_stream), _P(_vp)]),
    "sg_fri_prove": (ctypes.c_int, [_vp, _P(sg_fri), _vp, _sz, _P(sg_proof_stream), _P(_sz)]),
    "sg_fri_prove_dev": (ctypes.c_int, [_vp, _P(sg_fri), _vp, _sz, _P(sg_proof_stream), _P(_sz)]),
    "sg_fri_state_free": (None, [_vp, _vp]),
    "sg_fri_sample_indices": (ctypes.c_int, [_vp, _sz, _sz, _sz, _sz, _P(_sz)]),
    # row-sharded blocks (multi-GPU)
    "sg_ntt_rows_dev": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _sz, _vp, _sz]),
    "sg_scale_dev": (ctypes.c_int, [_vp, _vp, _sz, sg_fe]),
    "sg_mul_pow_dev": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _sz, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_uint64, ctypes.c_uint64]),
    "sg_transpose_dev": (ctypes.c_int, [_vp, _vp, _vp, _sz, _sz, _sz]),
    "sg_merkle_forest_dev": (ctypes.c_int, [_vp, _vp, _sz, _sz, _P(_vp)]),
    "sg_forest_roots_dev": (ctypes.c_int, [_vp, _vp, _vp]),
    "sg_forest_open": (ctypes.c_int, [_vp, _vp, _sz, _sz, _vp, _P(_sz)]),
    "sg_forest_free": (None, [_vp, _vp]),
    "sg_merkle_top_dev": (ctypes.c_int, [_vp, _vp, _sz, _P(_vp)]),
    "sg_fri_fold_runs_dev": (ctypes.c_int, [_vp, sg_fe, sg_fe, sg_fe, _vp, _sz, _sz, _sz, _sz, _sz, _vp]),
    # multi-GPU communicator (RCCL or a host-staged transport)
    "sg_dist_unique_id": (ctypes.c_int, [_vp]),
    "sg_dist_create": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _P(_vp)]),
    "sg_dist_create_transport": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _P(sg_dist_transport), _P(_vp)]),
    "sg_dist_destroy": (None, [_vp]),
    "sg_dist_set_timeout": (ctypes.c_int, [_vp, ctypes.c_double]),
    "sg_dist_poisoned": (ctypes.c_int, [_vp]),
    "sg_dist_counters": (ctypes.c_int, [_vp, _P(ctypes.c_uint64), _P(ctypes.c_uint64), _P(ctypes.c_uint64)]),
    "sg_dist_set_fri_tail": (ctypes.c_int, [_vp, ctypes.c_int]),
    "sg_dist_plan": (ctypes.c_int, [_sz, ctypes.c_int, _P(_sz), _P(_sz)]),
    "sg_dist_ntt": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _sz, _vp]),
    "sg_dist_intt": (ctypes.c_int, [_vp, sg_fe, _vp, _sz, _vp]),
    "sg_dist_coset_evaluate": (ctypes.c_int, [_vp, sg_fe, _sz, sg_fe, _vp, _sz, _vp]),
    "sg_dist_merkle_root": (ctypes.c_int, [_vp, _vp, _sz, _vp]),
    "sg_dist_fri_commit": (ctypes.c_int, [_vp, _P(sg_fri), _vp, _sz, _P(sg_proof_stream)]),
    "sg_dist_fri_prove": (ctypes.c_int, [_vp, _P(sg_fri), _vp, _sz, _P(sg_proof_stream), _P(_sz)]),
    # polynomial algebra (fft/ntt_arithmetics.rs)
    "sg_poly_create": (ctypes.c_int, [_vp, _vp, _sz, _P(_vp)]),
    "sg_poly_create_dev": (ctypes.c_int, [_vp, _vp, _sz, _P(_vp)]),
    "sg_poly_len": (_sz, [_vp]),
    "sg_poly_data_dev": (_vp, [_vp]),
    "sg_poly_read": (ctypes.c_int, [_vp, _vp, _vp]),
    "sg_poly_degree": (ctypes.c_int, [_vp, _vp, _P(ctypes.c_int64)]),
    "sg_poly_free": (None, [_vp]),
    "sg_fast_multiply": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, _vp, _vp, _P(_vp)]),
    "sg_fast_coset_divide": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, sg_fe, _vp, _vp, _P(_vp)]),
    "sg_fast_zerofier": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, _vp, _sz, _P(_vp)]),
    "sg_fast_interpolate_domain": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, _vp, _vp, _sz, _P(_vp)]),
    "sg_fast_zerofier_geometric": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, _sz, _P(_vp)]),
    "sg_fast_interpolate_geometric_dev": (ctypes.c_int, [_vp, sg_fe, ctypes.c_uint64, _vp, _sz, _P(_vp)]),
    # multivariate polynomials (m_polynomial.rs)
    "sg_mpoly_create": (ctypes.c_int, [_vp, _sz, _sz, _vp, _vp, _P(_vp)]),
    "sg_mpoly_constant": (ctypes.c_int, [_vp, sg_fe, _P(_vp)]),
    "sg_mpoly_variable": (ctypes.c_int, [_vp, _sz, _sz, _P(_vp)]),
    "sg_mpoly_lift": (ctypes.c_int, [_vp, _vp, _sz, _sz, _P(_vp)]),
    "sg_mpoly_lift_poly": (ctypes.c_int, [_vp, _vp, _sz, _P(_vp)]),
    "sg_mpoly_neg": (ctypes.c_int, [_vp, _vp, _P(_vp)]),
    "sg_mpoly_add": (ctypes.c_int, [_vp, _vp, _vp, _P(_vp)]),
    "sg_mpoly_sub": (ctypes.c_int, [_vp, _vp, _vp, _P(_vp)]),
    "sg_mpoly_mul": (ctypes.c_int, [_vp, _vp, _vp, _P(_vp)]),
    "sg_mpoly_pow": (ctypes.c_int, [_vp, _vp, sg_fe, _P(_vp)]),
    "sg_mpoly_is_zero": (ctypes.c_int, [_vp]),
    "sg_mpoly_evaluate": (ctypes.c_int, [_vp, _vp, _vp, _sz, _fep]),
    "sg_mpoly_shape": (ctypes.c_int, [_vp, _P(_sz), _P(_sz), _P(_sz)]),
    "sg_mpoly_export": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "sg_mpoly_free": (None, [_vp]),
    # Rescue-Prime (rescue_prime/rescue_prime.rs)
    "sg_rescue_create": (ctypes.c_int, [_vp, _sz, _sz, _sz, _sz, _P(_vp)]),
    "sg_rescue_free": (None, [_vp]),
    "sg_rescue_info": (ctypes.c_int, [_vp, _fep, _fep, _vp, _vp, _vp]),
    "sg_rescue_hash": (ctypes.c_int, [_vp, _vp, sg_fe, _fep]),
    "sg_rescue_trace": (ctypes.c_int, [_vp, _vp, sg_fe, _vp]),
    "sg_rescue_transition_constraints": (ctypes.c_int, [_vp, _vp, sg_fe, ctypes.c_uint64, _P(_vp)]),
    "sg_rescue_boundary_constraints": (ctypes.c_int, [_vp, sg_fe, _vp]),
    # STARK (stark/stark.rs)
    "sg_stark_create": (ctypes.c_int, [_vp, _sz, _sz, _sz, _sz, _sz, _sz, _P(_vp)]),
    "sg_stark_free": (None, [_vp]),
    "sg_stark_params": (ctypes.c_int, [_vp, _fep, _P(ctypes.c_uint64), _P(sg_fri), _P(_sz)]),
    "sg_stark_max_degree": (ctypes.c_int, [_vp, _vp, _vp, _sz, _P(ctypes.c_uint64)]),
    "sg_stark_degree_bounds": (ctypes.c_int, [_vp, _vp, _vp, _sz, _vp]),
    "sg_stark_prove": (ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp, _vp, _sz,
                                      _P(sg_proof_stream)]),
    "sg_stark_prove_dev": (ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp, _vp, _sz,
                                          _P(sg_proof_stream)]),
    "sg_dist_stark_prove": (ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp, _vp, _sz,
                                           _P(sg_proof_stream)]),
    "sg_dist_stark_prove_dev": (ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp, _vp, _sz,
                                               _P(sg_proof_stream)]),
}

_lib = None


def _prefer_torch_runtime():
    """Load PyTorch's HIP runtime before libstarkgpu's when torch is importable.

    torch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1 with the same
    sonames as /opt/rocm's; whichever is loaded first serves the whole process.
    torch only initializes on its own copy, so in a Python process that may
    also use torch (tests, bench) torch must be loaded first.  Processes that
    never import torch (e.g. a Rust binary) use /opt/rocm's runtime.
    """
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib():
    """Load libstarkgpu.so once (raises if it was not built)."""
    global _lib
    if _lib is None:
        _prefer_torch_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C zk-stark-tutor_amd` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            try:
                fn = getattr(l, name)
            except AttributeError:
                # an older build loaded through SG_LIB_PATH for a same-box A/B (tools/ab.sh) may lack
                # newer entry points; calling one raises.  The product library must export them all.
                if "SG_LIB_PATH" in os.environ:
                    continue
                raise
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib
