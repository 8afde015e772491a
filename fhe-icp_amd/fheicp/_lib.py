"""ctypes binding of libfheicp.so (include/fhe_icp.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no fallback: if the shared object is missing or fails to load, every
entry point raises, so a GPU run can never silently degrade to a CPU path.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import os

# FHEICP_LIB selects another build (A/B runs: tools/build_variant.sh); the
# default is the in-tree product library
LIB_PATH = Path(os.environ.get("FHEICP_LIB") or Path(__file__).resolve().parent / "libfheicp.so").resolve()

FHE_OK = 0
ERRORS = {-1: "FHE_E_ARG", -2: "FHE_E_DEVICE", -3: "FHE_E_STATE", -4: "FHE_E_NOMEM"}

PARAM_FIELDS = ("n", "k", "N", "pbs_base_log", "pbs_level", "ks_base_log", "ks_level",
                "lwe_noise_bits", "glwe_noise_bits", "msg_bits", "sign_digit_bits",
                "pbs_fast_base_log", "pbs_fast_level", "pbs_fast2_base_log", "pbs_fast2_level",
                "pbs_fast_group", "pbs_fast2_group", "pbs_mid_base_log", "pbs_mid_level",
                "pbs_mid2_base_log", "pbs_mid2_level", "pbs_mid_group", "pbs_mid2_group",
                "pbs_mid0_base_log", "pbs_mid0_level", "pbs_mid0_group")
# fields a caller may leave out (0 = auto / none)
OPTIONAL_FIELDS = PARAM_FIELDS[PARAM_FIELDS.index("sign_digit_bits"):]


class FheParams(C.Structure):
    # struct_size first (= sizeof(fhe_params), checked by the library:
    # include/fhe_icp.h), then the scheme parameters
    _fields_ = [("struct_size", C.c_int32)] + [(f, C.c_int32) for f in PARAM_FIELDS]


# (name, restype, argtypes) for every symbol declared in include/fhe_icp.h
_vp = C.c_void_p
_i64 = C.c_int64
_u64 = C.c_uint64
_i32 = C.c_int32
_P = C.POINTER(FheParams)
_CTXP = C.c_void_p
SIGNATURES = [
    ("fhe_ctx_create", C.c_int, [_P, C.c_int, C.POINTER(C.c_void_p)]),
    ("fhe_ctx_destroy", None, [_CTXP]),
    ("fhe_last_error", C.c_char_p, [_CTXP]),
    ("fhe_get_params", C.c_int, [_CTXP, _P]),
    ("fhe_set_msg_bits", C.c_int, [_CTXP, _i32]),
    ("fhe_bsk_words", C.c_size_t, [_P]),
    ("fhe_fast_bsk_words", C.c_size_t, [_P, _i32]),
    ("fhe_ksk_words", C.c_size_t, [_P]),
    ("fhe_big_lwe_words", C.c_size_t, [_P]),
    ("fhe_small_lwe_words", C.c_size_t, [_P]),
    ("fhe_keygen", C.c_int, [_CTXP, _u64, _vp]),
    ("fhe_keygen_key", C.c_int, [_CTXP, C.POINTER(C.c_uint32), _vp]),
    ("fhe_export_keys", C.c_int, [_CTXP, _vp, _vp, _vp, _vp]),
    ("fhe_import_keys", C.c_int, [_CTXP, _vp, _vp, _vp, _vp]),
    ("fhe_export_fast_bsk", C.c_int, [_CTXP, _i32, _vp]),
    ("fhe_encrypt_batch", C.c_int, [_CTXP, _vp, _i64, _u64, _u64, _vp, _vp]),
    ("fhe_encrypt_batch_key", C.c_int, [_CTXP, _vp, _i64, _vp, _u64, _vp, _vp]),
    ("fhe_decrypt_batch", C.c_int, [_CTXP, _vp, _i64, _vp, _vp]),
    ("fhe_decrypt_bits_batch", C.c_int, [_CTXP, _vp, _i64, _vp, _vp]),
    ("fhe_phase_batch", C.c_int, [_CTXP, _vp, _i64, _vp, _vp]),
    ("fhe_linear_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _i64, _vp, _vp]),
    ("fhe_encrypt_linear_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _u64, _u64, _vp, _i64, _vp, _vp]),
    ("fhe_encrypt_linear_batch_key", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _u64, _vp, _i64, _vp, _vp]),
    ("fhe_encrypt_packed_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _u64, _u64, _vp, _vp]),
    ("fhe_encrypt_packed_batch_key", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _u64, _vp, _vp]),
    ("fhe_linear_packed_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _i64, _vp, _vp]),
    ("fhe_keyswitch_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _u64, _vp, _vp]),
    ("fhe_pbs_batch", C.c_int, [_CTXP, _vp, _i64, _u64, _vp, _vp]),
    ("fhe_pbs_gadget_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _u64, _vp, _vp]),
    ("fhe_bit_extract_batch", C.c_int, [_CTXP, _vp, _i64, _vp, _vp, _vp]),
    ("fhe_sign_batch", C.c_int, [_CTXP, _vp, _i64, _vp, _vp]),
    ("fhe_sign_digit_bits", C.c_int, [_P]),
    ("fhe_sign_pbs_count", C.c_int, [_P]),
    ("fhe_sign_precise_rounds", C.c_int, [_P]),
    ("fhe_sign_plan", C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("fhe_sign_schedule", C.c_int, [_P, C.POINTER(C.c_int32), _i32]),
    ("fhe_sign_trace_batch", C.c_int, [_CTXP, _vp, _i64, C.POINTER(C.c_int32), _i32, _vp, _vp, _vp]),
    ("fhe_pbs_lut_batch", C.c_int, [_CTXP, _vp, _i64, _u64, _u64, _i32, _vp, _vp]),
    ("fhe_pbs_table_batch", C.c_int, [_CTXP, _vp, _i64, _vp, _i32, _vp, _vp]),
    ("fhe_pbs_table_gadget_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _i32, _vp, _vp]),
    ("fhe_pbs_table_gadget", C.c_int, [_P]),
    ("fhe_threshold_batch", C.c_int, [_CTXP, _vp, _i64, _i64, _vp, _vp]),
    ("fhe_compare_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _i64, _i64, _u64, _u64, _vp, _vp, _vp]),
    ("fhe_compare_batch_key", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _u64, _vp, _vp, _vp]),
    ("fhe_score_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _i64, _i64, _u64, _u64, _vp, _vp]),
    ("fhe_score_batch_key", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _u64, _vp, _vp]),
    ("fhe_encrypt_seeded_batch", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    ("fhe_expand_seeded_batch", C.c_int, [_CTXP, _vp, _vp, _i64, _i32, _vp, _vp, _vp]),
    ("fhe_linear_seeded_batch", C.c_int, [_CTXP, _vp, _vp, _i64, _i32, _vp, _vp, _i64, _vp, _vp]),
    ("fhe_compare_seeded_batch", C.c_int, [_CTXP, _vp, _vp, _i64, _i32, _vp, _vp, _i64, _i64, _vp, _vp, _vp]),
    ("fhe_key_from_seed", None, [_u64, _vp]),
    ("fhe_quantize_pairs", C.c_int, [_CTXP, _vp, _i32, _vp, _i32, _i64, _i32, C.c_double, _i64, _i64, _i64, _vp, _vp]),
    ("fhe_dequantize", C.c_int, [_CTXP, _vp, _i64, C.c_double, _vp, _vp]),
    ("fhe_pca_transform", C.c_int, [_CTXP, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]),
    ("fhe_topk", C.c_int, [_CTXP, _vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp]),
    ("fhe_dev_alloc", C.c_int, [_CTXP, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("fhe_dev_free", C.c_int, [_CTXP, _vp]),
    ("fhe_memcpy_h2d", C.c_int, [_CTXP, _vp, _vp, C.c_size_t, _vp]),
    ("fhe_memcpy_d2h", C.c_int, [_CTXP, _vp, _vp, C.c_size_t, _vp]),
    ("fhe_stream_sync", C.c_int, [_CTXP, _vp]),
    ("fhe_debug_v4_stamps", C.c_int, [_CTXP, _vp]),
    ("fhe_debug_el_stamps", C.c_int, [_CTXP, _vp]),
    ("fhe_profile_enable", C.c_int, [_CTXP, C.c_int]),
    ("fhe_profile_read", C.c_int, [_CTXP, C.c_char_p, C.POINTER(C.c_double), C.POINTER(_i64), C.POINTER(_i64)]),
    ("fhe_profile_kernel_name", C.c_int, [_CTXP, C.c_char_p, C.c_char_p, C.c_size_t]),
    ("fhe_build_info", C.c_char_p, []),
    # include/fhe_bert.h: the embedding stage's encoder (fheicp.bert)
    ("fhe_bert_create", C.c_int, [_vp, C.c_int, C.POINTER(C.c_void_p)]),
    ("fhe_bert_destroy", None, [_vp]),
    ("fhe_bert_last_error", C.c_char_p, [_vp]),
    ("fhe_bert_set_precision", C.c_int, [_vp, _i32]),
    ("fhe_bert_get_precision", C.c_int, [_vp]),
    ("fhe_bert_set_tensor", C.c_int, [_vp, _i32, _i32, _vp, _i64]),
    ("fhe_bert_ready", C.c_int, [_vp]),
    ("fhe_bert_forward", C.c_int, [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    ("fhe_bert_profile_enable", C.c_int, [_vp, C.c_int]),
    ("fhe_bert_profile_read", C.c_int, [_vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(_i64),
                                        C.POINTER(C.c_double)]),
]

_lib = None


class FheError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libfheicp.so (raises FheError if it is absent or broken)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise FheError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
        try:
            L = C.CDLL(str(LIB_PATH))
        except OSError as e:  # pragma: no cover - depends on the machine
            raise FheError(f"cannot load {LIB_PATH}: {e}") from e
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def ab_build() -> bool:
    """True for an A/B build (fhe_build_info: extra kernel shapes, timing kernels)."""
    return b"ab=1" in (lib().fhe_build_info() or b"")


def check(rc: int, ctx=None) -> None:
    if rc != FHE_OK:
        msg = lib().fhe_last_error(ctx)
        msg = msg.decode() if msg else ""
        raise FheError(f"{ERRORS.get(rc, rc)}: {msg}")


def params_struct(d: dict) -> FheParams:
    return FheParams(struct_size=C.sizeof(FheParams),
                     **{f: int(d.get(f, 0) if f in OPTIONAL_FIELDS else d[f]) for f in PARAM_FIELDS})
