"""ctypes binding of include/handel_gpu.h (libhandel_gpu.so, built in-tree).

There is no CPU fallback: if the HIP library is missing or fails to load,
every entry point raises. The oracle under oracle/ is never imported here.
"""

from __future__ import annotations

import ctypes
import os
import threading

from . import build as _build

_lock = threading.Lock()
_lib = None

# hg_code values (include/handel_gpu.h)
HG_OK = 0
HG_ERR_SIG_INVALID = 1
HG_ERR_HASH_EOF = 2
HG_ERR_LEVEL = 3
HG_ERR_PK_UNMARSHAL = 4
HG_ERR_SIG_UNMARSHAL = 5
HG_ERR_EMPTY_AGG = 6
HG_ERR_CF_EXCEEDS = 7
HG_ERR_CF_MALFORMED = 8
HG_ERR_CF_SHORT = 9
HG_ERR_SIG_CF_EXCEEDS = 10
HG_ERR_SIG_CF_MALFORMED = 11
HG_ERR_SIG_CF_SHORT = 12
HG_ERR_MULTI_SIZES = 13
HG_ERR_PKT_ORIGIN = 20
HG_ERR_PKT_LEVEL = 21
HG_ERR_PKT_EOF = 22
HG_ERR_PKT_UNEXPECTED_EOF = 23
HG_ERR_PKT_BITSET_SHORT = 24
HG_ERR_PKT_TYPE_MISMATCH = 25
HG_ERR_PKT_BITSET_SIZE = 26
HG_ERR_PKT_NO_SIG = 27
HG_ERR_PKT_ID_RANGE = 28
HG_PKT_NO_IND = 29
HG_PKT_HAS_IND = 1
HG_ERR_ARG = 100
HG_ERR_DEVICE = 101

HG_FLAVOR_GO = 0
HG_FLAVOR_CF = 1

HG_PHASE_VERIFY = 0
HG_PHASE_AGGREGATE = 1
HG_PHASE_SUBMIT = 2

# every symbol include/handel_gpu.h declares: name -> (restype, argtypes)
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_I = ctypes.c_int
SIGNATURES = {
    "hg_version": (_I, []),
    "hg_context_simds": (_I, [_P]),
    "hg_context_flavor": (_I, [_P]),
    "hg_create": (_I, [_I, _I, ctypes.POINTER(_P)]),
    "hg_destroy": (None, [_P]),
    "hg_last_error": (ctypes.c_char_p, [_P]),
    "hg_code_string": (ctypes.c_char_p, [_I, _I]),
    "hg_processing_error_string": (ctypes.c_char_p, [_I, _I]),
    "hg_registry_load": (_I, [_P, _P, _SZ, _P]),
    "hg_registry_size": (_SZ, [_P]),
    "hg_prepare_aggregate": (_I, [_P]),
    "hg_aggregate_tables": (_I, [_P]),
    "hg_prepare_aggregate_msg": (_I, [_P, _P, _SZ]),
    "hg_set_aggregate_level": (_I, [_P, _I]),
    "hg_set_table_budget": (_I, [_P, _SZ]),
    "hg_set_fold_overlap": (_I, [_P, _I]),
    "hg_set_verify_split": (_I, [_P, _I]),
    "hg_registry_non_g2": (_SZ, [_P]),
    "hg_set_message": (_I, [_P, _P, _SZ]),
    "hg_verify_batch": (_I, [_P, _P, _P, _SZ, _P]),
    "hg_verify_batch_msg": (_I, [_P, _P, _SZ, _P, _P, _SZ, _P]),
    "hg_verify_batch_device": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "hg_pack_verdicts_device": (_I, [_P, _P, _SZ, _P, _P]),
    "hg_verify_aggregate": (_I, [_P, _P, _SZ, _P, _SZ, _P, _P, _P]),
    "hg_verify_aggregate_device": (_I, [_P, _P, _SZ, _P, _P, _P, _P, _P]),
    "hg_verify_aggregate_device_bits": (_I, [_P, _P, _SZ, _P, _P, _P, _P, _P]),
    "hg_verify_aggregate_msg": (_I, [_P, _P, _SZ, _P, _SZ, _P, _SZ, _P, _P, _P]),
    "hg_verify_multisig": (_I, [_P, _P, _P, _SZ, _P, _SZ, _P, _P]),
    "hg_aggregate_pk": (_I, [_P, _P, _SZ, _P, _SZ, _P, _P]),
    "hg_combine_g1": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "hg_combine_g2": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "hg_pair": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "hg_keygen": (_I, [_P, _P, _SZ, _P]),
    "hg_sign": (_I, [_P, _P, _SZ, _P]),
    "hg_sign_msg": (_I, [_P, _P, _SZ, _P, _SZ, _P]),
    "hg_debug_fp_mul": (_I, [_P, _P, _P, _SZ, _P]),
    "hg_diag_read": (_I, [_P, _P, _SZ]),
    "hg_sig_pairing_device": (_I, [_P, _P, _SZ, _P, _I, _P]),
    "hg_debug_fp12": (_I, [_P, _I, _P, _P, _SZ, _P]),
    "hg_timing_enable": (_I, [_P, _I]),
    "hg_timing_read": (_I, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I)]),
    "hg_timing_read_phase": (_I, [_P, _I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I)]),
    "hg_sync": (_I, [_P]),
    "hg_context_bytes": (_SZ, [_P]),
    "hg_packet_stride_words": (_SZ, [_P]),
    "hg_parse_packets": (_I, [_P, _P, _SZ, _P, _SZ, _SZ, _P, _P, _P, _P]),
    "hg_parse_packets_device": (_I, [_P, _P, _SZ, _P, _SZ, _SZ, _P, _P, _P, _P, _P]),
    "hg_packet_error": (_I, [_P, _I, _P, ctypes.c_char_p, _SZ]),
    "hg_batcher_create": (_I, [_P, _SZ, ctypes.c_uint, ctypes.POINTER(_P)]),
    "hg_batcher_destroy": (None, [_P]),
    "hg_batcher_submit": (_I, [_P, _P, _SZ, _P, _P, _P, ctypes.POINTER(_P)]),
    "hg_batcher_wait": (_I, [_P, _P, _P]),
    "hg_batcher_verify_aggregate": (_I, [_P, _P, _SZ, _P, _P, _P, _P]),
    "hg_batcher_stats": (_I, [_P, _P, _P]),
    "hg_prepare_aggregate_level": (_I, [_P, _I]),
    "hg_lane_create": (_I, [_P, _SZ, _SZ, _I, ctypes.POINTER(_P)]),
    "hg_lane_destroy": (None, [_P]),
    "hg_lane_stage": (_I, [_P, _SZ, _SZ, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "hg_lane_submit": (_I, [_P]),
    "hg_lane_query": (_I, [_P]),
    "hg_lane_wait": (_I, [_P]),
    "hg_lane_codes": (ctypes.POINTER(ctypes.c_int32), [_P]),
    "hg_lane_submit_device": (_I, [_P, _P, _SZ, _P, _P, _P, _P, _P]),
    "hg_lane_set_pairing_padding": (_I, [_P, _I]),
    "hg_lane_set_latency_form": (_I, [_P, _I]),
    "hg_lane_stream": (_P, [_P]),
    "hg_service_config_init": (None, [_P]),
    "hg_service_create": (_I, [_P, ctypes.c_char_p, _P, ctypes.POINTER(_P)]),
    "hg_service_create_echo": (_I, [ctypes.c_char_p, _P, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_P)]),
    "hg_service_destroy": (None, [_P]),
    "hg_service_stats": (_I, [_P, _P, _P, _P]),
}


class HandelGPUError(RuntimeError):
    pass


def load(build_if_missing: bool = True):
    """Loads (building first if needed) the HIP library; raises on failure."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # HG_LIB selects the diagnostic build (tools/diag.py); default: the product library
        path = os.environ.get("HG_LIB") or _build.LIB
        if not os.path.exists(path):
            if not build_if_missing:
                raise HandelGPUError(f"HIP library not built: {path}")
            _build.build_library()
        try:
            L = ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on the box
            raise HandelGPUError(f"cannot load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)  # AttributeError = missing export: fail loudly
            fn.restype = res
            fn.argtypes = args
        _lib = L
        return L
