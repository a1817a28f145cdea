"""ctypes binding for oracle/_build/libbn256_ref.so — TEST INFRASTRUCTURE ONLY.

The C restatement of the reference path (see bn256_ref.c). Used by tests/ as
a fast checker at full batch sizes and by bench.py as the cpu_baseline
("port", timed on the host cores). Never imported by handel_amd.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libbn256_ref.so")

# result codes shared with bn256_ref.c
RC_OK, RC_SIG_INVALID, RC_HASH_EOF, RC_LEVEL, RC_PK_UNMARSHAL, RC_SIG_UNMARSHAL, RC_EMPTY_AGG = range(7)

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.c_void_p
        L.ref_init.restype = None
        L.ref_pair.argtypes = [u8p, u8p, u8p]
        L.ref_set_rehash.restype = None
        L.ref_set_rehash.argtypes = [ctypes.c_int]
        L.ref_verify_batch.restype = ctypes.c_long
        L.ref_verify_batch.argtypes = [u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_size_t, u8p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ref_verify_aggregate.restype = ctypes.c_long
        L.ref_verify_aggregate.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_size_t,
                                           u8p, u8p, u8p, u8p, u8p, u8p, u8p, u8p, ctypes.c_int,
                                           ctypes.c_int]
        L.ref_g2_scalar_base.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.ref_sign.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p]
        L.ref_g1_add.argtypes = [u8p, u8p, u8p]
        L.ref_g2_add.argtypes = [u8p, u8p, u8p]
        L.ref_decode_g2.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int]
        L.ref_decode_g1.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int]
        L.ref_hash_scalar.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.ref_init()
        _lib = L
    return _lib


def _buf(b: bytes):
    return ctypes.create_string_buffer(b, len(b)) if b else ctypes.create_string_buffer(1)


def pair(g1: bytes, g2: bytes) -> bytes:
    out = ctypes.create_string_buffer(384)
    rc = lib().ref_pair(_buf(g1), _buf(g2), out)
    if rc:
        raise ValueError(f"decode error {rc}")
    return out.raw


def set_rehash(on: bool) -> None:
    """Hash the message per check (the reference's VerifySignature does) instead of once per batch."""
    lib().ref_set_rehash(1 if on else 0)


def verify_batch(msg: bytes, pks: bytes, sigs: bytes, nthreads: int = 1, flavor: int = 0,
                 fast: bool = False) -> np.ndarray:
    n = len(sigs) // 64
    codes = np.zeros(n, dtype=np.int32)
    lib().ref_verify_batch(_buf(msg), len(msg), _buf(pks), _buf(sigs), n, codes.ctypes.data,
                           nthreads, flavor, int(fast))
    return codes


def verify_aggregate(msg: bytes, registry: bytes, off, bitlen, level_len, words, woff, sigs: bytes,
                     nthreads: int = 1, fast: bool = True, want_agg: bool = False):
    off = np.ascontiguousarray(off, dtype=np.uint32)
    bitlen = np.ascontiguousarray(bitlen, dtype=np.uint32)
    level_len = np.ascontiguousarray(level_len, dtype=np.uint32)
    words = np.ascontiguousarray(words, dtype=np.uint64)
    woff = np.ascontiguousarray(woff, dtype=np.uint64)
    n = len(off)
    codes = np.zeros(n, dtype=np.int32)
    agg = np.zeros(n * 128, dtype=np.uint8) if want_agg else None
    lib().ref_verify_aggregate(_buf(msg), len(msg), _buf(registry), len(registry) // 128, n,
                               off.ctypes.data, bitlen.ctypes.data, level_len.ctypes.data,
                               words.ctypes.data if len(words) else None, woff.ctypes.data,
                               _buf(sigs), codes.ctypes.data,
                               agg.ctypes.data if want_agg else None, nthreads, int(fast))
    return (codes, agg.tobytes()) if want_agg else codes


def g2_scalar_base(scalars_be: bytes) -> bytes:
    n = len(scalars_be) // 32
    out = ctypes.create_string_buffer(128 * n)
    lib().ref_g2_scalar_base(_buf(scalars_be), n, out)
    return out.raw


def sign(msg: bytes, scalars_be: bytes) -> bytes:
    n = len(scalars_be) // 32
    out = ctypes.create_string_buffer(64 * n)
    rc = lib().ref_sign(_buf(msg), len(msg), _buf(scalars_be), n, out)
    if rc:
        raise ValueError("EOF")
    return out.raw


def g1_add(a: bytes, b: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    rc = lib().ref_g1_add(_buf(a), _buf(b), out)
    if rc:
        raise ValueError(rc)
    return out.raw


def g2_add(a: bytes, b: bytes) -> bytes:
    out = ctypes.create_string_buffer(128)
    rc = lib().ref_g2_add(_buf(a), _buf(b), out)
    if rc:
        raise ValueError(rc)
    return out.raw
