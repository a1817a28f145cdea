"""The verifier service: one GPU-owning process, many client processes.

`Service` runs hg_service_* (include/handel_gpu.h) on an `Engine`: the
engine's context, registry and GT tables serve every client. `Client` binds
libhandel_client.so (include/handel_client.h), which has no GPU or HIP
dependency, so a process that runs Handel instances (simul/node/main.go:
63-131) submits each instance's verifySignature (processing.go:342-368)
through shared memory instead of opening a GPU context. `EchoService` serves
the same protocol with a CPU stand-in for the GPU (protocol tests only: its
codes are a checksum rule, not verification).
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import List, Optional, Tuple

import numpy as np

from . import _lib
from . import build as _build
from ._lib import HandelGPUError
from .engine import REQ_DTYPE, Engine, _ptr, _u8


class ServiceConfig(ctypes.Structure):
    """hg_service_config."""
    _fields_ = [("slots", ctypes.c_uint32), ("slot_bits", ctypes.c_uint32), ("channels", ctypes.c_uint32),
                ("lanes", ctypes.c_uint32), ("max_batch", ctypes.c_uint32), ("max_wait_us", ctypes.c_uint32),
                ("quiet_us", ctypes.c_uint32),
                ("prepare", ctypes.c_int32), ("overlap", ctypes.c_int32), ("follow", ctypes.c_int32)]


def _config(L, **kw) -> ServiceConfig:
    cfg = ServiceConfig()
    L.hg_service_config_init(ctypes.byref(cfg))
    for k, v in kw.items():
        if v is not None:
            setattr(cfg, k, int(v))
    return cfg


class _ServiceBase:
    L = None
    h = None

    def stats(self) -> Tuple[int, int, int]:
        """(batches launched, requests verified, most batches in flight at once)."""
        b, r, f = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self.L.hg_service_stats(self.h, ctypes.byref(b), ctypes.byref(r), ctypes.byref(f))
        return b.value, r.value, f.value

    def close(self):
        if getattr(self, "h", None):
            self.L.hg_service_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Service(_ServiceBase):
    """hg_service_create over an engine with a loaded registry. The engine
    must outlive the service and is not used by others while it runs."""

    def __init__(self, engine: Engine, name: str, **cfg):
        self.engine = engine
        self.L = engine.L
        self.name = name
        c = _config(self.L, **cfg)
        h = ctypes.c_void_p()
        rc = self.L.hg_service_create(engine.ctx, name.encode(), ctypes.byref(c), ctypes.byref(h))
        if rc != 0:
            raise HandelGPUError(f"hg_service_create({name}): code {rc}: {self.L.hg_last_error(engine.ctx)}")
        self.h = h


class EchoService(_ServiceBase):
    """hg_service_create_echo: the service protocol with a CPU stand-in for
    the GPU (no GPU calls). A request's code: HG_ERR_LEVEL (level check), 77
    (bitset words do not match sig[1..8]), HG_ERR_SIG_INVALID (sig[0] == 1),
    else HG_OK; every batch completes delay_us after launch."""

    def __init__(self, name: str, nreg: int, delay_us: int = 0, **cfg):
        self.L = _lib.load()
        self.name = name
        c = _config(self.L, **cfg)
        h = ctypes.c_void_p()
        rc = self.L.hg_service_create_echo(name.encode(), ctypes.byref(c), int(nreg), int(delay_us), ctypes.byref(h))
        if rc != 0:
            raise HandelGPUError(f"hg_service_create_echo({name}): code {rc}")
        self.h = h


def echo_signature(words, tampered: bool = False) -> bytes:
    """The 64-byte 'signature' EchoService accepts for these bitset words."""
    x = 0
    for w in np.asarray(words, dtype=np.uint64):
        x ^= int(w)
    return bytes([1 if tampered else 0]) + x.to_bytes(8, "little") + bytes(55)


# ---------------------------------------------------------------- client side
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
CLIENT_SIGNATURES = {
    "hg_client_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_P)]),
    "hg_client_close": (None, [_P]),
    "hg_client_submit": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _P, ctypes.POINTER(ctypes.c_uint64)]),
    "hg_client_wait": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int32)]),
    "hg_client_wait_any": (ctypes.c_int, [_P, _P, _P, _SZ, ctypes.c_long]),
    "hg_client_verify_aggregate": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _P, ctypes.POINTER(ctypes.c_int32)]),
    "hg_client_stats": (ctypes.c_int, [_P, _P, _P]),
    "hg_client_slot_bits": (ctypes.c_uint32, [_P]),
    "hg_client_flavor": (ctypes.c_int, [_P]),
    "hg_client_code_string": (ctypes.c_char_p, [_P, ctypes.c_int]),
    "hg_client_processing_error_string": (ctypes.c_char_p, [_P, ctypes.c_int]),
}
_client_lock = threading.Lock()
_client_lib = None


def load_client():
    """libhandel_client.so (built in-tree with the host compiler if missing)."""
    global _client_lib
    with _client_lock:
        if _client_lib is None:
            path = _build.CLIENT_LIB
            if not os.path.exists(path):
                _build.build_client(verbose=False)
            L = ctypes.CDLL(path)
            for name, (res, args) in CLIENT_SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _client_lib = L
        return _client_lib


class Client:
    """One handle on a service region (hg_client_open): a completion channel."""

    def __init__(self, name: str):
        self.L = load_client()
        h = ctypes.c_void_p()
        rc = self.L.hg_client_open(name.encode(), ctypes.byref(h))
        if rc != 0:
            raise HandelGPUError(f"hg_client_open({name}): code {rc}")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.hg_client_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def slot_bits(self) -> int:
        return int(self.L.hg_client_slot_bits(self.h))

    def submit(self, msg: bytes, offset: int, bitlen: int, level_size: int, words, sig: bytes) -> int:
        """Queues one verifySignature (hg_client_submit); returns the ticket."""
        m = _u8(msg)
        req = np.array([(offset, bitlen, level_size, 0)], dtype=REQ_DTYPE)
        w = np.ascontiguousarray(words, dtype=np.uint64)
        if len(w) < (int(bitlen) + 63) // 64:
            raise ValueError(f"{bitlen} bits need {(int(bitlen) + 63) // 64} words, got {len(w)}")
        sg = _u8(sig)
        if len(sg) != 64:
            raise ValueError("signature must be 64 bytes")
        t = ctypes.c_uint64()
        rc = self.L.hg_client_submit(self.h, _ptr(m) if len(m) else None, len(m), _ptr(req),
                                     _ptr(w) if len(w) else None, _ptr(sg), ctypes.byref(t))
        if rc != 0:
            raise HandelGPUError(f"hg_client_submit: code {rc}")
        return t.value

    def wait(self, ticket: int) -> int:
        """The request's hg_code (hg_client_wait)."""
        code = ctypes.c_int32(-1)
        rc = self.L.hg_client_wait(self.h, int(ticket), ctypes.byref(code))
        if rc != 0:
            raise HandelGPUError(f"hg_client_wait: code {rc}")
        return int(code.value)

    def wait_any(self, cap: int = 256, timeout_us: int = -1) -> List[Tuple[int, int]]:
        """Finished (ticket, code) pairs of this handle (hg_client_wait_any)."""
        t = np.zeros(cap, dtype=np.uint64)
        c = np.zeros(cap, dtype=np.int32)
        n = self.L.hg_client_wait_any(self.h, _ptr(t), _ptr(c), cap, int(timeout_us))
        if n < 0:
            raise HandelGPUError(f"hg_client_wait_any: code {-n}")
        return [(int(t[i]), int(c[i])) for i in range(n)]

    def verify(self, msg: bytes, offset: int, bitlen: int, level_size: int, words, sig: bytes) -> int:
        return self.wait(self.submit(msg, offset, bitlen, level_size, words, sig))

    def verify_many(self, msg: bytes, reqs: np.ndarray, words: np.ndarray, sigs: bytes) -> np.ndarray:
        """Submits every request (hg_request rows, words at word_offset), then
        collects all codes in request order."""
        reqs = np.ascontiguousarray(reqs, dtype=REQ_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint64)
        s = _u8(sigs)
        tickets = []
        for i, r in enumerate(reqs):
            nw = (int(r["bitlen"]) + 63) // 64
            wo = int(r["word_offset"])
            tickets.append(self.submit(msg, int(r["offset"]), int(r["bitlen"]), int(r["level_size"]),
                                       words[wo:wo + nw], s[64 * i:64 * i + 64]))
        return np.array([self.wait(t) for t in tickets], dtype=np.int32)

    def stats(self) -> Tuple[int, int]:
        b, r = ctypes.c_uint64(), ctypes.c_uint64()
        self.L.hg_client_stats(self.h, ctypes.byref(b), ctypes.byref(r))
        return b.value, r.value

    @property
    def flavor(self) -> int:
        return int(self.L.hg_client_flavor(self.h))

    def code_string(self, code: int) -> str:
        return self.L.hg_client_code_string(self.h, int(code)).decode()

    def processing_error_string(self, code: int) -> str:
        """processing.go verifySignature's text for a code (None-equivalent "" for HG_OK)."""
        return self.L.hg_client_processing_error_string(self.h, int(code)).decode()


def service_name(tag: Optional[str] = None) -> str:
    """A fresh region name for this process."""
    return f"/hg_{tag or 'svc'}_{os.getpid()}_{threading.get_ident() % 100000}"
