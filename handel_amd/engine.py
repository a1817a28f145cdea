"""Host wrapper around one hg_ctx (include/handel_gpu.h).

`Engine` is the batched replacement for the reference's one-at-a-time crypto
calls: it owns a GPU context, the decoded registry and the
hashed message, and exposes every C-ABI entry point with numpy/bytes
arguments. Device-resident variants take raw device pointers (e.g. from
torch tensors) and a HIP stream handle.
"""

from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import HandelGPUError

FLAVORS = {"go": _lib.HG_FLAVOR_GO, "bn256/go": _lib.HG_FLAVOR_GO,
           "cf": _lib.HG_FLAVOR_CF, "bn256/cf": _lib.HG_FLAVOR_CF, "bn256": _lib.HG_FLAVOR_CF}

REQ_DTYPE = np.dtype([("offset", "<u4"), ("bitlen", "<u4"), ("level_size", "<u4"), ("word_offset", "<u4")])
# hg_packet (include/handel_gpu.h): one received Handel packet, marshals as pool ranges
PACKET_DTYPE = np.dtype([("origin", "<i4"), ("receiver", "<u4"), ("level", "<u4"), ("flags", "<u4"),
                         ("ms_off", "<u4"), ("ms_len", "<u4"), ("ind_off", "<u4"), ("ind_len", "<u4")])


def _ptr(a) -> Optional[int]:
    if a is None:
        return None
    if isinstance(a, (bytes, bytearray)):
        return ctypes.cast(ctypes.c_char_p(bytes(a)), ctypes.c_void_p).value
    return a.ctypes.data


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


class Engine:
    """One verification context on one GPU (hg_create)."""

    def __init__(self, device: int = 0, flavor: str = "go"):
        self.L = _lib.load()
        self.flavor_name = flavor
        self.flavor = FLAVORS[flavor]
        h = ctypes.c_void_p()
        rc = self.L.hg_create(device, self.flavor, ctypes.byref(h))
        if rc != 0:
            raise HandelGPUError(f"hg_create failed: code {rc}")
        self.ctx = h
        self.device = device

    def close(self):
        if getattr(self, "ctx", None):
            self.L.hg_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str, ok=(0,)):
        if rc not in ok:
            err = self.L.hg_last_error(self.ctx)
            raise HandelGPUError(f"{what}: code {rc}: {err.decode() if err else ''}")
        return rc

    def code_string(self, code: int) -> str:
        return self.L.hg_code_string(int(code), self.flavor).decode()

    def processing_error_string(self, code: int) -> str:
        """The text processing.go's verifySignature returns for `code`
        (hg_processing_error_string): VerifySignature errors wrapped "handel: ..."."""
        return self.L.hg_processing_error_string(int(code), self.flavor).decode()

    # ----------------------------------------------------------- setup
    def set_message(self, msg: bytes) -> int:
        """hashedMessage once per message; returns HG_OK or HG_ERR_HASH_EOF."""
        m = _u8(msg)
        return self._check(self.L.hg_set_message(self.ctx, _ptr(m) if len(m) else None, len(m)),
                           "hg_set_message", ok=(0, _lib.HG_ERR_HASH_EOF))

    def prepare_aggregate(self) -> int:
        """Builds the GT tables of aggregate verification for the current
        message and registry now (hg_prepare_aggregate); HG_OK or HG_ERR_HASH_EOF."""
        return self._check(self.L.hg_prepare_aggregate(self.ctx), "hg_prepare_aggregate",
                           ok=(0, _lib.HG_ERR_HASH_EOF))

    def prepare_aggregate_msg(self, msg: bytes) -> int:
        """set_message + prepare_aggregate under one lock hold
        (hg_prepare_aggregate_msg); HG_OK or HG_ERR_HASH_EOF."""
        m = _u8(msg)
        return self._check(self.L.hg_prepare_aggregate_msg(self.ctx, _ptr(m) if len(m) else None, len(m)),
                           "hg_prepare_aggregate_msg", ok=(0, _lib.HG_ERR_HASH_EOF))

    def set_aggregate_level(self, level: int) -> None:
        """Pins the GT table level of aggregate submissions (0..2) or returns
        them to the volume policy (-1) (hg_set_aggregate_level)."""
        self._check(self.L.hg_set_aggregate_level(self.ctx, int(level)), "hg_set_aggregate_level")

    def set_fold_overlap(self, on: bool) -> None:
        """GT fold beside (True) or before (False) the pairing kernel
        (hg_set_fold_overlap); same verdicts."""
        self._check(self.L.hg_set_fold_overlap(self.ctx, int(bool(on))), "hg_set_fold_overlap")

    def set_verify_split(self, on: bool) -> None:
        """Config 2's form (hg_set_verify_split): True = the split form for
        batches in flight on several contexts; same verdicts."""
        self._check(self.L.hg_set_verify_split(self.ctx, int(bool(on))), "hg_set_verify_split")

    def set_table_budget(self, nbytes: int) -> None:
        """Upper bound for this context's GT tables (hg_set_table_budget)."""
        self._check(self.L.hg_set_table_budget(self.ctx, int(nbytes)), "hg_set_table_budget")

    def registry_non_g2(self) -> int:
        """Registry keys on the twist but outside G2 (hg_registry_non_g2)."""
        return int(self.L.hg_registry_non_g2(self.ctx))

    def context_bytes(self) -> int:
        """Device memory the context holds (hg_context_bytes)."""
        return int(self.L.hg_context_bytes(self.ctx))

    def aggregate_tables(self) -> int:
        """Table level aggregate requests run at (hg_aggregate_tables): 0 = G2
        fold, 1 = GT fold over 8-key windows, 2 = over 16-key windows."""
        return int(self.L.hg_aggregate_tables(self.ctx))

    def registry_load(self, pks: bytes) -> np.ndarray:
        a = _u8(pks)
        n = len(a) // 128
        codes = np.zeros(n, dtype=np.int32)
        rc = self.L.hg_registry_load(self.ctx, _ptr(a), n, _ptr(codes))
        self._check(rc, "hg_registry_load", ok=(0, _lib.HG_ERR_PK_UNMARSHAL))
        return codes

    # ----------------------------------------------------------- batch verification
    def verify_batch(self, pks: bytes, sigs: bytes) -> np.ndarray:
        a, b = _u8(pks), _u8(sigs)
        n = len(b) // 64
        if len(a) != 128 * n:
            raise ValueError("pks must hold 128 bytes per signature")
        codes = np.zeros(n, dtype=np.int32)
        self._check(self.L.hg_verify_batch(self.ctx, _ptr(a), _ptr(b), n, _ptr(codes)), "hg_verify_batch")
        return codes

    def verify_batch_msg(self, msg: bytes, pks: bytes, sigs: bytes) -> np.ndarray:
        """PublicKey.VerifySignature(msg, sig) x n, hashing and verifying under
        one lock hold of the context (hg_verify_batch_msg)."""
        m, a, b = _u8(msg), _u8(pks), _u8(sigs)
        n = len(b) // 64
        if len(a) != 128 * n:
            raise ValueError("pks must hold 128 bytes per signature")
        codes = np.zeros(n, dtype=np.int32)
        rc = self.L.hg_verify_batch_msg(self.ctx, _ptr(m) if len(m) else None, len(m), _ptr(a) if n else None,
                                        _ptr(b) if n else None, n, _ptr(codes) if n else None)
        self._check(rc, "hg_verify_batch_msg")
        return codes

    def verify_batch_device(self, d_pks: int, d_sigs: int, n: int, d_codes: int, stream: int = 0):
        self._check(self.L.hg_verify_batch_device(self.ctx, d_pks, d_sigs, n, d_codes, stream or None),
                    "hg_verify_batch_device")

    def pack_verdicts_device(self, d_codes: int, n: int, d_bits: int, stream: int = 0):
        """Device verdict bitset (hg_pack_verdicts_device): ceil(n/8) bytes,
        bit j of byte b = check 8b+j passed."""
        self._check(self.L.hg_pack_verdicts_device(self.ctx, d_codes, n, d_bits, stream or None),
                    "hg_pack_verdicts_device")

    # hg_sig_pairing_device kernels
    SIG_K16_PAD, SIG_K16, SIG_K12_PAD, SIG_K12, SIG_W2 = 0, 1, 2, 3, 4

    def sig_pairing_device(self, d_sigs: int, n: int, d_fe: int, kernel: int, stream: int = 0):
        """FE(Miller(G2Base at -sig)) of n signature marshals into d_fe (n x 480
        bytes) with one chosen pairing kernel (hg_sig_pairing_device): the
        per-kernel roofline and the cross-kernel check."""
        self._check(self.L.hg_sig_pairing_device(self.ctx, d_sigs, n, d_fe, int(kernel), stream or None),
                    "hg_sig_pairing_device")

    def verify_aggregate(self, reqs: np.ndarray, words: np.ndarray, sigs: bytes, want_agg: bool = False):
        reqs = np.ascontiguousarray(reqs, dtype=REQ_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint64)
        s = _u8(sigs)
        n = len(reqs)
        codes = np.zeros(n, dtype=np.int32)
        agg = np.zeros(n * 128, dtype=np.uint8) if want_agg else None
        self._check(self.L.hg_verify_aggregate(self.ctx, _ptr(reqs), n, _ptr(words) if len(words) else None,
                                               len(words), _ptr(s), _ptr(codes), _ptr(agg)),
                    "hg_verify_aggregate")
        return (codes, agg.tobytes()) if want_agg else codes

    # ------------------------------------------------------------ packet intake
    def packet_stride_words(self) -> int:
        """Bitset words per request slot of hg_parse_packets (largest level / 64)."""
        return int(self.L.hg_packet_stride_words(self.ctx))

    def parse_packets(self, pool, pkts: np.ndarray, stride: Optional[int] = None):
        """Handel.NewPacket's parse step for n packets (hg_parse_packets):
        returns (reqs[2n], words, sigs[2n*64], codes[2n]); slot i is packet i's
        multisignature, slot n + i its individual signature."""
        pkts = np.ascontiguousarray(pkts, dtype=PACKET_DTYPE)
        pool = _u8(pool)
        n = len(pkts)
        stride = self.packet_stride_words() if stride is None else int(stride)
        reqs, words, sigs, codes = _parse_outputs(n, stride)
        self._check(self.L.hg_parse_packets(self.ctx, _ptr(pool) if len(pool) else None, len(pool), _ptr(pkts), n,
                                            stride, _ptr(reqs), _ptr(words), _ptr(sigs), _ptr(codes)),
                    "hg_parse_packets")
        return reqs, words, sigs.tobytes(), codes

    def parse_packets_device(self, d_pool: int, pool_len: int, d_pkts: int, n: int, stride: int, d_reqs: int,
                             d_words: int, d_sigs: int, d_codes: int, stream: int = 0) -> None:
        """hg_parse_packets_device on raw device pointers (asynchronous)."""
        self._check(self.L.hg_parse_packets_device(self.ctx, d_pool or None, pool_len, d_pkts, n, stride, d_reqs,
                                                   d_words, d_sigs, d_codes, stream or None),
                    "hg_parse_packets_device")

    def packet_error(self, code: int, pkt) -> str:
        """The reference's text for a packet code (hg_packet_error)."""
        p = np.ascontiguousarray(np.asarray(pkt, dtype=PACKET_DTYPE).reshape(1))
        buf = ctypes.create_string_buffer(256)
        self.L.hg_packet_error(self.ctx, int(code), _ptr(p), buf, 256)
        return buf.value.decode()

    def verify_aggregate_msg(self, msg: bytes, reqs: np.ndarray, words: np.ndarray, sigs: bytes):
        """verify_aggregate with the message given per call: hashing and the
        batch under one lock hold of the context (hg_verify_aggregate_msg)."""
        reqs = np.ascontiguousarray(reqs, dtype=REQ_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint64)
        m, s = _u8(msg), _u8(sigs)
        n = len(reqs)
        codes = np.zeros(n, dtype=np.int32)
        self._check(self.L.hg_verify_aggregate_msg(self.ctx, _ptr(m) if len(m) else None, len(m),
                                                   _ptr(reqs) if n else None, n,
                                                   _ptr(words) if len(words) else None, len(words),
                                                   _ptr(s) if n else None, _ptr(codes) if n else None, None),
                    "hg_verify_aggregate_msg")
        return codes

    def verify_multisig(self, bitlens, word_offsets, words: np.ndarray, sigs: bytes) -> np.ndarray:
        """VerifyMultiSignature (crypto.go:120-137) x n (hg_verify_multisig)."""
        bl = np.ascontiguousarray(bitlens, dtype=np.uint32)
        wo = np.ascontiguousarray(word_offsets, dtype=np.uint32)
        words = np.ascontiguousarray(words, dtype=np.uint64)
        s = _u8(sigs)
        n = len(bl)
        codes = np.zeros(n, dtype=np.int32)
        if n:
            self._check(self.L.hg_verify_multisig(self.ctx, _ptr(bl), _ptr(wo), n, _ptr(words) if len(words) else None,
                                                  len(words), _ptr(s), _ptr(codes)), "hg_verify_multisig")
        return codes

    def verify_aggregate_device(self, d_reqs: int, n: int, d_words: int, d_sigs: int, d_codes: int,
                                d_agg: int = 0, stream: int = 0):
        self._check(self.L.hg_verify_aggregate_device(self.ctx, d_reqs, n, d_words, d_sigs, d_codes,
                                                      d_agg or None, stream or None),
                    "hg_verify_aggregate_device")

    def verify_aggregate_device_bits(self, d_reqs: int, n: int, d_words: int, d_sigs: int, d_codes: int,
                                     d_bits: int, stream: int = 0):
        """verify_aggregate_device + the verdict bitset in one submission."""
        self._check(self.L.hg_verify_aggregate_device_bits(self.ctx, d_reqs, n, d_words, d_sigs, d_codes, d_bits,
                                                           stream or None),
                    "hg_verify_aggregate_device_bits")

    def aggregate_pk(self, reqs: np.ndarray, words: np.ndarray) -> Tuple[bytes, np.ndarray]:
        reqs = np.ascontiguousarray(reqs, dtype=REQ_DTYPE)
        words = np.ascontiguousarray(words, dtype=np.uint64)
        n = len(reqs)
        codes = np.zeros(n, dtype=np.int32)
        out = np.zeros(n * 128, dtype=np.uint8)
        self._check(self.L.hg_aggregate_pk(self.ctx, _ptr(reqs), n, _ptr(words) if len(words) else None,
                                           len(words), _ptr(out), _ptr(codes)), "hg_aggregate_pk")
        return out.tobytes(), codes

    def combine_g1(self, a: bytes, b: bytes) -> Tuple[bytes, np.ndarray]:
        x, y = _u8(a), _u8(b)
        n = len(x) // 64
        out = np.zeros(n * 64, dtype=np.uint8)
        codes = np.zeros(n, dtype=np.int32)
        self._check(self.L.hg_combine_g1(self.ctx, _ptr(x), _ptr(y), n, _ptr(out), _ptr(codes)), "hg_combine_g1")
        return out.tobytes(), codes

    def combine_g2(self, a: bytes, b: bytes) -> Tuple[bytes, np.ndarray]:
        x, y = _u8(a), _u8(b)
        n = len(x) // 128
        out = np.zeros(n * 128, dtype=np.uint8)
        codes = np.zeros(n, dtype=np.int32)
        self._check(self.L.hg_combine_g2(self.ctx, _ptr(x), _ptr(y), n, _ptr(out), _ptr(codes)), "hg_combine_g2")
        return out.tobytes(), codes

    def pair(self, g1s: bytes, g2s: bytes) -> Tuple[bytes, np.ndarray]:
        x, y = _u8(g1s), _u8(g2s)
        n = len(x) // 64
        out = np.zeros(n * 384, dtype=np.uint8)
        codes = np.zeros(n, dtype=np.int32)
        self._check(self.L.hg_pair(self.ctx, _ptr(x), _ptr(y), n, _ptr(out), _ptr(codes)), "hg_pair")
        return out.tobytes(), codes

    def keygen(self, scalars_be: bytes) -> bytes:
        s = _u8(scalars_be)
        n = len(s) // 32
        out = np.zeros(n * 128, dtype=np.uint8)
        self._check(self.L.hg_keygen(self.ctx, _ptr(s), n, _ptr(out)), "hg_keygen")
        return out.tobytes()

    def sign(self, scalars_be: bytes) -> bytes:
        s = _u8(scalars_be)
        n = len(s) // 32
        out = np.zeros(n * 64, dtype=np.uint8)
        self._check(self.L.hg_sign(self.ctx, _ptr(s), n, _ptr(out)), "hg_sign")
        return out.tobytes()

    def sign_msg(self, msg: bytes, scalars_be: bytes) -> bytes:
        """SecretKey.Sign(msg) x n under one lock hold (hg_sign_msg); raises on EOF."""
        m, sc = _u8(msg), _u8(scalars_be)
        n = len(sc) // 32
        out = np.zeros(n * 64, dtype=np.uint8)
        rc = self.L.hg_sign_msg(self.ctx, _ptr(m) if len(m) else None, len(m), _ptr(sc) if n else None, n,
                                _ptr(out) if n else None)
        self._check(rc, "hg_sign_msg")
        return out.tobytes()

    def fp12_op(self, op: int, a: bytes, b: bytes = None) -> bytes:
        """Team Fp12 building-block probe (hg_debug_fp12); 384-byte GT marshals."""
        x = _u8(a)
        y = _u8(b) if b is not None else x
        n = len(x) // 384
        out = np.zeros(n * 384, dtype=np.uint8)
        self._check(self.L.hg_debug_fp12(self.ctx, op, _ptr(x), _ptr(y), n, _ptr(out)), "hg_debug_fp12")
        return out.tobytes()

    def fp_mul(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        n = a.shape[0]
        out = np.zeros((n, 8), dtype=np.uint32)
        self._check(self.L.hg_debug_fp_mul(self.ctx, _ptr(a), _ptr(b), n, _ptr(out)), "hg_debug_fp_mul")
        return out

    def timing_enable(self, on: bool = True):
        self._check(self.L.hg_timing_enable(self.ctx, int(on)), "hg_timing_enable")

    def timing_read(self) -> Tuple[float, int]:
        ms = ctypes.c_double()
        k = ctypes.c_int()
        self._check(self.L.hg_timing_read(self.ctx, ctypes.byref(ms), ctypes.byref(k)), "hg_timing_read")
        return ms.value, k.value

    def timing_read_phase(self, phase: int) -> Tuple[float, int]:
        ms = ctypes.c_double()
        k = ctypes.c_int()
        self._check(self.L.hg_timing_read_phase(self.ctx, int(phase), ctypes.byref(ms), ctypes.byref(k)),
                    "hg_timing_read_phase")
        return ms.value, k.value

    def sync(self):
        self._check(self.L.hg_sync(self.ctx), "hg_sync")


def _parse_outputs(n: int, stride: int):
    return (np.zeros(2 * n, dtype=REQ_DTYPE), np.zeros(2 * n * stride, dtype=np.uint64),
            np.zeros(2 * n * 64, dtype=np.uint8), np.zeros(2 * n, dtype=np.int32))


class Batcher:
    """The native launch-merging queue on one engine (hg_batcher_*): callers
    (one thread per Handel instance) submit single aggregate requests; a
    dispatcher thread merges what is queued into one launch per message.
    The engine must outlive the batcher."""

    def __init__(self, engine: Engine, max_batch: int = 4096, max_wait_us: int = 200):
        self.engine = engine
        self.L = engine.L
        h = ctypes.c_void_p()
        rc = self.L.hg_batcher_create(engine.ctx, max_batch, max_wait_us, ctypes.byref(h))
        if rc != 0:
            raise HandelGPUError(f"hg_batcher_create: code {rc}")
        self.b = h

    def close(self):
        if getattr(self, "b", None):
            self.L.hg_batcher_destroy(self.b)
            self.b = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def submit(self, msg: bytes, offset: int, bitlen: int, level_size: int, words, sig: bytes) -> int:
        """Queues one request (hg_batcher_submit); returns the ticket handle."""
        m = _u8(msg)
        req = np.array([(offset, bitlen, level_size, 0)], dtype=REQ_DTYPE)
        w = np.ascontiguousarray(words, dtype=np.uint64)
        if len(w) < (int(bitlen) + 63) // 64:  # hg_batcher_submit copies ceil(bitlen / 64) words
            raise ValueError(f"{bitlen} bits need {(int(bitlen) + 63) // 64} words, got {len(w)}")
        sg = _u8(sig)
        if len(sg) != 64:
            raise ValueError("signature must be 64 bytes")
        t = ctypes.c_void_p()
        rc = self.L.hg_batcher_submit(self.b, _ptr(m) if len(m) else None, len(m), _ptr(req),
                                      _ptr(w) if len(w) else None, _ptr(sg), ctypes.byref(t))
        if rc != 0:
            raise HandelGPUError(f"hg_batcher_submit: code {rc}")
        return t.value

    def wait(self, ticket: int) -> int:
        """The request's hg_code (hg_batcher_wait); releases the ticket."""
        code = ctypes.c_int32(-1)
        rc = self.L.hg_batcher_wait(self.b, ctypes.c_void_p(ticket), ctypes.byref(code))
        if rc != 0:
            raise HandelGPUError(f"hg_batcher_wait: code {rc}")
        return int(code.value)

    def verify(self, msg: bytes, offset: int, bitlen: int, level_size: int, words, sig: bytes) -> int:
        """One processing.go verifySignature through the queue (blocking)."""
        return self.wait(self.submit(msg, offset, bitlen, level_size, words, sig))

    def stats(self) -> Tuple[int, int]:
        """(batches launched, requests verified) so far."""
        b, r = ctypes.c_uint64(), ctypes.c_uint64()
        self.L.hg_batcher_stats(self.b, ctypes.byref(b), ctypes.byref(r))
        return b.value, r.value


class DeviceLane:
    """One hg_lane of an engine for batches already in HBM
    (hg_lane_submit_device): each lane has its own streams and workspaces over
    the engine's one registry and table set, so several lanes keep several
    batches in flight. pad=False: the unpadded pairing kernel (two batches'
    waves share the SIMDs). The engine must outlive the lane."""

    def __init__(self, engine: Engine, max_batch: int, pad: bool = True, overlap: bool = True):
        self.engine = engine
        self.L = engine.L
        h = ctypes.c_void_p()
        # staging capacity for host batches: 64 words (4096 bits) per request
        rc = self.L.hg_lane_create(engine.ctx, max_batch, max_batch * 64, 1 if overlap else 0, ctypes.byref(h))
        if rc != 0:
            raise HandelGPUError(f"hg_lane_create: code {rc}")
        self.h = h
        if not pad:
            engine._check(self.L.hg_lane_set_pairing_padding(self.h, 0), "hg_lane_set_pairing_padding")

    def set_latency_form(self, max_checks: int):
        """hg_lane_set_latency_form: padded batches of at most max_checks
        checks run the two-wave pairing kernel (0: never)."""
        self.engine._check(self.L.hg_lane_set_latency_form(self.h, int(max_checks)), "hg_lane_set_latency_form")

    def close(self):
        if getattr(self, "h", None):
            self.L.hg_lane_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def submit_device(self, d_reqs: int, n: int, d_words: int, d_sigs: int, d_codes: int, d_bits: int = 0,
                      stream: int = 0):
        """Enqueues the batch after `stream`'s earlier work; `stream` waits for its verdicts."""
        self.engine._check(self.L.hg_lane_submit_device(self.h, d_reqs, n, d_words, d_sigs, d_codes, d_bits or None,
                                                        stream or None), "hg_lane_submit_device")

    def wait(self):
        self.engine._check(self.L.hg_lane_wait(self.h), "hg_lane_wait")

    @property
    def stream(self) -> int:
        """The lane's launch stream (hipStream_t as int): as submit_device's
        `stream`, the batch is ordered only after the lane's own earlier ones."""
        return int(self.L.hg_lane_stream(self.h) or 0)


def requests_array(items: Sequence[Tuple[int, int, int, int]]) -> np.ndarray:
    return np.array(items, dtype=REQ_DTYPE)
