"""Batched replacement of Handel's evaluator verification.

processing.go's evaluatorProcessing verifies ONE incoming multisignature per
loop iteration (readTodos picks the best, verifyAndPublish checks it,
processing.go:171-287). `BatchVerifier` takes the same requests — a level,
its bitset and the aggregate signature — and verifies many per GPU launch:
the registry lives on the GPU, H(m) is computed once, and every request is a
(level range, bitset) -> aggregate key -> pairing check. Verdicts are a pure
function of (msg, range, bitset, sig), so batching cannot change them.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import partitioner as part
from ._lib import HG_ERR_SIG_UNMARSHAL, HG_OK
from .engine import REQ_DTYPE, Engine
from .sigprocessing import IncomingSig, MultiSig, bits_to_int, int_to_words


class BatchVerifier:
    def __init__(self, eng: Engine, registry_pks: bytes, msg: bytes, node_id: int = 0):
        self.eng = eng
        self.n = len(registry_pks) // 128
        codes = eng.registry_load(registry_pks)
        if codes.any():
            raise ValueError(f"registry key {int(np.flatnonzero(codes)[0])} fails to unmarshal")
        self.hash_rc = eng.set_message(msg)
        if self.hash_rc == 0:
            # the GT tables of aggregate verification for this message and
            # registry, now rather than in the first batch
            eng.prepare_aggregate()
        self.node_id = node_id

    def _pack(self, items):
        reqs = np.zeros(len(items), dtype=REQ_DTYPE)
        words: List[np.ndarray] = []
        nw = 0
        sigs = bytearray()
        for i, (lo, size, bits, sig) in enumerate(items):
            if isinstance(bits, MultiSig):
                w, bitlen = int_to_words(bits.bits, bits.bitlen), bits.bitlen
            else:
                w, bitlen = part.bits_to_words(bits), len(bits)
            reqs[i] = (lo, bitlen, size, nw)
            words.append(w)
            nw += len(w)
            s = bytes(sig)
            sigs += s[:64].ljust(64, b"\x00") if len(s) != 64 else s
        allw = np.concatenate(words) if words else np.zeros(0, dtype=np.uint64)
        return reqs, allw, bytes(sigs)

    def verify_levels(self, sigs: Sequence[IncomingSig]) -> List[Optional[str]]:
        """verifySignature (processing.go:342-368) for each incoming sig, as
        seen by node `node_id`; returns None or the reference's error text."""
        return self.verify_nodes([(self.node_id, s) for s in sigs])

    def verify_nodes(self, items_in: Sequence[Tuple[int, IncomingSig]]) -> List[Optional[str]]:
        """verify_levels for signatures addressed to different nodes of the
        same registry (several Handel instances in one process share a GPU
        context: sigprocessing.SharedBatcher)."""
        items, errs = [], []
        for node_id, s in items_in:
            try:
                lo, hi = part.range_level(node_id, self.n, s.level)
                items.append((lo, hi - lo, s.ms, s.ms.sig))
                errs.append(None)
            except part.PartitionerError as e:
                items.append((0, 0, [], bytes(64)))
                errs.append(str(e))
        codes = self.eng.verify_aggregate(*self._pack(items)) if items else []
        out = []
        for e, c in zip(errs, codes):
            if e is not None:
                out.append(e)
            elif c == HG_OK:
                out.append(None)
            else:
                # processing.go:350-352 returns the level error as is; only
                # VerifySignature's errors are wrapped "handel: ..." (:361-365)
                out.append(self.eng.processing_error_string(int(c)))
        return out

    def verify_packets(self, packets: Sequence[Tuple[int, bytes]]) -> List[Optional[str]]:
        """Packet-level batch: for each (level, MultiSig
        bytes) as handel.go:390-436 receives them, MultiSignature.Unmarshal
        (crypto.go:86-110: u16 length, WilffBitSet blob, 64-byte signature) on
        the host, then verifySignature for every well-formed packet in one GPU
        batch. Returns None or the error text the reference would log."""
        out: List[Optional[str]] = [None] * len(packets)
        todo, where = [], []
        for i, (level, buf) in enumerate(packets):
            try:
                bits, sig = part.multisig_unmarshal(buf)
            except ValueError as e:
                out[i] = str(e)
                continue
            if len(sig) != 64:  # x/crypto G1.Unmarshal wants exactly 64 bytes
                out[i] = self.eng.code_string(HG_ERR_SIG_UNMARSHAL)
                continue
            todo.append(IncomingSig(0, level, MultiSig(len(bits), bits_to_int(bits), sig)))
            where.append(i)
        for i, e in zip(where, self.verify_levels(todo) if todo else []):
            out[i] = e
        return out

    def verify_ranges(self, items) -> np.ndarray:
        """Raw codes for (offset, level_size, bits, sig) requests."""
        return self.eng.verify_aggregate(*self._pack(items))

    def verify_multisignature(self, bits: Sequence[bool], sig: bytes) -> Optional[str]:
        """crypto.go:120-137 VerifyMultiSignature over the whole registry
        (hg_verify_multisig: the size check and its error text are the C ABI's)."""
        return self.verify_multisignatures([(bits, sig)])[0]

    def verify_multisignatures(self, items) -> List[Optional[str]]:
        """VerifyMultiSignature for each (bits, sig) in one GPU batch."""
        words, bitlens, woffs, sigs = [], [], [], bytearray()
        nw = 0
        for bits, sig in items:
            w = part.bits_to_words(bits)
            words.append(w)
            bitlens.append(len(bits))
            woffs.append(nw)
            nw += len(w)
            s = bytes(sig)
            sigs += s[:64].ljust(64, b"\x00") if len(s) != 64 else s
        allw = np.concatenate(words) if words else np.zeros(0, dtype=np.uint64)
        codes = self.eng.verify_multisig(bitlens, woffs, allw, bytes(sigs))
        return [None if c == HG_OK else self.eng.code_string(int(c)) for c in codes]
