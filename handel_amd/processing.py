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
from ._lib import HG_ERR_SIG_CF_SHORT, HG_ERR_SIG_UNMARSHAL, HG_OK
from .engine import REQ_DTYPE, Engine
from .sigprocessing import IncomingSig, MultiSig, int_to_words


def sig_length_code(flavor: str, sig: bytes) -> int:
    """SigBLS.UnmarshalBinary's length rule: x/crypto's G1.Unmarshal wants
    exactly 64 bytes (bn256/go/bn256.go:182-190 -> "bn256: multisig can't
    unmarshal"); cloudflare's wants at least 64 and ignores the rest
    (bn256/cf/bn256.go:183-190 -> "...: bn256: not enough data"). HG_OK when
    the length passes (the point itself is checked on the GPU)."""
    n = len(sig)
    if flavor in ("cf", "bn256/cf", "bn256"):
        return HG_ERR_SIG_CF_SHORT if n < 64 else HG_OK
    return HG_ERR_SIG_UNMARSHAL if n != 64 else HG_OK


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
        """items whose signature passes the length rule go into one batch
        (cloudflare's extra bytes dropped, as its Unmarshal does); the others
        keep their unmarshal code and are never submitted"""
        pre = np.array([sig_length_code(self.eng.flavor_name, bytes(it[3])) for it in items], dtype=np.int32)
        keep = [i for i in range(len(items)) if pre[i] == HG_OK]
        reqs = np.zeros(len(keep), dtype=REQ_DTYPE)
        words: List[np.ndarray] = []
        nw = 0
        sigs = bytearray()
        for j, i in enumerate(keep):
            lo, size, bits, sig = items[i]
            if isinstance(bits, MultiSig):
                w, bitlen = int_to_words(bits.bits, bits.bitlen), bits.bitlen
            else:
                w, bitlen = part.bits_to_words(bits), len(bits)
            reqs[j] = (lo, bitlen, size, nw)
            words.append(w)
            nw += len(w)
            sigs += bytes(sig)[:64]
        allw = np.concatenate(words) if words else np.zeros(0, dtype=np.uint64)
        return (reqs, allw, bytes(sigs)), pre, keep

    def _codes(self, items) -> np.ndarray:
        """codes of (offset, level_size, bits, sig) items: the length rule's
        unmarshal codes, the GPU's for the rest"""
        batch, codes, keep = self._pack(items)
        if keep:
            codes[np.array(keep)] = self.eng.verify_aggregate(*batch)
        return codes

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
        codes = self._codes(items) if items else []
        out = []
        for e, c in zip(errs, codes):
            if e is not None:
                out.append(e)
            elif c == HG_OK:
                out.append(None)
            elif c in (HG_ERR_SIG_UNMARSHAL, HG_ERR_SIG_CF_SHORT):
                # the signature never parses (MultiSignature.Unmarshal, crypto.go:86-110)
                out.append(self.eng.code_string(int(c)))
            else:
                # processing.go:350-352 returns the level error as is; only
                # VerifySignature's errors are wrapped "handel: ..." (:361-365)
                out.append(self.eng.processing_error_string(int(c)))
        return out

    def verify_packets(self, packets) -> List[Optional[str]]:
        """Handel.NewPacket -> processing -> verifySignature for packets that
        node `node_id` received: the parse step on the GPU
        (hg_parse_packets: validatePacket and parseSignatures, handel.go:
        371-436), then ONE verification batch over every accepted packet's
        multisignature. Items are packets.Packet, or (level, MultiSig bytes)
        pairs (then sent by the first id of the level range, without an
        individual signature). Returns None or the error text: the parse error
        the packet is dropped with (handel.go:134-141), else verifySignature's."""
        from .packets import Packet, pack_packets

        pk = []
        for p in packets:
            if not isinstance(p, Packet):
                level, buf = p
                try:
                    origin = part.range_level(self.node_id, self.n, level)[0]
                except part.PartitionerError:
                    origin = 0
                p = Packet(origin, level, bytes(buf))
            pk.append(p)
        out: List[Optional[str]] = [None] * len(pk)
        if not pk:
            return out
        pool, recs = pack_packets(pk, [self.node_id] * len(pk))
        reqs, words, sigs, codes = self.eng.parse_packets(pool, recs)
        ok = [i for i in range(len(pk)) if codes[i] == HG_OK]
        for i in range(len(pk)):
            if codes[i] != HG_OK:
                out[i] = self.eng.packet_error(int(codes[i]), recs[i])
        if ok:
            vsigs = b"".join(sigs[64 * i:64 * i + 64] for i in ok)
            for i, c in zip(ok, self.eng.verify_aggregate(reqs[np.array(ok)], words, vsigs)):
                out[i] = None if c == HG_OK else self.eng.processing_error_string(int(c))
        return out

    def verify_ranges(self, items) -> np.ndarray:
        """Raw codes for (offset, level_size, bits, sig) requests."""
        return self._codes(items)

    def verify_multisignature(self, bits: Sequence[bool], sig: bytes) -> Optional[str]:
        """crypto.go:120-137 VerifyMultiSignature over the whole registry
        (hg_verify_multisig: the size check and its error text are the C ABI's)."""
        return self.verify_multisignatures([(bits, sig)])[0]

    def verify_multisignatures(self, items) -> List[Optional[str]]:
        """VerifyMultiSignature for each (bits, sig) in one GPU batch."""
        codes = np.array([sig_length_code(self.eng.flavor_name, bytes(sig)) for _, sig in items], dtype=np.int32)
        keep = [i for i in range(len(items)) if codes[i] == HG_OK]
        words, bitlens, woffs, sigs = [], [], [], bytearray()
        nw = 0
        for i in keep:
            bits, sig = items[i]
            w = part.bits_to_words(bits)
            words.append(w)
            bitlens.append(len(bits))
            woffs.append(nw)
            nw += len(w)
            sigs += bytes(sig)[:64]
        allw = np.concatenate(words) if words else np.zeros(0, dtype=np.uint64)
        if keep:
            codes[np.array(keep)] = self.eng.verify_multisig(bitlens, woffs, allw, bytes(sigs))
        return [None if c == HG_OK else self.eng.code_string(int(c)) for c in codes]
