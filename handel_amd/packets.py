"""Host side of the packet intake (hg_parse_packets): Handel's wire packet
(net.go:34-44) and the batch layout the C ABI takes — every marshal in one
byte pool, one hg_packet record per packet naming its ranges and the Handel
instance that received it."""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import HG_OK, HG_PKT_HAS_IND, HG_PKT_NO_IND
from .engine import PACKET_DTYPE, Engine


@dataclass
class Packet:
    """net.go Packet: the sender, the level byte, the MultiSignature marshal
    (crypto.go:65-82) and the optional individual signature (nil = None)."""
    origin: int
    level: int
    multisig: bytes
    individual: Optional[bytes] = None


def pack_packets(packets: Sequence[Packet], receivers: Sequence[int]) -> Tuple[bytes, np.ndarray]:
    """(pool, hg_packet records) for a batch; receivers[i] is the id of the
    instance packet i arrived at."""
    if len(receivers) != len(packets):
        raise ValueError("one receiver per packet")
    pool = bytearray()
    recs = np.zeros(len(packets), dtype=PACKET_DTYPE)
    for i, (p, r) in enumerate(zip(packets, receivers)):
        recs[i]["origin"] = p.origin
        recs[i]["receiver"] = r
        recs[i]["level"] = p.level
        recs[i]["ms_off"] = len(pool)
        recs[i]["ms_len"] = len(p.multisig)
        pool += p.multisig
        if p.individual is not None:
            recs[i]["flags"] = HG_PKT_HAS_IND
            recs[i]["ind_off"] = len(pool)
            recs[i]["ind_len"] = len(p.individual)
            pool += p.individual
    return bytes(pool), recs


@dataclass
class Parsed:
    """One packet after Handel.NewPacket's parse: err is the reference's text
    ('' = accepted); ms / ind are (offset, bitlen, level_size, words, sig)
    verification requests (ind None when the packet carried none)."""
    err: str
    ms: Optional[tuple]
    ind: Optional[tuple]


def parse(eng: Engine, packets: Sequence[Packet], receivers: Sequence[int]) -> List[Parsed]:
    """Parses a batch on the GPU and unpacks it per packet."""
    pool, recs = pack_packets(packets, receivers)
    reqs, words, sigs, codes = eng.parse_packets(pool, recs)
    n = len(packets)
    out = []
    for i in range(n):
        c = int(codes[i])
        if c != HG_OK:
            out.append(Parsed(eng.packet_error(c, recs[i]), None, None))
            continue
        slots = []
        for k in (i, n + i):
            r = reqs[k]
            nw = (int(r["bitlen"]) + 63) // 64
            wo = int(r["word_offset"])
            slots.append((int(r["offset"]), int(r["bitlen"]), int(r["level_size"]), words[wo:wo + nw].copy(),
                          sigs[64 * k:64 * k + 64]))
        out.append(Parsed("", slots[0], None if int(codes[n + i]) == HG_PKT_NO_IND else slots[1]))
    return out
