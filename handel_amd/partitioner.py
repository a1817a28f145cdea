"""Host-side mirror of the two pieces of Handel's protocol logic the batched
verifier needs: the binomial partitioner's level ranges and the willf bitset
layout. Both are integer bookkeeping."""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np


class PartitionerError(ValueError):
    pass


def log2_ceil(size: int) -> int:
    """utils.go:8-11 log2 = ceil(log2(size))."""
    r = 0
    while (1 << r) < size:
        r += 1
    return r


def range_level(node_id: int, size: int, level: int) -> Tuple[int, int]:
    """binomialPartitioner.rangeLevel (partitioner.go:133-178): [min, max) of
    the registry that node `node_id` contacts at `level`. Raises
    PartitionerError for an invalid or empty level."""
    bitsize = log2_ceil(size)
    if level < 0 or level > bitsize + 1:
        raise PartitionerError("handel: invalid level for computing candidate set")
    lo, hi = 0, 1 << bitsize
    inverse_idx = level - 1
    idx = bitsize - 1
    while idx >= inverse_idx and idx >= 0 and lo < hi:
        middle = (hi + lo) // 2
        bit = (node_id >> idx) & 1
        if (bit == 1) == (idx == inverse_idx):
            hi = middle
        else:
            lo = middle
        idx -= 1
    if lo >= size:
        raise PartitionerError("empty level")
    return lo, min(hi, size)


def level_sizes(node_id: int, size: int) -> List[Tuple[int, int, int]]:
    """(level, min, max) for every non-empty level 1..log2(size) (Partitioner.Levels)."""
    out = []
    for lvl in range(1, log2_ceil(size) + 1):
        try:
            lo, hi = range_level(node_id, size, lvl)
        except PartitionerError:
            continue
        out.append((lvl, lo, hi))
    return out


def bits_to_words(bits: Sequence[bool]) -> np.ndarray:
    """willf/bitset in-memory layout: bit i = word[i >> 6] bit (i & 63)."""
    b = np.asarray(bits, dtype=bool)
    n = len(b)
    nw = (n + 63) // 64
    padded = np.zeros(nw * 64, dtype=np.uint8)
    padded[:n] = b
    return np.packbits(padded.reshape(nw, 64)[:, ::-1], axis=1).view(">u8").astype(np.uint64).ravel()


def words_to_bits(words: np.ndarray, n: int) -> List[bool]:
    w = np.asarray(words, dtype=np.uint64)
    return [bool((int(w[i >> 6]) >> (i & 63)) & 1) for i in range(n)]


def bitset_marshal(bits: Sequence[bool]) -> bytes:
    """WilffBitSet.MarshalBinary (bitset.go:150-162): u16 BE bit length, then
    willf's blob (u64 BE length + u64 BE words)."""
    n = len(bits)
    out = n.to_bytes(2, "big") + n.to_bytes(8, "big")
    for w in bits_to_words(bits):
        out += int(w).to_bytes(8, "big")
    return out


def bitset_unmarshal(buf: bytes) -> List[bool]:
    """WilffBitSet.UnmarshalBinary (bitset.go:166-177)."""
    if len(buf) < 10:
        raise ValueError("bitset too short")
    n = int.from_bytes(buf[0:2], "big")
    blen = int.from_bytes(buf[2:10], "big")
    nw = (blen + 63) // 64
    if len(buf) < 10 + 8 * nw:
        raise ValueError("bitset truncated")
    words = np.array([int.from_bytes(buf[10 + 8 * i:18 + 8 * i], "big") for i in range(nw)], dtype=np.uint64)
    return words_to_bits(words, n)


def multisig_unmarshal(buf: bytes) -> Tuple[List[bool], bytes]:
    """MultiSignature.Unmarshal (crypto.go:86-110): (bits, signature bytes)."""
    if len(buf) < 2:
        raise ValueError("EOF")
    length = int.from_bytes(buf[0:2], "big")
    blob = buf[2:2 + length]
    if len(blob) < length:
        raise ValueError("bitset received smaller than expected")
    return bitset_unmarshal(blob), buf[2 + length:]


def multisig_marshal(bits: Sequence[bool], sig: bytes) -> bytes:
    """MultiSignature.MarshalBinary (crypto.go:65-82)."""
    bs = bitset_marshal(bits)
    return len(bs).to_bytes(2, "big") + bs + sig
