"""Deterministic fixture builders for the parity tests (test infrastructure).

Keys come from a seeded reader fed to the NewKeyPair rule
and signatures from SecretKey.Sign, both computed by the oracle; nothing here
is used by the product path.
"""

from __future__ import annotations

import hashlib

import numpy as np

from oracle import bn256_oracle as O
from oracle import ref_lib as R

LIB_MESSAGE = (b"Everything that is beautiful and noble is the product of reason and calculation."
               )  # simul/lib/config.go:37 lib.Message (81 bytes)
TEST_MESSAGES = [b"Peaches and Cream", b"Get Funky Tonight", b"Sun is Shining..."]
REJECT_MESSAGES = [b"hello world", b"Hello World"]


def scalars(n: int, seed: bytes = b"handel-amd") -> list:
    """n secret keys drawn by the RandomG2 rule from a SHA-256 counter reader."""
    r = O.SeededReader(seed)
    out = []
    for _ in range(n):
        k, err = O.random_scalar(r)
        assert err is None
        out.append(k)
    return out


def scalar_bytes(ks) -> bytes:
    return b"".join(k.to_bytes(32, "big") for k in ks)


def keys_and_sigs(n: int, msg: bytes = LIB_MESSAGE, seed: bytes = b"handel-amd"):
    ks = scalars(n, seed)
    kb = scalar_bytes(ks)
    pks = R.g2_scalar_base(kb)
    sigs = R.sign(msg, kb)
    return ks, pks, sigs


def tamper(sigs: bytes, every: int = 8) -> bytes:
    """Adds G1 to every `every`-th signature (config 2: 1/8 tampered)."""
    g1 = O.g1_marshal(O.G1_GEN)
    out = bytearray(sigs)
    for i in range(0, len(sigs) // 64, every):
        out[64 * i:64 * i + 64] = R.g1_add(bytes(sigs[64 * i:64 * i + 64]), g1)
    return bytes(out)


def random_bitsets(rng: np.random.Generator, sizes, density=(0.5, 1.0)):
    out = []
    for s in sizes:
        d = rng.uniform(*density)
        bits = rng.random(s) < d
        out.append([bool(b) for b in bits])
    return out


def pack_requests(ranges, bitsets):
    """(offset, level_size) ranges + bit lists -> (reqs tuples, words array)."""
    reqs = []
    words = []
    for (off, size), bits in zip(ranges, bitsets):
        w = O.bitset_words(bits)
        reqs.append((off, len(bits), size, len(words)))
        words.extend(w)
    return reqs, np.array(words, dtype=np.uint64)


def digest(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def non_g2_points(k: int, seed: int = 1) -> list:
    """k twist points outside the order-n subgroup G2 (random x, y = sqrt(x^3 + b')):
    keys x/crypto's G2.Unmarshal accepts (bn256/go/bn256.go:113-120) and
    cloudflare's rejects."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < k:
        x = (int.from_bytes(rng.bytes(32), "big") % O.P, int.from_bytes(rng.bytes(32), "big") % O.P)
        q = O.twist_point(x)
        if q is not None and not O.g2_in_subgroup(q):
            out.append(q)
    return out
