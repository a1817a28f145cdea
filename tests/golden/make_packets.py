#!/usr/bin/env python3
"""Generates tests/golden/packet_vectors.json (test infrastructure): Handel
packets and the result of Handel.NewPacket's parse step for them, from the
pure-Python restatement `oracle.bn256_oracle.parse_packet` (handel.go:371-436,
crypto.go:86-110, bitset.go:166-177, willf/bitset v1.1.10 ReadFrom).

The reference's own tests fix the expected accept/reject of the cases marked
"ref:" (handel_test.go:335-406 TestHandelParsePacket, crypto_test.go:9-24
TestMultiSignatureMarshalling, bitset_test.go:52-64 TestBitSetWilffMarshalling);
the exact error texts, the bit masking and the willf corner cases come from
the restatement alone (the Go reference cannot run here: parity of those is
unpinned by the reference, pinned to the restatement).

Usage: python tests/golden/make_packets.py   (a few seconds)
"""

from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import bn256_oracle as O  # noqa: E402

SEED = 20261017


def sig(k: int) -> bytes:
    return O.g1_marshal(O.g1_mul(O.G1_GEN, k))


def willf_blob(wl: int, flen: int, words) -> bytes:
    return wl.to_bytes(2, "big") + flen.to_bytes(8, "big") + b"".join(w.to_bytes(8, "big") for w in words)


def ms_raw(blob: bytes, s: bytes) -> bytes:
    return len(blob).to_bytes(2, "big") + blob + s


def multisig(bits, s: bytes) -> bytes:
    return ms_raw(O.bitset_marshal(bits), s)


def case(name, nreg, flavor, receiver, origin, level, ms, ind=None):
    r = O.parse_packet(nreg, flavor, receiver, origin, level, ms, ind)
    return {"name": name, "nreg": nreg, "flavor": flavor, "receiver": receiver, "origin": origin, "level": level,
            "ms": ms.hex(), "ind": None if ind is None else ind.hex(), "err": r["err"] or "",
            "range": list(r["range"]), "bitlen": r["bitlen"], "bits": hex(r["bits"]), "sig": r["sig"].hex(),
            "ind_bit": r["ind_bit"]}


def main():
    rnd = random.Random(SEED)
    s1, s2 = sig(5), sig(7)
    off_curve = (1).to_bytes(32, "big") + (3).to_bytes(32, "big")  # 9 != 1 + 3
    over_p = (O.P + 1).to_bytes(32, "big") + (2).to_bytes(32, "big")
    out = []
    # ref: TestHandelParsePacket (n = 16, receiver 1, shuffling off)
    full2 = multisig([True, True], s1)
    full5 = multisig([True] * 5, s1)
    out += [case("ref:origin 65000", 16, "go", 1, 65000, 0, full2),
            case("ref:level 254", 16, "go", 1, 3, 254, full2),
            case("ref:multisig 0x01", 16, "go", 1, 3, 1, b"\x01"),
            case("ref:correct level 2", 16, "go", 1, 3, 2, full2),
            case("ref:5-bit bitset at level 2", 16, "go", 1, 3, 2, full5)]
    # ref: TestMultiSignatureMarshalling / TestBitSetWilffMarshalling (10-bit
    # bitsets: the top level of ids 0..15 in a 26-node registry)
    b10 = [i in (1, 9) for i in range(10)]
    b10b = [i in (1, 4) for i in range(10)]
    out += [case("ref:multisig 10 bits {1, 9}", 26, "go", 0, 16, 5, multisig(b10, s1)),
            case("ref:bitset 10 bits {1, 4}", 26, "cf", 3, 20, 5, multisig(b10b, s2))]
    # validatePacket
    out += [case("origin -1", 16, "go", 1, -1, 2, full2),
            case("origin == N", 16, "go", 1, 16, 2, full2),
            case("level 0", 16, "go", 1, 3, 0, full2),
            case("level MaxLevel + 1", 16, "go", 1, 3, 5, full2),
            case("empty level (N = 5, id 4, level 2)", 5, "go", 4, 0, 2, full2),
            case("level MaxLevel", 16, "go", 1, 9, 4, multisig([True] * 8, s1))]
    # MultiSignature.Unmarshal / WilffBitSet / willf ReadFrom
    good = O.bitset_marshal([True, False])
    out += [case("empty multisig", 16, "go", 1, 3, 2, b""),
            case("blob length cut", 16, "go", 1, 3, 2, len(good).to_bytes(2, "big") + good[:-1]),
            case("blob length 0", 16, "go", 1, 3, 2, ms_raw(b"", s1)),
            case("blob length 1", 16, "go", 1, 3, 2, ms_raw(b"\x00", s1)),
            case("no willf length", 16, "go", 1, 3, 2, ms_raw(b"\x00\x02", s1)),
            case("willf length cut", 16, "go", 1, 3, 2, ms_raw(b"\x00\x02\x00\x00\x00", s1)),
            case("willf words missing", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 2, []), s1)),
            case("willf words cut", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 70, [3])[:-3], s1)),
            case("willf length 2^60 (type mismatch)", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 1 << 60, []), s1)),
            case("willf length 2^64-1", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, (1 << 64) - 1, []), s1)),
            case("willf length 0, no words", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 0, []), s1)),
            case("willf shorter than w.l", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 1, [3]), s1)),
            case("willf longer than w.l", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 128, [7, 1]), s1)),
            case("bits only past w.l (not None)", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 64, [4]), s1)),
            case("bits only past willf length", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 1, [2]), s1)),
            case("trailing blob bytes", 16, "go", 1, 3, 2, ms_raw(willf_blob(2, 2, [1]) + b"\xff" * 5, s1)),
            case("none set", 16, "go", 1, 3, 2, multisig([False, False], s1)),
            case("bitset size", 16, "go", 1, 3, 2, multisig([True] * 3, s1))]
    # signatures, per flavor
    for fl in ("go", "cf"):
        out += [case(f"{fl}: sig 63 B", 16, fl, 1, 3, 2, multisig([True, True], s1[:63])),
                case(f"{fl}: sig 65 B", 16, fl, 1, 3, 2, multisig([True, True], s1 + b"\x00")),
                case(f"{fl}: sig empty", 16, fl, 1, 3, 2, multisig([True, True], b"")),
                case(f"{fl}: sig off curve", 16, fl, 1, 3, 2, multisig([True, True], off_curve)),
                case(f"{fl}: sig x >= p", 16, fl, 1, 3, 2, multisig([True, True], over_p)),
                case(f"{fl}: sig infinity", 16, fl, 1, 3, 2, multisig([True, True], bytes(64))),
                case(f"{fl}: individual ok", 16, fl, 1, 3, 2, full2, s2),
                case(f"{fl}: individual bad", 16, fl, 1, 3, 2, full2, off_curve),
                case(f"{fl}: individual short", 16, fl, 1, 3, 2, full2, s2[:10]),
                case(f"{fl}: individual, origin outside the level", 16, fl, 1, 9, 2, full2, s2),
                case(f"{fl}: individual, bad multisig first", 16, fl, 1, 9, 2, multisig([True], s1), off_curve)]
    # random Handel-shaped packets (N = 4000: levels up to 2048 bits)
    n = 4000
    pts = [sig(k) for k in range(2, 10)]
    for t in range(48):
        recv = rnd.randrange(n)
        lv = O.log2_ceil(n)
        levels = [(l, O.range_level(recv, n, l)[0]) for l in range(1, lv + 1) if O.range_level(recv, n, l)[0]]
        level, (lo, hi) = rnd.choice(levels)
        bits = [rnd.random() < rnd.uniform(0.3, 1.0) for _ in range(hi - lo)]
        origin = rnd.randrange(lo, hi) if rnd.random() < 0.8 else rnd.randrange(n)
        ind = pts[t % 8] if rnd.random() < 0.5 else None
        out.append(case(f"random {t}", n, "go" if t % 2 == 0 else "cf", recv, origin, level,
                        multisig(bits, pts[(t + 3) % 8]), ind))
    path = os.path.join(HERE, "packet_vectors.json")
    with open(path, "w") as f:
        json.dump({"source": "oracle/bn256_oracle.py parse_packet", "cases": out}, f, indent=0)
    print(path, len(out), "cases")


if __name__ == "__main__":
    main()
