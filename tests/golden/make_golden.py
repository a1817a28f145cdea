#!/usr/bin/env python3
"""Generates the committed golden vectors in tests/golden/ (test infrastructure).

The reference (Go, un-vendored golang.org/x/crypto/bn256 and cloudflare/bn256)
cannot be built or run in this environment and its own bn256 tests hold no
known-answer bytes, so these vectors are produced by the
pure-Python restatement `oracle/bn256_oracle.py`, whose algorithms follow the
reference's call sites (bn256/go/bn256.go, crypto.go, processing.go,
partitioner.go) and are pinned in tests/test_oracle.py by the reference's own
property tests and the published upstream constants. Every vector below is
data: inputs and the outputs the reference's code path returns for them.

Files written:
  bn256_vectors.json   curve / pairing / hash / sign / verify / combine /
                       unmarshal / multisig vectors (hex, codes = include/handel_gpu.h)
  registry_50.csv      a 50-node registry in simul/lib/parser.go's CSV layout
                       (id, addr, hex(sk.MarshalBinary), hex(pk.MarshalBinary))

Usage: python tests/golden/make_golden.py   (≈1 min, pure Python)
"""

from __future__ import annotations

import csv
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import bn256_oracle as O  # noqa: E402

SEED = b"handel-amd-golden-v1"
LIB_MESSAGE = b"Everything that is beautiful and noble is the product of reason and calculation."
N_REG = 50

# result codes (include/handel_gpu.h)
OK, SIG_INVALID, HASH_EOF, LEVEL, PK_UNMARSHAL, SIG_UNMARSHAL, EMPTY_AGG = range(7)
CF_EXCEEDS, CF_MALFORMED, CF_SHORT = 7, 8, 9

_ERR_TO_CODE = {
    None: OK,
    O.ERR_SIG_INVALID: SIG_INVALID,
    O.ERR_EOF: HASH_EOF,
    O.ERR_LEVEL: LEVEL,
    O.ERR_GO_PK_UNMARSHAL: PK_UNMARSHAL,
    O.ERR_GO_SIG_UNMARSHAL: SIG_UNMARSHAL,
    O.ERR_EMPTY_AGGREGATE: EMPTY_AGG,
    O.ERR_CF_EXCEEDS: CF_EXCEEDS,
    O.ERR_CF_MALFORMED: CF_MALFORMED,
    O.ERR_CF_NOT_ENOUGH: CF_SHORT,
}


def code_of(err) -> int:
    if err is not None and err.startswith("handel: ") and err != O.ERR_LEVEL:
        err = err[len("handel: "):]
    return _ERR_TO_CODE[err]


def hx(b: bytes) -> str:
    return b.hex()


def verify_code(pk_bytes: bytes, sig_bytes: bytes, msg: bytes, flavor: str = "go") -> int:
    """Reference precedence: pk unmarshal (registry/packet), sig unmarshal, then
    PublicKey.VerifySignature (bn256/go/bn256.go:82-94), two full pairings."""
    P, e1 = O.g2_unmarshal(pk_bytes, flavor)
    if e1 is not None:
        return PK_UNMARSHAL if flavor == "go" else code_of(e1)
    S, e2 = O.g1_unmarshal(sig_bytes, flavor)
    if e2 is not None:
        return SIG_UNMARSHAL if flavor == "go" else code_of(e2)
    return code_of(O.verify_signature(P, msg, S))


def main():
    reader = O.SeededReader(SEED)
    sks, pks = [], []
    for _ in range(N_REG):
        sk, pk = O.new_key_pair(reader)
        sks.append(sk)
        pks.append(pk)
    pk_bytes = [O.g2_marshal(p) for p in pks]

    # registry CSV (simul/lib/parser.go:105-155, nodes.go:25-40)
    with open(os.path.join(HERE, "registry_50.csv"), "w", newline="") as f:
        w = csv.writer(f)
        for i in range(N_REG):
            w.writerow([i, f"127.0.0.1:{3000 + i}", hx(O.sk_marshal(sks[i])), hx(pk_bytes[i])])

    out = {"generator": "tests/golden/make_golden.py", "seed": SEED.decode(), "oracle": "oracle/bn256_oracle.py",
           "codes": "include/handel_gpu.h hg_code", "registry_csv": "registry_50.csv"}

    # ---- curve and pairing (bn256.Pair(...).Marshal(), bn256/go/bn256.go:88-89)
    g1 = O.g1_marshal(O.G1_GEN)
    g2 = O.g2_marshal(O.G2_GEN)
    P5, Q9 = O.g1_mul(O.G1_GEN, 5), O.g2_mul(O.G2_GEN, 9)
    out["pair"] = [
        {"g1": hx(g1), "g2": hx(g2), "gt": hx(O.f12_marshal(O.pair(O.G1_GEN, O.G2_GEN)))},
        {"g1": hx(O.g1_marshal(P5)), "g2": hx(O.g2_marshal(Q9)), "gt": hx(O.f12_marshal(O.pair(P5, Q9)))},
        {"g1": hx(bytes(64)), "g2": hx(g2), "gt": hx(O.f12_marshal(O.F12_ONE))},
    ]

    # ---- hashedMessage (bn256/go/bn256.go:210-218)
    hashes = []
    for m in [LIB_MESSAGE, b"Peaches and Cream", b"Get Funky Tonight", b"Sun is Shining...",
              b"hello world", b"Hello World", b""]:
        h, err = O.hashed_message(m)
        hashes.append({"msg": hx(m), "h": None if h is None else hx(O.g1_marshal(h)), "code": code_of(err)})
    out["hash"] = hashes

    # ---- keygen / sign (NewKeyPair, SecretKey.Sign: bn256/go/bn256.go:129-154)
    h_lib, _ = O.hashed_message(LIB_MESSAGE)
    sigs = [O.g1_mul(h_lib, k) for k in sks]
    sig_bytes = [O.g1_marshal(s) for s in sigs]
    out["sign"] = {"msg": hx(LIB_MESSAGE), "sk": [hx(O.sk_marshal(k)) for k in sks], "pk": [hx(b) for b in pk_bytes],
                   "sig": [hx(b) for b in sig_bytes]}

    # ---- single-signature verification (config 2 shape, 1/8 tampered, plus edge cases)
    g1_pt = O.G1_GEN
    single = []
    for i in range(16):
        s = sigs[i]
        if i % 8 == 0:
            s = O.g1_add(s, g1_pt)
        sb = O.g1_marshal(s)
        single.append({"pk": hx(pk_bytes[i]), "sig": hx(sb), "msg": hx(LIB_MESSAGE),
                       "code": verify_code(pk_bytes[i], sb, LIB_MESSAGE)})
    off_g1 = (1).to_bytes(32, "big") + (1).to_bytes(32, "big")
    off_g2 = bytes(127) + b"\x01"
    edge = [
        (pk_bytes[0], sig_bytes[1]),   # wrong key
        (bytes(128), bytes(64)),       # infinity pk, infinity sig: GT 1 == GT 1
        (bytes(128), sig_bytes[2]),    # infinity pk
        (pk_bytes[3], bytes(64)),      # infinity sig
        (off_g2, sig_bytes[4]),        # pk off the twist
        (pk_bytes[5], off_g1),         # sig off the curve
        (pk_bytes[6], O.g1_marshal(O.g1_neg(sigs[6]))),  # negated sig
    ]
    for p, s in edge:
        single.append({"pk": hx(p), "sig": hx(s), "msg": hx(LIB_MESSAGE), "code": verify_code(p, s, LIB_MESSAGE)})
    # a hash-rejected message: every check fails with the hash error
    single.append({"pk": hx(pk_bytes[0]), "sig": hx(sig_bytes[0]), "msg": hx(b"hello world"),
                   "code": verify_code(pk_bytes[0], sig_bytes[0], b"hello world")})
    out["verify"] = single

    # ---- Combine (PublicKey.Combine bn256/go:97-105, SigBLS.Combine :192-200)
    out["combine_g2"] = [
        {"a": hx(pk_bytes[0]), "b": hx(pk_bytes[1]), "out": hx(O.g2_marshal(O.g2_add(pks[0], pks[1])))},
        {"a": hx(pk_bytes[2]), "b": hx(pk_bytes[2]), "out": hx(O.g2_marshal(O.g2_add(pks[2], pks[2])))},
        {"a": hx(pk_bytes[3]), "b": hx(O.g2_marshal(O.g2_neg(pks[3]))), "out": hx(bytes(128))},
        {"a": hx(bytes(128)), "b": hx(pk_bytes[4]), "out": hx(pk_bytes[4])},
    ]
    out["combine_g1"] = [
        {"a": hx(sig_bytes[0]), "b": hx(sig_bytes[1]), "out": hx(O.g1_marshal(O.g1_add(sigs[0], sigs[1])))},
        {"a": hx(sig_bytes[2]), "b": hx(sig_bytes[2]), "out": hx(O.g1_marshal(O.g1_add(sigs[2], sigs[2])))},
        {"a": hx(sig_bytes[3]), "b": hx(O.g1_marshal(O.g1_neg(sigs[3]))), "out": hx(bytes(64))},
        {"a": hx(bytes(64)), "b": hx(sig_bytes[4]), "out": hx(sig_bytes[4])},
    ]

    # ---- Unmarshal rules per flavor (bn256/go:113-120,179-190; bn256/cf:112-121,183-190)
    p_be = O.P.to_bytes(32, "big")
    unm = []
    g1_cases = [g1, bytes(64), off_g1, p_be + g1[32:], g1[:63]]
    g2_cases = [g2, bytes(128), off_g2, p_be + g2[32:], g2[:127]]
    for flavor in ("go", "cf"):
        for b in g1_cases:
            _, err = O.g1_unmarshal(b, flavor)
            unm.append({"kind": "g1", "flavor": flavor, "bytes": hx(b), "err": err})
        for b in g2_cases:
            _, err = O.g2_unmarshal(b, flavor)
            unm.append({"kind": "g2", "flavor": flavor, "bytes": hx(b), "err": err})
    out["unmarshal"] = unm

    # ---- multisignatures over the 50-node registry (processing.go:342-368,
    # crypto.go:59-137, partitioner.go:133-178), seen from node 3
    multis = []
    rng_reader = O.SeededReader(SEED + b"/bits")
    node = 3
    levels = []
    for lvl in range(1, O.log2_ceil(N_REG) + 1):
        rl, err = O.range_level(node, N_REG, lvl)
        if err is None:
            levels.append((lvl, rl[0], rl[1]))
    levels.append((None, 0, N_REG))  # VerifyMultiSignature over the whole registry
    for j, (lvl, lo, hi) in enumerate(levels):
        size = hi - lo
        rb = rng_reader.read_full(size)
        bits = [b >= 64 for b in rb]  # density ~3/4
        if j == 0:
            bits = [True] * size
        agg_sig = None
        for i, b in enumerate(bits):
            if b:
                agg_sig = sigs[lo + i] if agg_sig is None else O.g1_add(agg_sig, sigs[lo + i])
        if j == 2:  # one bad aggregate: + G1
            agg_sig = O.g1_add(agg_sig, g1_pt)
        status, agg_pk = O.aggregate_pk(pks[lo:hi], bits)
        err = O.verify_request(pks, lo, hi, bits, agg_sig, LIB_MESSAGE, fast=False)
        multis.append({"level": lvl, "lo": lo, "hi": hi, "bitlen": size,
                       "bitset": hx(O.bitset_marshal(bits)),
                       "multisig": hx(O.multisig_marshal(bits, agg_sig)),
                       "agg_pk": hx(O.g2_marshal(agg_pk)) if status == "ok" else None,
                       "agg_sig": hx(O.g1_marshal(agg_sig)), "code": code_of(err)})
    # empty bitset (the reference panics on the nil aggregate) and a bitlen != level size
    lvl, lo, hi = levels[3]
    bits = [False] * (hi - lo)
    multis.append({"level": lvl, "lo": lo, "hi": hi, "bitlen": hi - lo, "bitset": hx(O.bitset_marshal(bits)),
                   "multisig": hx(O.multisig_marshal(bits, sigs[0])), "agg_pk": None,
                   "agg_sig": hx(sig_bytes[0]), "code": EMPTY_AGG})
    bits = [True] * 3
    multis.append({"level": levels[2][0], "lo": levels[2][1], "hi": levels[2][2], "bitlen": 3,
                   "bitset": hx(O.bitset_marshal(bits)), "multisig": hx(O.multisig_marshal(bits, sigs[0])),
                   "agg_pk": None, "agg_sig": hx(sig_bytes[0]), "code": LEVEL})
    out["multisig"] = {"node": node, "registry_size": N_REG, "msg": hx(LIB_MESSAGE), "requests": multis}

    # ---- rangeLevel table for a 4000-node registry (config 3 level sizes)
    rl = []
    for nid in (0, 1, 2047, 2048, 3999):
        for lvl in range(0, O.log2_ceil(4000) + 2):
            r, err = O.range_level(nid, 4000, lvl)
            rl.append({"id": nid, "level": lvl, "range": list(r) if r else None, "err": err})
    out["range_level_4000"] = rl

    path = os.path.join(HERE, "bn256_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    with open(path, "rb") as f:
        print(path, len(f.read()), "bytes; sha256", hashlib.sha256(open(path, "rb").read()).hexdigest()[:16])


if __name__ == "__main__":
    main()
