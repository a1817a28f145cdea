"""Packet intake (hg_parse_packets), CPU side: the restatement of Handel's
packet parse (oracle.bn256_oracle.parse_packet) against the reference's own
tests of that code (handel_test.go:335-406, crypto_test.go:9-24,
bitset_test.go:52-64) and the committed vectors, and the host packing."""

import importlib.util
import json
import os

import numpy as np
import pytest

from oracle import bn256_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def pv():
    with open(os.path.join(GOLD, "packet_vectors.json")) as f:
        return json.load(f)["cases"]


def test_generator_reproduces_committed_vectors(tmp_path, monkeypatch):
    spec = importlib.util.spec_from_file_location("make_packets", os.path.join(GOLD, "make_packets.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    monkeypatch.setattr(mod, "HERE", str(tmp_path))
    mod.main()
    with open(os.path.join(GOLD, "packet_vectors.json"), "rb") as f1, open(tmp_path / "packet_vectors.json", "rb") as f2:
        assert f1.read() == f2.read()


def test_reference_parse_packet_expectations(pv):
    """TestHandelParsePacket: packets 0, 1, 2, 4 rejected (validatePacket or
    parseSignatures), packet 3 accepted; the marshalling tests' bitsets round
    trip (bits and the u16 length)."""
    by = {c["name"]: c for c in pv}
    assert by["ref:origin 65000"]["err"]
    assert by["ref:level 254"]["err"]
    assert by["ref:multisig 0x01"]["err"]
    assert by["ref:correct level 2"]["err"] == ""
    assert by["ref:5-bit bitset at level 2"]["err"]
    a, b = by["ref:multisig 10 bits {1, 9}"], by["ref:bitset 10 bits {1, 4}"]
    assert a["err"] == b["err"] == ""
    assert (a["bitlen"], int(a["bits"], 16)) == (10, (1 << 1) | (1 << 9))
    assert (b["bitlen"], int(b["bits"], 16)) == (10, (1 << 1) | (1 << 4))


def test_error_order_follows_the_reference(pv):
    """validatePacket before parseSignatures; inside it the wire parse, the
    signature, the bit length, the empty set, then the individual signature."""
    by = {c["name"]: c for c in pv}
    assert by["origin -1"]["err"] == O.ERR_PKT_ORIGIN
    assert by["level 0"]["err"] == O.ERR_PKT_LEVEL % 0
    assert by["empty level (N = 5, id 4, level 2)"]["err"] == O.ERR_PKT_LEVEL % 2
    assert by["go: individual, bad multisig first"]["err"] == O.ERR_PKT_BITSET_SIZE
    assert by["cf: sig x >= p"]["err"].endswith("coordinate exceeds modulus")
    assert by["go: sig x >= p"]["err"] == ""  # x/crypto takes coordinates mod p
    assert by["willf length 2^60 (type mismatch)"]["err"] == O.ERR_PKT_TYPE_MISMATCH
    assert by["willf words cut"]["err"] == O.ERR_READ_UNEXPECTED_EOF
    assert by["willf words missing"]["err"] == O.ERR_READ_EOF
    # the empty-set check sees willf's whole words, BitSet.Get only bits < w.l
    assert by["bits only past w.l (not None)"]["err"] == "" and by["bits only past w.l (not None)"]["bits"] == "0x0"
    assert by["willf shorter than w.l"]["bits"] == "0x1"


def test_oracle_matches_handel_mirror():
    """handel_amd.partitioner's wire helpers (the host mirror) agree with the
    restatement on a well-formed packet."""
    from handel_amd import partitioner as HP

    bits = [True, False, True] + [False] * 60 + [True]
    s = O.g1_marshal(O.g1_mul(O.G1_GEN, 3))
    wire = HP.multisig_marshal(bits, s)
    assert wire == O.multisig_marshal(bits, O.g1_mul(O.G1_GEN, 3))
    got_bits, got_sig = HP.multisig_unmarshal(wire)
    assert got_bits == bits and got_sig == s
    r = O.parse_packet(128, "go", 0, 64, 7, wire)
    assert r["err"] is None and r["range"] == (64, 128) and r["bitlen"] == 64


def test_pack_packets_layout():
    from handel_amd.engine import PACKET_DTYPE
    from handel_amd.packets import Packet, pack_packets

    ps = [Packet(3, 2, b"abc"), Packet(-1, 7, b"", b"x" * 64), Packet(5, 1, b"zz", None)]
    pool, recs = pack_packets(ps, [1, 2, 3])
    assert recs.dtype == PACKET_DTYPE and PACKET_DTYPE.itemsize == 32
    assert pool == b"abc" + b"x" * 64 + b"zz"
    assert list(recs["ms_off"]) == [0, 3, 67] and list(recs["ms_len"]) == [3, 0, 2]
    assert list(recs["flags"]) == [0, 1, 0] and recs[1]["ind_off"] == 3 and recs[1]["ind_len"] == 64
    assert list(recs["origin"]) == [3, -1, 5] and list(recs["receiver"]) == [1, 2, 3]
    with pytest.raises(ValueError):
        pack_packets(ps, [1])
